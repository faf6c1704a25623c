set -o pipefail
# round 6: where the v2 pass's time goes (measurement modes), and the
# shallow A/B once more on this box
D=gpurun_out/r06e; mkdir -p $D
timeout -k 10 300 python3 profiles/nl_dbg_probe.py 20 3 > $D/nl_dbg.json 2> $D/nl_dbg.err || { tail -20 $D/nl_dbg.err; exit 2; }
cat $D/nl_dbg.json
timeout -k 10 300 python3 profiles/nl_ab.py 20 4 OPENR_NL_SHALLOW > $D/shallow_ab.json 2> $D/shallow_ab.err || { tail -20 $D/shallow_ab.err; exit 3; }
python3 -c "import json; d=json.load(open('$D/shallow_ab.json')); print({k:v for k,v in d.items() if k!='raw'})"
