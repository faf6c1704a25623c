set -o pipefail
# final bench line at HEAD (gteps moved under "derived") + smoke
D=gpurun_out/r06bc; mkdir -p $D
timeout -k 10 600 python3 bench.py > $D/bench_full.json 2> $D/bench_full.err || { tail -20 $D/bench_full.err; exit 3; }
python3 -c "
import json; b=json.loads(open('$D/bench_full.json').read().strip().splitlines()[-1])
print(b['metric'], b['value'], b['ms_per_step'], b['roofline']['frac'], 'gteps' in json.dumps({k: v for k, v in b.items() if k != 'derived' and k != 'table_path'}), b['derived'])"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 5; }
tail -1 $D/smoke.log
