set -o pipefail
# round 6: patch kernel persistent-grid sweep (ticks + batch ms)
D=gpurun_out/r06k; mkdir -p $D
for GR in 1024 256 4096; do
  OPENR_SPF_WHATIF_PATCH_GRID=$GR OPENR_SPF_WHATIF_STATS=1 timeout -k 10 300 python3 profiles/whatif_probe.py 1 > $D/wi_stats$GR.json 2> $D/wi_stats$GR.err || { tail -20 $D/wi_stats$GR.err; exit 4; }
  grep "whatif patch" $D/wi_stats$GR.err | tail -2
  OPENR_SPF_WHATIF_PATCH_GRID=$GR timeout -k 10 300 python3 profiles/whatif_probe.py 5 > $D/wi$GR.json 2> $D/wi$GR.err || { tail -20 $D/wi$GR.err; exit 3; }
  python3 -c "import json; d=json.loads(open('$D/wi$GR.json').read().strip().splitlines()[-1]); print('grid=$GR', d['ms'], d['device_ms'], d['value'], d['parity_check'])"
done
