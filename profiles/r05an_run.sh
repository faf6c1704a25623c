set -o pipefail
# what-if repair stats per area (OPENR_SPF_WHATIF_STATS=1)
D=gpurun_out/r05an; mkdir -p $D
OPENR_SPF_WHATIF_STATS=1 timeout -k 10 300 python3 profiles/whatif_probe.py 2 > $D/probe.json 2> $D/probe.err || { tail -5 $D/probe.err; exit 3; }
grep "whatif" $D/probe.err | tail -8
python3 -c "import json; d=json.load(open('$D/probe.json')); print({k: d.get(k) for k in ('ms','device_ms','screened_queries','per_area')})"
