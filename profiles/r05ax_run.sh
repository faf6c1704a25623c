set -o pipefail
# what-if: the pull kernel beside the SSSP (default) vs in order before it
D=gpurun_out/r05ax; mkdir -p $D
for m in 1 0 1 0; do
  OPENR_SPF_WHATIF_HEAVY_STREAM=$m timeout -k 10 200 python3 profiles/whatif_probe.py 5 > $D/probe_$m.json 2> $D/probe_$m.err || exit 3
  python3 -c "import json; d=json.load(open('$D/probe_$m.json')); print('side=$m', {k: d.get(k) for k in ('ms','device_ms','value','parity_check')})"
done
