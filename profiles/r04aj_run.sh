set -o pipefail
# round 4: plain MS-BFS instance (ignore / wrec / zero-metric paths compiled
# out: 320 -> 100 B scratch) vs the general one, fabric step A/B/A/B
D=gpurun_out/r04aj; mkdir -p $D
B="bench.py --no-cpu-baseline --no-route-db --no-whatif --no-wan --steps 20 --warmup 3"
for i in 1 2; do
for g in 0 1; do
OPENR_MS_GEN=$g timeout -k 10 300 python3 $B > $D/fabric_gen$g.$i.json 2> $D/fabric_gen$g.$i.err || { tail -5 $D/fabric_gen$g.$i.err; exit 2; }
python3 -c "import json,sys; d=json.load(open('$D/fabric_gen$g.$i.json')); print('gen=$g', d['value'], d['ms_per_step'], d.get('kernels') or {k:v for k,v in d.items() if 'ms' in k and not isinstance(v,(dict,list))})"
done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -15 $D/gpu_tests.log; exit 3; }
tail -1 $D/gpu_tests.log
