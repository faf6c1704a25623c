set -o pipefail
# round 5: where the v2 next-hop pass spends its time (measurement knobs:
# OPENR_NL_V2_DBG bit 0 = no solo items, 1 = no groups, 2 = no stores)
D=gpurun_out/r05d; mkdir -p $D
B="bench.py --no-cpu-baseline --no-route-db --no-whatif --no-wan --steps 20 --warmup 3"
for v in 0 1 2 4 3 5 6; do
OPENR_NL_V2_DBG=$v timeout -k 10 300 python3 $B > $D/fabric.d$v.json 2> $D/fabric.d$v.err || { tail -5 $D/fabric.d$v.err; exit 2; }
python3 -c "import json,sys; d=json.load(open('$D/fabric.d$v.json')); print('dbg=$v', d['ms_per_step'], {k: v['avg_ms'] for k, v in d['kernels'].items()}, d.get('parity_spot_check'))"
done
