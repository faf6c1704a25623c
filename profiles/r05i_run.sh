set -o pipefail
# round 5: link-flap update breakdown (spf_graph_update phases, splice, memo
# screen) and the v2 pass's store floor (OPENR_NL_V2_DBG bit 3: stores only)
D=gpurun_out/r05i; mkdir -p $D
OPENR_SPF_CREATE_TIMING=1 timeout -k 10 300 python3 profiles/linkflap_probe.py > $D/linkflap.json 2> $D/linkflap.err || { tail -5 $D/linkflap.err; exit 4; }
python3 -c "import json; d=json.load(open('$D/linkflap.json')); print({k: d.get(k) for k in ('ms_median','update_ms_median','build_ms_median','parity_check','per_build_us')})"
grep "spf_graph_update" $D/linkflap.err | tail -9
B="bench.py --no-cpu-baseline --no-route-db --no-whatif --no-wan --steps 20 --warmup 3"
for v in 0 8 9 10; do
OPENR_NL_V2_ORDER=3 OPENR_NL_V2_DBG=$v timeout -k 10 300 python3 $B > $D/fabric.d$v.json 2> $D/fabric.d$v.err || { tail -5 $D/fabric.d$v.err; exit 2; }
python3 -c "import json,sys; d=json.load(open('$D/fabric.d$v.json')); print('dbg=$v', d['ms_per_step'], {k: v['avg_ms'] for k, v in d['kernels'].items()})"
done
