set -o pipefail
# round 5: the v2 pass's store floor by block order and by stream
# (OPENR_NL_V2_DBG 8 = stores only; +16 no distance rows; +32 no masks)
D=gpurun_out/r05j; mkdir -p $D
B="bench.py --no-cpu-baseline --no-route-db --no-whatif --no-wan --steps 20 --warmup 3"
for cfg in "3 8" "4 8" "1 8" "3 24" "3 40" "4 24" "4 40" "3 0" "4 0" "3 9" "3 10" "4 9" "4 10"; do
set -- $cfg
OPENR_NL_V2_ORDER=$1 OPENR_NL_V2_DBG=$2 timeout -k 10 300 python3 $B > $D/fabric.o$1.d$2.json 2> $D/fabric.o$1.d$2.err || { tail -5 $D/fabric.o$1.d$2.err; exit 2; }
python3 -c "import json,sys; d=json.load(open('$D/fabric.o$1.d$2.json')); print('order=$1 dbg=$2', d['ms_per_step'], {k: v['avg_ms'] for k, v in d['kernels'].items()}, d.get('parity_spot_check'))"
done
