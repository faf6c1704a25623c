set -o pipefail
# round 4: held next-hop pass with non-temporal mask / distance-row stores (A/B)
D=gpurun_out/r04ao; mkdir -p $D
B="bench.py --no-cpu-baseline --no-route-db --no-whatif --no-wan --steps 20 --warmup 3"
for i in 1 2; do
for n in 1 0; do
OPENR_NL_NT=$n timeout -k 10 300 python3 $B > $D/fabric_nt$n.$i.json 2> $D/fabric_nt$n.$i.err || { tail -5 $D/fabric_nt$n.$i.err; exit 2; }
python3 -c "import json,sys; d=json.load(open('$D/fabric_nt$n.$i.json')); print('nt=$n', d['value'], d['ms_per_step'], {k: v['avg_ms'] for k, v in d['kernels'].items()})"
done
done
OPENR_NL_NT=1 timeout -k 10 300 python -u -m pytest tests/test_abi_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $D/abi_nt.log 2>&1 || { tail -15 $D/abi_nt.log; exit 3; }
tail -1 $D/abi_nt.log
