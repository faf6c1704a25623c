set -o pipefail
# round 4: A/B of the held next-hop kernel's block order (OPENR_NL_ORDER=0 chunk-major
# default vs 1 XCD-contiguous, cost-balanced source ranges) on the fabric step, with
# the bench's own parity spot check and the all-sources parity tests under ORDER=1
D=gpurun_out/r04v; mkdir -p $D
B="bench.py --no-cpu-baseline --no-route-db --no-whatif --no-wan --steps 30 --warmup 5"
for o in 0 1 0 1; do
  OPENR_NL_ORDER=$o timeout -k 10 200 python3 $B > $D/bench_o$o.json 2> $D/bench_o$o.err || exit 3
  python3 -c "import json;d=json.load(open('$D/bench_o$o.json'));print('order $o', d['ms_per_step'], d['value'], d['kernels'], d['parity_spot_check'])"
done
OPENR_NL_ORDER=1 timeout -k 10 400 python -u -m pytest tests/test_abi_gpu.py -k "all_sources or fabric or msbfs" tests/test_config_sized_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/tests_o1.log 2>&1; rc=$?
tail -2 $D/tests_o1.log
exit $rc
