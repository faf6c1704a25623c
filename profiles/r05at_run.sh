set -o pipefail
# v2 next-hop pass: item-major (4) vs the XCD class map (5), same box, A/B/A/B
D=gpurun_out/r05at; mkdir -p $D
B="bench.py --no-cpu-baseline --no-route-db --no-whatif --no-wan --steps 20 --warmup 3"
OPENR_NL_V2_ORDER=5 timeout -k 10 600 python -u -m pytest tests/test_config_sized_gpu.py -k "fabric" -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -30 $D/gpu_tests.log; exit 2; }
tail -1 $D/gpu_tests.log
for o in 4 5 4 5; do
  OPENR_NL_V2_ORDER=$o timeout -k 10 200 python3 $B > $D/fabric.o$o.json 2> $D/fabric.o$o.err || exit 3
  python3 -c "import json; b=json.loads(open('$D/fabric.o$o.json').read().strip().splitlines()[-1]); print('order $o', b['ms_per_step'], b['kernels'])"
done
