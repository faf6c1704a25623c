set -o pipefail
# round 4: link-flap RouteDb with the parallel engine flatten (+ parity tests of the engine)
D=gpurun_out/r04r; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_routedb_golden_gpu.py tests/test_engine_parity_gpu.py tests/test_trace_paths_gpu.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1; rc=$?
tail -2 $D/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 profiles/linkflap_probe.py > $D/linkflap.log 2>&1 || exit 3
grep '^{' $D/linkflap.log
