set -o pipefail
# round 4: link flaps in place in LinkState (patchStructure) -- engine parity vs the oracle,
# RouteDb goldens (incl. link flaps), then the link-flap RouteDb loop
D=gpurun_out/r04s; mkdir -p $D
timeout -k 10 700 python -u -m pytest tests/test_engine_parity_gpu.py tests/test_routedb_golden_gpu.py tests/test_trace_paths_gpu.py \
  tests/test_all_sources_table_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1; rc=$?
tail -3 $D/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 profiles/linkflap_probe.py > $D/linkflap.log 2>&1 || exit 3
grep '^{' $D/linkflap.log
