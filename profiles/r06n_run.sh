set -o pipefail
# AllSourcesTable with several source blocks (halo rows for next hops)
D=gpurun_out/r06n; mkdir -p $D
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_all_sources_table_gpu.py > $D/gpu_tests.log 2>&1 || { tail -40 $D/gpu_tests.log; exit 3; }
tail -3 $D/gpu_tests.log
