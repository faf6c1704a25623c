set -o pipefail
# smoke + ABI / what-if / trace tests on the clean-rebuilt libraries
D=gpurun_out/r05ay; mkdir -p $D
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 2; }
tail -1 $D/smoke.log
timeout -k 10 600 python -u -m pytest tests/test_abi_gpu.py tests/test_abi_lifetime_gpu.py tests/test_whatif_repair_gpu.py tests/test_trace_paths_gpu.py tests/test_graph_update_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -30 $D/gpu_tests.log; exit 3; }
tail -1 $D/gpu_tests.log
