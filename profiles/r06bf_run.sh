set -o pipefail
# closing check at HEAD: full GPU suite + smoke with the in-tree libraries
D=gpurun_out/r06bf; mkdir -p $D
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $D/gpu_tests.log 2>&1 || { tail -40 $D/gpu_tests.log; exit 4; }
tail -1 $D/gpu_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 5; }
tail -1 $D/smoke.log
