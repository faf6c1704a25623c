set -o pipefail
# round 4: the whole GPU suite and smoke at HEAD (batched cursor trace)
D=gpurun_out/r04ai; mkdir -p $D
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -15 $D/gpu_tests.log; exit 2; }
tail -2 $D/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.log 2>&1 || { tail -5 $D/smoke.log; exit 3; }
tail -1 $D/smoke.log
