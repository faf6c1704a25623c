set -o pipefail
# round 4: the whole GPU suite + smoke at HEAD
D=gpurun_out/r04w; mkdir -p $D
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1; rc=$?
tail -3 $D/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.log 2>&1 || exit 4
tail -1 $D/smoke.log
