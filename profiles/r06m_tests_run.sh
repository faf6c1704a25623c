set -o pipefail
# round 6 HEAD: full GPU suite + smoke, headline kernel trace + PMC, what-if
# plan PMC (now with spf_whatif_pull_kernel), full bench
R=$(pwd)
D=gpurun_out/r06m; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -30 $D/gpu_tests.log; exit 2; }
tail -1 $D/gpu_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 2; }
tail -1 $D/smoke.log
