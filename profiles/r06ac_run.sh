set -o pipefail
# round-6 final validation: full GPU suite + smoke, headline kernel trace + PMC
D=gpurun_out/r06ac; mkdir -p $D
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $D/gpu_tests.log 2>&1 || { tail -40 $D/gpu_tests.log; exit 3; }
tail -1 $D/gpu_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 4; }
tail -1 $D/smoke.log
timeout -k 10 700 bash profiles/prof_fabric.sh r06ac || exit 5
cp gpurun_out/prof_r06ac/final/* $D/
head -4 $D/kernel_stats.csv | cut -c1-120
