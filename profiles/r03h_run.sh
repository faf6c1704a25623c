set -o pipefail
D=gpurun_out/r03h; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1; rc=$?
tail -3 $D/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 bash profiles/prof_fabric.sh r03h > $D/prof.log 2>&1 || exit 5
timeout -k 10 300 bash profiles/prof_fabric_sq.sh r03h > $D/sq.log 2>&1 || exit 6
tail -3 $D/sq.log
mkdir -p profiles/r03h && cp gpurun_out/prof_r03h/final/* profiles/r03h/ && cp gpurun_out/prof_r03h/sq_counters.json profiles/r03h/
timeout -k 10 400 python bench.py > $D/bench.json 2> $D/bench.err || exit 7
python -c "import json;d=json.load(open('$D/bench.json'));print(d['ms_per_step'],d['value'],d.get('kernels'));print(d.get('roofline'))"
