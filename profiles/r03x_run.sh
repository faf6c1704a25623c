set -o pipefail
D=gpurun_out/r03x; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1; rc=$?
tail -3 $D/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.log 2>&1 || exit 4
tail -1 $D/smoke.log
bash profiles/prof_fabric.sh r03x > $D/prof.log 2>&1 || exit 6
mkdir -p $D/prof && cp gpurun_out/prof_r03x/final/* $D/prof/
timeout -k 10 600 python bench.py > $D/bench_full.json 2> $D/bench_full.err || exit 5
python -c "import json;d=json.load(open('$D/bench_full.json'));print(d['value'], d['ms_per_step'], d['roofline'])"
