set -o pipefail
D=gpurun_out/r03a; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread $PYTEST_EXTRA > $D/gpu_tests.log 2>&1; rc=$?
tail -3 $D/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $D/bench.json 2> $D/bench.err || exit 6
cut -c1-600 $D/bench.json
Q="--no-cpu-baseline --no-route-db --no-wan --no-whatif --no-repair --steps 20 --warmup 3"
for v in "1 1" "0 0"; do set -- $v
  OPENR_NL_XCD=$1 OPENR_NL_HELD=$2 timeout -k 10 200 python bench.py $Q > $D/fab_xcd$1_held$2.json 2> $D/fab_xcd$1_held$2.err || exit 7
  python -c "import json;d=json.load(open('$D/fab_xcd$1_held$2.json'));print('xcd',$1,'held',$2,d['ms_per_step'],d.get('kernels',d.get('roofline')))" | cut -c1-400
done
