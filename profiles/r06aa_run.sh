set -o pipefail
# v2 store tile 3 vs 2 words (occupancy 6 -> 7 waves / SIMD): A/B same process
D=gpurun_out/r06aa; mkdir -p $D
timeout -k 10 300 python profiles/nl_ab.py 20 6 OPENR_NL_TILEW 3,2 > $D/tilew_ab.json 2> $D/tilew_ab.err || { tail -20 $D/tilew_ab.err; exit 3; }
python3 -c "
import json; d=json.load(open('$D/tilew_ab.json')); print({k: v for k, v in d.items() if k not in ('raw','kernels')})"
OPENR_NL_TILEW=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_nl_trit_gpu.py tests/test_abi_gpu.py > $D/tests_tw2.log 2>&1 || { tail -30 $D/tests_tw2.log; exit 4; }
tail -1 $D/tests_tw2.log
