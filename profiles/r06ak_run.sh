set -o pipefail
# distance rows on a side stream beside the v2 pass (OPENR_NL_DIST_SIDE)
D=gpurun_out/r06ak; mkdir -p $D
timeout -k 10 300 python profiles/nl_ab.py 20 6 OPENR_NL_DIST_SIDE 0,1 > $D/dside_ab.json 2> $D/dside_ab.err || { tail -20 $D/dside_ab.err; exit 3; }
python3 -c "
import json; d=json.load(open('$D/dside_ab.json')); print({k: v for k, v in d.items() if k not in ('raw','kernels')})"
OPENR_NL_DIST_SIDE=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_nl_trit_gpu.py tests/test_abi_gpu.py tests/test_config_sized_gpu.py > $D/tests_dside.log 2>&1 || { tail -30 $D/tests_dside.log; exit 4; }
tail -1 $D/tests_dside.log
