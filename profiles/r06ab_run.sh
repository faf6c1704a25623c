set -o pipefail
# what-if: the screen pre-copies the repairs' baseline rows
D=gpurun_out/r06ab; mkdir -p $D
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_whatif_firsthop_gpu.py tests/test_whatif_repair_gpu.py tests/test_abi_gpu.py tests/test_config_sized_gpu.py > $D/gpu_tests.log 2>&1 || { tail -40 $D/gpu_tests.log; exit 3; }
tail -1 $D/gpu_tests.log
for v in base pc0 base2 pc02; do
  case $v in base|base2) E="";; pc0|pc02) E="OPENR_SPF_WHATIF_PRECOPY=0";; esac
  env $E timeout -k 10 200 python profiles/whatif_probe.py 5 > $D/wi_$v.json 2> $D/wi_$v.err || { tail -20 $D/wi_$v.err; exit 4; }
  python3 -c "
import json
d=json.loads(open('$D/wi_$v.json').read().strip().splitlines()[-1]); print('$v', d['ms'], d['device_ms'], d['value'], d['parity_check'])"
done
OPENR_SPF_WHATIF_STATS=1 timeout -k 10 200 python profiles/whatif_probe.py 1 > $D/wi_stats.json 2> $D/wi_stats.err || exit 5
grep "whatif stats" $D/wi_stats.err | tail -2
