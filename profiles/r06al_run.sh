set -o pipefail
# what-if screen with 1,024-thread blocks (OPENR_SPF_SCREEN_BS) vs 256
D=gpurun_out/r06al; mkdir -p $D
for v in b256 b1024 b256x b1024x; do
  case $v in b256*) E="OPENR_SPF_SCREEN_BS=256";; b1024*) E="OPENR_SPF_SCREEN_BS=1024";; esac
  env $E timeout -k 10 200 python profiles/whatif_probe.py 8 > $D/wi_$v.json 2> $D/wi_$v.err || { tail -20 $D/wi_$v.err; exit 4; }
  python3 -c "
import json
d=json.loads(open('$D/wi_$v.json').read().strip().splitlines()[-1]); print('$v', d['ms'], d['device_ms'], d['value'], d['parity_check'])"
done
OPENR_SPF_SCREEN_BS=1024 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_whatif_firsthop_gpu.py tests/test_whatif_repair_gpu.py > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 5; }
tail -1 $D/tests.log
