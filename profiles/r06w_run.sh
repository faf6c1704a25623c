set -o pipefail
# what-if repair work list: what-if tests + batch; WAN baseline knobs
D=gpurun_out/r06w; mkdir -p $D
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_whatif_firsthop_gpu.py tests/test_whatif_repair_gpu.py > $D/gpu_tests.log 2>&1 || { tail -40 $D/gpu_tests.log; exit 3; }
tail -1 $D/gpu_tests.log
for v in base wl0 ls6 ls8 ls10 few0; do
  case $v in
    base) E="";; wl0) E="OPENR_SPF_WHATIF_WORKLIST=0";; ls6) E="OPENR_SPF_DSTEP_LSHIFT=6";;
    ls8) E="OPENR_SPF_DSTEP_LSHIFT=8";; ls10) E="OPENR_SPF_DSTEP_LSHIFT=10";; few0) E="OPENR_SPF_FEW_DSTEP=0";;
  esac
  env $E timeout -k 10 200 python profiles/whatif_probe.py 5 > $D/wi_$v.json 2> $D/wi_$v.err || { tail -20 $D/wi_$v.err; exit 4; }
  python3 -c "
import json
d=json.loads(open('$D/wi_$v.json').read().strip().splitlines()[-1]); print('$v', d['ms'], d['device_ms'], d['value'], d['parity_check'])"
done
