set -o pipefail
# v2 pass, persistent form (OPENR_NL_V2_PERSIST=1) vs one block per item-chunk
D=gpurun_out/r06ah; mkdir -p $D
timeout -k 10 300 python profiles/nl_ab.py 20 6 OPENR_NL_V2_PERSIST 0,1 > $D/persist_ab.json 2> $D/persist_ab.err || { tail -20 $D/persist_ab.err; exit 3; }
python3 -c "
import json; d=json.load(open('$D/persist_ab.json')); print({k: v for k, v in d.items() if k not in ('raw','kernels')})"
for pc in 3 4 8; do
  OPENR_NL_V2_PER_CU=$pc timeout -k 10 300 python profiles/nl_ab.py 20 4 OPENR_NL_V2_PERSIST 0,1 > $D/persist_ab_pc$pc.json 2> $D/persist_ab_pc$pc.err || { tail -20 $D/persist_ab_pc$pc.err; exit 4; }
  python3 -c "
import json; d=json.load(open('$D/persist_ab_pc$pc.json')); print($pc, d['OPENR_NL_V2_PERSIST=0']['nh_ms'], d['OPENR_NL_V2_PERSIST=1']['nh_ms'], d['masks_equal'])"
done
OPENR_NL_V2_PERSIST=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_nl_trit_gpu.py tests/test_abi_gpu.py > $D/tests_persist.log 2>&1 || { tail -30 $D/tests_persist.log; exit 5; }
tail -1 $D/tests_persist.log
