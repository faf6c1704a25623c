set -o pipefail
# v2 pass: 1,280-node chunks, chunk c on XCD c (OPENR_NL_V2_XCD=1) vs default
R=$(pwd)
D=gpurun_out/r06ag; mkdir -p $D
timeout -k 10 300 python profiles/nl_ab.py 20 6 OPENR_NL_V2_XCD 0,1 > $D/xcd_ab.json 2> $D/xcd_ab.err || { tail -20 $D/xcd_ab.err; exit 3; }
python3 -c "
import json; d=json.load(open('$D/xcd_ab.json')); print({k: v for k, v in d.items() if k not in ('raw','kernels')})"
OPENR_NL_V2_XCD=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_nl_trit_gpu.py tests/test_abi_gpu.py > $D/tests_xcd.log 2>&1 || { tail -30 $D/tests_xcd.log; exit 4; }
tail -1 $D/tests_xcd.log
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --no-cpu-baseline --no-route-db --no-whatif --no-wan --steps 3 --warmup 1"
for m in 0 1; do
  OPENR_NL_V2_XCD=$m timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -T -d $R/$D/pmc_f$m -o run --output-format csv -- python3 $B > $R/$D/pf$m.json 2> $R/$D/pf$m.err || exit 5
  OPENR_NL_V2_XCD=$m timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -T -d $R/$D/pmc_w$m -o run --output-format csv -- python3 $B > $R/$D/pw$m.json 2> $R/$D/pw$m.err || exit 6
  cd $R && python3 profiles/collect_pmc.py $D/pmc_f$m $D/pmc_w$m $D/pmc_xcd$m.json > /dev/null && cd /tmp
done
cd $R
python3 -c "
import json
for m in (0, 1):
    d=json.load(open('$D/pmc_xcd%d.json' % m))
    for k, v in d['kernels'].items():
        if 'v2' in k: print(m, k, v['FETCH_SIZE_kB'], v['WRITE_SIZE_kB'], v['hbm_bytes_per_launch'])"
