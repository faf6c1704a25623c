set -o pipefail
# round 4: LDS-row WAN kernel sweep + byte-granular next-hop masks, full GPU suite, bench
D=gpurun_out/r04c; mkdir -p $D
timeout -k 10 500 python -u profiles/quick_wan.py 8192 LDSROW=0 base LG=1 LG=2 LG=8 LG=1,LSHIFT=5 LG=1,LSHIFT=7 LG=2,LSHIFT=5 LG=2,LSHIFT=7 LSHIFT=5 LSHIFT=7 base > $D/quick_wan.log 2>&1 || exit 3
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1; rc=$?
tail -5 $D/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --no-cpu-baseline > $D/bench.json 2> $D/bench.err || exit 5
python -c "import json;d=json.load(open('$D/bench.json'));print(d['value'], d['ms_per_step'], d['roofline'])"
