set -o pipefail
# round 5: v2 pass with constant-space tables (scalar-loaded entries) and multiply-free distance rows (no per-lane 64-bit
# addresses): A/B vs held, SQ instruction counts, parity tests
D=gpurun_out/r05m; mkdir -p $D
R=$(pwd)
B="bench.py --no-cpu-baseline --no-route-db --no-whatif --no-wan --steps 20 --warmup 3"
for cfg in "1 4" "0 4" "1 4" "0 4" "1 3"; do
set -- $cfg
OPENR_NL_V2=$1 OPENR_NL_V2_ORDER=$2 timeout -k 10 300 python3 $B > $D/fabric.v$1.o$2.json 2> $D/fabric.v$1.o$2.err || { tail -5 $D/fabric.v$1.o$2.err; exit 2; }
python3 -c "import json,sys; d=json.load(open('$D/fabric.v$1.o$2.json')); print('v2=$1 order=$2', d['ms_per_step'], {k: v['avg_ms'] for k, v in d['kernels'].items()}, d.get('parity_spot_check'))"
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES -T -d $R/$D/sq -o run --output-format csv -- \
  python3 $R/$B --steps 3 --warmup 1 > $R/$D/sq.json 2> $R/$D/sq.err || { tail -3 $R/$D/sq.err; exit 3; }
cd $R
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(set)
for f in glob.glob('gpurun_out/r05m/sq/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'].split('(')[0].split('<')[0].split('::')[-1]
        acc[k][r['Counter_Name']] += float(r['Counter_Value'] or 0)
        cnt[k].add(r.get('Dispatch_Id'))
for k, v in acc.items():
    if 'nh_levels' in k:
        n = max(1, len(cnt[k]))
        print(k, n, {c: round(x / n) for c, x in sorted(v.items())})
PY
timeout -k 10 600 python -u -m pytest tests/test_config_sized_gpu.py tests/test_abi_gpu.py tests/test_graph_update_gpu.py tests/test_zero_metric_plan.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -30 $D/gpu_tests.log; exit 4; }
tail -1 $D/gpu_tests.log
