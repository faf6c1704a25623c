set -o pipefail
# round 5: v2 pass with LDS-staged wide mask tiles: A/B vs register-layout
# stores (OPENR_NL_V2_DBG=64), store floor, parity, and one SQ counter pass
D=gpurun_out/r05k; mkdir -p $D
R=$(pwd)
B="bench.py --no-cpu-baseline --no-route-db --no-whatif --no-wan --steps 20 --warmup 3"
for cfg in "3 0" "3 64" "4 0" "4 64" "3 8" "3 72" "3 0" "4 0"; do
set -- $cfg
OPENR_NL_V2_ORDER=$1 OPENR_NL_V2_DBG=$2 timeout -k 10 300 python3 $B > $D/fabric.o$1.d$2.json 2> $D/fabric.o$1.d$2.err || { tail -5 $D/fabric.o$1.d$2.err; exit 2; }
python3 -c "import json,sys; d=json.load(open('$D/fabric.o$1.d$2.json')); print('order=$1 dbg=$2', d['ms_per_step'], {k: v['avg_ms'] for k, v in d['kernels'].items()}, d.get('parity_spot_check'))"
done
cd /tmp && export TMPDIR=/tmp
OPENR_NL_V2_ORDER=4 timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES -T -d $R/$D/sq -o run --output-format csv -- \
  python3 $R/$B --steps 3 --warmup 1 > $R/$D/sq.json 2> $R/$D/sq.err || { tail -3 $R/$D/sq.err; exit 3; }
cd $R
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(set)
for f in glob.glob('gpurun_out/r05k/sq/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'].split('(')[0].split('<')[0].split('::')[-1]
        acc[k][r['Counter_Name']] += float(r['Counter_Value'] or 0)
        cnt[k].add(r.get('Dispatch_Id'))
for k, v in acc.items():
    n = max(1, len(cnt[k]))
    print(k, n, {c: round(x / n) for c, x in sorted(v.items())})
PY
