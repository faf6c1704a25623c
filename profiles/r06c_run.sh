set -o pipefail
# round 6: A/B of the 2-bit neighbour rows and of per-thread route node
# recycling (both opt-in switches), kernel trace of the step with both modes
R=$(pwd)
D=gpurun_out/r06c; mkdir -p $D
timeout -k 10 300 python3 profiles/trit_ab.py 20 4 > $D/trit_ab.json 2> $D/trit_ab.err || { tail -20 $D/trit_ab.err; exit 2; }
cat $D/trit_ab.json | python3 -c "import json,sys; d=json.load(sys.stdin); print({k:v for k,v in d.items() if k!='raw'})"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$D/kt -o run --output-format csv -- python3 $R/profiles/trit_ab.py 10 2 > $R/$D/kt.log 2>&1 || { tail -20 $R/$D/kt.log; exit 3; }
cd $R
find $D/kt -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $D/kernel_stats.csv
python3 - <<PY
import csv
for r in csv.DictReader(open("$D/kernel_stats.csv")):
    print(r["Name"][:60], r["Calls"], r["AverageNs"])
PY
for M in 0 1; do
  OPENR_ROUTE_RECYCLE=$M timeout -k 10 300 python3 profiles/route_db_probe.py 6 > $D/rdb_recycle$M.json 2> $D/rdb_recycle$M.err || { tail -20 $D/rdb_recycle$M.err; exit 4; }
done
for M in 1 0; do
  OPENR_ROUTE_RECYCLE=$M timeout -k 10 300 python3 profiles/route_db_probe.py 6 > $D/rdb2_recycle$M.json 2> $D/rdb2_recycle$M.err || { tail -20 $D/rdb2_recycle$M.err; exit 4; }
done
python3 - <<PY
import json
for f in ("rdb_recycle0","rdb_recycle1","rdb2_recycle1","rdb2_recycle0"):
    d=json.loads(open("$D/"+f+".json").read().strip().splitlines()[-1])
    r=d["route_db_rebuild"]; k=d["ksp2_route_db"]
    print(f, r["ms_median"], r["build_ms_median"], r.get("release_ms_median"), "ksp2", k["ms_median"], k["build_ms_median"], k.get("release_ms_median"))
PY
