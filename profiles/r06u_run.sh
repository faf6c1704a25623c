set -o pipefail
# route shards on fixed pool workers (parallelShards) vs dynamic hand-out:
# RouteDb rebuild loops A/B/A/B on one box
D=gpurun_out/r06u; mkdir -p $D
B="python bench.py --no-wan --no-whatif --no-cpu-baseline --no-repair --steps 3 --warmup 1"
for i in 1 2; do
  for m in 0 1; do
    OPENR_SHARD_DYNAMIC=$m timeout -k 10 300 $B > $D/rdb_dyn$m.$i.json 2> $D/rdb_dyn$m.$i.err || { tail -20 $D/rdb_dyn$m.$i.err; exit 3; }
  done
done
python3 - <<PY
import json
for i in (1, 2):
    for m in (0, 1):
        b = json.loads(open("$D/rdb_dyn%d.%d.json" % (m, i)).read().strip().splitlines()[-1])
        out = []
        for k in ("route_db_rebuild", "route_db_rebuild_lfa", "ksp2_route_db", "route_db_link_flap"):
            v = b.get(k, {})
            out.append("%s %s/%s/%s" % (k, v.get("ms_median"), v.get("build_ms_median"), v.get("release_ms_median")))
        print("dyn=%d" % m, i, b["value"], " | ".join(out))
PY
