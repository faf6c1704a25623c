set -o pipefail
# round 5 HEAD: full GPU suite + smoke + full bench (KSP2 heavy launch with
# the reachability walk, budget 1024)
D=gpurun_out/r05ag; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -30 $D/gpu_tests.log; exit 3; }
tail -1 $D/gpu_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 4; }
tail -1 $D/smoke.log
timeout -k 10 600 python3 bench.py > $D/bench_full.json 2> $D/bench_full.err || { tail -20 $D/bench_full.err; exit 6; }
python3 - <<PY
import json
b=json.loads(open("$D/bench_full.json").read().strip().splitlines()[-1])
print(b["value"], b["ms_median"] if "ms_median" in b else b["ms_per_step"], b["roofline"]["frac"])
for k in ("route_db_rebuild","ksp2_route_db","route_db_link_flap","whatif_batch","wan_all_sources","grid_route_db"):
    v=b.get(k,{}); print(k, {x: v.get(x) for x in ("ms_median","build_ms_median","update_ms_median","ms","engine")})
print({x:y for x,y in b["ksp2_route_db"]["per_build"].items() if "kth" in x})
PY
