set -o pipefail
# round 6: LFA fast path parity (every loop state) + full bench at N=1 with
# the LFA-on rebuild line and the spf_table path line
D=gpurun_out/r06a; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_routedb_golden_gpu.py tests/test_engine_parity_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -30 $D/gpu_tests.log; exit 2; }
tail -1 $D/gpu_tests.log
timeout -k 10 600 python3 bench.py > $D/bench_full.json 2> $D/bench_full.err || { tail -20 $D/bench_full.err; exit 6; }
python3 - <<PY
import json
b=json.loads(open("$D/bench_full.json").read().strip().splitlines()[-1])
print(b["value"], b["n_gpus"], b["ms_per_step"], b["roofline"]["frac"], b.get("table_path"))
for k in ("route_db_rebuild_lfa","route_db_rebuild","ksp2_route_db","route_db_link_flap","whatif_batch","wan_all_sources","grid_route_db"):
    v=b.get(k,{}); print(k, {x: v.get(x) for x in ("ms_median","build_ms_median","update_ms_median","release_ms_median","parity_check","ms","value","engine","error")})
print(b["cpu_baseline"].get("route_db_rebuild_lfa"))
PY
