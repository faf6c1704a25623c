set -o pipefail
# round 6: trit next-hop rows parity + LFA fast path parity + recycled route
# nodes + ADVICE fixes, then the full bench
D=gpurun_out/r06b; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests/test_nl_trit_gpu.py tests/test_abi_gpu.py tests/test_graph_update_gpu.py tests/test_whatif_repair_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests_abi.log 2>&1 || { tail -40 $D/gpu_tests_abi.log; exit 2; }
tail -1 $D/gpu_tests_abi.log
timeout -k 10 900 python -u -m pytest tests/test_routedb_golden_gpu.py tests/test_config_sized_gpu.py tests/test_engine_parity_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests_rdb.log 2>&1 || { tail -40 $D/gpu_tests_rdb.log; exit 3; }
tail -1 $D/gpu_tests_rdb.log
timeout -k 10 600 python3 bench.py > $D/bench_full.json 2> $D/bench_full.err || { tail -20 $D/bench_full.err; exit 6; }
python3 - <<PY
import json
b=json.loads(open("$D/bench_full.json").read().strip().splitlines()[-1])
print(b["value"], b["n_gpus"], b["ms_per_step"], b["roofline"]["frac"], b["kernels"], b.get("table_path"))
for k in ("route_db_rebuild_lfa","route_db_rebuild","ksp2_route_db","route_db_link_flap","whatif_batch","wan_all_sources","grid_route_db"):
    v=b.get(k,{}); print(k, {x: v.get(x) for x in ("ms_median","build_ms_median","update_ms_median","release_ms_median","parity_check","ms","value","engine","error")})
print(b["cpu_baseline"].get("route_db_rebuild_lfa"))
PY
