set -o pipefail
# round 5: link-flap update after the host-pass fixes (sorted-row fast path,
# kept scratch, reused splice arrays) + parity of the flap / update / set_edges
# tests; the MS-BFS without its scattered level-row stores (measurement)
D=gpurun_out/r05p; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_graph_update_gpu.py tests/test_engine_parity_gpu.py tests/test_table_repair.py tests/test_all_sources_table_gpu.py -k "update or link_flap or selective_memo or incremental or set_edges or repair or table" -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -30 $D/gpu_tests.log; exit 3; }
tail -1 $D/gpu_tests.log
OPENR_SPF_CREATE_TIMING=1 timeout -k 10 300 python3 profiles/linkflap_probe.py > $D/linkflap.json 2> $D/linkflap.err || { tail -5 $D/linkflap.err; exit 4; }
python3 -c "import json; d=json.load(open('$D/linkflap.json')); print({k: d.get(k) for k in ('ms_median','update_ms_median','build_ms_median','parity_check','per_build_us')})"
grep "spf_graph_update" $D/linkflap.err | tail -9
B="bench.py --no-cpu-baseline --no-route-db --no-whatif --no-wan --steps 20 --warmup 3"
for n in 0 1; do
OPENR_MS_NOREC=$n timeout -k 10 300 python3 $B > $D/fabric.n$n.json 2> $D/fabric.n$n.err || { tail -5 $D/fabric.n$n.err; exit 2; }
python3 -c "import json,sys; d=json.load(open('$D/fabric.n$n.json')); print('norec=$n', d['ms_per_step'], {k: v['avg_ms'] for k, v in d['kernels'].items()})"
done
