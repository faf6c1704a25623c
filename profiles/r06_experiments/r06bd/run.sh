set -o pipefail
# MPLS label splice on a thread beside the collision pass: RouteDb loops A/B
# (OPENR_ROUTE_MPLS_MERGE_INLINE=1 vs 0, interleaved), then the RouteDb
# goldens and engine parity
D=gpurun_out/r06bd; mkdir -p $D
timeout -k 10 500 python3 profiles/rdb_ab.py OPENR_ROUTE_MPLS_MERGE_INLINE 1 0 2 > $D/ab.log 2>&1 || { tail -5 $D/ab.log; exit 3; }
grep "^OPENR" $D/ab.log
timeout -k 10 600 python3 -u -m pytest tests/test_routedb_golden_gpu.py tests/test_engine_parity_gpu.py tests/test_golden.py tests/test_route_table.py -x -q --timeout 200 --timeout-method thread > $D/t.log 2>&1 || { tail -30 $D/t.log; exit 6; }
tail -1 $D/t.log
