set -o pipefail
# KSP2 todo lookups on the host pool: KSP2 goldens + bench breakdown
D=gpurun_out/${TAG:-r06ae}; mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -k "ksp2 or kth or trace" tests/ > $D/gpu_tests.log 2>&1 || { tail -40 $D/gpu_tests.log; exit 3; }
tail -1 $D/gpu_tests.log
timeout -k 10 400 python bench.py --no-wan --no-whatif --no-cpu-baseline --no-repair --steps 3 --warmup 1 > $D/b.json 2> $D/b.err || { tail -20 $D/b.err; exit 4; }
python3 -c "
import json
b=json.loads(open('$D/b.json').read().strip().splitlines()[-1])
k=b['ksp2_route_db']; print(k['ms_median'], k['build_ms_median'], k['release_ms_median'], k['parity_check']); p=k['per_build']; print({x: p[x] for x in ('route_prefetch_us','kth_todo_us','kth_lists_us','spf_batch_us','kth_fill_us')})"
