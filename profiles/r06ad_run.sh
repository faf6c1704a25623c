set -o pipefail
# KSP2 prefetch breakdown (kth_todo / kth_lists / kth_fill counters)
D=gpurun_out/r06ad; mkdir -p $D
timeout -k 10 400 python bench.py --no-wan --no-whatif --no-cpu-baseline --no-repair --steps 3 --warmup 1 > $D/b.json 2> $D/b.err || { tail -20 $D/b.err; exit 3; }
python3 -c "
import json
b=json.loads(open('$D/b.json').read().strip().splitlines()[-1])
k=b['ksp2_route_db']; print(k['ms_median'], k['build_ms_median'], k['release_ms_median']); print(json.dumps(k['per_build']))"
