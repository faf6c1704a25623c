set -o pipefail
# round 5 HEAD: headline kernel trace + FETCH/WRITE PMC (v2 next-hop pass),
# what-if plan PMC, then the default bench line
R=$(pwd)
D=gpurun_out/r05w; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_trace_paths_gpu.py tests/test_graph_update_gpu.py tests/test_engine_parity_gpu.py tests/test_routedb_golden_gpu.py -k "trace or ksp2 or update or link_flap or selective_memo or incremental" -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -30 $D/gpu_tests.log; exit 2; }
tail -1 $D/gpu_tests.log
OPENR_SPF_CREATE_TIMING=1 timeout -k 10 300 python3 profiles/linkflap_probe.py > $D/linkflap.json 2> $D/linkflap.err || { tail -5 $D/linkflap.err; exit 2; }
python3 -c "import json; d=json.load(open('$D/linkflap.json')); print({k: d.get(k) for k in ('ms_median','update_ms_median','build_ms_median','parity_check','per_build_us')})"
timeout -k 10 700 bash profiles/prof_fabric.sh r05w || exit 3
cp gpurun_out/prof_r05w/final/* $D/
cd /tmp && export TMPDIR=/tmp
for P in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $P -T -d $R/$D/wi_$P -o run --output-format csv -- \
    python3 $R/profiles/whatif_probe.py 2 --batches-out $R/$D/wi_batches.json > $R/$D/wi_$P.log 2>&1 || exit 4
done
cd $R
python3 profiles/collect_pmc.py $D/wi_FETCH_SIZE $D/wi_WRITE_SIZE $D/pmc_whatif.json || exit 5
python3 - <<PY
import json
D="$D"
wi=json.load(open(D+"/pmc_whatif.json")); wi["batches"]=json.load(open(D+"/wi_batches.json"))["batches"]
wi["what"]+="; what-if batch alone at round-5 HEAD (profiles/whatif_probe.py 2: warm-up + 2 timed batches)"
json.dump(wi,open(D+"/pmc_whatif.json","w"),indent=1)
print({k: (v["dispatches"], v["hbm_bytes_per_launch"]) for k, v in wi["kernels"].items()})
PY
timeout -k 10 600 python3 bench.py > $D/bench_full.json 2> $D/bench_full.err || { tail -20 $D/bench_full.err; exit 6; }
cut -c1-1500 $D/bench_full.json
