set -o pipefail
# round 5: PMC passes of the what-if plan as it runs at HEAD (the kernel set
# is recorded by collect_pmc; bench.py refuses a file whose set differs from
# the plan's spf_query_kernels), then the v2 time split
D=gpurun_out/r05e; mkdir -p $D/final
R=$(pwd); cd /tmp && export TMPDIR=/tmp
for P in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $P -T -d $R/$D/wi_$P -o run --output-format csv -- \
    python3 $R/profiles/whatif_probe.py 2 --batches-out $R/$D/wi_batches.json > $R/$D/wi_$P.log 2>&1 || exit 3
done
cd $R
python3 profiles/collect_pmc.py $D/wi_FETCH_SIZE $D/wi_WRITE_SIZE $D/final/pmc_whatif.json || exit 4
python3 - <<PY
import json
D="$D"
wi=json.load(open(D+"/final/pmc_whatif.json")); wi["batches"]=json.load(open(D+"/wi_batches.json"))["batches"]
wi["what"]+="; what-if batch alone at round-5 HEAD (profiles/whatif_probe.py 2: warm-up + 2 timed batches)"
json.dump(wi,open(D+"/final/pmc_whatif.json","w"),indent=1)
print({k: (v["dispatches"], v["hbm_bytes_per_launch"]) for k, v in wi["kernels"].items()})
PY
tail -1 $D/wi_WRITE_SIZE.log | cut -c1-600
bash profiles/r05d_run.sh
