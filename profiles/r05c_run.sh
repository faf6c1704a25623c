set -o pipefail
# round 5: fabric-step profile with the v2 next-hop pass (kernel trace,
# FETCH / WRITE passes)
D=gpurun_out/r05c; mkdir -p $D
timeout -k 10 600 bash profiles/prof_fabric.sh r05c > $D/prof.log 2>&1 || { tail -5 $D/prof.log; exit 3; }
mkdir -p $D/prof && cp gpurun_out/prof_r05c/final/* $D/prof/
cat $D/prof/kernel_stats.csv
python3 -c "import json; d=json.load(open('$D/prof/pmc_traffic.json')); print(json.dumps(d, indent=0)[:3000])"
