set -o pipefail
# small-area MS-BFS plan for few-source batches (OPENR_SPF_MSBFS_SMALL): grid
# RouteDb A/B, then the GPU tests
R=$(pwd)
D=gpurun_out/r06ao; mkdir -p $D
OPENR_SPF_MSBFS_SMALL=0 timeout -k 10 200 python3 profiles/grid_probe.py --iters 300 > $D/grid_off.json 2> $D/grid_off.err || exit 3
timeout -k 10 200 python3 profiles/grid_probe.py --iters 300 > $D/grid_on.json 2> $D/grid_on.err || exit 4
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$D/kt -o run --output-format csv -- python3 $R/profiles/grid_probe.py --iters 50 > $R/$D/grid_prof.json 2> $R/$D/grid_prof.err || { tail -20 $R/$D/grid_prof.err; exit 5; }
cd $R
python3 - <<PY
import csv, glob, json
for t in ("off", "on"):
    j = json.load(open("$D/grid_%s.json" % t))
    print(t, j["engine"]["ms_median"], j["engine"]["per_build_us"].get("decision.spf_batch_us"), j["engine"]["per_build_us"].get("decision.spf_device_us"), "oracle", j["cpu_oracle"]["ms_median"])
f = glob.glob("$D/kt/**/run_kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:14]:
    print(r["Name"][:80], r["Calls"], r["AverageNs"])
PY
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $D/gpu_tests.log 2>&1 || { tail -30 $D/gpu_tests.log; exit 6; }
tail -3 $D/gpu_tests.log
