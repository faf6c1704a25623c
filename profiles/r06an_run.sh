set -o pipefail
# grid RouteDb (BASELINE configs[0]): kernel trace of the engine's builds
R=$(pwd)
D=gpurun_out/r06an; mkdir -p $D
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$D/kt -o run --output-format csv -- python3 $R/profiles/grid_probe.py --iters 50 > $R/$D/grid.json 2> $R/$D/grid.err || { tail -20 $R/$D/grid.err; exit 3; }
cd $R
python3 - <<PY
import csv, glob
f = glob.glob("$D/kt/**/run_kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:14]:
    print(r["Name"][:80], r["Calls"], r["AverageNs"])
t = glob.glob("$D/kt/**/run_kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(t)), key=lambda r: int(r["Start_Timestamp"]))
t0 = int(rows[-12]["Start_Timestamp"])
for r in rows[-12:]:
    print("%-60s %8.1f %8.1f" % (r["Kernel_Name"][:60], (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
PY
