set -o pipefail
# first-hop what-if: kernel trace of the batch
R=$(pwd)
D=gpurun_out/${TAG:-r06p}; mkdir -p $D
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$D/kt -o run --output-format csv -- python3 $R/profiles/whatif_probe.py 3 > $R/$D/kt.log 2>&1 || { tail -20 $R/$D/kt.log; exit 3; }
cd $R
python3 - <<PY
import csv, glob
f = glob.glob("$D/kt/**/run_kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:16]:
    print(r["Name"][:70], r["Calls"], r["AverageNs"], r["TotalDurationNs"])
t = glob.glob("$D/kt/**/run_kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(t)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the last batch: from the last spf_ms_ign_kernel / dlds on
names = [r["Kernel_Name"][:40] for r in rows]
last = max(i for i, r in enumerate(rows) if "spf_dlds_kernel" in r["Kernel_Name"])
first = max(i for i, r in enumerate(rows[:last]) if "spf_dlds_kernel" in r["Kernel_Name"]) if sum("spf_dlds_kernel" in r["Kernel_Name"] for r in rows) > 1 else 0
t0 = int(rows[last]["Start_Timestamp"])
lo = max(0, last - 20)
for r in rows[lo:last + 25]:
    print("%-48s q%-3s %8.1f %8.1f" % (r["Kernel_Name"][:48], r.get("Queue_Id", "?"), (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
PY
