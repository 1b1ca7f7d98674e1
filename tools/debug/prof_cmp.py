"""Compare rocprofv3 kernel stats of two profile directories (gpurun_out/prof_<a>, prof_<b>): per-kernel average."""
import csv
import sys

def load(tag):
    return {r["Name"][:70]: r for r in csv.DictReader(open(f"gpurun_out/prof_{tag}/run_kernel_stats.csv"))}

a, b = load(sys.argv[1]), load(sys.argv[2])
for k in sorted(b, key=lambda k: -float(b[k]["TotalDurationNs"]))[:int(sys.argv[3]) if len(sys.argv) > 3 else 16]:
    ra = a.get(k)
    av = float(ra["AverageNs"]) / 1e3 if ra else float("nan")
    print("%-70s %7s %9.2f -> %9.2f us" % (k, b[k]["Calls"], av, float(b[k]["AverageNs"]) / 1e3))
