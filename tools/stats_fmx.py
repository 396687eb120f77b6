"""Filter a rocprofv3 --stats kernel summary to the fmx kernels (short names).

Usage: python tools/stats_fmx.py <run_kernel_stats.csv> > out.csv
The full summary also lists the torch kernels of the synthetic-scan generator,
which run before the timed region."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
w = csv.writer(sys.stdout)
w.writerow(["kernel", "calls", "total_us", "avg_us", "min_us", "max_us", "percent"])
for r in rows:
    n = r["Name"]
    if "fmx::" not in n and "__amd_rocclr" not in n:
        continue
    short = n.replace("(anonymous namespace)::", "").replace("void ", "")
    short = re.sub(r"\(.*", "", short).replace("fmx::", "")
    w.writerow([short, r["Calls"], round(float(r["TotalDurationNs"]) / 1e3, 1), round(float(r["AverageNs"]) / 1e3, 2),
                round(float(r["MinNs"]) / 1e3, 2), round(float(r["MaxNs"]) / 1e3, 2), r["Percentage"]])
