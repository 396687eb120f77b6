"""Summarise a rocprofv3 kernel_trace.csv: busy vs idle time over the last steps and
the per-kernel launch sequence of one register_scan (bench.py C4 run)."""
import csv
import re
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
def short(n):
    m = re.search(r"(k_\w+|__amd_rocclr_\w+)(<[^>(]*>)?", n)
    return (m.group(1) + (m.group(2) or "")) if m else n[:40]


ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows)
print("kernels:", len(ev))
# steps start at the extraction kernel
starts = [i for i, e in enumerate(ev) if "k_extract_rows" in e[2]]
print("steps seen:", len(starts))
# argv[2]: which step to print, counted from the end (default 3: the third-to-last start)
back = int(sys.argv[2]) if len(sys.argv) > 2 else 3
if len(starts) >= back:
    a, b = starts[-back], starts[-back + 1]
    seg = ev[a:b]
    t0 = seg[0][0]
    span = ev[b][0] - t0
    busy = 0
    last_end = t0
    for s, e, n in seg:
        busy += e - max(s, last_end) if e > last_end else 0
        last_end = max(last_end, e)
    print(f"one step: span {span/1e3:.1f} us, kernel-busy {busy/1e3:.1f} us, launches {len(seg)}")
    prev_end = t0
    for s, e, n in seg:
        print(f"  +{(s - t0)/1e3:8.1f}  gap {(s - prev_end)/1e3:7.1f}  dur {(e - s)/1e3:7.1f}  {n}")
        prev_end = max(prev_end, e)
    tot = defaultdict(float)
    for s, e, n in ev[starts[1]:starts[-1]]:
        tot[n] += (e - s) / 1e3
    nsteps = len(starts) - 2
    print("per-step kernel time (us):")
    for k, v in sorted(tot.items(), key=lambda x: -x[1]):
        print(f"  {v / nsteps:8.1f}  {k}")
# step spans (extraction start to the next extraction start) over the timed steps:
# the last `timed` steps of the trace (bench.py --steps), robust to one odd step
timed = int(sys.argv[2]) if len(sys.argv) > 2 else 20
spans = sorted((ev[starts[i + 1]][0] - ev[starts[i]][0]) / 1e3 for i in range(max(0, len(starts) - 1 - timed), len(starts) - 1))
if spans:
    import statistics
    print(f"step span over the last {len(spans)} steps: median {statistics.median(spans):.1f} us, "
          f"p10 {spans[len(spans) // 10]:.1f}, p90 {spans[(9 * len(spans)) // 10]:.1f}, mean {sum(spans) / len(spans):.1f}")
