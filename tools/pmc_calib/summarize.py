"""Measured (FETCH_SIZE, WRITE_SIZE in KiB -> bytes) vs known bytes per launch."""
import csv, glob, os, sys
from collections import defaultdict

D = sys.argv[1]
known = {l.split()[0]: (int(l.split()[1]), int(l.split()[2])) for l in open(os.path.join(D, "known.txt"))}
meas = defaultdict(lambda: defaultdict(list))
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob(os.path.join(D, c, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = next((n for n in known if n + "(" in r["Kernel_Name"] or r["Kernel_Name"].endswith(n)), None)
            if k and r["Counter_Name"] == c:
                meas[k][c].append(float(r["Counter_Value"]) * 1024)
print(f"{'kernel':10s} {'known B':>12s} {'FETCH B':>12s} {'F/known':>8s} {'WRITE B':>12s} {'W/known':>8s}")
for k, (n, b) in known.items():
    f = sum(meas[k]["FETCH_SIZE"]) / max(len(meas[k]["FETCH_SIZE"]), 1)
    w = sum(meas[k]["WRITE_SIZE"]) / max(len(meas[k]["WRITE_SIZE"]), 1)
    print(f"{k:10s} {b:12d} {f:12.0f} {f / b:8.3f} {w:12.0f} {w / b:8.3f}")
