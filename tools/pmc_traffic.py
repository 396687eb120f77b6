"""Summarize rocprofv3 --pmc passes into per-kernel HBM bytes per launch.

Usage: python tools/pmc_traffic.py <workload> <out.json> <pass_dir> [<pass_dir> ...]

Each pass dir holds a rocprofv3 `*counter_collection.csv` of one counter pass
(FETCH_SIZE, WRITE_SIZE and TCC hit/miss are collected in separate runs, as
MI355X_MICROARCH.md §rocprofv3 PMC slots requires).  Per MI355X_MICROARCH.md §HBM:
FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports 1/2 of the bytes
of wide coalesced reads, so hbm_bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024
(the raw sum is kept beside it).  Kernel names are mapped to the fmx profile ids
bench.py uses for the roofline.
"""
from __future__ import annotations

import csv
import glob
import json
import os
import sys
from collections import defaultdict

# fmx kernel symbol fragment -> bench.py profile id
KMAP = {
    "k_match": "match",
    "k_extract_rows": "extract_rows",
    "k_normals": "fit",  # find_closest + compute_normal, fused (C <= 2048)
    "k_closest": "closest",
    "k_fit": "fit",
    "k_linearize_total": "linearize",  # register_scan's fused linearization
    "k_linearize<1>": "linearize_pairs",
    "k_linearize<0>": "linearize_full",
    "k_map_insert": "map_build_insert",
    "k_map_scatter": "map_build_scatter",
    "k_insert": "insert",
    "k_win_linearize": "window",  # smoothing mode: many pairs per launch
    "k_pair_scatter": "pair_sort",
}


def kernel_id(name: str):
    for frag, kid in KMAP.items():
        if frag in name:
            return kid
    return None


def main():
    workload, out = sys.argv[1], sys.argv[2]
    sums = defaultdict(lambda: defaultdict(float))
    counts = defaultdict(lambda: defaultdict(int))
    for d in sys.argv[3:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    kid = kernel_id(row.get("Kernel_Name", ""))
                    if not kid:
                        continue
                    cn = row.get("Counter_Name")
                    sums[kid][cn] += float(row.get("Counter_Value", 0) or 0)
                    counts[kid][cn] += 1
    kernels = {}
    for kid, cs in sums.items():
        avg = {cn: cs[cn] / max(counts[kid][cn], 1) for cn in cs}
        ent = {"counters_per_launch": avg, "launches": max(counts[kid].values())}
        if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
            ent["hbm_bytes_raw_per_launch"] = (avg["FETCH_SIZE"] + avg["WRITE_SIZE"]) * 1024.0
            ent["hbm_bytes_per_launch"] = (2.0 * avg["FETCH_SIZE"] + avg["WRITE_SIZE"]) * 1024.0
        hit, miss = avg.get("TCC_HIT_sum"), avg.get("TCC_MISS_sum")
        if hit is not None and miss is not None and hit + miss > 0:
            ent["l2_hit_rate"] = hit / (hit + miss)
        kernels[kid] = ent
    res = {"workload": workload, "correction": "hbm = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950, MI355X_MICROARCH.md §HBM)",
           "kernels": kernels}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
