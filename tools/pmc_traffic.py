"""Summarize rocprofv3 --pmc passes into per-kernel HBM bytes per launch.

Usage: python tools/pmc_traffic.py <workload> <out.json> <pass_dir> [<pass_dir> ...]

Each pass dir holds a rocprofv3 `*counter_collection.csv` of one counter pass
(FETCH_SIZE, WRITE_SIZE and TCC hit/miss are collected in separate runs, as
MI355X_MICROARCH.md §rocprofv3 PMC slots requires).  FETCH_SIZE / WRITE_SIZE are in
KiB.  Corrections, per access pattern (MI355X_MICROARCH.md §HBM for coalesced streams;
the rest calibrated on known byte counts with tools/pmc_calib, committed as
profiles/r2_pmc_calibration.txt):
  * coalesced reads (16 B per lane, or a group's consecutive 32-B records): FETCH_SIZE
    reports 1/2 of the bytes -> 2 * FETCH_SIZE;
  * random 64-B lines (brick probes, one record per line): FETCH_SIZE = the bytes of
    the 64-B lines fetched (calibrated 1.03 and 2.06 x the 64-B / 32-B useful bytes)
    -> 1 * FETCH_SIZE;
  * WRITE_SIZE = bytes for both coalesced and scattered 32-B stores (1.00).
Per kernel: hbm_bytes_per_launch uses the correction of its dominant read pattern
(GATHER kernels: 1 x FETCH, the others 2 x FETCH); hbm_bytes_hi / hbm_bytes_lo keep
both bounds (a gather kernel's coalesced share is undercounted by up to 2x in lo).
Kernel names are mapped to the fmx profile ids bench.py uses for the roofline.
"""
from __future__ import annotations

import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import provenance  # noqa: E402

# fmx kernel symbol fragment -> bench.py profile id
KMAP = {
    "k_match<false, true>": "match_linearize",  # C5: match + single-pose linearization fused
    "k_match<true, true>": "match_linearize",
    "k_match": "match",
    "k_extract_rows": "extract_rows",
    "k_normals": "fit",  # find_closest + compute_normal, fused (C <= 2048)
    "k_closest": "closest",
    "k_fit": "fit",
    "k_linearize_total": "linearize",  # register_scan's fused linearization
    "k_linearize<1>": "linearize_pairs",
    "k_linearize<0>": "linearize_full",
    "k_map_insert": "map_build_insert",
    "k_map_count": "map_build_count",
    "k_map_alloc": "map_build_alloc",
    "k_map_scatter": "map_build_scatter",
    "k_map_dense": "map_build_dense",
    "k_insert": "insert",
    "k_win_linearize": "window",  # smoothing mode: many pairs per launch
    "k_pair_scatter": "pair_sort",
}


# kernels whose HBM reads are dominated by random 64-B lines (1 x FETCH_SIZE)
GATHER = {"match", "match_linearize"}


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
            lo = (avg["FETCH_SIZE"] + avg["WRITE_SIZE"]) * 1024.0
            hi = (2.0 * avg["FETCH_SIZE"] + avg["WRITE_SIZE"]) * 1024.0
            ent["hbm_bytes_lo"] = lo
            ent["hbm_bytes_hi"] = hi
            ent["correction"] = "1 x FETCH (random 64-B lines)" if kid in GATHER else "2 x FETCH (coalesced)"
            ent["hbm_bytes_per_launch"] = lo if kid in GATHER else hi
        hit, miss = avg.get("TCC_HIT_sum"), avg.get("TCC_MISS_sum")
        if hit is not None and miss is not None and hit + miss > 0:
            ent["l2_hit_rate"] = hit / (hit + miss)
        kernels[kid] = ent
    # the map build as one class (bench.py's "map_build": its four kernels, once each per
    # build): insert / alloc / scatter mix coalesced record streams with random table
    # lines, so the sum keeps both bounds and takes the upper one
    parts = [kernels[k] for k in ("map_build_insert", "map_build_count", "map_build_alloc", "map_build_scatter", "map_build_dense")
             if k in kernels and "hbm_bytes_lo" in kernels[k]]
    if parts:
        lo = sum(p["hbm_bytes_lo"] for p in parts)
        hi = sum(p["hbm_bytes_hi"] for p in parts)
        kernels["map_build"] = {"parts": len(parts), "launches": min(p["launches"] for p in parts), "hbm_bytes_lo": lo,
                                "hbm_bytes_hi": hi, "correction": "sum of the build kernels (upper bound)",
                                "hbm_bytes_per_launch": hi}
    res = {"workload": workload,
           "correction": "per kernel (see 'correction'): coalesced 2 x FETCH_SIZE, random 64-B lines 1 x FETCH_SIZE "
                         "(calibrated, profiles/r2_pmc_calibration.txt), + WRITE_SIZE; KiB -> bytes",
           "kernels": kernels}
    provenance.stamp(res)  # the sources this run measured (bench.py marks stale profiles)
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
