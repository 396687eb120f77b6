"""Per-step wall times of the C4 smoothing stream (bench.py's timed loop), to tell host
jitter (a few slow steps) from a uniformly slower run.  Diagnostic only.

  python tools/step_times.py [--runs 3] [--steps 40] [--pin]
--pin: bind the process to the CPU it starts on (sched_setaffinity) for the runs.
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from form_amd import fmx, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--runs", type=int, default=3)
ap.add_argument("--steps", type=int, default=40)
ap.add_argument("--warmup", type=int, default=10)
ap.add_argument("--pin", action="store_true")
ap.add_argument("--pin-local", type=int, default=None, help="pin to the k-th CPU of the GPU's NUMA-local list")
a = ap.parse_args()
geo = synth.GEOMETRIES["c4"]
params = synth.default_params(geo)
w = synth.World()
n = a.warmup + a.steps
scans = [synth.raycast(w, synth.trajectory_pose(k), geo, synth.SEED + 7919 * (k + 1), "cuda:0") for k in range(n)]
torch.cuda.synchronize()
allowed = sorted(os.sched_getaffinity(0))
print(f"allowed cpus: {len(allowed)} ({allowed[:4]}...)", flush=True)
if a.pin:
    with open("/proc/self/stat") as f:
        cpu = int(f.read().split()[38])
    os.sched_setaffinity(0, {cpu})
    print("pinned to cpu", cpu, flush=True)
if a.pin_local is not None:
    pr = torch.cuda.get_device_properties(0)
    bdf = f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}.0"
    cpus = []
    for part in open(f"/sys/bus/pci/devices/{bdf}/local_cpulist").read().strip().split(","):
        lo, _, hi = part.partition("-")
        cpus += list(range(int(lo), int(hi or lo) + 1))
    os.sched_setaffinity(0, {cpus[a.pin_local]})
    print("pinned to GPU-local cpu", cpus[a.pin_local], "of", bdf, flush=True)
for r in range(a.runs):
    ctx = fmx.Context(fmx.EstimatorParams(extraction=fmx.KeypointExtractionParams(**params)))
    for k in range(a.warmup):
        ctx.register_scan(scans[k])
    ctx.sync()
    t = []
    t0 = time.perf_counter()
    for k in range(a.warmup, n):
        s = time.perf_counter()
        ctx.register_scan(scans[k])
        t.append(time.perf_counter() - s)
    ctx.sync()
    tot = time.perf_counter() - t0
    t = np.array(t) * 1e3
    print(f"run {r}: {a.steps / tot:.1f} scans/s  step ms p10 {np.percentile(t, 10):.3f} p50 {np.median(t):.3f} "
          f"p90 {np.percentile(t, 90):.3f} max {t.max():.3f} (> 2 ms: {(t > 2).sum()})", flush=True)
    ctx.close()
