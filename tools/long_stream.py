"""Long-stream check: N scans of the C4 stream through the GPU path and through the CPU
oracle (test infrastructure, the checker only), poses compared scan by scan.  Covers
what a 40-step bench never reaches: window-store compaction, keypoint-pool
compaction, many marginalizations.  Diagnostic; prints max pose difference and ATE
of both paths against the synthetic trajectory.

  python tools/long_stream.py [--scans 300] [--config c4] [--pipeline]

--pipeline announces every next scan (fmx_next_scan), as bench.py does.
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle_py as O  # noqa: E402  (checker only)
from form_amd import fmx, metrics, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--scans", type=int, default=300)
ap.add_argument("--config", default="c4")
ap.add_argument("--pipeline", action="store_true")
a = ap.parse_args()
geo = synth.GEOMETRIES[a.config]
p = synth.default_params(geo)
w = synth.World()
ctx = fmx.Context(fmx.EstimatorParams(extraction=fmx.KeypointExtractionParams(**p)))
threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
est = O.Estimator(O.default_params(p), threads)
gpu, cpu, gt = [], [], []
worst, t0 = 0.0, time.time()


def scan(k):
    return synth.raycast(w, synth.trajectory_pose(k), geo, synth.SEED + 7919 * (k + 1), "cuda:0")


nxt = scan(0)
for k in range(a.scans):
    s = nxt
    nxt = scan(k + 1) if k + 1 < a.scans else None
    if a.pipeline and nxt is not None:
        ctx.next_scan(nxt)
    ctx.register_scan(s)
    Tg = ctx.current_pose()
    To, _, _ = est.register_scan(s.cpu().numpy())
    gpu.append(Tg)
    cpu.append(To)
    gt.append(synth.trajectory_pose(k))
    worst = max(worst, float(np.abs(Tg - To).max()))
    if k % 50 == 49:
        print(f"scan {k + 1}: max |T_gpu - T_oracle| so far {worst:.3e}  ({time.time() - t0:.0f} s)", flush=True)
print(f"{a.scans} scans{' (pipelined)' if a.pipeline else ''}: max pose difference {worst:.3e}; ATE gpu {metrics.ate_rmse(gpu, gt):.6f} m, "
      f"oracle {metrics.ate_rmse(cpu, gt):.6f} m")
assert worst < 1e-6, "GPU path drifted from the oracle"
