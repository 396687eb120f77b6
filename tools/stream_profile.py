"""Per-scan wall time and work along a long stream (bench.py's pipelined smoothing loop),
in blocks of scans: tells a slower stretch of the synthetic trajectory (more ICP
iterations, larger maps) from a slowdown that grows with the run (something
accumulating).  Diagnostic only.

  python tools/stream_profile.py [--config c2] [--scans 360] [--block 40] [--k0 0]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from form_amd import fmx, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c2")
ap.add_argument("--scans", type=int, default=360)
ap.add_argument("--block", type=int, default=40)
ap.add_argument("--k0", type=int, default=0, help="first trajectory index")
a = ap.parse_args()
geo = synth.GEOMETRIES[a.config]
params = synth.default_params(geo)
w = synth.World()
scans = [synth.raycast(w, synth.trajectory_pose(a.k0 + k), geo, synth.SEED + 7919 * (a.k0 + k + 1), "cuda:0")
         for k in range(a.scans)]
torch.cuda.synchronize()
ctx = fmx.Context(fmx.EstimatorParams(extraction=fmx.KeypointExtractionParams(**params)))
ts, st = [], []
for k in range(a.scans):
    if k + 1 < a.scans:
        ctx.next_scan(scans[k + 1])
    t0 = time.perf_counter()
    ctx.register_scan(scans[k])
    ts.append(time.perf_counter() - t0)
    st.append(ctx.last_stats())
ctx.close()
rows = []
for b0 in range(0, a.scans, a.block):
    sl = slice(b0, min(a.scans, b0 + a.block))
    blk = st[sl]
    rows.append({"scans": [a.k0 + b0, a.k0 + sl.stop], "ms_p50": round(float(np.median(ts[sl])) * 1e3, 3),
                 "ms_mean": round(float(np.mean(ts[sl])) * 1e3, 3),
                 **{k: round(float(np.mean([s[k] for s in blk])), 2)
                    for k in ("icp_iters", "lm_iters", "linearizations", "map_planar", "map_point", "matched_planar",
                              "window_poses", "map_scans")}})
for r in rows:
    print(json.dumps(r))
