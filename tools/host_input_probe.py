"""Host-resident scan input on C4: what the staging copy costs (diagnostic).

  python tools/host_input_probe.py [--scans 40] [--prefill 90]

Times register_scan over the same steady-state C4 scans fed as (a) device tensors,
pipelined (fmx_next_scan) and sequential, (b) pageable numpy arrays (the reference's
host std::vector<PointXYZf> boundary), pipelined and sequential, (c) scans the caller
assembles in fmx_scan_buffer's pinned memory (the copy into it is timed); plus the raw 4-MiB copies (pageable / pinned H2D, a host
memcpy into pinned memory).  One JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from form_amd import fmx, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scans", type=int, default=40)
    ap.add_argument("--prefill", type=int, default=90)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--modes", default="device_sequential,device_pipelined,host_sequential,host_pipelined,"
                                       "pinned_sequential,pinned_pipelined")
    a = ap.parse_args()
    geo = synth.GEOMETRIES["c4"]
    params = synth.default_params(geo)
    w = synth.World()
    total = a.prefill + a.scans + 1
    dscans = [synth.raycast(w, synth.trajectory_pose(k), geo, synth.SEED + 7919 * (k + 1), "cuda:0")
              for k in range(total)]
    torch.cuda.synchronize()
    hscans = [s.cpu().numpy().copy() for s in dscans]
    out = {}
    # raw copies
    n = hscans[0].nbytes
    dst = torch.empty_like(dscans[0])
    pin = torch.empty(dscans[0].shape, dtype=torch.float32).pin_memory()
    for name, fn in (("pageable_h2d_us", lambda h: dst.copy_(torch.from_numpy(h))),
                     ("pinned_h2d_us", lambda h: dst.copy_(pin, non_blocking=True)),
                     ("memcpy_to_pinned_us", lambda h: pin.numpy().__setitem__(Ellipsis, h))):
        ts = []
        for k in range(20):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn(hscans[k])
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        out[name] = round(float(np.median(ts[2:])) * 1e6, 1)
    out["bytes"] = n

    def run(mode):
        ctx = fmx.Context(fmx.EstimatorParams(extraction=fmx.KeypointExtractionParams(**params)))
        for k in range(a.prefill):
            ctx.register_scan(dscans[k])
        ctx.sync()
        pipeline = mode.endswith("pipelined")
        scans = dscans if mode.startswith("device") else hscans
        pinned = mode.startswith("pinned")
        bufs = {}

        def get(k):  # pinned: the caller assembles scan k in an fmx_scan_buffer (timed)
            if not pinned:
                return scans[k]
            if k not in bufs:
                b = ctx.scan_buffer()
                np.copyto(b, hscans[k])
                bufs[k] = b
            return bufs[k]
        t0 = time.perf_counter()
        for k in range(a.prefill, a.prefill + a.scans):
            if pipeline:
                ctx.next_scan(get(k + 1))
            ctx.register_scan(get(k))
            bufs.pop(k - 1, None)
        ctx.sync()
        dt = time.perf_counter() - t0
        T = ctx.current_pose()
        ctx.close()
        return a.scans / dt, T

    modes = [m for m in a.modes.split(",") if m]
    res = {m: [] for m in modes}
    poses = {}
    for _ in range(a.reps):
        for m in modes:
            v, T = run(m)
            res[m].append(round(v, 1))
            poses[m] = T
    out["scans_per_s"] = res
    out["env"] = {k: v for k, v in os.environ.items() if k.startswith("FMX_")}
    ref = poses[modes[0]]
    out["max_pose_diff_vs_" + modes[0]] = {m: float(np.abs(T - ref).max()) for m, T in poses.items()}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
