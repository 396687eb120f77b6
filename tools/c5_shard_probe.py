"""VERDICT r5 "next round" 6: the per-rank work of the sharded C5 path measured on ONE GPU,
for the multi-GPU prediction in DESIGN.md §Multi-GPU.

For N = 1, 2, 4, 8 and every shard r of the 2M-point query set (bench.py's contiguous
shards, form_amd/shard.py): the fused match + 7x7 linearization of the shard
(fmx_match without counts + fmx_linearize_matched at the same pose: one k_match<.., FUSED>
launch) behind a 1-rank RCCL communicator (the all-reduce + publish path, no peers), timed
per ICP iteration at the identity pose and at the converged pose; plus the full
registration of the whole set (fmx_register_points) for the iteration count.
Prints one JSON line."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402  (first: libfmx binds torch's HIP runtime)

from form_amd import fmx, shard, synth  # noqa: E402


def main():
    side = int(os.environ.get("C5_SIDE", "7071"))
    nq = int(os.environ.get("C5_QUERIES", str(2 * 1024 * 1024)))
    reps = int(os.environ.get("REPS", "20"))
    w = 0.8
    pos4, nrm4 = shard.terrain_map(side, w, synth.SEED, "cuda:0")
    n_map = pos4.shape[0]
    ctx = fmx.Context(fmx.EstimatorParams(keypoint_pool_capacity=n_map + 1024))
    ctx.comm_init(fmx.comm_unique_id(), 1, 0)
    ctx.keypoints_add_device(0, pos4, nrm4)
    I34 = np.hstack([np.eye(3), np.zeros((3, 1))])
    ctx.map_build([0], I34[None], w)
    out = {"map_voxels": int(n_map), "queries": nq, "per_iteration_ms": {}, "registration": {}}
    for dist in ("local", "wholemap"):
        if dist == "local":
            Ttrue = shard.c5_offset()
            q4, n4 = shard.make_queries(pos4, nrm4, nq, Ttrue, 0.03, synth.SEED + 1)
        else:
            Ttrue = shard.c5_offset(shard.C5_WHOLEMAP_ROT_SCALE)
            q4, n4 = shard.make_queries_wholemap(pos4, nrm4, nq, Ttrue, 0.03, synth.SEED + 2)
        # the whole set: iterations to convergence and the converged pose
        ctx.set_queries_device(q4, n4)
        torch.cuda.synchronize()
        Tc, iters = ctx.register_points(I34, w, 0.1, 30, 1e-4)
        t0 = time.perf_counter()
        for _ in range(reps):
            Tc, iters = ctx.register_points(I34, w, 0.1, 30, 1e-4)
        reg_ms = (time.perf_counter() - t0) / reps * 1e3
        out["registration"][dist] = {"iters": int(iters), "ms": round(reg_ms, 4)}
        rows = {}
        for N in (1, 2, 4, 8):
            per = []
            for r in range(N):
                b, e = shard.shard_bounds(nq, r, N)
                ctx.set_queries_device(q4[b:e].contiguous(), n4[b:e].contiguous())
                torch.cuda.synchronize()
                ts = []
                for T in (I34, Tc):
                    for k in range(reps + 2):
                        t0 = time.perf_counter()
                        ctx.match(T, w, counts=False)
                        ctx.linearize_matched(T, 0.1)
                        if k >= 2:
                            ts.append(time.perf_counter() - t0)
                per.append(float(np.median(ts)) * 1e3)
            rows[str(N)] = {"max_over_shards_ms": round(max(per), 4), "min_ms": round(min(per), 4),
                            "shards_ms": [round(x, 4) for x in per]}
        out["per_iteration_ms"][dist] = rows
        del q4, n4
    ctx.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
