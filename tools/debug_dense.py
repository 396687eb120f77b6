"""Scratch: dense-cell match mismatches per scenario (GPU vs oracle)."""
import sys, os
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import oracle_py as O
from form_amd import fmx, synth

I34 = np.hstack([np.eye(3), np.zeros((3, 1))])
p = synth.default_params(synth.GEOMETRIES["tiny"])


def planar(xyz, rng):
    n = rng.normal(size=(len(xyz), 3))
    n /= np.linalg.norm(n, axis=1, keepdims=True)
    return np.ascontiguousarray(np.hstack([xyz, n]).astype(np.float32))


def run(name, blocks, queries, subdiv=1, w=0.8):
    rng = np.random.default_rng(3)
    ctx = fmx.Context(fmx.EstimatorParams(extraction=fmx.KeypointExtractionParams(**p), voxel_subdivision=subdiv))
    om = O.VoxelMap(w, 0)
    ids, poses = [], []
    for k, b in enumerate(blocks):
        pl = planar(b, rng)
        ctx.keypoints_add(k, pl, np.zeros((0, 3), np.float32))
        om.add_scan(k, I34, pl)
        ids.append(k)
        poses.append(I34)
    ctx.map_build(ids, np.stack(poses), w)
    q = planar(queries, rng)
    ctx.set_queries(q, np.zeros((0, 3), np.float32), 99)
    ctx.match(I34, w)
    got = ctx.match_download()
    ref = om.match(q, I34)
    acc = ref["found"] & (ref["d2"] < w * w)
    bad = np.nonzero((got["d2"][acc] != ref["d2"][acc]))[0]
    print(name, "queries", acc.sum(), "bad", len(bad), flush=True)
    if len(bad):
        i = np.nonzero(acc)[0][bad[0]]
        print("  q", q[i, :3], "gpu d2", got["d2"][i], "ref", ref["d2"][i], "gpu pi", got["pi"][i], "ref pi", ref["pi"][i])


rng = np.random.default_rng(1)
box = lambda n, lo, hi: rng.uniform(lo, hi, (n, 3))
qbox = box(2000, 3.25, 3.95) + np.array([0, 0.8, 0.8])
for n in (200, 1000, 4000, 8000, 9000):
    run(f"one cell {n}", [box(n, 3.25, 3.95) + np.array([0, 0.8, 0.8])], qbox)
run("cluster 6x2500", [box(2500, -0.8, 0.8) for _ in range(6)], box(3000, -1.2, 1.2))
run("one cell 4000 split 4 scans", [box(1000, 3.25, 3.95) + np.array([0, 0.8, 0.8]) for _ in range(4)], qbox)
run("one cell 9000 subdiv2", [box(9000, 3.25, 3.95) + np.array([0, 0.8, 0.8])], qbox, subdiv=2)
