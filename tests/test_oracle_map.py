"""Oracle voxel map + matcher vs a brute-force numpy nearest neighbour restricted to
the 27 voxels around the query (map.tpp:54-91), and the world->local round trip
(matcher.hpp:92-96)."""
import numpy as np

import np_ref
from scenario import perturb


def test_match_vs_bruteforce(oracle):
    rng = np.random.default_rng(2)
    w = 0.8
    m = oracle.VoxelMap(w, 0)
    poses, locs, worlds = [], [], []
    for s in range(3):
        T = np_ref.compose(np_ref.pose(np.eye(3), rng.normal(size=3)), np_ref.expmap(rng.normal(size=6) * 0.2))
        f = np.zeros((400, 6), np.float32)
        f[:, :3] = rng.uniform(-6, 6, (400, 3))
        n = rng.normal(size=(400, 3))
        f[:, 3:] = n / np.linalg.norm(n, axis=1, keepdims=True)
        m.add_scan(s, T, f)
        poses.append(T)
        locs.append(f)
        worlds.append((T[:, :3] @ f[:, :3].astype(np.float64).T).T + T[:, 3])
    allw = np.concatenate(worlds)
    scan_of = np.repeat(np.arange(3), 400)
    q = np.zeros((300, 6), np.float32)
    q[:, :3] = rng.uniform(-6, 6, (300, 3))
    Tj = perturb(np_ref.pose(np.eye(3), np.zeros(3)), rng, 0.1, 0.5)
    res = m.match(q, Tj)
    qw = (Tj[:, :3] @ q[:, :3].astype(np.float64).T).T + Tj[:, 3]
    for i in range(len(q)):
        j, d2 = np_ref.voxel_nn(allw, qw[i], w)
        assert res["found"][i] == (j >= 0)
        if j < 0:
            continue
        assert np.isclose(res["d2"][i], d2, rtol=1e-12, atol=1e-15)
        assert res["scan"][i] == scan_of[j]
        # the matched point moved back into its scan's frame ~= the stored local point
        assert np.allclose(res["pi"][i], locs[scan_of[j]][j % 400, :3], atol=1e-9)
        assert np.allclose(res["ni"][i], locs[scan_of[j]][j % 400, 3:], atol=1e-9)
    assert m.num_voxels() > 100
