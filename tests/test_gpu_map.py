"""Voxel map build + nearest-neighbour match edge cases, HIP path vs the oracle.

* exact distance ties: the reference keeps the first record in its fixed shift order
  (map.tpp:54-68), then in insertion order inside a voxel (map.tpp:41-52, 77-88);
  k_match's argmin key (d^2, shift rank, build order) must pick the same record even
  when build order and shift order disagree;
* dense cells (> 64 records: sorted into 4 x 4 x 4 sub-cells with a header; > 8192:
  left unsorted and scanned whole), on plain and subdivided maps;
* repeated builds on one context: the brick table is never cleared between builds
  (epoch-tagged keys), so stale bricks of earlier builds — including across the
  63-build epoch wrap — must never be found.
Bar: bit-exact (pair, d^2, p_i, n_i, insert decision, per-pair counts).
"""
import numpy as np
import pytest

from form_amd import synth

pytestmark = pytest.mark.gpu

I34 = np.hstack([np.eye(3), np.zeros((3, 1))])


def _ctx(fmx_mod, subdiv=1):
    p = synth.default_params(synth.GEOMETRIES["tiny"])
    return fmx_mod.Context(fmx_mod.EstimatorParams(extraction=fmx_mod.KeypointExtractionParams(**p),
                                                   voxel_subdivision=subdiv))


def _planar(xyz, rng=None):
    xyz = np.asarray(xyz, np.float32).reshape(-1, 3)
    if rng is None:
        n = np.tile(np.array([0, 0, 1], np.float32), (len(xyz), 1))
    else:
        n = rng.normal(size=(len(xyz), 3))
        n = (n / np.linalg.norm(n, axis=1, keepdims=True)).astype(np.float32)
    return np.ascontiguousarray(np.hstack([xyz, n]).astype(np.float32))


def _check(ctx, oracle, scans, poses, qpl, qpt, Tj, w, max_dist):
    """Build, match and compare against the oracle VoxelMap (both feature types)."""
    omaps = [oracle.VoxelMap(w, 0), oracle.VoxelMap(w, 1)]
    for k, (pl, pt) in enumerate(scans):
        omaps[0].add_scan(k, poses[k], pl)
        omaps[1].add_scan(k, poses[k], pt)
    ctx.map_build(list(range(len(scans))), np.stack(poses), w)
    ctx.set_queries(qpl, qpt, len(scans))
    cpl, cpt = ctx.match(Tj, max_dist)
    got = ctx.match_download()
    npl = len(qpl)
    for t, (om, Q) in enumerate(zip(omaps, (qpl, qpt))):
        ref = om.match(Q, Tj)
        sl = slice(0, npl) if t == 0 else slice(npl, None)
        acc = ref["found"] & (ref["d2"] < max_dist * max_dist)
        pair = got["pair"][sl]
        assert np.array_equal(pair >= 0, acc)
        assert np.array_equal(pair[acc].astype(np.uint64), ref["scan"][acc])
        bad = np.nonzero(got["d2"][sl][acc] != ref["d2"][acc])[0]
        assert len(bad) == 0, (t, len(bad), Q[acc][bad[:4]], got["d2"][sl][acc][bad[:4]], ref["d2"][acc][bad[:4]],
                               got["pi"][sl][acc][bad[:4]], ref["pi"][acc][bad[:4]])
        assert np.array_equal(got["pi"][sl][acc], ref["pi"][acc])
        if t == 0:
            assert np.array_equal(got["ni"][acc], ref["ni"][acc])
        assert np.array_equal(got["d2"][sl] > 0.01, ~ref["found"] | (ref["d2"] > 0.01))
        counts = np.bincount(ref["scan"][acc].astype(np.int64), minlength=len(scans))
        assert np.array_equal(cpl if t == 0 else cpt, counts)
    return got


def _tie_cases():
    """(scan 0 records, scan 1 records, query) per region; every coordinate exact in
    fp32 and every tied distance exact in fp64.  Build order puts scan 0 first."""
    cases = [
        # faces +x (rank 1) vs -x (rank 2): the reference takes +x, which is in scan 1
        ([(-0.25, 0.5, 0.5)], [(1.25, 0.5, 0.5)], (0.5, 0.5, 0.5)),
        # own voxel (rank 0, scan 1) vs the +z face (rank 5, scan 0)
        ([(0.5, 0.5, 1.125)], [(0.5, 0.5, 0.625)], (0.5, 0.5, 0.875)),
        # edges (1, 1, 0) (rank 7, scan 1) vs (-1, -1, 0) (rank 10, scan 0)
        ([(-0.25, -0.25, 0.5)], [(1.25, 1.25, 0.5)], (0.5, 0.5, 0.5)),
        # corners (1, 1, 1) (rank 19, scan 1) vs (-1, -1, -1) (rank 26, scan 0)
        ([(-0.25, -0.25, -0.25)], [(1.25, 1.25, 1.25)], (0.5, 0.5, 0.5)),
        # one voxel, two scans: insertion order (scan 0 first)
        ([(0.75, 0.5, 0.5)], [(0.25, 0.5, 0.5)], (0.5, 0.5, 0.5)),
        # the face -y (rank 4, scan 1) vs the edge (1, 1, 0) (rank 7, scan 0) at the same
        # distance 1.25 (> the voxel width: found by the unbounded search, max_dist 1.3)
        ([(1.25, 1.5, 0.5)], [(0.5, -0.75, 0.5)], (0.5, 0.5, 0.5)),
    ]
    return cases


@pytest.mark.parametrize("kind", ["planar", "point"])
def test_exact_ties_follow_reference_shift_order(fmx_mod, oracle, kind):
    w = 1.0
    s0, s1, q = [], [], []
    for r, (a, b, qq) in enumerate(_tie_cases()):
        off = np.array([8.0 * r, 0.0, 0.0])
        s0 += [np.add(p, off) for p in a]
        s1 += [np.add(p, off) for p in b]
        q.append(np.add(qq, off))
    empty_pl, empty_pt = np.zeros((0, 6), np.float32), np.zeros((0, 3), np.float32)
    if kind == "planar":
        scans = [(_planar(s0), empty_pt), (_planar(s1), empty_pt)]
        qpl, qpt = _planar(q), empty_pt
    else:
        scans = [(empty_pl, np.asarray(s0, np.float32)), (empty_pl, np.asarray(s1, np.float32))]
        qpl, qpt = empty_pl, np.asarray(q, np.float32)
    ctx = _ctx(fmx_mod)
    for k, (pl, pt) in enumerate(scans):
        ctx.keypoints_add(k, pl, pt)
    got = _check(ctx, oracle, scans, [I34, I34], qpl, qpt, I34, w, 1.3)
    pair = got["pair"]
    # the cases' winners: scan 1 except the same-voxel case (insertion order: scan 0)
    assert list(pair) == [1, 1, 1, 1, 0, 1]


@pytest.mark.parametrize("subdiv,max_dist", [(1, 0.8), (2, 0.8), (1, 1.0)])
def test_dense_cells_match_oracle(fmx_mod, oracle, subdiv, max_dist):
    """Clusters of thousands of records per 0.8 m cell (sub-cell headers) and one cell
    with 9000 records of one scan (> 8192: scanned unsorted), queries in and around
    them at a perturbed pose.  max_dist 1.0 > the voxel width: the unbounded search
    (no prune bound until the first record is found)."""
    rng = np.random.default_rng(11)
    w = 0.8
    scans, poses = [], []
    for k in range(6):
        c = rng.uniform(-0.8, 0.8, (2500, 3))                       # ~1500 per cell
        flat = np.c_[rng.uniform(2, 6, 1500), rng.uniform(-1, 1, 1500), rng.normal(0, 0.01, 1500) - 1.5]
        pl = np.vstack([c, flat])
        if k == 2:
            pl = np.vstack([pl, np.c_[rng.uniform(3.25, 3.95, 9000), rng.uniform(4.05, 4.75, (9000, 2))]])
        pt = rng.uniform(-0.8, 0.8, (600, 3))
        T = I34.copy()
        T[:, 3] = rng.normal(0, 0.01, 3)
        poses.append(T)
        scans.append((_planar(pl, rng), np.asarray(pt, np.float32)))
    qpl = _planar(np.vstack([rng.uniform(-1.2, 1.2, (3000, 3)),
                             np.c_[rng.uniform(2, 6, 1000), rng.uniform(-1, 1, 1000), np.full(1000, -1.45)],
                             np.c_[rng.uniform(3.1, 4.1, 1000), rng.uniform(3.9, 4.9, (1000, 2))]]), rng)
    qpt = np.asarray(rng.uniform(-1.2, 1.2, (1500, 3)), np.float32)
    ctx = _ctx(fmx_mod, subdiv)
    for k, (pl, pt) in enumerate(scans):
        ctx.keypoints_add(k, pl, pt)
    Tj = I34.copy()
    Tj[:, 3] = [0.003, -0.002, 0.001]
    _check(ctx, oracle, scans, poses, qpl, qpt, Tj, w, max_dist)


def test_repeated_builds_epoch_wrap(fmx_mod, oracle):
    """70 builds on one context alternating two window sets and voxel widths (the brick
    table is reused with a new epoch each build and cleared when the epoch wraps at 63):
    every match equals the oracle's for the current build only."""
    rng = np.random.default_rng(5)
    feats = []
    for k in range(4):
        pl = rng.uniform(-3, 3, (400, 3))
        feats.append((_planar(pl, rng), np.asarray(rng.uniform(-3, 3, (100, 3)), np.float32)))
    qpl = _planar(rng.uniform(-3.5, 3.5, (500, 3)), rng)
    qpt = np.asarray(rng.uniform(-3.5, 3.5, (200, 3)), np.float32)
    ctx = _ctx(fmx_mod)
    for k, (pl, pt) in enumerate(feats):
        ctx.keypoints_add(k, pl, pt)
    sets = [[0, 1, 2, 3], [1, 3]]
    for b in range(70):
        ids = sets[b % 2]
        w = 0.8 if b % 3 else 0.6
        poses = []
        for k in ids:
            T = I34.copy()
            T[:, 3] = [0.01 * b, 0.0, 0.02 * k]
            poses.append(T)
        # the oracle numbers scans 0..n-1 in build order; the context keeps the real ids
        ctx.map_build(ids, np.stack(poses), w)
        ctx.set_queries(qpl, qpt, 9)
        cpl, cpt = ctx.match(I34, w)
        got = ctx.match_download()
        for t, Q in enumerate((qpl, qpt)):
            om = oracle.VoxelMap(w, t)
            for k, T in zip(ids, poses):
                om.add_scan(k, T, feats[k][t])
            ref = om.match(Q, I34)
            sl = slice(0, len(qpl)) if t == 0 else slice(len(qpl), None)
            acc = ref["found"] & (ref["d2"] < w * w)
            pair = got["pair"][sl]
            assert np.array_equal(pair >= 0, acc), b
            assert np.array_equal(np.asarray(ids, np.uint64)[pair[acc]], ref["scan"][acc]), b
            assert np.array_equal(got["d2"][sl][acc], ref["d2"][acc]), b


def test_dense_cells_warm_from_cell_cache(fmx_mod, oracle):
    """The dense-cell fixture above matched at several poses on ONE map and query set:
    every match after the first is warm (bounded by the previous NN record, the own cell
    — range and dense bit — from the per-query cell cache, no brick probe).  Each match
    is bit-exact to the oracle; the fixture puts thousands of queries in dense own cells;
    and the warm match probes at least half a brick fewer per query than a cold match
    at the same pose (the cache is hit)."""
    rng = np.random.default_rng(11)
    w = 0.8
    scans, poses = [], []
    for k in range(6):
        c = rng.uniform(-0.8, 0.8, (2500, 3))
        flat = np.c_[rng.uniform(2, 6, 1500), rng.uniform(-1, 1, 1500), rng.normal(0, 0.01, 1500) - 1.5]
        pl = np.vstack([c, flat])
        if k == 2:
            pl = np.vstack([pl, np.c_[rng.uniform(3.25, 3.95, 9000), rng.uniform(4.05, 4.75, (9000, 2))]])
        pt = rng.uniform(-0.8, 0.8, (600, 3))
        T = I34.copy()
        T[:, 3] = rng.normal(0, 0.01, 3)
        poses.append(T)
        scans.append((_planar(pl, rng), np.asarray(pt, np.float32)))
    qpl = _planar(np.vstack([rng.uniform(-1.2, 1.2, (3000, 3)),
                             np.c_[rng.uniform(2, 6, 1000), rng.uniform(-1, 1, 1000), np.full(1000, -1.45)],
                             np.c_[rng.uniform(3.1, 4.1, 1000), rng.uniform(3.9, 4.9, (1000, 2))]]), rng)
    qpt = np.asarray(rng.uniform(-1.2, 1.2, (1500, 3)), np.float32)
    ctx = _ctx(fmx_mod)
    for k, (pl, pt) in enumerate(scans):
        ctx.keypoints_add(k, pl, pt)
    omaps = [oracle.VoxelMap(w, 0), oracle.VoxelMap(w, 1)]
    for k, (pl, pt) in enumerate(scans):
        omaps[0].add_scan(k, poses[k], pl)
        omaps[1].add_scan(k, poses[k], pt)
    ctx.map_build(list(range(len(scans))), np.stack(poses), w)
    # queries whose own cell is dense (> 128 records) in the world map
    wp = np.vstack([pl[:, :3].astype(np.float64) @ poses[k][:, :3].T + poses[k][:, 3]
                    for k, (pl, _) in enumerate(scans)])
    cells, cnt = np.unique(np.floor(wp / w).astype(np.int64), axis=0, return_counts=True)
    dense = {tuple(c) for c in cells[cnt > 128]}
    assert sum(tuple(c) in dense for c in np.floor(qpl[:, :3].astype(np.float64) / w).astype(np.int64)) > 2000

    def match_cmp(Tj):
        cpl, cpt = ctx.match(Tj, w)
        got = ctx.match_download()
        npl = len(qpl)
        for t, (om, Q) in enumerate(zip(omaps, (qpl, qpt))):
            ref = om.match(Q, Tj)
            sl = slice(0, npl) if t == 0 else slice(npl, None)
            acc = ref["found"] & (ref["d2"] < w * w)
            pair = got["pair"][sl]
            assert np.array_equal(pair >= 0, acc)
            assert np.array_equal(pair[acc].astype(np.uint64), ref["scan"][acc])
            assert np.array_equal(got["d2"][sl][acc], ref["d2"][acc])
            assert np.array_equal(got["pi"][sl][acc], ref["pi"][acc])
            if t == 0:
                assert np.array_equal(got["ni"][acc], ref["ni"][acc])
            assert np.array_equal(got["d2"][sl] > 0.01, ~ref["found"] | (ref["d2"] > 0.01))
        return ctx.match_work()

    ctx.profile(True)
    ctx.set_queries(qpl, qpt, 6)
    steps = [(0.003, -0.002, 0.001), (0.0031, -0.0021, 0.0012), (0.0031, -0.0021, 0.00121), (0.05, 0.04, -0.03),
             (0.0031, -0.0021, 0.00121)]
    warm = None
    for i, tr in enumerate(steps):
        Tj = I34.copy()
        Tj[:, 3] = tr
        wk = match_cmp(Tj)
        if i == 2:
            warm = wk
    nq = len(qpl) + len(qpt)
    ctx.set_queries(qpl, qpt, 6)  # same features, new query set: a cold match
    Tj = I34.copy()
    Tj[:, 3] = steps[2]
    cold = match_cmp(Tj)
    ctx.profile(False)
    assert warm["probes"] < cold["probes"] - 0.5 * nq, (warm, cold, nq)
    assert warm["candidates"] <= cold["candidates"], (warm, cold)
