"""The voxel map build (voxelmap.hip: k_map_insert / count / alloc / scatter / dense) at
its edges, checked through bit-exact matches against the oracle's VoxelMap::find_closest
(map.tpp:70-91): 70 rebuilds of one context (the 6-bit build epoch wraps and the table is
cleared once, claim slots / counts reused across builds of different sizes), and maps
whose cells hold hundreds and more than 8192 records (the dense path: sub-cell sort, and
a cell too large to sort, walked whole), and a 7.9M-record two-scan map of both
feature types (the interleaved record layout of the C5 maps)."""
import numpy as np
import pytest

from scenario import perturb, stream_features

pytestmark = pytest.mark.gpu

W = 0.8
I34_ = np.hstack([np.eye(3), np.zeros((3, 1))])


def _check(ctx, omaps, Q, Tj, K):
    cpl, cpt = ctx.match(Tj, W)
    got = ctx.match_download()
    npl = len(Q[0])
    for t, (om, q) in enumerate(zip(omaps, Q)):
        ref = om.match(q, Tj)
        sl = slice(0, npl) if t == 0 else slice(npl, None)
        acc = ref["found"] & (ref["d2"] < W * W)
        pair = got["pair"][sl]
        assert np.array_equal(pair >= 0, acc)
        assert np.array_equal(pair[acc].astype(np.uint64), ref["scan"][acc])
        assert np.array_equal(got["d2"][sl][acc], ref["d2"][acc])
        assert np.array_equal(got["pi"][sl][acc], ref["pi"][acc])
        if t == 0:
            assert np.array_equal(got["ni"][acc], ref["ni"][acc])
        counts = np.bincount(ref["scan"][acc].astype(np.int64), minlength=K)
        assert np.array_equal(cpl if t == 0 else cpt, counts)


def test_rebuilds_across_epoch_wrap(fmx_mod, oracle):
    feats = stream_features(oracle, "tiny", 8)
    p = feats[0]["params"]
    ctx = fmx_mod.Context(fmx_mod.EstimatorParams(extraction=fmx_mod.KeypointExtractionParams(**p),
                                                  voxel_subdivision=1))
    for k in range(7):
        ctx.keypoints_add(k, feats[k]["planar"], feats[k]["point"])
    q = feats[7]
    ctx.set_queries(q["planar"], q["point"], 7)
    rng = np.random.default_rng(3)
    checked = 0
    for b in range(70):
        scans = list(range(7 - b % 7))  # 7..1 scans: biggest first, so storage never grows and only the epoch resets
        poses = [perturb(feats[k]["pose"], rng, 0.002, 0.01) for k in scans]
        ctx.map_build(scans, np.stack(poses), W)
        if b in (0, 1, 61, 62, 63, 64, 69):  # build 63 wraps the epoch (kEpochMax) and clears the table
            omaps = [oracle.VoxelMap(W, 0), oracle.VoxelMap(W, 1)]
            for k, T in zip(scans, poses):
                omaps[0].add_scan(k, T, feats[k]["planar"])
                omaps[1].add_scan(k, T, feats[k]["point"])
            _check(ctx, omaps, (q["planar"], q["point"]), perturb(q["pose"], rng, 0.005, 0.03), len(scans))
            checked += 1
    assert checked == 7


@pytest.mark.parametrize("n_big", [300, 9000])
def test_dense_and_oversized_cells(fmx_mod, oracle, n_big):
    """One cell with n_big planar records (dense: > 128, sub-cell sorted; > 8192: left
    unsorted and walked whole), sparse cells around it, queries inside and beside it."""
    rng = np.random.default_rng(n_big)
    c0 = np.array([0.4, 0.4, 0.4])
    big = c0 + rng.uniform(-0.39, 0.39, size=(n_big, 3))
    sparse = rng.uniform(-3.0, 3.0, size=(2000, 3))
    pos = np.vstack([big, sparse]).astype(np.float32)
    nrm = rng.normal(size=pos.shape)
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    planar = np.hstack([pos, nrm.astype(np.float32)])
    point = rng.uniform(-3.0, 3.0, size=(1500, 3)).astype(np.float32)
    point[:400] = (c0 + rng.uniform(-0.39, 0.39, size=(400, 3))).astype(np.float32)  # a dense point cell too
    prm = fmx_mod.EstimatorParams(voxel_subdivision=1, keypoint_pool_capacity=len(planar) + len(point) + 1024)
    ctx = fmx_mod.Context(prm)
    ctx.keypoints_add(0, planar, point)
    I34 = np.hstack([np.eye(3), np.zeros((3, 1))])
    ctx.map_build([0], I34[None], W)
    omaps = [oracle.VoxelMap(W, 0), oracle.VoxelMap(W, 1)]
    omaps[0].add_scan(0, I34, planar)
    omaps[1].add_scan(0, I34, point)
    qpl = np.vstack([c0 + rng.uniform(-0.6, 0.6, size=(500, 3)), rng.uniform(-3, 3, size=(500, 3))])
    qn = rng.normal(size=qpl.shape)
    qn /= np.linalg.norm(qn, axis=1, keepdims=True)
    Qpl = np.hstack([qpl, qn]).astype(np.float32)
    Qpt = np.vstack([c0 + rng.uniform(-0.6, 0.6, size=(300, 3)), rng.uniform(-3, 3, size=(300, 3))]).astype(np.float32)
    ctx.set_queries(Qpl, Qpt, 1)
    _check(ctx, omaps, (Qpl, Qpt), I34, 1)


def test_large_build_two_scans_both_types(fmx_mod, oracle):
    """A C5-sized map shape (run_map_build's interleaved record layout, >= 4M records)
    from two scans at different poses and both feature types: 5.3M planar + 2.6M point
    records, every match of 24k queries bit-exact against the oracle's VoxelMap, and a
    rebuild of the same context (new epoch, the cells' record order set by the atomics
    again) giving the same matches."""
    import torch
    from form_amd import shard, synth
    side = 2300
    pos4, nrm4 = shard.terrain_map(side, W, synth.SEED + 5, "cuda:0")
    n = pos4.shape[0]
    h = n // 2
    pt4 = pos4[::2].contiguous()  # the point features: every second terrain sample
    hp = pt4.shape[0] // 2
    T1 = shard.expmap(np.array([0.001, -0.002, 0.003, 0.4, -0.3, 0.05]))
    poses = np.stack([I34_, T1])
    T1inv = np.linalg.inv(np.vstack([T1, [0, 0, 0, 1]]))[:3]

    def to_local(x4, T):  # scan 1's records are stored in its own frame
        x = x4[:, :3].double() @ torch.tensor(T[:, :3].T, device=x4.device) + torch.tensor(T[:, 3], device=x4.device)
        return torch.cat([x.float(), x4[:, 3:]], 1).contiguous()
    T1inv_rot = np.hstack([T1inv[:, :3], np.zeros((3, 1))])
    pl0, nl0 = pos4[:h].contiguous(), nrm4[:h].contiguous()
    pl1, nl1 = to_local(pos4[h:], T1inv), to_local(nrm4[h:], T1inv_rot)
    pp0, pp1 = pt4[:hp].contiguous(), to_local(pt4[hp:], T1inv)
    torch.cuda.synchronize()
    ctx = fmx_mod.Context(fmx_mod.EstimatorParams(keypoint_pool_capacity=n + 1024, voxel_subdivision=1))
    ctx.keypoints_add_device(0, pl0, nl0, pp0)
    ctx.keypoints_add_device(1, pl1, nl1, pp1)
    omaps = [oracle.VoxelMap(W, 0), oracle.VoxelMap(W, 1)]
    for k, (pl, nl, pp) in enumerate(((pl0, nl0, pp0), (pl1, nl1, pp1))):
        omaps[0].add_scan(k, poses[k], torch.cat([pl[:, :3], nl[:, :3]], 1).cpu().numpy())
        omaps[1].add_scan(k, poses[k], pp[:, :3].cpu().numpy())
    rng = np.random.default_rng(3)
    qi = rng.choice(n, 16000, replace=False)
    qp = rng.choice(pt4.shape[0], 8000, replace=False)
    Qpl = np.concatenate([pos4[qi, :3].cpu().numpy(), nrm4[qi, :3].cpu().numpy()], 1)
    Qpl[:, :3] += rng.normal(0, 0.05, (len(qi), 3)).astype(np.float32)
    Qpt = pt4[qp, :3].cpu().numpy() + rng.normal(0, 0.05, (len(qp), 3)).astype(np.float32)
    ctx.set_queries(Qpl, Qpt, 2)
    Tj = shard.expmap(np.array([0.0003, 0.0002, -0.0004, 0.01, -0.02, 0.005]))
    got = []
    for _ in range(2):
        ctx.map_build([0, 1], poses, W)
        _check(ctx, omaps, (Qpl, Qpt), Tj, 2)
        got.append(ctx.match_download())
    for k in ("pair", "d2", "pi", "ni"):
        assert np.array_equal(got[0][k], got[1][k]), k
    ctx.close()
