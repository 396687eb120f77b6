"""C5 scale: the full 50M-voxel terrain submap on the
device, a sampled 64k-point scan, bit-exact against the CPU oracle's VoxelMap; the
registration converges from the injected offset; the sharded exchange step (RCCL
communicator on the context stream; two ranks each running the HIP path on its shard)
reproduces the unsharded normal equations.

The oracle cannot hold 50M voxels cheaply, and does not need to: a query's nearest
neighbour lies in its 27 voxels (map.tpp:54-91), so the oracle map is built from every
terrain feature within +-3 grid columns of a sampled query — a superset of those 27
voxels' contents — while the device matches against the whole map.
"""
import os
import socket

import numpy as np
import pytest

from form_amd import shard, synth

pytestmark = pytest.mark.gpu

SIDE, W = 7071, 0.8  # 50M voxels, the bench's C5 map
I34 = np.hstack([np.eye(3), np.zeros((3, 1))])


@pytest.fixture(scope="module")
def c5_map():
    import torch
    pos4, nrm4 = shard.terrain_map(SIDE, W, synth.SEED, "cuda:0")
    torch.cuda.synchronize()
    return pos4, nrm4


def _ctx(fmx, n_map):
    return fmx.Context(fmx.EstimatorParams(keypoint_pool_capacity=n_map + 1024, voxel_subdivision=1))


def _near_features(pos4, nrm4, qw):
    """Every terrain feature within +-3 grid columns of the world points qw (numpy)."""
    import torch
    ic = np.rint(qw[:, 0] / W + 0.5 * SIDE - 0.5).astype(np.int64)
    jc = np.rint(qw[:, 1] / W + 0.5 * SIDE - 0.5).astype(np.int64)
    d = np.arange(-3, 4)
    ii = np.clip(ic[:, None, None] + d[None, :, None], 0, SIDE - 1)
    jj = np.clip(jc[:, None, None] + d[None, None, :], 0, SIDE - 1)
    idx = np.unique((ii * SIDE + jj).ravel())
    t = torch.as_tensor(idx, device=pos4.device)
    feats = torch.cat([pos4[t, :3], nrm4[t, :3]], 1).cpu().numpy()
    return np.ascontiguousarray(feats)


@pytest.mark.parametrize("dist", ["local", "wholemap"])
def test_c5_match_full_map_matches_oracle(fmx_mod, oracle, c5_map, dist):
    """The bench's two C5 query sets: a 240 m terrain scan (samples with replacement)
    and distinct features drawn across the whole 50M-voxel map (up to ~4 km away, so
    the rotation of the ICP iterate is scaled down as in the bench)."""
    pos4, nrm4 = c5_map
    n_map = pos4.shape[0]
    assert n_map == SIDE * SIDE > 50_000_000 - 100_000
    rs = 1.0 if dist == "local" else shard.C5_WHOLEMAP_ROT_SCALE
    Tt = shard.c5_offset(rs)
    make = shard.make_queries if dist == "local" else shard.make_queries_wholemap
    q4, n4 = make(pos4, nrm4, 65536, Tt, 0.03, 77)
    ctx = _ctx(fmx_mod, n_map)
    ctx.keypoints_add_device(0, pos4, nrm4)
    ctx.map_build([0], I34[None], W)
    ctx.set_queries_device(q4, n4)
    Tj = shard.expmap(np.array([0.0005 * rs, -0.0003 * rs, 0.0008 * rs, 0.02, 0.01, -0.01]))  # an ICP iterate
    cpl, _ = ctx.match(Tj, W)
    got = ctx.match_download()
    Q = np.concatenate([q4[:, :3].cpu().numpy(), n4[:, :3].cpu().numpy()], 1)
    qw = Q[:, :3].astype(np.float64) @ Tj[:, :3].T + Tj[:, 3]
    om = oracle.VoxelMap(W, 0)
    om.add_scan(0, I34, _near_features(pos4, nrm4, qw))
    ref = om.match(Q, Tj)
    acc = ref["found"] & (ref["d2"] < W * W)
    assert acc.sum() > 60000
    assert np.array_equal(got["pair"] >= 0, acc)
    assert np.array_equal(got["d2"][acc], ref["d2"][acc])
    assert np.array_equal(got["pi"][acc], ref["pi"][acc])
    assert np.array_equal(got["ni"][acc], ref["ni"][acc])
    assert cpl[0] == acc.sum()
    # the summed single-pose system over those matches
    S, e = ctx.linearize_matched(Tj, 0.1)
    G, er = oracle.linearize(np.array([acc.sum()], np.uint32), ref["pi"][acc], ref["ni"][acc],
                             Q[acc, :3].astype(np.float64), np.array([0], np.uint32), np.zeros((0, 3)),
                             np.zeros((0, 3)), I34[None], Tj[None], 0.1, True)
    assert np.all(np.abs(S - G[0]) <= 1e-10 * np.abs(G[0]).max())
    assert abs(e - er[0]) <= 1e-10 * er[0]


def test_c5_registration_converges(fmx_mod, c5_map):
    """ICP from the identity against the full map recovers the injected 5 cm / 0.1 deg
    offset to well below it (the terrain constrains x, y and yaw too)."""
    pos4, nrm4 = c5_map
    Tt = shard.c5_offset()
    q4, n4 = shard.make_queries(pos4, nrm4, 262144, Tt, 0.03, 78)
    ctx = _ctx(fmx_mod, pos4.shape[0])
    ctx.keypoints_add_device(0, pos4, nrm4)
    ctx.map_build([0], I34[None], W)
    ctx.set_queries_device(q4, n4)
    T = I34.copy()
    for it in range(30):
        if it == 0:  # the counting, waiting call and the no-wait call give the same system
            ctx.match(T, W)
            S0, e0 = ctx.linearize_matched(T, 0.1)
        ctx.match(T, W, counts=False)  # as bench.py's c5_register
        S, err = ctx.linearize_matched(T, 0.1)
        if it == 0:  # fused match + linearization vs the stored-results path: summation order only
            assert np.all(np.abs(S - S0) <= 1e-10 * np.abs(S0).max()) and abs(err - e0) <= 1e-10 * e0
        dx = shard.gauss_newton_step(S)
        T = shard.compose(T, shard.expmap(dx))
        if np.linalg.norm(dx) < 1e-4:
            break
    et, er = shard.pose_error(T, Tt)
    e0t, e0r = shard.pose_error(I34, Tt)
    assert it < 10
    assert et < 0.02 * e0t and er < 0.02 * e0r, (et, er, e0t, e0r)


def test_register_points_equals_python_loop(fmx_mod, c5_map):
    """fmx_register_points (the ICP loop inside libfmx, bench.py's C5 step) follows the
    same iterates as the loop driven from Python over fmx_match + fmx_linearize_matched
    (its 6 x 6 solve is a Cholesky instead of numpy's LU: iterates agree to 1e-9), on
    the fused (large query set) and the materialized (small set) paths."""
    pos4, nrm4 = c5_map
    Tt = shard.c5_offset()
    for n in (300000, 50000):
        q4, n4 = shard.make_queries(pos4, nrm4, n, Tt, 0.03, 83)
        ctx = _ctx(fmx_mod, pos4.shape[0])
        ctx.keypoints_add_device(0, pos4, nrm4)
        ctx.map_build([0], I34[None], W)
        ctx.set_queries_device(q4, n4)
        T = I34.copy()
        for it in range(30):
            ctx.match(T, W, counts=False)
            S, _ = ctx.linearize_matched(T, 0.1)
            dx = shard.gauss_newton_step(S)
            T = shard.compose(T, shard.expmap(dx))
            if np.linalg.norm(dx) < 1e-4:
                break
        T2, iters = ctx.register_points(I34, W, 0.1, 30, 1e-4)
        assert iters == it + 1, (n, iters, it + 1)
        assert np.abs(T2 - T).max() < 1e-9, (n, np.abs(T2 - T).max())
        et, _ = shard.pose_error(T2, Tt)
        assert et < 0.001
        got = ctx.match_download()  # the last iterate's match is still available
        assert (got["pair"] >= 0).sum() > 0.9 * n
        ctx.close()


def test_fused_match_linearize(fmx_mod, oracle, c5_map):
    """fmx_match without counts on a large query set is deferred; fmx_linearize_matched
    at the same pose then runs match + linearization in one launch (no per-query
    results): the system equals the two-step path's to 1e-10 (summation order), the
    profile shows the fused kernel, and a later fmx_match_download still gets the
    match (launched on demand), bit-equal to a counted match."""
    pos4, nrm4 = c5_map
    q4, n4 = shard.make_queries(pos4, nrm4, 300000, shard.c5_offset(), 0.03, 81)
    ctx = _ctx(fmx_mod, pos4.shape[0])
    ctx.keypoints_add_device(0, pos4, nrm4)
    ctx.map_build([0], I34[None], W)
    ctx.set_queries_device(q4, n4)
    Tj = shard.expmap(np.array([0.0005, -0.0003, 0.0008, 0.02, 0.01, -0.01]))
    ctx.match(Tj, W)
    ref = ctx.match_download()
    S0, e0 = ctx.linearize_matched(Tj, 0.1)
    ctx.profile(True)
    ctx.profile_reset()
    ctx.match(Tj, W, counts=False)
    S1, e1 = ctx.linearize_matched(Tj, 0.1)
    S2, e2 = ctx.linearize_matched(Tj, 0.1)  # the match is still deferred: fused again, same sums
    prof = ctx.profile_read()
    ctx.profile(False)
    assert prof["match_linearize"]["launches"] == 2 and prof["match"]["launches"] == 0
    assert prof["linearize"]["launches"] == 0
    assert np.all(np.abs(S1 - S0) <= 1e-10 * np.abs(S0).max()) and abs(e1 - e0) <= 1e-10 * e0
    assert np.array_equal(S1, S2) and e1 == e2
    got = ctx.match_download()  # settles the deferred match
    for k in ("pair", "d2", "pi", "ni"):
        assert np.array_equal(got[k], ref[k]), k
    # at another pose the deferred match is launched first, then linearized as stored
    ctx.match(Tj, W, counts=False)
    T2 = shard.expmap(np.array([0.0004, -0.0003, 0.0008, 0.02, 0.01, -0.01]))
    S3, _ = ctx.linearize_matched(T2, 0.1)
    ctx.match(Tj, W)
    S4, _ = ctx.linearize_matched(T2, 0.1)
    assert np.array_equal(S3, S4)


def test_fused_first_match_with_profiling(fmx_mod, c5_map):
    """A fresh context whose first match is the deferred one, consumed fused while
    profiling (the bench's C5 loop): the work counters of the fused launch are read
    (byte model) and the system equals the two-step path's of a second context."""
    pos4, nrm4 = c5_map
    q4, n4 = shard.make_queries(pos4, nrm4, 200000, shard.c5_offset(), 0.03, 82)
    out = []
    for fused in (True, False):
        ctx = _ctx(fmx_mod, pos4.shape[0])
        ctx.keypoints_add_device(0, pos4, nrm4)
        ctx.map_build([0], I34[None], W)
        ctx.set_queries_device(q4, n4)
        ctx.profile(True)
        ctx.profile_reset()
        ctx.match(I34, W, counts=not fused)
        out.append(ctx.linearize_matched(I34, 0.1))
        ctx.sync()
        prof = ctx.profile_read()
        work = ctx.match_work()
        assert prof["match_linearize" if fused else "match"]["launches"] == 1
        ctx.profile(False)
        ctx.close()
        assert work["candidates"] > 0 and work["probes"] > 0
    (S0, e0), (S1, e1) = out
    assert np.all(np.abs(S0 - S1) <= 1e-10 * np.abs(S1).max()) and abs(e0 - e1) <= 1e-10 * e1


def test_comm_single_rank_is_identity(fmx_mod, c5_map):
    """A one-rank RCCL communicator (the device all-reduce path on a 1-GPU box): the
    all-reduced systems equal the plain ones bit for bit."""
    pos4, nrm4 = c5_map
    q4, n4 = shard.make_queries(pos4, nrm4, 100000, shard.c5_offset(), 0.03, 79)
    out = []
    for use_comm in (False, True):
        ctx = _ctx(fmx_mod, pos4.shape[0])
        if use_comm:
            ctx.comm_init(fmx_mod.comm_unique_id(), 1, 0)
        ctx.keypoints_add_device(0, pos4, nrm4)
        ctx.map_build([0], I34[None], W)
        ctx.set_queries_device(q4, n4)
        ctx.match(I34, W, counts=False)
        Sf, ef = ctx.linearize_matched(I34, 0.1)  # fused
        ctx.match(I34, W)
        S, e = ctx.linearize_matched(I34, 0.1)
        G, err = ctx.linearize(I34[None], I34[None], 0.1, False)
        out.append((S, e, G, err, Sf, ef))
        ctx.close()
    (S0, e0, G0, r0, F0, f0), (S1, e1, G1, r1, F1, f1) = out
    assert np.array_equal(S0, S1) and e0 == e1
    assert np.array_equal(G0, G1) and np.array_equal(r0, r1)
    assert np.array_equal(F0, F1) and f0 == f1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shard_worker(rank, world, port, out_dir):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import torch
    import torch.distributed as dist

    from form_amd import fmx
    from form_amd import shard as sh
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    side = 1501  # 2.25M voxels: the sharding logic, not the map size, is under test
    pos4, nrm4 = sh.terrain_map(side, W, synth.SEED, "cuda:0")
    q4, n4 = sh.make_queries(pos4, nrm4, 200000, sh.c5_offset(), 0.03, 80)
    b, e = sh.shard_bounds(q4.shape[0], rank, world)
    ctx = fmx.Context(fmx.EstimatorParams(keypoint_pool_capacity=pos4.shape[0] + 1024))
    ctx.keypoints_add_device(0, pos4, nrm4)
    ctx.map_build([0], I34[None], W)
    ctx.set_queries_device(q4[b:e].contiguous(), n4[b:e].contiguous())
    Tj = sh.expmap(np.array([0.0005, -0.0003, 0.0008, 0.02, 0.01, -0.01]))
    ctx.match(Tj, W)
    S, err = ctx.linearize_matched(Tj, 0.1)
    Ssum = sh.allreduce_sum(np.append(S, err))  # the host exchange (gloo) over the HIP results
    np.save(os.path.join(out_dir, f"S_{rank}.npy"), Ssum)
    torch.cuda.synchronize()
    ctx.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_shards_match_unsharded(fmx_mod, tmp_path):
    """World size 2 (gloo for the exchange, both ranks on this box's GPU): each rank
    runs the HIP match + linearization on its half of the points; the all-reduced
    system equals one process's unsharded system to 1e-10 and is identical on both
    ranks."""
    import torch.multiprocessing as mp
    world = 2
    mp.spawn(_shard_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    S = [np.load(tmp_path / f"S_{r}.npy") for r in range(world)]
    assert np.array_equal(S[0], S[1])
    pos4, nrm4 = shard.terrain_map(1501, W, synth.SEED, "cuda:0")
    q4, n4 = shard.make_queries(pos4, nrm4, 200000, shard.c5_offset(), 0.03, 80)
    ctx = _ctx(fmx_mod, pos4.shape[0])
    ctx.keypoints_add_device(0, pos4, nrm4)
    ctx.map_build([0], I34[None], W)
    ctx.set_queries_device(q4, n4)
    Tj = shard.expmap(np.array([0.0005, -0.0003, 0.0008, 0.02, 0.01, -0.01]))
    ctx.match(Tj, W)
    S1, e1 = ctx.linearize_matched(Tj, 0.1)
    ref = np.append(S1, e1)
    assert np.all(np.abs(S[0] - ref) <= 1e-10 * np.abs(ref).max())


def test_register_points_with_comm_is_identity(fmx_mod, c5_map):
    """fmx_register_points with a one-rank RCCL communicator attached (every ICP
    iteration's system all-reduced on the device, then published behind the completion
    word) follows the no-communicator iterates bit for bit."""
    pos4, nrm4 = c5_map
    q4, n4 = shard.make_queries(pos4, nrm4, 300000, shard.c5_offset(), 0.03, 84)
    out = []
    for use_comm in (False, True):
        ctx = _ctx(fmx_mod, pos4.shape[0])
        if use_comm:
            ctx.comm_init(fmx_mod.comm_unique_id(), 1, 0)
        ctx.keypoints_add_device(0, pos4, nrm4)
        ctx.map_build([0], I34[None], W)
        ctx.set_queries_device(q4, n4)
        out.append(ctx.register_points(I34, W, 0.1, 30, 1e-4))
        ctx.close()
    (T0, i0), (T1, i1) = out
    assert i0 == i1 and np.array_equal(T0, T1)


def test_dropped_deferred_match_is_never_launched(fmx_mod, c5_map):
    """a registration leaves its last match deferred; a new query set drops
    it instead of launching a 300k-query match nobody reads (the streaming C5 loop:
    set_queries -> register_points -> set_queries -> register_points)."""
    pos4, nrm4 = c5_map
    ctx = _ctx(fmx_mod, pos4.shape[0])
    ctx.keypoints_add_device(0, pos4, nrm4)
    ctx.map_build([0], I34[None], W)
    ctx.profile(True)
    ctx.profile_reset()
    for seed in (85, 86):
        q4, n4 = shard.make_queries(pos4, nrm4, 300000, shard.c5_offset(), 0.03, seed)
        ctx.set_queries_device(q4, n4)
        ctx.register_points(I34, W, 0.1, 30, 1e-4)
    prof = ctx.profile_read()
    assert prof["match"]["launches"] == 0 and prof["match_linearize"]["launches"] >= 4
    got = ctx.match_download()  # the last registration's match is still available on demand
    assert (got["pair"] >= 0).sum() > 0.9 * 300000
    assert ctx.profile_read()["match"]["launches"] == 1
    ctx.close()


def test_failed_call_after_deferred_match_serves_no_stale_results(fmx_mod, c5_map):
    """an immediate match, then a deferred one (no count outputs, >= 128k
    queries), then an extraction that fails its size check: the deferred match was
    dropped with its results, so fmx_match_download reports FMX_E_STATE instead of
    serving the older immediate match's outputs as if they were the dropped one's."""
    pos4, nrm4 = c5_map
    ctx = _ctx(fmx_mod, pos4.shape[0])
    ctx.keypoints_add_device(0, pos4, nrm4)
    ctx.map_build([0], I34[None], W)
    q4, n4 = shard.make_queries(pos4, nrm4, 200000, shard.c5_offset(), 0.03, 87)
    ctx.set_queries_device(q4, n4)
    ctx.match(I34, W)  # immediate
    ctx.match(shard.expmap(np.array([0.0, 0.0, 0.001, 0.01, 0.0, 0.0])), W, counts=False)  # deferred
    with pytest.raises(fmx_mod.FmxError) as e:
        ctx.extract(np.zeros((16, 4), np.float32), 1)
    assert e.value.status == 2  # FMX_E_SIZE
    with pytest.raises(fmx_mod.FmxError) as e:
        ctx.match_download()
    assert e.value.status == 5  # FMX_E_STATE
    ctx.close()


def test_deferred_match_validates_its_arguments(fmx_mod):
    """fmx_match reports a bad max_dist itself (a radius beyond the voxel
    width of a subdivided map), before it defers the launch; the next call is unaffected."""
    import torch
    pos4, nrm4 = shard.terrain_map(801, W, synth.SEED, "cuda:0")
    q4, n4 = shard.make_queries(pos4, nrm4, 200000, shard.c5_offset(), 0.03, 87)
    torch.cuda.synchronize()
    ctx = fmx_mod.Context(fmx_mod.EstimatorParams(keypoint_pool_capacity=pos4.shape[0] + 1024, voxel_subdivision=2))
    ctx.keypoints_add_device(0, pos4, nrm4)
    ctx.map_build([0], I34[None], W)
    ctx.set_queries_device(q4, n4)
    with pytest.raises(fmx_mod.FmxError, match="FMX_E_INVAL"):
        ctx.match(I34, 1.5 * W, counts=False)
    ctx.map_build([0], I34[None], W)  # not poisoned by the rejected match
    ctx.match(I34, W, counts=False)
    S, e = ctx.linearize_matched(I34, 0.1)
    assert e > 0 and np.isfinite(S).all()
    ctx.close()


_WITHHELD = r'''
import sys, time
import numpy as np
sys.path.insert(0, sys.argv[1])
from form_amd import fmx, shard, synth
W = 0.8
I34 = np.hstack([np.eye(3), np.zeros((3, 1))])
pos4, nrm4 = shard.terrain_map(301, W, synth.SEED, "cuda:0")
q4, n4 = shard.make_queries(pos4, nrm4, 20000, shard.c5_offset(), 0.03, 81)
ctx = fmx.Context(fmx.EstimatorParams(keypoint_pool_capacity=pos4.shape[0] + 1024))
ctx.comm_init(fmx.comm_unique_id(), 1, 0)
ctx.keypoints_add_device(0, pos4, nrm4)
ctx.map_build([0], I34[None], W)
ctx.set_queries_device(q4, n4)
ctx.match(I34, W)
t0 = time.time()
try:
    ctx.linearize_matched(I34, 0.1)
    print("RESULT ok", time.time() - t0)
except fmx.FmxError as e:
    print("RESULT err", e.status, round(time.time() - t0, 3), str(e))
# ADVICE r5: a retry must not return this rank's shard as the global system
t1 = time.time()
try:
    ctx.linearize_matched(I34, 0.1)
    print("RETRY ok")
except fmx.FmxError as e:
    print("RETRY err", e.status, round(time.time() - t1, 3))
ctx.close()
'''


@pytest.mark.timeout(120)
def test_withheld_allreduce_fails_within_bound(tmp_path):
    """a sharded wait must fail, not hang.  A test switch
    (FMX_TEST_WITHHOLD_FLAG) keeps the publish kernel behind ncclAllReduce on the stream
    without storing the completion word — a collective that never completes, on a 1-rank
    communicator.  With FMX_COMM_TIMEOUT_S=2 the call returns FMX_E_RCCL after ~2 s (the
    communicator aborted, the held kernel released).  ADVICE r5: a second sharded call on
    the same context fails at once with FMX_E_RCCL too (its queries are only this rank's
    shard), instead of returning the rank-local system."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = tmp_path / "withheld.py"
    script.write_text(_WITHHELD)
    env = dict(os.environ, FMX_TEST_WITHHOLD_FLAG="1", FMX_COMM_TIMEOUT_S="2")
    r = subprocess.run([sys.executable, str(script), root], env=env, capture_output=True, text=True, timeout=100)
    print(r.stdout, r.stderr[-2000:])
    assert r.returncode == 0, r.stderr[-2000:]
    res = [ln.split() for ln in r.stdout.splitlines() if ln.startswith("RESULT")][0]
    assert res[1] == "err" and int(res[2]) == 7, r.stdout  # FMX_E_RCCL
    assert 1.9 <= float(res[3]) < 10.0, r.stdout  # the bound, not a hang (the held kernel itself gives up at 20 s)
    retry = [ln.split() for ln in r.stdout.splitlines() if ln.startswith("RETRY")][0]
    assert retry[1] == "err" and int(retry[2]) == 7 and float(retry[3]) < 1.0, r.stdout
