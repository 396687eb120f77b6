"""World-size-2 gloo tests of the sharded path (form_amd/shard.py): shards cover the
queries exactly once, and the all-reduced per-shard normal equations equal the
unsharded ones — the exchange step bench.py's C5 workload runs over RCCL."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from form_amd import shard


def test_shard_bounds_cover():
    for n in (0, 1, 7, 1000, 2097152):
        for world in (1, 2, 3, 4, 8):
            spans = [shard.shard_bounds(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            for (b0, e0), (b1, _) in zip(spans, spans[1:]):
                assert e0 == b1
            sizes = [e - b for b, e in spans]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "oracle"))
    sys.path.insert(0, os.path.join(root, "tests"))
    import torch.distributed as dist

    import oracle_py as O
    from scenario import random_corr
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(42)  # same data on every rank
    np_, ppi, pni, ppj, nt, tpi, tpj, Pi, Pj = random_corr(rng, 2, max_rows=5000)
    # keep pair 1 only (pair 0 is made empty by random_corr)
    ppi, pni, ppj = ppi[np_[0]:], pni[np_[0]:], ppj[np_[0]:]
    tpi, tpj = tpi[nt[0]:], tpj[nt[0]:]
    np_, nt, Pi, Pj = np_[1:], nt[1:], Pi[1:], Pj[1:]
    assert np_[0] > 100 and nt[0] > 10
    # shard both row types of the single pair contiguously
    b, e = shard.shard_bounds(int(np_[0]), rank, world)
    bt, et = shard.shard_bounds(int(nt[0]), rank, world)
    for single in (True, False):
        G, err = O.linearize(np.array([e - b], np.uint32), ppi[b:e], pni[b:e], ppj[b:e],
                             np.array([et - bt], np.uint32), tpi[bt:et], tpj[bt:et], Pi, Pj, 0.1, single)
        Gs = shard.allreduce_sum(G[0])
        Gf, errf = O.linearize(np_, ppi, pni, ppj, nt, tpi, tpj, Pi, Pj, 0.1, single)
        assert np.allclose(Gs, Gf[0], rtol=1e-11, atol=1e-9), (rank, single)
        if single:
            dx = shard.gauss_newton_step(Gs)
            np.save(os.path.join(out_dir, f"dx_{rank}.npy"), dx)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_sharded_normal_equations_gloo(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    dx = [np.load(tmp_path / f"dx_{r}.npy") for r in range(world)]
    # bitwise-identical all-reduced sums -> identical steps on every rank
    assert np.array_equal(dx[0], dx[1])


def test_gauss_newton_recovers_offset(oracle):
    """One sharded-style GN step on a synthetic plane-point set recovers a small pose
    offset (sanity of the host solve used by the C5 bench)."""
    import np_ref
    rng = np.random.default_rng(8)
    n = 4000
    pts = rng.uniform(-20, 20, (n, 3))
    nrm = rng.normal(size=(n, 3))
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    Ttrue = np_ref.expmap(np.array([0.004, -0.003, 0.005, 0.03, -0.02, 0.01]))
    Rt, tt = Ttrue[:, :3], Ttrue[:, 3]
    pj = (pts - tt) @ Rt  # local coordinates of the same points in frame Ttrue
    I = np.hstack([np.eye(3), np.zeros((3, 1))])
    G, _ = oracle.linearize(np.array([n], np.uint32), pts, nrm, pj, np.array([0], np.uint32),
                            np.zeros((0, 3)), np.zeros((0, 3)), I[None], I[None], 0.1, True)
    T = I
    for _ in range(3):
        dx = shard.gauss_newton_step(G[0])
        T = shard.compose(T, shard.expmap(dx))
        G, _ = oracle.linearize(np.array([n], np.uint32), pts, nrm, pj, np.array([0], np.uint32),
                                np.zeros((0, 3)), np.zeros((0, 3)), I[None], T[None], 0.1, True)
    assert np.abs(T - Ttrue).max() < 1e-9
