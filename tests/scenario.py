"""Shared synthetic scenarios for the parity tests (CPU oracle vs HIP path)."""
from __future__ import annotations

import numpy as np

from form_amd import synth


def stream_features(oracle, config: str, n_scans: int, world=None):
    """Oracle features (planar (F,6), point (F,3)) and GT poses of the first n scans."""
    world = world or synth.World()
    out = []
    for k in range(n_scans):
        scan, T, geo = synth.make_scan(config, k, world=world)
        p = synth.default_params(geo)
        ex = oracle.extract(scan.numpy(), p)
        pl, pt = oracle.features_from(scan.numpy(), ex)
        out.append(dict(scan=scan.numpy(), pose=T, planar=pl, point=pt, params=p))
    return out


def perturb(T: np.ndarray, rng: np.random.Generator, rot=0.01, trans=0.05) -> np.ndarray:
    """T * Exp(xi) with a small random xi (GTSAM right perturbation)."""
    w = rng.normal(size=3) * rot
    v = rng.normal(size=3) * trans
    th = np.linalg.norm(w)
    W = np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]])
    R = np.eye(3) + np.sin(th) / th * W + (1 - np.cos(th)) / th**2 * W @ W
    out = np.zeros((3, 4))
    out[:, :3] = T[:, :3] @ R
    out[:, 3] = T[:, :3] @ v + T[:, 3]
    return out


def random_corr(rng: np.random.Generator, K: int, max_rows: int = 3000, empty_every: int = 4):
    """Random pair-major correspondence sets (plane rows + point pairs) and poses."""
    np_ = rng.integers(0, max_rows, K).astype(np.uint32)
    nt = rng.integers(0, max_rows // 4, K).astype(np.uint32)
    for k in range(0, K, empty_every):
        np_[k] = 0
        if k % 8 == 0:
            nt[k] = 0
    Np, Nt = int(np_.sum()), int(nt.sum())
    ppi = rng.uniform(-30, 30, (Np, 3))
    n = rng.normal(size=(Np, 3))
    pni = n / np.linalg.norm(n, axis=1, keepdims=True)
    ppj = ppi + rng.normal(scale=0.3, size=(Np, 3))
    tpi = rng.uniform(-30, 30, (Nt, 3))
    tpj = tpi + rng.normal(scale=0.3, size=(Nt, 3))
    poses_i = np.stack([perturb(np.hstack([np.eye(3), rng.normal(size=(3, 1)) * 5]), rng, 0.5, 1.0)
                        for _ in range(K)])
    poses_j = np.stack([perturb(np.hstack([np.eye(3), rng.normal(size=(3, 1)) * 5]), rng, 0.5, 1.0)
                        for _ in range(K)])
    return np_, ppi, pni, ppj, nt, tpi, tpj, poses_i, poses_j
