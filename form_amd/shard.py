"""Multi-GPU C5 path: 2M query points sharded over ranks against a
replicated 50M-voxel submap; the only exchange is one all-reduce of the normal
equations per linearization.

* Each rank builds the same voxel map locally (building is cheaper than broadcasting
  ~3 GB over xGMI) and owns a contiguous, equal shard of the queries.
* Per linearization a rank reduces its shard to the packed 7x7 (single pose, 28
  doubles) or 13x13 (91 doubles) augmented Hessian; the sum over ranks is one
  ``all_reduce(SUM)`` of a few hundred bytes — latency-bound, so a single small
  fp64 collective (RCCL picks its low-latency protocol), not a bucketed ring.
* Every rank then runs the identical host solve: the all-reduced sums are bitwise
  identical on all ranks, so accept/converge decisions agree without a broadcast.
"""
from __future__ import annotations

import math

import numpy as np
import torch


def shard_bounds(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous, equal (+-1) shard [b, e) of n items for `rank`."""
    q, r = divmod(n, world)
    b = rank * q + min(rank, r)
    return b, b + q + (1 if rank < r else 0)


def allreduce_sum(x: np.ndarray, device=None) -> np.ndarray:
    """Sum a small fp64 array over all ranks (RCCL on GPUs, gloo on CPU)."""
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return x
    t = torch.as_tensor(np.ascontiguousarray(x, np.float64), device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.cpu().numpy()


def unpack_sym(G: np.ndarray) -> np.ndarray:
    """Packed upper triangle (row-major) -> full symmetric matrix."""
    m = int(round((math.sqrt(8 * len(G) + 1) - 1) / 2))
    M = np.zeros((m, m))
    iu = np.triu_indices(m)
    M[iu] = G
    M.T[iu] = G
    return M


def gauss_newton_step(G28: np.ndarray, lam: float = 0.0) -> np.ndarray:
    """Solve (H + lam I) dx = g from the packed single-pose 7x7 [H_j b]^T[H_j b]
    (H = A^T A, g = A^T b): the increment in GTSAM's tangent [w; v]."""
    M = unpack_sym(G28)
    H, g = M[:6, :6], M[:6, 6]
    return np.linalg.solve(H + lam * np.eye(6), g)


def expmap(xi: np.ndarray) -> np.ndarray:
    w, v = xi[:3], xi[3:]
    th = float(np.linalg.norm(w))
    W = np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]])
    if th < 1e-12:
        R, V = np.eye(3) + W, np.eye(3) + 0.5 * W
    else:
        R = np.eye(3) + math.sin(th) / th * W + (1 - math.cos(th)) / th**2 * W @ W
        V = np.eye(3) + (1 - math.cos(th)) / th**2 * W + (th - math.sin(th)) / th**3 * W @ W
    T = np.zeros((3, 4))
    T[:, :3] = R
    T[:, 3] = V @ v
    return T


def compose(A: np.ndarray, B: np.ndarray) -> np.ndarray:
    T = np.zeros((3, 4))
    T[:, :3] = A[:, :3] @ B[:, :3]
    T[:, 3] = A[:, :3] @ B[:, 3] + A[:, 3]
    return T


# ----------------------------------------------------------------- C5 synthetic data
def terrain_map(n_side: int, w: float, seed: int, device="cpu"):
    """Jittered terrain grid: one planar feature per w-voxel over n_side x n_side
    voxels, heights within +-0.2 m, normals of the height field.  Returns (pos4,
    nrm4) float32 tensors (N, 4) in the map scan's frame."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    n = n_side * n_side
    ij = torch.arange(n, device=device)
    i = (ij // n_side).to(torch.float64)
    j = (ij % n_side).to(torch.float64)
    jit = torch.rand((n, 2), generator=g, dtype=torch.float64).to(device)
    x = (i + 0.1 + 0.8 * jit[:, 0]) * w - 0.5 * n_side * w
    y = (j + 0.1 + 0.8 * jit[:, 1]) * w - 0.5 * n_side * w
    a, b = 0.7, 0.9
    z = 0.1 * torch.sin(a * x) + 0.1 * torch.cos(b * y)  # |z| <= 0.2
    nx = -0.1 * a * torch.cos(a * x)
    ny = 0.1 * b * torch.sin(b * y)
    nrm = torch.stack([-nx, -ny, torch.ones_like(x)], 1)
    nrm = nrm / nrm.norm(dim=1, keepdim=True)
    pos4 = torch.zeros((n, 4), dtype=torch.float32, device=device)
    pos4[:, 0], pos4[:, 1], pos4[:, 2] = x.float(), y.float(), (z + 0.2).float()
    nrm4 = torch.zeros((n, 4), dtype=torch.float32, device=device)
    nrm4[:, :3] = nrm.float()
    return pos4, nrm4


def make_queries(pos4, nrm4, n_query: int, offset: np.ndarray, noise: float, seed: int):
    """n_query map features perturbed by N(0, noise) and expressed in the frame of a
    sensor offset by `offset` (3x4): q_local = offset^-1 * (p + e)."""
    dev = pos4.device
    g = torch.Generator(device="cpu").manual_seed(seed)
    # a random subset of the map features, kept in map (grid) order: a LiDAR scan's
    # points arrive spatially coherent, not shuffled
    sel = torch.randperm(pos4.shape[0], generator=g)[:n_query].sort().values.to(dev)
    p = pos4[sel, :3].double() + noise * torch.randn((n_query, 3), generator=g, dtype=torch.float64).to(dev)
    R = torch.as_tensor(offset[:, :3], dtype=torch.float64, device=dev)
    t = torch.as_tensor(offset[:, 3], dtype=torch.float64, device=dev)
    ql = (p - t) @ R  # R^T (p - t)
    nl = nrm4[sel, :3].double() @ R
    q4 = torch.zeros((n_query, 4), dtype=torch.float32, device=dev)
    n4 = torch.zeros((n_query, 4), dtype=torch.float32, device=dev)
    q4[:, :3] = ql.float()
    n4[:, :3] = nl.float()
    return q4, n4
