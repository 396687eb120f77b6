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


_TRIU: dict[int, tuple[np.ndarray, np.ndarray]] = {}


def unpack_sym(G: np.ndarray) -> np.ndarray:
    """Packed upper triangle (row-major) -> full symmetric matrix."""
    m = int(round((math.sqrt(8 * len(G) + 1) - 1) / 2))
    iu = _TRIU.get(m)
    if iu is None:
        iu = _TRIU[m] = np.triu_indices(m)
    M = np.empty((m, m))
    M[iu] = G
    M.T[iu] = G
    return M


def gauss_newton_step(G28: np.ndarray, lam: float = 0.0) -> np.ndarray:
    """Solve (H + lam I) dx = g from the packed single-pose 7x7 [H_j b]^T[H_j b]
    (H = A^T A, g = A^T b): the increment in GTSAM's tangent [w; v]."""
    M = unpack_sym(G28)
    H = M[:6, :6]
    if lam:
        H = H + lam * np.eye(6)
    return np.linalg.solve(H, M[:6, 6])


def expmap(xi) -> np.ndarray:
    """SE(3) exponential of [w; v] as a 3x4 [R | t] (Rodrigues; scalar arithmetic, the
    per-iteration host step of the C5 loop)."""
    wx, wy, wz, vx, vy, vz = (float(v) for v in xi)
    th2 = wx * wx + wy * wy + wz * wz
    th = math.sqrt(th2)
    if th < 1e-12:
        a, b, c = 1.0, 0.5, 1.0 / 6.0
    else:
        a, b, c = math.sin(th) / th, (1 - math.cos(th)) / th2, (th - math.sin(th)) / (th2 * th)
    # W, W^2 entries
    W = ((0.0, -wz, wy), (wz, 0.0, -wx), (-wy, wx, 0.0))
    W2 = ((-(wy * wy + wz * wz), wx * wy, wx * wz), (wx * wy, -(wx * wx + wz * wz), wy * wz),
          (wx * wz, wy * wz, -(wx * wx + wy * wy)))
    v = (vx, vy, vz)
    T = np.empty((3, 4))
    for r in range(3):
        for s in range(3):
            T[r, s] = (1.0 if r == s else 0.0) + a * W[r][s] + b * W2[r][s]
        T[r, 3] = sum(((1.0 if r == s else 0.0) + b * W[r][s] + c * W2[r][s]) * v[s] for s in range(3))
    return T


def compose(A: np.ndarray, B: np.ndarray) -> np.ndarray:
    T = np.empty((3, 4))
    T[:, :3] = A[:, :3] @ B[:, :3]
    T[:, 3] = A[:, :3] @ B[:, 3] + A[:, 3]
    return T


# ----------------------------------------------------------------- C5 synthetic data
# Terrain: z = A (sin(2 pi x / LX) + cos(2 pi y / LY)).  The wavelengths are a few
# voxels and incommensurate, so the surface normals vary in x AND y (slopes up to
# ~0.4 per term): point-to-plane residuals then constrain x, y and yaw as well as
# z / roll / pitch (a flat or nearly flat field leaves them unobservable).
TERRAIN_A, TERRAIN_LX, TERRAIN_LY = 0.6, 9.7, 13.3
# Sensor range of the 2M-point "scan" (OS2-128 class, ~240 m): queries are map
# surface samples within this radius of the sensor.  With the injected rotation
# (C5_OFFSET) the farthest points start <= ~0.45 m from their surface, inside the
# 0.8 m match radius, so ICP converges from the offset pose.
C5_RANGE_M = 240.0


def c5_offset(rot_scale: float = 1.0) -> np.ndarray:
    """The injected sensor-pose error (truth): 5 cm translation, 0.1 deg yaw, 0.05 deg
    roll and pitch (GTSAM tangent [w; v]); rot_scale scales the rotation (the whole-map
    query set reaches ~4 km, where 0.1 deg is 7 m: it uses 1/20 of it)."""
    d = np.radians
    return expmap(np.array([d(0.05) * rot_scale, d(-0.05) * rot_scale, d(0.1) * rot_scale, 0.03, -0.04, 0.0]))


# the whole-map query set (2M features drawn across the whole map)
C5_WHOLEMAP_ROT_SCALE = 0.05
C5_RINGS = 128


def terrain_map(n_side: int, w: float, seed: int, device="cpu"):
    """Jittered terrain grid: one planar feature per w-column over n_side x n_side
    columns (centred on the origin), on the height field above with its normals.
    Returns (pos4, nrm4) float32 tensors (N, 4) in the map scan's frame."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    n = n_side * n_side
    ij = torch.arange(n, device=device)
    i = (ij // n_side).to(torch.float64)
    j = (ij % n_side).to(torch.float64)
    jit = torch.rand((n, 2), generator=g, dtype=torch.float64).to(device)
    x = (i + 0.1 + 0.8 * jit[:, 0]) * w - 0.5 * n_side * w
    y = (j + 0.1 + 0.8 * jit[:, 1]) * w - 0.5 * n_side * w
    kx, ky = 2 * math.pi / TERRAIN_LX, 2 * math.pi / TERRAIN_LY
    z = TERRAIN_A * (torch.sin(kx * x) + torch.cos(ky * y))
    dzdx = TERRAIN_A * kx * torch.cos(kx * x)
    dzdy = -TERRAIN_A * ky * torch.sin(ky * y)
    nrm = torch.stack([-dzdx, -dzdy, torch.ones_like(x)], 1)
    nrm = nrm / nrm.norm(dim=1, keepdim=True)
    pos4 = torch.zeros((n, 4), dtype=torch.float32, device=device)
    pos4[:, 0], pos4[:, 1], pos4[:, 2] = x.float(), y.float(), z.float()
    nrm4 = torch.zeros((n, 4), dtype=torch.float32, device=device)
    nrm4[:, :3] = nrm.float()
    return pos4, nrm4


def make_queries(pos4, nrm4, n_query: int, offset: np.ndarray, noise: float, seed: int,
                 radius: float = C5_RANGE_M):
    """An n_query-point scan taken from a sensor at pose `offset` (3x4, world <- sensor):
    map surface samples within `radius` of the origin (drawn with replacement, each
    with N(0, noise) range noise), in the sensor frame: q = offset^-1 (p + e).  Returned
    in map (grid) order: a LiDAR scan's points arrive spatially coherent."""
    dev = pos4.device
    g = torch.Generator(device="cpu").manual_seed(seed)
    r2 = (pos4[:, 0].double() ** 2 + pos4[:, 1].double() ** 2)
    inside = torch.nonzero(r2 <= radius * radius).squeeze(1)
    pick = torch.randint(0, inside.shape[0], (n_query,), generator=g).to(dev)
    sel = inside[pick].sort().values
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


def make_queries_wholemap(pos4, nrm4, n_query: int, offset: np.ndarray, noise: float, seed: int,
                          rings: int = C5_RINGS):
    """n_query DISTINCT map features drawn uniformly over the whole map,
    each with N(0, noise) noise, in the sensor frame (q = offset^-1 (p + e)), ordered
    like a spinning LiDAR's output: `rings` range bands of equal counts, each in azimuth
    order.  Unlike make_queries (a 240 m scan drawn with replacement, grid order), most
    queries here touch bricks no other query touches: the match reads the map from HBM."""
    dev = pos4.device
    g = torch.Generator(device="cpu").manual_seed(seed)
    n = pos4.shape[0]
    sel = torch.randperm(n, generator=g)[:n_query].to(dev)
    p = pos4[sel, :3].double() + noise * torch.randn((n_query, 3), generator=g, dtype=torch.float64).to(dev)
    R = torch.as_tensor(offset[:, :3], dtype=torch.float64, device=dev)
    t = torch.as_tensor(offset[:, 3], dtype=torch.float64, device=dev)
    ql = (p - t) @ R  # R^T (p - t)
    nl = nrm4[sel, :3].double() @ R
    rng = torch.sqrt(ql[:, 0] ** 2 + ql[:, 1] ** 2)
    az = torch.atan2(ql[:, 1], ql[:, 0])
    ring = torch.empty(n_query, dtype=torch.int64, device=dev)
    ring[torch.argsort(rng)] = torch.arange(n_query, device=dev) * rings // n_query
    order = torch.argsort(ring.double() * 8.0 + (az + math.pi))  # ring-major, azimuth inside a ring
    q4 = torch.zeros((n_query, 4), dtype=torch.float32, device=dev)
    n4 = torch.zeros((n_query, 4), dtype=torch.float32, device=dev)
    q4[:, :3] = ql[order].float()
    n4[:, :3] = nl[order].float()
    return q4, n4


def pose_error(T: np.ndarray, Ttrue: np.ndarray) -> tuple[float, float]:
    """(translation error m, rotation error rad) of T against Ttrue."""
    D = compose(np.hstack([Ttrue[:, :3].T, -(Ttrue[:, :3].T @ Ttrue[:, 3])[:, None]]), T)
    ang = math.acos(max(-1.0, min(1.0, (np.trace(D[:, :3]) - 1) / 2)))
    return float(np.linalg.norm(D[:, 3])), ang
