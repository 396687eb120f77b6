"""Independent numpy restatement of the reference path, used only to cross-check
the C++ oracle (oracle/form_oracle.cpp).  Written separately from the oracle, from
the reference files:
  extraction.tpp:136-222 (masks), :226-261 (curvature), :44-96 + :332-399
  (selection), :263-329 + :402-448 (normals); map.tpp:35-91 (voxel NN);
  factor.cpp:30-128 (residuals/Jacobians); gtsam.hpp:67-139 (whitened G).
Pure Python loops: small inputs only.
"""
from __future__ import annotations

import numpy as np

f32 = np.float32


def sqnorm4f(d):
    """vec4().squaredNorm() in float with zero pad: (x*x + z*z) + y*y (SSE2 predux)."""
    d = d.astype(f32)
    return (d[..., 0] * d[..., 0] + d[..., 2] * d[..., 2]) + d[..., 1] * d[..., 1]


def masks(scan, p):
    R, C, k = p["num_rows"], p["num_columns"], p["neighbor_points"]
    pts = scan.reshape(R, C, 4)[..., :3].astype(f32)
    r2 = sqnorm4f(pts).astype(np.float64)
    col = np.arange(C)[None, :].repeat(R, 0)
    inwin = (col >= k) & (col < C - k)
    oor = inwin & ((r2 < p["min_norm_squared"]) | (r2 > p["max_norm_squared"]))
    point_valid = inwin & ~oor
    planar = point_valid.copy()
    for d in range(1, k + 1):
        planar[:, d:] &= ~oor[:, :-d]
        planar[:, :-d] &= ~oor[:, d:]
    return planar.reshape(-1), point_valid.reshape(-1)


def curvature(scan, p, planar):
    R, C, k = p["num_rows"], p["num_columns"], p["neighbor_points"]
    pts = scan.reshape(R, C, 4)[..., :3].astype(np.float64)
    out = np.full((R, C), np.finfo(f32).max, f32)
    acc = -(2.0 * k) * pts[:, k:C - k]
    for n in range(1, k + 1):
        acc = acc + pts[:, k - n:C - k - n] + pts[:, k + n:C - k + n]
    cv = ((acc[..., 0] * acc[..., 0] + acc[..., 1] * acc[..., 1]) + acc[..., 2] * acc[..., 2]).astype(f32)
    inner = out[:, k:C - k]
    m = planar.reshape(R, C)[:, k:C - k]
    inner[m] = cv[m]
    return out.reshape(-1)


def select(scan, p):
    R, C, k, S = p["num_rows"], p["num_columns"], p["neighbor_points"], p["num_sectors"]
    planar, pointv = masks(scan, p)
    curv = curvature(scan, p, planar)
    used = planar.copy()
    pps = C // S
    sel = []
    for r in range(R):
        for s in range(S):
            b = r * C + s * pps
            e = (r + 1) * C if s == S - 1 else b + pps
            order = sorted(range(b, e), key=lambda i: (curv[i], i))
            nf = 0
            for i in order:
                if used[i] and float(curv[i]) < p["planar_threshold"]:
                    sel.append(i)
                    for n in range(k):
                        used[i + n] = False
                        used[i - n] = False
                    nf += 1
                if nf > p["planar_feats_per_sector"]:
                    break
    elig = (used == planar) & pointv
    pts = []
    P = p["point_feats_per_sector"]
    for r in range(R):
        for s in range(S):
            b = r * C + s * pps
            e = (r + 1) * C if s == S - 1 else b + pps
            if P == 0:
                continue
            U = [i for i in range(b, e) if elig[i]]
            factor = 1 + len(U) // P
            nf = 0
            for off in range(factor):
                for ui in range(off, len(U), factor):
                    i = U[ui]
                    if elig[i]:
                        pts.append(i)
                        for n in range(k):
                            elig[i + n] = False
                            elig[i - n] = False
                        nf += 1
                    if nf > P:
                        break
    return np.array(sel, np.int64), np.array(pts, np.int64), planar, curv


def dist2f(a, b):
    return sqnorm4f((a.astype(f32) - b.astype(f32)))


def normal(scan, p, idx, planar):
    """(ok, normal via numpy eigh in float64) for one selected index; neighbour
    sequence exactly as extraction.tpp:263-329."""
    R, C, k = p["num_rows"], p["num_columns"], p["neighbor_points"]
    pts = scan[:, :3].astype(f32)
    r2 = p["radius"] ** 2

    def nbrs(j, out):
        for i in range(1, k + 1):
            if float(dist2f(pts[j + i], pts[j])) < r2:
                out.append(pts[j + i])
            else:
                break
        for i in range(1, k + 1):
            if float(dist2f(pts[j - i], pts[j])) < r2:
                out.append(pts[j - i])
            else:
                break

    row = idx // C
    q = []
    nbrs(idx, q)
    other = False
    for rr in (row - 1, row + 1):
        if rr < 0 or rr >= R:
            continue
        cand = np.arange(rr * C, (rr + 1) * C)
        cand = cand[planar[cand]]
        if len(cand) == 0:
            continue
        d = dist2f(pts[cand], pts[idx][None, :])
        j = int(cand[int(np.argmin(d))])  # first index on exact ties
        other = True
        q.append(pts[j])
        nbrs(j, q)
    if not other or len(q) < p["min_points"]:
        return False, None, None
    A = (np.array(q, np.float64) - pts[idx].astype(np.float64)) / len(q)
    cov = A.T @ A
    w, V = np.linalg.eigh(cov)
    return True, V[:, 0], w


# ---------------------------------------------------------------- factors
def RzRyRx(x, y, z):
    """gtsam Rot3::RzRyRx(x, y, z) = Rz(z) Ry(y) Rx(x) (external API)."""
    cx, sx, cy, sy, cz, sz = np.cos(x), np.sin(x), np.cos(y), np.sin(y), np.cos(z), np.sin(z)
    Rx = np.array([[1, 0, 0], [0, cx, -sx], [0, sx, cx]])
    Ry = np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]])
    Rz = np.array([[cz, -sz, 0], [sz, cz, 0], [0, 0, 1]])
    return Rz @ Ry @ Rx


def pose(R, t):
    T = np.zeros((3, 4))
    T[:, :3] = R
    T[:, 3] = t
    return T


def plane_residual(Ti, Tj, pi, ni, pj):
    wn = Ti[:, :3] @ ni
    return float(wn @ ((Tj[:, :3] @ pj + Tj[:, 3]) - (Ti[:, :3] @ pi + Ti[:, 3])))


def point_residual(Ti, Tj, pi, pj):
    return (Tj[:, :3] @ pj + Tj[:, 3]) - (Ti[:, :3] @ pi + Ti[:, 3])


def skew(w):
    return np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]])


def expmap(xi):
    w, v = xi[:3], xi[3:]
    th = np.linalg.norm(w)
    W = skew(w)
    if th < 1e-12:
        R = np.eye(3) + W
        V = np.eye(3) + 0.5 * W
    else:
        R = np.eye(3) + np.sin(th) / th * W + (1 - np.cos(th)) / th**2 * W @ W
        V = np.eye(3) + (1 - np.cos(th)) / th**2 * W + (th - np.sin(th)) / th**3 * W @ W
    return pose(R, V @ v)


def compose(A, B):
    return pose(A[:, :3] @ B[:, :3], A[:, :3] @ B[:, 3] + A[:, 3])


def numeric_jacobian(f, Ti, Tj, h=1e-6):
    """Central differences of f(Ti, Tj) under T * Exp(xi) (GTSAM right perturbation)."""
    r0 = np.atleast_1d(f(Ti, Tj))
    J = np.zeros((r0.size, 12))
    for c in range(12):
        xi = np.zeros(6)
        xi[c % 6] = h
        if c < 6:
            rp, rm = f(compose(Ti, expmap(xi)), Tj), f(compose(Ti, expmap(-xi)), Tj)
        else:
            rp, rm = f(Ti, compose(Tj, expmap(xi))), f(Ti, compose(Tj, expmap(-xi)))
        J[:, c] = (np.atleast_1d(rp) - np.atleast_1d(rm)) / (2 * h)
    return r0, J


def packed_G(J, r, sigma, single=False):
    A = J[:, 6:] / sigma if single else J / sigma
    Ab = np.hstack([A, (-r / sigma)[:, None]])
    G = Ab.T @ Ab
    iu = np.triu_indices(G.shape[0])
    return G[iu]


# ---------------------------------------------------------------- voxel NN
def voxel_nn(map_pts, q, w):
    """Exact NN of q among map points in the 27 voxels around floor(q/w) (map.tpp:70-91)."""
    vq = np.floor(q / w).astype(np.int64)
    vm = np.floor(map_pts / w).astype(np.int64)
    near = np.all(np.abs(vm - vq[None, :]) <= 1, axis=1)
    if not near.any():
        return -1, np.inf
    idx = np.nonzero(near)[0]
    d = map_pts[idx] - q[None, :]
    d2 = (d[:, 0] * d[:, 0] + d[:, 2] * d[:, 2]) + d[:, 1] * d[:, 1]
    j = int(np.argmin(d2))
    return int(idx[j]), float(d2[j])
