"""Pair moments (moments.hpp, fmx_moments_contract): DenseFactor::linearize of a pair
(gtsam.hpp:67-86, factor.cpp:30-128) evaluated from its 16-feature row moments, on the
host, against the oracle's per-row linearization at the same poses.

The features are formed here exactly as k_win_moments forms them (window.hip): plane rows
[r0 = n.(q0 - p_i), n x q0, n, n (x) p_j] with q0 = R_i0^T (R_j0 p_j + t_j0 - t_i0);
point rows [e0, p_i, p_j, 1] with e0 the world residual at the reference poses.  Bar:
G within 1e-10 of max |G| per pair, errors within 1e-10 relative — the same bar as the
device linearization (summation order only), also far from the reference poses.
"""
import numpy as np
import pytest

from form_amd import fmx

I34 = np.hstack([np.eye(3), np.zeros((3, 1))])


def _rot(w):
    th = np.linalg.norm(w)
    if th == 0:
        return np.eye(3)
    K = np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]]) / th
    return np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K


def _pose(rng, sr, st):
    return np.hstack([_rot(rng.normal(size=3) * sr), (rng.normal(size=3) * st)[:, None]])


def _perturb(T, rng, sr, st):
    return np.hstack([_rot(rng.normal(size=3) * sr) @ T[:, :3], (T[:, 3] + rng.normal(size=3) * st)[:, None]])


def _packed16(M):
    return M[np.triu_indices(16)]


def _moments(pl, pt, Ti0, Tj0):
    """(272,) packed plane then point moments of one pair (the kernel's features)."""
    pi, ni, pj = pl
    Ri, ti, Rj, tj = Ti0[:, :3], Ti0[:, 3], Tj0[:, :3], Tj0[:, 3]
    out = np.zeros(272)
    if len(pi):
        q0 = ((Rj @ pj.T).T + tj - ti) @ Ri
        f = np.zeros((len(pi), 16))
        f[:, 0] = np.sum(ni * (q0 - pi), 1)
        f[:, 1:4] = np.cross(ni, q0)
        f[:, 4:7] = ni
        f[:, 7:16] = (ni[:, :, None] * pj[:, None, :]).reshape(-1, 9)
        out[:136] = _packed16(f.T @ f)
    qi, qj = pt
    if len(qi):
        f = np.zeros((len(qi), 16))
        f[:, 0:3] = ((Rj @ qj.T).T + tj) - ((Ri @ qi.T).T + ti)
        f[:, 3:6] = qi
        f[:, 6:9] = qj
        f[:, 9] = 1.0
        out[136:] = _packed16(f.T @ f)
    return out


def _scene(rng, K, npl, npt, Tref):
    """K pairs of matched rows consistent with the reference poses (p_i near p_j's image)."""
    pairs = []
    for k in range(K):
        Ti0, Tj0 = Tref[k]
        n1 = 0 if k == K - 1 else npl + k  # the last pair: point rows only
        n2 = 0 if k == 0 else npt + k      # the first pair: plane rows only
        pj = rng.normal(size=(n1, 3)) * 25
        q = ((Tj0[:, :3] @ pj.T).T + Tj0[:, 3] - Ti0[:, 3]) @ Ti0[:, :3]
        pi = q + rng.normal(size=(n1, 3)) * 0.2
        ni = rng.normal(size=(n1, 3))
        ni /= np.linalg.norm(ni, axis=1)[:, None]
        qj = rng.normal(size=(n2, 3)) * 25
        qq = ((Tj0[:, :3] @ qj.T).T + Tj0[:, 3] - Ti0[:, 3]) @ Ti0[:, :3]
        qi = qq + rng.normal(size=(n2, 3)) * 0.2
        pairs.append(((pi, ni, pj), (qi, qj)))
    return pairs


@pytest.mark.parametrize("sr,st", [(0.0, 0.0), (2e-3, 0.02), (0.05, 0.5), (0.4, 5.0)])
def test_contract_matches_oracle_linearize(oracle, sr, st):
    rng = np.random.default_rng(int(1e4 * sr) + 7)
    K = 9  # more than one 8-pair SIMD block
    Tref = [(_pose(rng, 0.6, 30), _pose(rng, 0.6, 30)) for _ in range(K)]
    pairs = _scene(rng, K, 300, 60, Tref)
    mom = np.stack([_moments(pl, pt, *Tref[k]) for k, (pl, pt) in enumerate(pairs)])
    Ti = np.stack([_perturb(Tref[k][0], rng, sr, st) for k in range(K)])
    Tj = np.stack([_perturb(Tref[k][1], rng, sr, st) for k in range(K)])
    ri = np.stack([t[0] for t in Tref])
    rj = np.stack([t[1] for t in Tref])
    G, err = fmx.moments_contract(mom, ri, rj, Ti, Tj, 0.1)
    cat = lambda i, w: np.vstack([p[w][i] for p in pairs])
    npl = np.array([len(p[0][0]) for p in pairs])
    npt = np.array([len(p[1][0]) for p in pairs])
    Go, eo = oracle.linearize(npl, cat(0, 0), cat(1, 0), cat(2, 0), npt, cat(0, 1), cat(1, 1),
                              Ti.reshape(K, 12), Tj.reshape(K, 12), 0.1)
    for k in range(K):
        scale = np.abs(Go[k]).max()
        assert np.abs(G[k] - Go[k]).max() <= 1e-10 * scale, (k, np.abs(G[k] - Go[k]).max() / scale)
        assert abs(err[k] - eo[k]) <= 1e-10 * eo[k], (k, err[k], eo[k])
        assert err[k] == 0.5 * G[k][90]


def test_zero_moments_give_zero_system():
    K = 3
    G, err = fmx.moments_contract(np.zeros((K, 272)), np.stack([I34] * K), np.stack([I34] * K),
                                  np.stack([I34] * K), np.stack([I34] * K), 0.1)
    assert not G.any() and not err.any()


def test_contract_rejects_bad_arguments():
    L = fmx.lib()
    assert L.fmx_moments_contract(0, None, None, None, None, None, fmx.C.c_double(0.1), None, None) == 0
    with pytest.raises(fmx.FmxError):
        fmx.moments_contract(np.zeros((1, 272)), I34, I34, I34, I34, 0.0)
