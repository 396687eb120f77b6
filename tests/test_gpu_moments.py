"""Pair moments on the device (k_win_moments, fmx_moments) against the same moments
formed in numpy (tests/test_moments.py), and their host contraction against the oracle's
per-row linearization (orc_linearize: DenseFactor::linearize, gtsam.hpp:67-86) at poses
near and far from the reference.  Bars: moments within 1e-12 relative (fp64 sums in a
different order); G within 1e-10 of max |G| per pair; errors 1e-10 relative."""
import numpy as np
import pytest

from scenario import perturb, random_corr
from test_moments import _moments

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("K,max_rows,seed", [(5, 700, 3), (40, 3000, 4), (3, 9000, 5)])
def test_device_moments_and_contraction(fmx_mod, oracle, K, max_rows, seed):
    rng = np.random.default_rng(seed)
    np_, ppi, pni, ppj, nt, tpi, tpj, Pi, Pj = random_corr(rng, K, max_rows)
    ctx = fmx_mod.Context(fmx_mod.EstimatorParams())
    ctx.corr_set(np_, ppi, pni, ppj, nt, tpi, tpj)
    mom = ctx.moments(Pi, Pj)
    ob = np.concatenate([[0], np.cumsum(np_)]).astype(int)
    tb = np.concatenate([[0], np.cumsum(nt)]).astype(int)
    for k in range(K):
        ref = _moments((ppi[ob[k]:ob[k + 1]], pni[ob[k]:ob[k + 1]], ppj[ob[k]:ob[k + 1]]),
                       (tpi[tb[k]:tb[k + 1]], tpj[tb[k]:tb[k + 1]]), Pi[k], Pj[k])
        scale = max(np.abs(ref).max(), 1e-300)
        assert np.abs(mom[k] - ref).max() <= 1e-12 * scale, (k, np.abs(mom[k] - ref).max() / scale)
        if np_[k] == 0:
            assert not mom[k][:136].any()
        if nt[k] == 0:
            assert not mom[k][136:].any()
    for sr, st in [(0.0, 0.0), (1e-3, 0.01), (0.3, 3.0)]:
        Ti = np.stack([perturb(Pi[k], rng, sr, st) if sr else Pi[k] for k in range(K)])
        Tj = np.stack([perturb(Pj[k], rng, sr, st) if sr else Pj[k] for k in range(K)])
        G, err = fmx_mod.moments_contract(mom, Pi, Pj, Ti, Tj, 0.1)
        Go, eo = oracle.linearize(np_, ppi, pni, ppj, nt, tpi, tpj, Ti.reshape(K, 12), Tj.reshape(K, 12), 0.1)
        Gd, ed = ctx.linearize(Ti, Tj, 0.1)  # the per-row device linearization, for comparison
        for k in range(K):
            if np_[k] + nt[k] == 0:
                assert not G[k].any() and err[k] == 0
                continue
            scale = np.abs(Go[k]).max()
            assert np.abs(G[k] - Go[k]).max() <= 1e-10 * scale, (sr, k)
            assert np.abs(G[k] - Gd[k]).max() <= 1e-10 * scale, (sr, k)
            assert abs(err[k] - eo[k]) <= 1e-10 * eo[k], (sr, k, err[k], eo[k])
    ctx.close()
