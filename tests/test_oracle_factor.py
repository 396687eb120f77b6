"""Oracle residuals / Jacobians / whitened normal equations (factor.cpp, gtsam.hpp).

Known answers at the reference's own test poses and points
(tests/test_SeparateFactor.cpp:26-30, 53-59: x0 = (RzRyRx(0.1,0.2,0.3), (1,2,3)),
x1 = (RzRyRx(0.4,0.5,0.6), (4,5,6)), p_i = (1,2,3), n_i = (0,0,1), p_j = (4,5,6)),
recomputed here independently in numpy (that test pins no numbers and does not
compile against the current tree); Jacobians against central differences under
GTSAM's right perturbation T * Exp([w; v]).
"""
import numpy as np
import pytest

import np_ref

X0 = np_ref.pose(np_ref.RzRyRx(0.1, 0.2, 0.3), [1, 2, 3])
X1 = np_ref.pose(np_ref.RzRyRx(0.4, 0.5, 0.6), [4, 5, 6])
PI = np.array([1.0, 2.0, 3.0])
NI = np.array([0.0, 0.0, 1.0])
PJ = np.array([4.0, 5.0, 6.0])


def test_plane_point_known_answer(oracle):
    r, J = oracle.factor_rows(PI, NI, PJ, np.zeros((0, 3)), np.zeros((0, 3)), X0, X1)
    r_np = np_ref.plane_residual(X0, X1, PI, NI, PJ)
    assert abs(r[0] - r_np) <= 1e-12 * max(1.0, abs(r_np))
    _, Jn = np_ref.numeric_jacobian(lambda a, b: np_ref.plane_residual(a, b, PI, NI, PJ), X0, X1)
    assert np.allclose(J, Jn, atol=1e-7, rtol=1e-7)


def test_point_point_known_answer(oracle):
    # the reference test stacks the same pair four times
    pis = np.tile(PI, (4, 1))
    pjs = np.tile(PJ, (4, 1))
    r, J = oracle.factor_rows(np.zeros((0, 3)), np.zeros((0, 3)), np.zeros((0, 3)), pis, pjs, X0, X1)
    r_np = np_ref.point_residual(X0, X1, PI, PJ)
    assert np.allclose(r.reshape(4, 3), r_np[None, :], atol=1e-12)
    _, Jn = np_ref.numeric_jacobian(lambda a, b: np_ref.point_residual(a, b, PI, PJ), X0, X1)
    for k in range(4):
        assert np.allclose(J[3 * k:3 * k + 3], Jn, atol=1e-7, rtol=1e-7)


def test_jacobians_random(oracle):
    rng = np.random.default_rng(3)
    for _ in range(20):
        Ti = np_ref.compose(np_ref.pose(np.eye(3), rng.normal(size=3)), np_ref.expmap(rng.normal(size=6) * 0.5))
        Tj = np_ref.compose(np_ref.pose(np.eye(3), rng.normal(size=3)), np_ref.expmap(rng.normal(size=6) * 0.5))
        pi, pj = rng.normal(size=3) * 5, rng.normal(size=3) * 5
        n = rng.normal(size=3)
        n /= np.linalg.norm(n)
        r, J = oracle.factor_rows(pi, n, pj, pi[None], pj[None], Ti, Tj)
        _, Jp = np_ref.numeric_jacobian(lambda a, b: np_ref.plane_residual(a, b, pi, n, pj), Ti, Tj)
        _, Jt = np_ref.numeric_jacobian(lambda a, b: np_ref.point_residual(a, b, pi, pj), Ti, Tj)
        assert np.allclose(J[0], Jp[0], atol=2e-6)
        assert np.allclose(J[1:4], Jt, atol=2e-6)


@pytest.mark.parametrize("single", [False, True])
def test_normal_equations(oracle, single):
    """G = [A b]^T [A b], A = J / sigma, b = -r / sigma (DenseFactor::linearize +
    FastIsotropic); err = 0.5 ||r / sigma||^2 = 0.5 G[last]."""
    rng = np.random.default_rng(5)
    K = 3
    npl = np.array([5, 0, 7], np.uint32)
    npt = np.array([2, 3, 0], np.uint32)
    ppi = rng.normal(size=(12, 3)) * 10
    pni = rng.normal(size=(12, 3))
    pni /= np.linalg.norm(pni, axis=1, keepdims=True)
    ppj = ppi + rng.normal(size=(12, 3)) * 0.1
    tpi = rng.normal(size=(5, 3)) * 10
    tpj = tpi + rng.normal(size=(5, 3)) * 0.1
    Pi = np.stack([np_ref.expmap(rng.normal(size=6) * 0.3) for _ in range(K)])
    Pj = np.stack([np_ref.expmap(rng.normal(size=6) * 0.3) for _ in range(K)])
    G, err = oracle.linearize(npl, ppi, pni, ppj, npt, tpi, tpj, Pi, Pj, 0.1, single)
    op = ot = 0
    for k in range(K):
        r, J = oracle.factor_rows(ppi[op:op + npl[k]], pni[op:op + npl[k]], ppj[op:op + npl[k]],
                                  tpi[ot:ot + npt[k]], tpj[ot:ot + npt[k]], Pi[k], Pj[k])
        op += npl[k]
        ot += npt[k]
        Gn = np_ref.packed_G(J, r, 0.1, single)
        assert np.allclose(G[k], Gn, rtol=1e-10, atol=1e-9)
        assert np.isclose(err[k], 0.5 * np.sum((r / 0.1) ** 2), rtol=1e-12)
        assert np.isclose(err[k], 0.5 * G[k][-1], rtol=1e-12)


def test_se3_exp_log(oracle):
    rng = np.random.default_rng(11)
    for _ in range(50):
        xi = rng.normal(size=6) * np.array([1, 1, 1, 3, 3, 3])
        T = oracle.expmap(xi)
        assert np.allclose(T, np_ref.expmap(xi), atol=1e-12)
        assert np.allclose(oracle.logmap(T), xi, atol=1e-9)
    assert np.allclose(oracle.logmap(oracle.expmap(np.zeros(6))), 0)
