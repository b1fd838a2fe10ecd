"""Fronts beyond LDS (m > 128): the blocked large-front factorization (kkt_kernels.hip k_big_*: panels
of 32 pivots with the threshold rule of the small-front kernels, trailing updates on
v_mfma_f64_16x16x4f64) against the oracle and numpy's eigenvalues.  MUMPS factors such fronts with BLAS3
(MUMPSSolver.cpp:85-89, JOB=2); the inertia must be exact and the solve accurate."""
import numpy as np
import pytest

from oracle_ffi import OracleKKT

pytestmark = pytest.mark.gpu


def dense_coo(A):
    r, c = np.nonzero(np.tril(A))
    return r.astype(np.int64), c.astype(np.int64), A[r, c]


def check(n, r, c, v, S, rng, **opt):
    import uno_amd
    uno_amd.load_library()
    ev = np.linalg.eigvalsh(S)
    g = uno_amd.HipKKT(0, **opt)
    g.analyze(n, r, c)
    g.factorize(v)
    o = OracleKKT()
    o.analyze(n, r, c)
    o.factorize(v)
    expect = (int((ev > 0).sum()), int((ev < 0).sum()), 0)
    assert g.inertia() == o.inertia() == expect
    b = rng.standard_normal(n)
    x = g.solve(b)
    cond = np.abs(ev).max() / np.abs(ev).min()
    assert np.abs(S @ x - b).max() <= 1e-13 * cond * np.abs(b).max() * n ** 0.5
    np.testing.assert_allclose(x, o.solve(b), rtol=1e-12 * cond, atol=1e-12 * cond * np.abs(x).max())
    return g.stats()


@pytest.mark.parametrize("n", [129, 200, 513, 1024])
def test_dense_indefinite(n):
    """One dense front of order n (every column fully summed): random symmetric indefinite."""
    rng = np.random.default_rng(n)
    A = rng.standard_normal((n, n))
    S = (A + A.T) / 2 + np.diag(rng.uniform(-3, 3, n))
    r, c, v = dense_coo(S)
    st = check(n, r, c, v, S, rng)
    assert st["max_front"] == n


@pytest.mark.parametrize("nv,m", [(200, 120), (500, 300)])
def test_dense_kkt_2x2(nv, m):
    """Dense saddle point [[H, J^T], [J, 0]]: the zero block forces 2x2 pivots and interchanges, i.e. the
    panel's full-search path (flush, search, swap) inside the blocked factorization."""
    rng = np.random.default_rng(nv + m)
    H = rng.standard_normal((nv, nv)) * 0.1
    H = H + H.T + np.diag(rng.uniform(0.5, 2.0, nv))
    J = rng.standard_normal((m, nv))
    S = np.block([[H, J.T], [J, np.zeros((m, m))]])
    # constraints first: their zero diagonals fail the 1x1 test at once
    P = np.concatenate([np.arange(nv, nv + m), np.arange(nv)])
    S = S[np.ix_(P, P)]
    n = nv + m
    r, c, v = dense_coo(S)
    # keep the zero diagonal entries in the pattern (Uno's regularization slots)
    r = np.concatenate([r, np.arange(m)])
    c = np.concatenate([c, np.arange(m)])
    v = np.concatenate([v, np.zeros(m)])
    st = check(n, r, c, v, S, rng)
    assert st["pivots_2x2"] > 0


def test_arrow_root_front():
    """A banded system with 160 dense (arrow) rows: small fronts below, a root front of order >= 160 on
    the large-front path; the children's contribution blocks are assembled into it."""
    rng = np.random.default_rng(7)
    nb, k, bw = 3000, 160, 4
    n = nb + k
    S = np.zeros((n, n))
    for d in range(bw + 1):
        vals = rng.standard_normal(nb - d) * (0.3 if d else 1.0)
        S[np.arange(d, nb), np.arange(nb - d)] = vals
    S[:nb, :nb] += np.diag(rng.uniform(-2, 2, nb))
    S[nb:, :nb] = rng.standard_normal((k, nb)) * 0.05
    S[nb:, nb:] = np.tril(rng.standard_normal((k, k)))
    S = np.tril(S)
    S = S + S.T - np.diag(np.diag(S))
    r, c, v = dense_coo(S)
    st = check(n, r, c, v, S, rng)
    assert st["max_front"] > 128 and st["n_dense"] == k


def test_big_front_refactorization_and_retry():
    """Refactorizing with new values (and a device-side diagonal shift, as in the inertia-correction loop)
    re-runs the large-front path from its per-front state: results as from a fresh handle."""
    import uno_amd
    uno_amd.load_library()
    rng = np.random.default_rng(11)
    n = 300
    A = rng.standard_normal((n, n))
    S = (A + A.T) / 2
    r, c, v = dense_coo(S)
    r = np.concatenate([np.arange(n), r])
    c = np.concatenate([np.arange(n), c])
    v = np.concatenate([np.zeros(n), v])
    g = uno_amd.HipKKT(0)
    g.analyze(n, r, c)
    g.factorize(v)
    for shift in (0.0, 5.0, 50.0):
        g.fill_values(0, n, shift)
        g.factorize()
        ev = np.linalg.eigvalsh(S + shift * np.eye(n))
        assert g.inertia() == (int((ev > 0).sum()), int((ev < 0).sum()), 0)
        b = rng.standard_normal(n)
        x = g.solve(b)
        assert np.abs((S + shift * np.eye(n)) @ x - b).max() < 1e-8 * np.abs(x).max()
