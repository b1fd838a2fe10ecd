"""GPU parity tests: the HIP path (through the C ABI) against the oracle and the reference's known
answers.  Integer results (inertia, singularity, rank) must match exactly; solutions are checked
against the oracle and by residual, with tolerances stated in each test (north_star: primal/dual
residuals within 1e-10 relative)."""
import json
import os

import numpy as np
import pytest

from oracle_ffi import OracleKKT

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
KATS = json.load(open(os.path.join(HERE, "golden", "kats.json")))
RES_TOL = 1e-10  # relative residual ||Kx-b||_inf / (||K||_inf ||x||_inf + ||b||_inf)


@pytest.fixture(scope="module")
def uno_amd():
    import uno_amd as ua
    ua.load_library()
    return ua


def rel_residual(n, r, c, v, x, b):
    from uno_amd import coo_symv
    res = coo_symv(n, r, c, v, x) - b
    absv = coo_symv(n, r, c, np.abs(v), np.ones(n))  # row sums of |K|
    return np.abs(res).max() / (absv.max() * np.abs(x).max() + np.abs(b).max())


def componentwise_backward_error(n, r, c, v, x, b):
    """omega = max_i |b - K x|_i / (|K| |x| + |b|)_i: the smallest relative perturbation of every entry of K
    and b for which x is exact.  A backward-stable LDL^T solve gives omega of a few eps."""
    from uno_amd import coo_symv
    res = np.abs(coo_symv(n, r, c, v, x) - b)
    den = coo_symv(n, r, c, np.abs(v), np.abs(x)) + np.abs(b)
    return float(np.max(np.where(den > 0, res / np.where(den > 0, den, 1.0), np.where(res > 0, np.inf, 0.0))))


OMEGA_TOL = 1e-12  # componentwise backward error bar of one solve (GPU and oracle alike; the oracle measures 6e-14 at C2)


def both(n, r, c, v, **opt):
    from uno_amd import HipKKT
    g = HipKKT(0, **opt)
    g.analyze(n, r, c)
    g.factorize(v)
    o = OracleKKT()
    o.analyze(n, r, c)
    o.factorize(v)
    return g, o


@pytest.mark.parametrize("pack", [1, 0])
@pytest.mark.parametrize("case", ["c2", "random", "hub"])
def test_scaling_bit_identical(uno_amd, case, pack):
    """The equilibration (ICNTL(8)=8 restated as 3 symmetric infinity-norm sweeps, MUMPSSolver.cpp:82) is
    the oracle's to the bit: every scaling factor equal, and ||A_pre||_inf (whose summation order differs)
    within 1e-14 relative, so the null-pivot threshold eps * 1e-5 * ||A_pre||_inf is the oracle's."""
    from uno_amd import arrowband, SEEDS
    from kkt_cases import null_threshold_case
    if case == "c2":
        n, _, _, r, c, v, _ = arrowband(10000, SEEDS["C2"])
    elif case == "hub":  # long (chunked) rows, power-of-two scalings
        n, r, c, v, _, _ = null_threshold_case(100_000, [2, 8], 2.0 ** 30)
    else:
        rr, cc, vv, _ = random_sym(np.random.default_rng(5), 60, 0.3, zero_diag_frac=0.5)
        n, r, c, v = 60, rr, cc, vv * np.exp(np.random.default_rng(6).uniform(-20, 20, len(vv)))
    g, o = both(n, r, c, v, sweep_pack=pack)  # pack 0: the flat k_pack before the sweeps (option sweep_pack)
    sg, anorm = g.debug_scaling()
    so, thres = o.scaling()
    assert np.isfinite(sg).all() and (sg > 0).all()
    np.testing.assert_array_equal(sg, so)
    assert abs(np.finfo(float).eps * 1e-5 * anorm - thres) <= 1e-14 * thres


def test_kat_5x5(uno_amd):
    k = KATS["mumps_5x5"]
    g, o = both(k["n"], k["rows"], k["cols"], k["vals"])
    assert g.inertia() == tuple(k["inertia"]) == o.inertia()
    np.testing.assert_allclose(g.solve(k["rhs"]), k["solution"], atol=k["solution_tol"], rtol=0)


def test_kat_singular(uno_amd):
    k = KATS["mumps_singular"]
    g, o = both(k["n"], k["rows"], k["cols"], k["vals"])
    assert g.inertia() == tuple(k["inertia"]) == o.inertia()
    s = uno_amd.HipLDLSolver()
    m = uno_amd.SparseSymmetricMatrix(k["n"], len(k["rows"]), 0)
    for r, c, v in zip(k["rows"], k["cols"], k["vals"]):
        m.insert(r, c, v)
    s.initialize_memory(k["n"], 0, len(k["rows"]), 0)
    s.do_symbolic_analysis(m)
    s.do_numerical_factorization(m)
    assert s.matrix_is_singular() and s.rank() == 2 and s.number_negative_eigenvalues() == 1


@pytest.mark.parametrize("name", ["hs015_kkt0", "hs015_lsq"])
def test_hs015_systems(uno_amd, name):
    k = KATS[name]
    g, o = both(k["n"], k["rows"], k["cols"], k["vals"])
    assert g.inertia() == o.inertia()
    b = np.arange(1.0, k["n"] + 1)
    xg, xo = g.solve(b), o.solve(b)
    np.testing.assert_allclose(xg, xo, rtol=1e-9, atol=1e-12)
    assert rel_residual(k["n"], k["rows"], k["cols"], k["vals"], xg, b) < RES_TOL


def test_hs015_inertia_correction_trace(uno_amd):
    """PrimalDualRegularization loop (PrimalDualRegularization.hpp:133-219) driven by the GPU and by
    the oracle must visit the same (delta_w, delta_c, inertia) sequence."""
    from uno_amd import SparseSymmetricMatrix, HipLDLSolver, regularize_augmented_matrix
    k = KATS["hs015_kkt0"]

    class OracleSolver(HipLDLSolver):
        def __init__(self):
            self.kkt = None
            self.o = OracleKKT()

        def do_symbolic_analysis(self, m):
            r, c, _ = m.arrays()
            self.o.analyze(m.dimension(), r, c)

        def do_numerical_factorization(self, m):
            self.o.factorize(m.arrays()[2])

        def get_inertia(self):
            return self.o.inertia()

        def number_zero_eigenvalues(self):
            return self.o.inertia()[2]

    traces = []
    for solver in (HipLDLSolver(), OracleSolver()):
        m = SparseSymmetricMatrix(k["n"], len(k["rows"]) - 6, 6)
        for r, c, v in zip(k["rows"][6:], k["cols"][6:], k["vals"][6:]):
            m.insert(r, c, v)
        tr = []
        regularize_augmented_matrix(m, range(4), range(2), 1e-2, (4, 2, 0), solver, {}, trace=tr)
        traces.append(tr)
    assert traces[0] == traces[1]
    assert traces[0][-1][2] == (4, 2, 0)


def random_sym(rng, n, dens, zero_diag_frac):
    A = np.where(rng.random((n, n)) < dens, rng.standard_normal((n, n)), 0.0)
    A = np.tril(A)
    d = np.diag(A).copy()
    d[rng.random(n) < zero_diag_frac] = 0.0
    np.fill_diagonal(A, d)
    r, c = np.nonzero(A)
    rr = np.concatenate([r, np.arange(n)])
    cc = np.concatenate([c, np.arange(n)])
    vv = np.concatenate([A[r, c], np.zeros(n)])
    return rr, cc, vv, A + A.T - np.diag(np.diag(A))


@pytest.mark.parametrize("nmax,dens", [(40, 0.3), (150, 0.05), (300, 0.6)])
def test_random_indefinite(uno_amd, nmax, dens):
    """Random sparse/dense symmetric indefinite systems, including fronts beyond the LDS limit
    (n up to 300 dense -> k_factor_global)."""
    rng = np.random.default_rng(nmax)
    done = 0
    for trial in range(12):
        n = int(rng.integers(max(2, nmax // 3), nmax + 1))
        rr, cc, vv, S = random_sym(rng, n, dens, zero_diag_frac=0.5)
        ev = np.linalg.eigvalsh(S)
        if np.min(abs(ev)) < 1e-8 * max(1.0, abs(ev).max()):
            continue
        g, o = both(n, rr, cc, vv)
        assert g.inertia() == o.inertia() == (int((ev > 0).sum()), int((ev < 0).sum()), 0)
        b = rng.standard_normal(n)
        xg = g.solve(b)
        np.testing.assert_allclose(S @ xg, b, atol=1e-8 * np.linalg.cond(S) * np.abs(b).max())
        done += 1
    assert done >= 6


def test_small_dense_fronts(uno_amd):
    """One-wave fronts (register-grid kernels): inertia equal to the oracle's and the residual bar, on
    dense indefinite fronts up to 64 rows with zero diagonals (2x2 pivots, interchanges, LDS steps in the
    middle of a panel) and on the C2 arrowband KKT (level launches + dataflow launch)."""
    from uno_amd import arrowband, SEEDS
    rng = np.random.default_rng(17)
    done = 0
    for trial in range(16):
        n = int(rng.integers(5, 65))
        rr, cc, vv, S = random_sym(rng, n, 0.5, zero_diag_frac=0.6)
        ev = np.linalg.eigvalsh(S)
        if np.min(abs(ev)) < 1e-8 * max(1.0, abs(ev).max()):
            continue
        g, o = both(n, rr, cc, vv)
        assert g.inertia() == o.inertia() == (int((ev > 0).sum()), int((ev < 0).sum()), 0)
        b = rng.standard_normal(n)
        np.testing.assert_allclose(S @ g.solve(b), b, atol=1e-8 * np.linalg.cond(S) * np.abs(b).max())
        done += 1
    assert done >= 8
    n, nv, m, r, c, v, b = arrowband(10000, SEEDS["C2"])
    g, o = both(n, r, c, v)
    assert g.inertia() == o.inertia()
    xg = g.solve(b)
    assert rel_residual(n, r, c, v, xg, b) < RES_TOL


@pytest.mark.parametrize("rg", [0, 1, 2])
def test_dataflow_solve_kernels_bit_identical(uno_amd, rg):
    """C3-shaped arrowband at N = 1e5 (fronts of up to 72 rows, 2x2 pivots): the dataflow solve kernels
    (rg = 1: register-resident k_solve_fwd_rg + LDS-panel k_solve_bwd_df, the default; rg = 2: both register
    kernels, whose backward sums the rectangle in another order, so the level schedule follows it through
    k_solve_bwd_w2; rg = 0: the LDS-panel k_solve_*_df) give
    solutions bit-identical to the level-scheduled launches, over repeated solves (the arrival counters'
    epochs) and after a refactorization with new values."""
    from uno_amd import arrowband, SEEDS, HipKKT
    n, nv, m, r, c, v, b = arrowband(100000, SEEDS["C3"])
    opt = dict(solve_rg=int(rg > 0), solve_rg_bwd=int(rg == 2))
    gd, gl = HipKKT(0, **opt), HipKKT(0, dataflow_solve=0, **opt)
    for g in (gd, gl):
        g.analyze(n, r, c)
        g.factorize(v)
    assert gd.inertia() == gl.inertia()
    assert gd.stats()["solve_grid"] > 0
    for rep in range(3):
        np.testing.assert_array_equal(gd.solve(b * (rep + 1)), gl.solve(b * (rep + 1)))
    v2 = np.array(v)
    v2[:n] += 0.5
    for g in (gd, gl):
        g.factorize(v2)
    assert gd.inertia() == gl.inertia()
    np.testing.assert_array_equal(gd.solve(b), gl.solve(b))
    assert gd.stats()["solve_aborts"] == 0


@pytest.mark.parametrize("levels", [1, 2, 3])
def test_forward_flat_levels_bit_identical(uno_amd, levels):
    """Round 6: the walks' bottom levels as flat launches (k_solve_fwd_flat before the forward walk, k_solve_bwd_flat
    after the backward walk, one per level;
    option solve_flat_levels, default 2) give solutions bit-identical to the walk that solves every front itself
    (solve_flat_levels = 0), over repeated solves, in the plugin's relaxed mode, and after a refactorization; the
    walk's fronts then wait only for their walk children."""
    from uno_amd import arrowband, SEEDS, HipKKT
    n, nv, m, r, c, v, b = arrowband(100000, SEEDS["C3"])
    gl = HipKKT(0, solve_flat_levels=levels, delay_relaxed=0)
    gw = HipKKT(0, solve_flat_levels=0, delay_relaxed=0)
    for g in (gl, gw):
        g.analyze(n, r, c)
        g.factorize(v)
    assert gl.inertia() == gw.inertia()
    for rep in range(3):
        np.testing.assert_array_equal(gl.solve(b * (rep + 1)), gw.solve(b * (rep + 1)))
    v2 = np.array(v)
    v2[:n] -= 0.25
    for g in (gl, gw):
        g.factorize(v2)
    assert gl.inertia() == gw.inertia()
    xl = gl.solve(b)
    np.testing.assert_array_equal(xl, gw.solve(b))
    assert rel_residual(n, r, c, v2, xl, b) < RES_TOL
    assert gl.stats()["solve_aborts"] == 0 and gw.stats()["solve_aborts"] == 0


def test_arrowband_c2(uno_amd):
    """C2: arrowband KKT N=1e4; first factorization has wrong inertia (negative
    curvature), so the values of one regularized retry are compared too."""
    from uno_amd import arrowband, SEEDS
    n, nv, m, r, c, v, b = arrowband(10000, SEEDS["C2"])
    g, o = both(n, r, c, v)
    assert g.inertia() == o.inertia()
    xg = g.solve(b)
    assert rel_residual(n, r, c, v, xg, b) < RES_TOL
    # the bar is backward stability: each solution exact for a matrix within a few eps of K entrywise.  The two
    # solutions then differ only through K's conditioning (different orderings, different rounding); the
    # forward comparison below is a coarse sanity check, not the parity bar.
    xo = o.solve(b)
    assert componentwise_backward_error(n, r, c, v, xg, b) < OMEGA_TOL
    assert componentwise_backward_error(n, r, c, v, xo, b) < OMEGA_TOL
    np.testing.assert_allclose(xg, xo, rtol=1e-6, atol=1e-9 * np.abs(xg).max())
    # device-side diagonal update (inertia correction): delta_w on the primal block, -delta_c dual
    g.fill_values(0, nv, 1e-2)
    g.fill_values(nv, m, -1e-9)
    g.factorize()
    v2 = v.copy()
    v2[:nv] = 1e-2
    v2[nv:n] = -1e-9
    o.factorize(v2)
    assert g.inertia() == o.inertia()
    xg = g.solve(b)
    assert rel_residual(n, r, c, v2, xg, b) < RES_TOL
    st = g.stats()
    assert st["n_dense"] == 6 and st["factorizations"] == 2


def test_staged_values_match_host_upload(uno_amd):
    """uno_kkt_stage_values (the plugin's StagedCOOMatrix, integration/StagedCOOMatrix.hpp): the values staged
    in chunks out of order while "assembling", the first 50 positions (the regularization diagonal, stored
    first by COOFormat) edited and re-staged afterwards, then uno_kkt_factorize(NULL): inertia and solution
    bit-identical to a host-pointer factorization of the same values; then a second set of values staged over
    the first (the next IPM iteration) against a fresh host upload."""
    from uno_amd import HipKKT, arrowband, SEEDS
    n, _, _, r, c, v, b = arrowband(10000, SEEDS["C2"])
    nnz = len(v)
    host = HipKKT(0)
    host.analyze(n, r, c)
    host.factorize(v)
    x_host, in_host = host.solve(b), host.inertia()
    g = HipKKT(0)
    g.analyze(n, r, c)
    vals = np.array(v, dtype=np.float64)
    vals[:50] = 0.0
    bounds = list(range(0, nnz, 70_001)) + [nnz]
    for lo, hi in reversed(list(zip(bounds[:-1], bounds[1:]))):
        g.stage_values(vals, lo, hi - lo)
    vals[:50] = v[:50]
    g.stage_values(vals, 0, 50)
    g.factorize()
    assert g.inertia() == in_host
    np.testing.assert_array_equal(g.solve(b), x_host)
    v2 = np.array(v) * 1.5
    vals[:] = v2
    g.stage_values(vals, 0, nnz)
    g.factorize()
    host.factorize(v2)
    assert g.inertia() == host.inertia()
    np.testing.assert_array_equal(g.solve(b), host.solve(b))


def test_staged_then_device_edit_ordered(uno_amd):
    """Staged chunks and device-side value edits take effect in call order: chunks of a new set
    of values are staged (asynchronously, page-locked source), then uno_kkt_fill_values / uno_kkt_set_values
    edit the regularization prefix on the device before the factorization -- the edit wins over the staged
    chunk of the same positions, as a sequential copy would have it.  Inputs converted on the fly (float32,
    strided) stay referenced until the factorization is queried."""
    from uno_amd import HipKKT, arrowband, SEEDS
    n, nv, m, r, c, v, b = arrowband(20000, SEEDS["C2"])
    nnz = len(v)
    g = HipKKT(0, pin_host_values=1)
    g.analyze(n, r, c)
    g.factorize(v)
    g.inertia()
    ref = HipKKT(0)
    ref.analyze(n, r, c)
    for rep, dw in enumerate((1e-4, 3e-2)):
        v2 = np.array(v) * (1.0 + 0.25 * rep)
        vals = v2.copy()
        bounds = list(range(0, nnz, 1 << 16)) + [nnz]
        for lo, hi in zip(bounds[:-1], bounds[1:]):
            g.stage_values(vals, lo, hi - lo)
        g.fill_values(0, nv, dw)
        g.set_values(np.arange(nv, n, dtype=np.int64), np.full(n - nv, -1e-8))
        g.factorize()
        expect = v2.copy()
        expect[:nv] = dw
        expect[nv:n] = -1e-8
        ref.factorize(expect)
        assert g.inertia() == ref.inertia()
        np.testing.assert_array_equal(g.solve(b), ref.solve(b))
    # a float32 source: every chunk is a converted temporary, kept alive by the wrapper until inertia()
    v32 = (np.array(v) * 0.5).astype(np.float32)
    g.stage_values(v32, 0, nnz // 2)
    g.stage_values(v32, nnz // 2, nnz - nnz // 2)
    g.factorize()
    ref.factorize(v32.astype(np.float64))
    assert g.inertia() == ref.inertia()
    np.testing.assert_array_equal(g.solve(b), ref.solve(b))


def test_empty_and_tiny(uno_amd):
    from uno_amd import HipKKT
    g = HipKKT()
    g.analyze(3, [], [])
    g.factorize(np.zeros(0))
    assert g.inertia() == (0, 0, 3)
    np.testing.assert_array_equal(g.solve([1.0, 2.0, 3.0]), 0.0)
    g.analyze(1, [0], [0])
    g.factorize([-2.0])
    assert g.inertia() == (0, 1, 0)
    np.testing.assert_allclose(g.solve([4.0]), [-2.0])


@pytest.mark.parametrize("n", [10000, 200000])
def test_dataflow_matches_level_schedule(uno_amd, n):
    """The one-launch dataflow factorization of the upper tree (k_factor_df) and dataflow solves
    (k_solve_*_df: fronts wait on arrival counters inside the launch) do the same arithmetic as the
    level-scheduled launches: inertia equal and solutions bit-identical, over repeated solves
    (cumulative epoch counters) and after a refactorization with other values (new pivoting)."""
    from uno_amd import HipKKT, arrowband, SEEDS
    N, nv, m, r, c, v, b = arrowband(n, SEEDS["C2"])
    gd, gl = HipKKT(0), HipKKT(0, dataflow_solve=0, dataflow_factor=0)
    for g in (gd, gl):
        g.analyze(N, r, c)
        g.factorize(v)
    assert gd.inertia() == gl.inertia()
    sd, sl = gd.stats(), gl.stats()
    assert sd["solve_grid"] > 0 and sl["solve_grid"] == 0
    assert sd["factor_df_fronts"] > 0 and sl["factor_df_fronts"] == 0
    xl = gl.solve(b)
    for rep in range(3):
        xd = gd.solve(b * (rep + 1))
        np.testing.assert_array_equal(xd, gl.solve(b * (rep + 1)) if rep else xl)
    assert rel_residual(N, r, c, v, xl, b) < RES_TOL
    v2 = v.copy()
    v2[:nv] = 1e-2
    v2[nv:N] = -1e-9
    for g in (gd, gl):
        g.factorize(v2)
    assert gd.inertia() == gl.inertia()
    b2 = np.cos(np.arange(N))
    np.testing.assert_array_equal(gd.solve(b2), gl.solve(b2))
    assert gd.stats()["solve_aborts"] == 0 and gd.stats()["factor_df_aborts"] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("window", [74, 160, 400])
def test_dataflow_panel_windows(uno_amd, window):
    """Panels larger than the LDS window are solved in column windows (forward first to last, backward
    last to first, later windows loaded from L): bit-identical to the level schedule, with 2x2 pivots."""
    from uno_amd import HipKKT, arrowband, SEEDS
    N, nv, m, r, c, v, b = arrowband(20000, SEEDS["C2"])
    gd, gl = HipKKT(0, solve_window=window), HipKKT(0, dataflow_solve=0)
    for g in (gd, gl):
        g.analyze(N, r, c)
        g.factorize(v)
    assert gd.inertia() == gl.inertia()
    assert gd.stats()["pivots_2x2"] > 0
    for rep in range(2):
        np.testing.assert_array_equal(gd.solve(b * (rep + 1)), gl.solve(b * (rep + 1)))
    assert gd.stats()["solve_aborts"] == 0


@pytest.mark.slow
def test_c3_full_size(uno_amd):
    """The headline configuration itself (BASELINE.json configs[2], SURVEY.md 8(d) C3: arrowband KKT
    n = 1e6, nnz = 2e7, seed 0x5EED0003): inertia identical to the oracle's, solution within 1e-6 of the
    oracle's (different orderings: ND vs RCM), relative residual <= 1e-10; then one inertia-correction
    retry (delta_w / delta_c edited on the device, PrimalDualRegularization.hpp:178-179) with the same
    checks, and a second solve that must be bit-identical to the first (deterministic kernels)."""
    from uno_amd import HipKKT, arrowband, SEEDS
    n, nv, m, r, c, v, b = arrowband(1_000_000, SEEDS["C3"])
    g, o = both(n, r, c, v)
    assert g.inertia() == o.inertia()
    xg = g.solve(b)
    assert rel_residual(n, r, c, v, xg, b) < RES_TOL
    # backward stability is the bar (test_arrowband_c2); the forward comparison is a sanity check
    xo = o.solve(b)
    assert componentwise_backward_error(n, r, c, v, xg, b) < OMEGA_TOL
    assert componentwise_backward_error(n, r, c, v, xo, b) < OMEGA_TOL
    np.testing.assert_allclose(xg, xo, rtol=1e-6, atol=1e-9 * np.abs(xg).max())
    np.testing.assert_array_equal(g.solve(b), xg)
    g.fill_values(0, nv, 1e-4)
    g.fill_values(nv, m, -1e-8)
    g.factorize()
    v2 = v.copy()
    v2[:nv] = 1e-4
    v2[nv:n] = -1e-8
    o.factorize(v2)
    assert g.inertia() == o.inertia()
    xg = g.solve(b)
    assert rel_residual(n, r, c, v2, xg, b) < RES_TOL
    np.testing.assert_allclose(xg, o.solve(b), rtol=1e-6, atol=1e-9 * np.abs(xg).max())
    st = g.stats()
    assert st["solve_aborts"] == 0 and st["factor_df_aborts"] == 0


def test_threshold_relaxation_with_refinement(uno_amd):
    """delay_relaxed = 0 (the Uno plugin's setting, integration/HIPLDLSolver.cpp): a front whose fully-summed
    block has no pivot passing u relaxes the threshold instead of delaying the columns to its parent (no
    re-analysis); the factorization is then followed by one step of iterative refinement.  Inertia equal
    to the oracle's (which delays, as MUMPS); residual within the 1e-10 bar after refinement."""
    from uno_amd import HipKKT, arrowband, SEEDS
    n, nv, m, r, c, v, b = arrowband(10000, SEEDS["C2"])
    g, o = both(n, r, c, v, delay_relaxed=0)
    assert g.inertia() == o.inertia()
    st = g.stats()
    assert st["pivots_relaxed"] > 0 and st["fronts_merged"] == 0
    xg = g.solve(b)
    assert rel_residual(n, r, c, v, xg, b) < RES_TOL
    np.testing.assert_allclose(xg, o.solve(b), rtol=1e-6, atol=1e-9 * np.abs(xg).max())
    # aliasing device solve with refinement keeps the right-hand side for the residual
    import torch
    bd = torch.from_numpy(b.copy()).to("cuda")
    g.solve_device(bd.data_ptr(), bd.data_ptr())
    torch.cuda.synchronize()
    np.testing.assert_allclose(bd.cpu().numpy(), xg, rtol=1e-12, atol=1e-14 * np.abs(xg).max())


def test_refinement_residual_over_fronts(uno_amd):
    """The refinement residual r = A x - b over the fronts' packed slots (launch_resid: per-front LDS partials,
    then per-row sums in front order; the default) against the row-wise COO symv it replaced (resid_fronts =
    0): both refined solutions meet the residual bar and agree to rounding; the chunked path of the dense
    rows (forced here on every row with more than 4 partials) gives the same; a repeated solve is
    bit-identical (the per-front accumulation is one wave's, the row sums are in a fixed order)."""
    from uno_amd import arrowband, SEEDS
    n, nv, m, r, c, v, b = arrowband(10000, SEEDS["C2"])
    g1, o = both(n, r, c, v, delay_relaxed=0)
    g0, _ = both(n, r, c, v, delay_relaxed=0, resid_fronts=0)
    g2, _ = both(n, r, c, v, delay_relaxed=0, resid_long=4)
    assert g1.stats()["pivots_relaxed"] > 0
    x1, x0, x2 = g1.solve(b), g0.solve(b), g2.solve(b)
    for x in (x1, x0, x2):
        assert rel_residual(n, r, c, v, x, b) < RES_TOL
    assert g1.stats()["refinements"] == 1 and g0.stats()["refinements"] == 1
    np.testing.assert_allclose(x1, x0, rtol=1e-9, atol=1e-12 * np.abs(x0).max())
    np.testing.assert_allclose(x2, x1, rtol=1e-9, atol=1e-12 * np.abs(x1).max())
    np.testing.assert_array_equal(g1.solve(b), x1)
    np.testing.assert_array_equal(g2.solve(b), x2)


def test_refine_tol_non_finite(uno_amd):
    """Option refine_tol skips the refinement step only when the componentwise backward error of x is
    finite and below the bound: a NaN in the right-hand side makes omega NaN, which must count as
    +infinity (the step runs and last_backward_error reports inf), never as a near-perfect solve."""
    from uno_amd import arrowband, SEEDS
    n, nv, m, r, c, v, b = arrowband(10000, SEEDS["C2"])
    g, o = both(n, r, c, v, delay_relaxed=0, refine_tol=1e-6)
    assert g.stats()["pivots_relaxed"] > 0
    g.solve(b)
    st = g.stats()
    assert 0.0 <= st["last_backward_error"] < np.inf
    bn = np.array(b)
    bn[n // 2] = np.nan
    x = g.solve(bn)
    st2 = g.stats()
    assert st2["last_backward_error"] == np.inf
    assert st2["refinements"] == st["refinements"] + 1 and st2["refinements_skipped"] == st["refinements_skipped"]
    assert np.isnan(x).any()


def test_factorize_update_prefix(uno_amd):
    """uno_kkt_factorize_update (the plugin's inertia-correction retries): after a host-pointer
    factorization, uploading only positions [0, n) (the regularization diagonal Uno stores first,
    COOFormat.hpp:102-110) gives the factorization of the edited array: same inertia and solution as a
    full upload and as the oracle; page-locked host values (pin_host_values) give the same results."""
    from uno_amd import HipKKT, arrowband, SEEDS
    n, nv, m, r, c, v, b = arrowband(20000, SEEDS["C2"])
    g = HipKKT(0, pin_host_values=1)
    full = HipKKT(0)
    g.analyze(n, r, c)
    full.analyze(n, r, c)
    o = OracleKKT()
    o.analyze(n, r, c)
    vals = v.copy()
    g.factorize(vals)
    for dw in (1e-4, 8e-4, 6.4e-3, 1.0):
        vals[:nv] = dw
        vals[nv:n] = -1e-8
        g.factorize_update(vals, 0, n)
        full.factorize(vals.copy())
        o.factorize(vals)
        assert g.inertia() == full.inertia() == o.inertia()
        np.testing.assert_array_equal(g.solve(b), full.solve(b))
    with pytest.raises(RuntimeError):
        g.factorize_update(vals, n - 1, len(vals))  # range beyond the array


def test_dataflow_abort_redone_and_rearmed(uno_amd):
    """A dataflow solve whose dependency waits give up (forced here: option debug_abort_solves starts the
    walk with its abort flag set) is redone level by level within the same call -- same solution, bit for
    bit, also for an aliasing device solve -- and the dataflow solve stays armed for the next solve
    (one abort used to disable it for the handle's lifetime)."""
    import torch
    from uno_amd import HipKKT, arrowband, SEEDS
    N, nv, m, r, c, v, b = arrowband(20000, SEEDS["C2"])
    g, ref = HipKKT(0), HipKKT(0, dataflow_solve=0)
    for h in (g, ref):
        h.analyze(N, r, c)
        h.factorize(v)
    x_ref = ref.solve(b)
    g.set_option("debug_abort_solves", 1)
    np.testing.assert_array_equal(g.solve(b), x_ref)
    st = g.stats()
    assert st["solve_aborts"] == 1 and st["solve_grid"] > 0  # redone, and still armed
    g.set_option("debug_abort_solves", 1)
    bd = torch.from_numpy(b.copy()).to("cuda")
    g.solve_device(bd.data_ptr(), bd.data_ptr())  # x aliases the rhs: the redo must still see b
    torch.cuda.synchronize()
    np.testing.assert_array_equal(bd.cpu().numpy(), x_ref)
    np.testing.assert_array_equal(g.solve(b), x_ref)  # a normal dataflow solve again
    st = g.stats()
    assert st["solve_aborts"] == 2 and st["solve_grid"] > 0


@pytest.mark.gpu
def test_children_assembly_positions_bitwise(uno_amd):
    """Children assembly through the precomputed packed positions (option cbpos, default on; rebuilt with the
    structure after delays) adds the same entries in the same order as the relmap-gather form: same inertia,
    same solution bit for bit, default and relaxed (plugin) mode."""
    from uno_amd import HipKKT, arrowband, SEEDS
    N, nv, m, r, c, v, b = arrowband(20000, SEEDS["C2"])
    for opts in ({}, {"delay_relaxed": 0}):
        g, ref = HipKKT(0, **opts), HipKKT(0, cbpos=0, **opts)
        for h in (g, ref):
            h.analyze(N, r, c)
            h.factorize(v)
        assert g.inertia() == ref.inertia()
        np.testing.assert_array_equal(g.solve(b), ref.solve(b))
        g.close()
        ref.close()
