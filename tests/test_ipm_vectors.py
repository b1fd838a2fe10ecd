"""Device-side vector work around the KKT solve against the CPU oracle
(oracle/ipm_oracle.py, a restatement of the reference loops in their floating-point order).

Bars: the right-hand side and the direction (with both step lengths) are bit-identical to the oracle
(same operation order, no FMA contraction); symv / quadratic_product differ from the reference's COO
order only by summation order: relative error <= 1e-13 (symv, per entry against the row's |A| |x|
sum) and 1e-12 (quadratic product)."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import ipm_oracle  # noqa: E402


def random_ipm_point(rng, n, m, nnz_per_con=8):
    jc = np.repeat(np.arange(m), nnz_per_con)
    jv = rng.integers(0, n, size=m * nnz_per_con)
    perm = rng.permutation(len(jc))          # entries in arbitrary stored order
    jc, jv = jc[perm], jv[perm]
    jval = rng.uniform(-2, 2, size=len(jc))
    grad = rng.standard_normal(n)
    cons = rng.standard_normal(m)
    y = rng.standard_normal(m)
    y[rng.random(m) < 0.2] = 0.0             # zero multipliers are skipped by the reference
    return grad, cons, y, jc, jv, jval


def test_oracle_rhs_matches_dense():
    rng = np.random.default_rng(1)
    n, m = 60, 25
    grad, cons, y, jc, jv, jval = random_ipm_point(rng, n, m)
    J = np.zeros((m, n))
    np.add.at(J, (jc, jv), jval)
    rhs = ipm_oracle.assemble_augmented_rhs(grad, cons, y, jc, jv, jval)
    np.testing.assert_allclose(rhs[:n], -grad + J.T @ y, rtol=1e-13, atol=1e-13)
    np.testing.assert_array_equal(rhs[n:], -cons)


def test_oracle_direction_small():
    # one lower-bounded, one upper-bounded, one free variable, one constraint
    sol = np.array([-1.0, 2.0, 5.0, 3.0])
    x = np.array([1.0, 0.0, 0.0])
    lb = np.array([0.0, -np.inf, -np.inf])
    ub = np.array([np.inf, 1.0, np.inf])
    zl = np.array([0.5, 0.0, 0.0])
    zu = np.array([0.0, 0.25, 0.0])
    dx, dy, dzl, dzu, (ap, ad) = ipm_oracle.assemble_direction(sol, x, lb, ub, zl, zu, 0.1, 0.99)
    tau = 0.99
    ap_ref = min(1.0, -tau * 1.0 / -1.0, -tau * (0.0 - 1.0) / 2.0)
    assert ap == pytest.approx(ap_ref)
    assert dy[0] == pytest.approx(-3.0 * ap)
    dzl0 = (0.1 - (-1.0) * 0.5) / 1.0 - 0.5
    assert dzl[0] == pytest.approx(dzl0 * ad)


def test_oracle_symv_matches_dense():
    rng = np.random.default_rng(2)
    n = 30
    r = rng.integers(0, n, 120)
    c = rng.integers(0, n, 120)
    v = rng.standard_normal(120)
    A = np.zeros((n, n))
    for a, b, w in zip(r, c, v):
        A[a, b] += w
        if a != b:
            A[b, a] += w
    x, yv = rng.standard_normal(n), rng.standard_normal(n)
    np.testing.assert_allclose(ipm_oracle.symv(n, r, c, v, x), A @ x, rtol=1e-12, atol=1e-12)
    assert ipm_oracle.quadratic_product(r, c, v, x, yv) == pytest.approx(x @ A @ yv, rel=1e-12)


@pytest.mark.gpu
def test_device_rhs_and_direction_bitwise():
    import torch
    import uno_amd
    rng = np.random.default_rng(3)
    n, m = 20000, 7000
    grad, cons, y, jc, jv, jval = random_ipm_point(rng, n, m)
    g = uno_amd.HipKKT(0)
    g.rhs_setup(n, m, jc, jv)
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).cuda()
    G, C, Y, JV = d(grad), d(cons), d(y), d(jval)
    rhs = torch.empty(n + m, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()  # torch's copies run on its own stream; the solver has its own
    g.assemble_rhs(G.data_ptr(), C.data_ptr(), Y.data_ptr(), JV.data_ptr(), rhs.data_ptr())
    torch.cuda.synchronize()
    ref = ipm_oracle.assemble_augmented_rhs(grad, cons, y, jc, jv, jval)
    np.testing.assert_array_equal(rhs.cpu().numpy(), ref)

    sol = rng.standard_normal(n + m)
    x = rng.uniform(-1, 1, n)
    lb = np.where(rng.random(n) < 0.6, x - rng.uniform(0.01, 2, n), -np.inf)
    ub = np.where(rng.random(n) < 0.4, x + rng.uniform(0.01, 2, n), np.inf)
    zl = np.where(np.isfinite(lb), rng.uniform(0.01, 1, n), 0.0)
    zu = np.where(np.isfinite(ub), rng.uniform(0.01, 1, n), 0.0)
    out = [torch.empty(k, dtype=torch.float64, device="cuda") for k in (n, m, n, n)]
    ins = [d(a) for a in (sol, x, lb, ub, zl, zu)]  # kept alive across the call
    torch.cuda.synchronize()
    steps = g.assemble_direction(n, m, *[t.data_ptr() for t in ins], 1e-3, 0.99, *[o.data_ptr() for o in out])
    dx, dy, dzl, dzu, (ap, ad) = ipm_oracle.assemble_direction(sol, x, lb, ub, zl, zu, 1e-3, 0.99)
    assert steps == (ap, ad) and 0.0 < ap <= 1.0 and 0.0 < ad <= 1.0
    for got, want in zip(out, (dx, dy, dzl, dzu)):
        np.testing.assert_array_equal(got.cpu().numpy(), want)


@pytest.mark.gpu
def test_device_rhs_long_variables_bitwise():
    """Variables in more than kRhsLong (1024) constraints -- the arrowband's linking variables are in all of
    them -- take the one-wave ordered sum (k_rhs_long): bit-identical to the reference's accumulation,
    zero multipliers skipped, list lengths that are and are not multiples of 64."""
    import torch
    import uno_amd
    rng = np.random.default_rng(8)
    n, m = 3000, 5000
    grad, cons, y, jc, jv, jval = random_ipm_point(rng, n, m, nnz_per_con=4)
    dense = np.array([7, 1500, 2999])                # in every constraint
    half = np.array([11])                            # in the first 1088 = 17 x 64 constraints
    jc = np.concatenate([jc, np.repeat(np.arange(m), len(dense)), np.arange(1088)])
    jv = np.concatenate([jv, np.tile(dense, m), np.repeat(half, 1088)])
    perm = rng.permutation(len(jc))
    jc, jv = jc[perm], jv[perm]
    jval = rng.uniform(-2, 2, size=len(jc))
    g = uno_amd.HipKKT(0)
    g.rhs_setup(n, m, jc, jv)
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).cuda()
    G, C, Y, JV = d(grad), d(cons), d(y), d(jval)
    rhs = torch.empty(n + m, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    g.assemble_rhs(G.data_ptr(), C.data_ptr(), Y.data_ptr(), JV.data_ptr(), rhs.data_ptr())
    torch.cuda.synchronize()
    ref = ipm_oracle.assemble_augmented_rhs(grad, cons, y, jc, jv, jval)
    np.testing.assert_array_equal(rhs.cpu().numpy(), ref)


@pytest.mark.gpu
def test_device_symv_and_quadratic_product():
    import torch
    import uno_amd
    n, nv, m, r, c, v, b = uno_amd.arrowband(3000, uno_amd.SEEDS["C2"])
    g = uno_amd.HipKKT(0)
    g.analyze(n, r, c)
    g.factorize(v)
    g.inertia()
    rng = np.random.default_rng(4)
    x, w = rng.standard_normal(n), rng.standard_normal(n)
    X = torch.from_numpy(x).cuda()
    W = torch.from_numpy(w).cuda()
    Y = torch.from_numpy(w.copy()).cuda()     # y += A x on top of w
    torch.cuda.synchronize()
    g.symv(X.data_ptr(), Y.data_ptr())
    torch.cuda.synchronize()
    ref = w + ipm_oracle.symv(n, r, c, v, x)
    scale = ipm_oracle.symv(n, r, c, np.abs(v), np.abs(x)) + np.abs(w)
    assert (np.abs(Y.cpu().numpy() - ref) <= 1e-13 * scale + 1e-300).all()
    q = g.quadratic_product(W.data_ptr(), X.data_ptr())
    qref = ipm_oracle.quadratic_product(r, c, v, w, x)
    assert abs(q - qref) <= 1e-12 * abs(np.abs(w) @ ipm_oracle.symv(n, r, c, np.abs(v), np.abs(x)))
    # values edited on the device are picked up (the packed copy is refreshed)
    g.fill_values(0, nv, 2.0)
    Y.zero_()
    torch.cuda.synchronize()
    g.symv(X.data_ptr(), Y.data_ptr())
    v2 = v.copy()
    v2[:nv] = 2.0
    torch.cuda.synchronize()
    np.testing.assert_allclose(Y.cpu().numpy(), ipm_oracle.symv(n, r, c, v2, x), rtol=1e-12, atol=1e-12)


@pytest.mark.gpu
def test_device_symv_long_rows():
    """Rows with more than 2048 entries (the arrowband's 6 dense rows carry m = 25 000 Jacobian entries
    each here) take the chunked reduction (k_symv_long + k_symv_long_fin); the product and the quadratic
    form agree with the COO product, and two calls give bit-identical results (fixed chunk order)."""
    import torch
    import uno_amd
    n, nv, m, r, c, v, b = uno_amd.arrowband(100000, uno_amd.SEEDS["C2"])
    g = uno_amd.HipKKT(0)
    g.analyze(n, r, c)
    g.factorize(v)
    g.inertia()
    rng = np.random.default_rng(5)
    x, w = rng.standard_normal(n), rng.standard_normal(n)
    X = torch.from_numpy(x).cuda()
    W = torch.from_numpy(w).cuda()
    ys = []
    for _ in range(2):
        Y = torch.zeros(n, dtype=torch.float64, device="cuda")
        torch.cuda.synchronize()
        g.symv(X.data_ptr(), Y.data_ptr())
        torch.cuda.synchronize()
        ys.append(Y.cpu().numpy())
    np.testing.assert_array_equal(ys[0], ys[1])
    ref = uno_amd.coo_symv(n, r, c, v, x)  # the generator's C COO product (same as ipm_oracle.symv)
    scale = uno_amd.coo_symv(n, r, c, np.abs(v), np.abs(x))
    assert (np.abs(ys[0] - ref) <= 1e-13 * scale + 1e-300).all()
    dense = np.argsort(-np.abs(scale))[:6]  # the long rows dominate |A||x|
    assert np.all(np.abs(ref[dense]) > 0.0)
    q = g.quadratic_product(W.data_ptr(), X.data_ptr())
    assert abs(q - w @ ref) <= 1e-12 * abs(np.abs(w) @ scale)


@pytest.mark.gpu
def test_device_barrier_diagonal_bitwise():
    """Sigma on the device (uno_kkt_assemble_barrier) equals the host expression of
    PrimalDualInteriorPointProblem.cpp:62-77 bit for bit: 0 + zl / (x - lb) [finite lb] + zu / (x - ub)
    [finite ub], one entry per variable with a finite bound, ascending, written at the barrier block of the
    COO value array (the rest of the array untouched)."""
    import torch
    import uno_amd
    rng = np.random.default_rng(9)
    n = 50000
    x = rng.uniform(-1, 1, n)
    lb = np.where(rng.random(n) < 0.6, x - 10.0 ** rng.uniform(-8, 1, n), -np.inf)
    ub = np.where(rng.random(n) < 0.4, x + 10.0 ** rng.uniform(-8, 1, n), np.inf)
    zl = rng.uniform(1e-9, 1, n)
    zu = -rng.uniform(1e-9, 1, n)
    bounded = np.isfinite(lb) | np.isfinite(ub)
    ref = []
    for i in np.nonzero(bounded)[0]:
        d = 0.0
        if np.isfinite(lb[i]):
            d += zl[i] / (x[i] - lb[i])
        if np.isfinite(ub[i]):
            d += zu[i] / (x[i] - ub[i])
        ref.append(d)
    g = uno_amd.HipKKT(0)
    assert g.barrier_setup(lb, ub) == bounded.sum()
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).cuda()
    X, ZL, ZU = d(x), d(zl), d(zu)
    vals = torch.full((bounded.sum() + 10,), 7.0, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    g.assemble_barrier(X.data_ptr(), ZL.data_ptr(), ZU.data_ptr(), vals.data_ptr() + 8 * 5)
    torch.cuda.synchronize()
    out = vals.cpu().numpy()
    np.testing.assert_array_equal(out[5:5 + bounded.sum()], np.array(ref))
    assert (out[:5] == 7.0).all() and (out[5 + bounded.sum():] == 7.0).all()


# ---- reference-generated golden vectors (tests/golden/make_ipm_fixtures.sh: the Uno core compiled from
# /root/reference calls PrimalDualInteriorPointProblem::evaluate_lagrangian_hessian,
# Subproblem::assemble_augmented_rhs and Subproblem::assemble_primal_dual_direction on seeded inputs) ----
def _ref_cases():
    import json
    raw = json.load(open(os.path.join(ROOT, "tests", "golden", "ipm_reference_vectors.json")))
    conv = lambda a: np.array([float(v) for v in a])  # "inf" / "-inf" strings for unbounded sides
    out = []
    for c in raw:
        d = dict(c)
        for k in ("lb", "ub", "x", "zl", "zu", "y", "sigma", "grad", "cons", "jac_val", "rhs", "solution", "dx", "dy",
                  "dzl", "dzu"):
            d[k] = conv(c[k])
        for k in ("sigma_var", "jac_con", "jac_var"):
            d[k] = np.array(c[k], dtype=np.int64)
        out.append(d)
    return out


REF_CASES = _ref_cases()


def test_reference_vectors_cover_every_bound_kind():
    for c in REF_CASES:
        fl, fu = np.isfinite(c["lb"]), np.isfinite(c["ub"])
        assert (fl & ~fu).any() and (fu & ~fl).any() and (fl & fu).any() and (~fl & ~fu).any()
        assert (c["y"] == 0.0).any() and len(np.unique(c["jac_var"])) < len(c["jac_var"])  # skipped terms, repeats


@pytest.mark.parametrize("k", range(len(REF_CASES)))
def test_oracle_reproduces_reference_vectors(k):
    """oracle/ipm_oracle.py against the reference's own outputs, bit for bit (the restatement is pinned)."""
    c = REF_CASES[k]
    var, sig = ipm_oracle.barrier_diagonal(c["x"], c["lb"], c["ub"], c["zl"], c["zu"])
    np.testing.assert_array_equal(var, c["sigma_var"])
    np.testing.assert_array_equal(sig, c["sigma"])
    rhs = ipm_oracle.assemble_augmented_rhs(c["grad"], c["cons"], c["y"], c["jac_con"], c["jac_var"], c["jac_val"])
    np.testing.assert_array_equal(rhs, c["rhs"])
    dx, dy, dzl, dzu, _ = ipm_oracle.assemble_direction(c["solution"], c["x"], c["lb"], c["ub"], c["zl"], c["zu"],
                                                        c["mu"], c["tau_min"])
    for got, key in ((dx, "dx"), (dy, "dy"), (dzl, "dzl"), (dzu, "dzu")):
        np.testing.assert_array_equal(got, c[key], err_msg=key)


@pytest.mark.gpu
@pytest.mark.parametrize("k", range(len(REF_CASES)))
def test_device_reproduces_reference_vectors(k):
    """The HIP kernels (uno_kkt_assemble_barrier / _rhs / _direction) on the reference's inputs give the
    reference's outputs bit for bit."""
    import torch
    import uno_amd
    c = REF_CASES[k]
    n, m = c["n"], c["m"]
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).cuda()
    g = uno_amd.HipKKT(0)
    assert g.barrier_setup(c["lb"], c["ub"]) == len(c["sigma"])
    X, ZL, ZU = d(c["x"]), d(c["zl"]), d(c["zu"])
    vals = torch.zeros(len(c["sigma"]), dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    g.assemble_barrier(X.data_ptr(), ZL.data_ptr(), ZU.data_ptr(), vals.data_ptr())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(vals.cpu().numpy(), c["sigma"])
    g.rhs_setup(n, m, c["jac_con"], c["jac_var"])
    G, C, Y, JV = d(c["grad"]), d(c["cons"]), d(c["y"]), d(c["jac_val"])
    rhs = torch.empty(n + m, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    g.assemble_rhs(G.data_ptr(), C.data_ptr(), Y.data_ptr(), JV.data_ptr(), rhs.data_ptr())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(rhs.cpu().numpy(), c["rhs"])
    out = [torch.empty(k2, dtype=torch.float64, device="cuda") for k2 in (n, m, n, n)]
    ins = [d(a) for a in (c["solution"], c["x"], c["lb"], c["ub"], c["zl"], c["zu"])]
    torch.cuda.synchronize()
    g.assemble_direction(n, m, *[t.data_ptr() for t in ins], c["mu"], c["tau_min"], *[o.data_ptr() for o in out])
    torch.cuda.synchronize()
    for got, key in zip(out, ("dx", "dy", "dzl", "dzu")):
        np.testing.assert_array_equal(got.cpu().numpy(), c[key], err_msg=key)


# ---- the augmented (KKT) value array, SURVEY.md 8(f)2 (tests/golden/augmented_reference_vectors.json: the
# reference's COOFormat::reset + Subproblem::assemble_augmented_matrix for the arrowband model through the ipopt
# reformulation chain, with the inputs of the device assembly; tests/golden/make_ipm_fixtures.sh) ----
def _aug_cases():
    import json
    raw = json.load(open(os.path.join(ROOT, "tests", "golden", "augmented_reference_vectors.json")))
    out = []
    for c in raw:
        d = dict(c)
        for k in ("lb", "ub", "x", "zl", "zu", "hess", "hess_sigma", "jac", "values"):
            d[k] = np.array([float(v) for v in c[k]])
        for k in ("rows", "cols"):
            d[k] = np.array(c[k], dtype=np.int64)
        out.append(d)
    return out


AUG_CASES = _aug_cases()


@pytest.mark.parametrize("k", range(len(AUG_CASES)))
def test_oracle_reproduces_reference_augmented_matrix(k):
    """oracle/ipm_oracle.assemble_augmented on the reference's inputs gives the reference's COO values bit for
    bit; the Hessian terms at objective multiplier sigma are sigma times those at 1 (ArrowbandModel inserts
    sigma * H), so hess_scale carries the objective multiplier."""
    c = AUG_CASES[k]
    vals = ipm_oracle.assemble_augmented(c["reg_size"], 1.0, c["hess"], c["jac"], c["x"], c["lb"], c["ub"], c["zl"], c["zu"])
    np.testing.assert_array_equal(vals, c["values"])
    np.testing.assert_array_equal(c["sigma"] * c["hess"], c["hess_sigma"])
    var, sig = ipm_oracle.barrier_diagonal_vec(c["x"], c["lb"], c["ub"], c["zl"], c["zu"])
    np.testing.assert_array_equal(sig, ipm_oracle.barrier_diagonal(c["x"], c["lb"], c["ub"], c["zl"], c["zu"])[1])


def test_reference_augmented_pattern_is_the_bench_layout():
    """The bench / parity generator (uno_amd/csrc/arrowband.c) lays its COO out exactly as the reference assembles
    the arrowband model's KKT (equality case): same (row, col) sequence, entry for entry."""
    import uno_amd
    c = next(c for c in AUG_CASES if c["model"] == "arrowband")
    n, nv, m, r, cc, _, _ = uno_amd.arrowband(c["N"], uno_amd.SEEDS["C2"])
    assert (n, nv, m) == (c["n"] + c["m"], c["n"], c["m"])
    np.testing.assert_array_equal(r, c["rows"])
    np.testing.assert_array_equal(cc, c["cols"])


@pytest.mark.gpu
@pytest.mark.parametrize("k", range(len(AUG_CASES)))
def test_device_assembly_reproduces_reference_augmented_matrix(k):
    """uno_kkt_assemble_augmented (device iterate, multipliers and model terms) writes the reference's
    augmented COO values bit for bit -- every segment: regularization zeros, sigma * H (the objective multiplier
    applied on the device), Sigma, J -- then factors them on the device with the same inertia as the host copy."""
    import torch
    import uno_amd
    c = AUG_CASES[k]
    n, m, N = c["n"], c["m"], c["n"] + c["m"]
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).cuda()
    g = uno_amd.HipKKT(0)
    g.analyze(N, c["rows"], c["cols"])
    assert g.barrier_setup(c["lb"], c["ub"]) == n
    g.augmented_setup(c["reg_size"], len(c["hess"]), len(c["jac"]))
    with pytest.raises(RuntimeError):
        g.augmented_setup(c["reg_size"], len(c["hess"]) + 1, len(c["jac"]))  # layout != analysed nnz
    g.augmented_setup(c["reg_size"], len(c["hess"]), len(c["jac"]))
    H, J, X, ZL, ZU = d(c["hess"]), d(c["jac"]), d(c["x"]), d(c["zl"]), d(c["zu"])
    vals = torch.full((len(c["values"]),), np.nan, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    g.assemble_augmented(1.0, H.data_ptr(), J.data_ptr(), X.data_ptr(), ZL.data_ptr(), ZU.data_ptr(), vals.data_ptr())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(vals.cpu().numpy(), c["values"])
    g.assemble_augmented(c["sigma"], H.data_ptr(), J.data_ptr(), X.data_ptr(), ZL.data_ptr(), ZU.data_ptr(), vals.data_ptr())
    torch.cuda.synchronize()
    out = vals.cpu().numpy()
    lo = c["reg_size"]
    np.testing.assert_array_equal(out[lo:lo + len(c["hess"])], c["hess_sigma"])
    g.assemble_augmented(1.0, H.data_ptr(), J.data_ptr(), X.data_ptr(), ZL.data_ptr(), ZU.data_ptr(), vals.data_ptr())
    g.factorize(device_ptr=vals.data_ptr())
    host = uno_amd.HipKKT(0)
    host.analyze(N, c["rows"], c["cols"])
    host.factorize(c["values"])
    assert g.inertia() == host.inertia()


@pytest.mark.gpu
def test_device_assembly_full_size_c3():
    """configs[2] size (KKT dimension 1e6, 2e7 values): the device assembly equals the oracle restatement bit for
    bit on the arrowband layout (Hessian band and Jacobian from the C3 generator, a random interior iterate with
    the late-IPM multiplier spread)."""
    import torch
    import uno_amd
    N = 1_000_000
    n, nv, m, r, cc, v, _ = uno_amd.arrowband(N, uno_amd.SEEDS["C3"])
    nh = sum(min(j, 12) + 1 for j in range(nv))
    hess, jac = v[n:n + nh], v[n + nh + nv:]
    rng = np.random.default_rng(3)
    lb, ub = np.full(nv, -10.0000001), np.full(nv, 10.0000001)
    x = rng.uniform(-9.9, 9.9, nv)
    zl = 10.0 ** rng.uniform(-8, 8, nv)
    zu = -(10.0 ** rng.uniform(-8, 8, nv))
    g = uno_amd.HipKKT(0)
    g.analyze(n, r, cc)
    assert g.barrier_setup(lb, ub) == nv
    g.augmented_setup(n, nh, len(jac))
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).cuda()
    H, J, X, ZL, ZU = d(hess), d(jac), d(x), d(zl), d(zu)
    vals = torch.empty(len(v), dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    g.assemble_augmented(1.0, H.data_ptr(), J.data_ptr(), X.data_ptr(), ZL.data_ptr(), ZU.data_ptr(), vals.data_ptr())
    torch.cuda.synchronize()
    ref = ipm_oracle.assemble_augmented(n, 1.0, hess, jac, x, lb, ub, zl, zu)
    got = vals.cpu().numpy()
    assert got.view(np.uint64).tobytes() == ref.view(np.uint64).tobytes()
