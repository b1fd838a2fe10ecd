"""CPU oracle (test infrastructure only) for the device-side vector work around the KKT solve,
restating the reference loops in the same floating-point order:

- barrier_diagonal         PrimalDualInteriorPointProblem.cpp:56-78 (Sigma)
- assemble_augmented       uno/ingredients/subproblem/Subproblem.cpp:57-70 after COOFormat::reset (COOFormat.hpp:78-89):
                           the whole augmented COO value array in Uno's insertion order
- assemble_augmented_rhs   uno/ingredients/subproblem/Subproblem.cpp:80-99
- assemble_direction       uno/ingredients/inequality_handling_methods/interior_point_methods/
                           PrimalDualInteriorPointProblem.cpp:173-194 (assemble_primal_dual_direction),
                           :262-278 (compute_bound_dual_direction), :281-325 (fraction-to-boundary)
- symv / quadratic_product uno/linear_algebra/SymmetricMatrix.hpp:100-130 (COO order)

Pinned to the reference itself: tests/golden/ipm_reference_vectors.json and augmented_reference_vectors.json hold the outputs of those very
reference functions (compiled from /root/reference, tests/golden/make_ipm_fixtures.sh) on seeded inputs, and
tests/test_ipm_vectors.py requires this restatement to reproduce them bit for bit.

Only tests/ may import this module; the product path is uno_amd/csrc/ipm_kernels.hip.
"""
import numpy as np


def barrier_diagonal(x, lb, ub, zl, zu):
    """(variables, Sigma): for every variable with a finite bound, ascending, 0 + zl/(x - lb) [finite lb]
    + zu/(x - ub) [finite ub] (PrimalDualInteriorPointProblem.cpp:62-77, the order Uno inserts them)."""
    var, sig = [], []
    for i in range(len(x)):
        fl, fu = np.isfinite(lb[i]), np.isfinite(ub[i])
        if fl or fu:
            d = 0.0
            if fl:
                d += zl[i] / (x[i] - lb[i])
            if fu:
                d += zu[i] / (x[i] - ub[i])
            var.append(i)
            sig.append(d)
    return np.array(var, dtype=np.int64), np.array(sig)


def assemble_augmented(reg_size, hess_scale, hess, jac, x, lb, ub, zl, zu):
    """[0] * reg_size (the regularization diagonal COOFormat::reset re-inserts) ++ hess_scale * hess (the model's
    Lagrangian Hessian terms, its insertion order; ArrowbandModel inserts sigma * H) ++ Sigma (barrier_diagonal)
    ++ jac (constraint-major, Subproblem.cpp:64-69).  Elementwise IEEE products, so numpy's vector multiply is the
    scalar loop's result."""
    _, sig = barrier_diagonal(x, lb, ub, zl, zu)
    return np.concatenate([np.zeros(int(reg_size)), float(hess_scale) * np.asarray(hess, dtype=np.float64), sig,
                           np.asarray(jac, dtype=np.float64)])


def barrier_diagonal_vec(x, lb, ub, zl, zu):
    """barrier_diagonal for large inputs (same operations, vectorised: 0 + a + b with the absent terms skipped)."""
    x, lb, ub, zl, zu = (np.asarray(a, dtype=np.float64) for a in (x, lb, ub, zl, zu))
    fl, fu = np.isfinite(lb), np.isfinite(ub)
    with np.errstate(all="ignore"):
        a = np.where(fl, zl / (x - lb), 0.0)
        b = np.where(fu, zu / (x - ub), 0.0)
    d = np.where(fl, 0.0 + a, 0.0)
    d = np.where(fu, d + b, d)
    keep = fl | fu
    return np.nonzero(keep)[0], d[keep]


def assemble_augmented_rhs(grad, cons, y, jac_con, jac_var, jac_val):
    """rhs = -grad; for each constraint j (ascending), for its Jacobian entries (stored order):
    rhs[var] += y_j * d if y_j != 0; rhs[n + j] = -c_j (Subproblem.cpp:83-96).  np.add.at is
    unbuffered and applies repeated indices in array order, i.e. the reference's order."""
    grad = np.asarray(grad, dtype=np.float64)
    n, m = len(grad), len(cons)
    rhs = np.empty(n + m)
    rhs[:n] = -grad
    order = np.argsort(np.asarray(jac_con), kind="stable")          # constraint-major, stored order
    con = np.asarray(jac_con)[order]
    var = np.asarray(jac_var)[order]
    val = np.asarray(jac_val, dtype=np.float64)[order]
    yj = np.asarray(y, dtype=np.float64)[con]
    keep = yj != 0.0
    np.add.at(rhs, var[keep], yj[keep] * val[keep])
    rhs[n:] = -np.asarray(cons, dtype=np.float64)
    return rhs


def assemble_direction(sol, x, lb, ub, zl, zu, mu, tau_min):
    """dx, dy, dzl, dzu (scaled) and (primal, dual) step lengths, scalar loops as in the reference."""
    n, m = len(x), len(sol) - len(x)
    tau = max(tau_min, 1.0 - mu)
    dx = np.array(sol[:n], dtype=np.float64)
    dy = -np.array(sol[n:n + m], dtype=np.float64)
    dzl, dzu = np.zeros(n), np.zeros(n)
    for i in range(n):
        if np.isfinite(lb[i]):
            dist = x[i] - lb[i]
            dzl[i] = (mu - dx[i] * zl[i]) / dist - zl[i]
        if np.isfinite(ub[i]):
            dist = x[i] - ub[i]
            dzu[i] = (mu - dx[i] * zu[i]) / dist - zu[i]
    ap = 1.0
    for i in range(n):
        if np.isfinite(lb[i]) and dx[i] < 0.0:
            d = -tau * (x[i] - lb[i]) / dx[i]
            if 0.0 < d:
                ap = min(ap, d)
        if np.isfinite(ub[i]) and 0.0 < dx[i]:
            d = -tau * (x[i] - ub[i]) / dx[i]
            if 0.0 < d:
                ap = min(ap, d)
    ad = 1.0
    for i in range(n):
        if np.isfinite(lb[i]) and dzl[i] < 0.0:
            d = -tau * zl[i] / dzl[i]
            if 0.0 < d:
                ad = min(ad, d)
        if np.isfinite(ub[i]) and 0.0 < dzu[i]:
            d = -tau * zu[i] / dzu[i]
            if 0.0 < d:
                ad = min(ad, d)
    return dx * ap, dy * ap, dzl * ad, dzu * ad, (ap, ad)


def symv(n, rows, cols, vals, x):
    """SymmetricMatrix::product over COO entries in stored order (off-diagonals twice)."""
    y = np.zeros(n)
    for r, c, v in zip(rows, cols, vals):
        y[r] += v * x[c]
        if r != c:
            y[c] += v * x[r]
    return y


def quadratic_product(rows, cols, vals, x, y):
    res = 0.0
    for r, c, v in zip(rows, cols, vals):
        res += v * x[r] * y[r] if r == c else v * (x[r] * y[c] + x[c] * y[r])
    return res
