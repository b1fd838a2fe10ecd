"""Hand-built systems whose inertia hinges on the null-pivot threshold and on the equilibration.

MUMPSSolver.cpp:36,82 asks MUMPS for null-pivot detection (ICNTL(24)=1, CNTL(3)=0: a pivot column whose
magnitude is at most eps * 1e-5 * ||A_pre||_inf counts as a zero eigenvalue) on the matrix scaled by
ICNTL(8)=8.  SURVEY.md 8(c) showed that this classification changes Uno's iterate sequence, so the
product and the oracle must take the same decision at the threshold.  Every value below is a power of
two or 1 - k*eps, so the scaled matrix is exact in binary64 and the decision does not depend on the
elimination order: only on ||A_pre||_inf, i.e. on the scaling.

null_threshold_case(N, ks, block_scale)
  * a hub (dense row, ordered last by both orderings) joined to N spokes: spoke diagonal 2^-16, hub
    entry 2^-8, hub diagonal 1.  Symmetric infinity-norm sweeps rescale the spokes by 2^4, 2^2, 2^1, so
    the scaled hub entries are 2^-4 after one sweep and 2^-1 after three: ||A_pre||_inf = 1 + N/2 with
    the 3 sweeps of the oracle (1 + N/16 with one sweep).
  * independent 2x2 blocks b*[[4, 4], [4, 4 - 4k eps]] (b = block_scale^2, a power of 4): scaled to
    [[1, 1], [1, 1 - k eps]] whatever b, whose second pivot is -k eps (either elimination order).  It is a
    null pivot iff k <= 1e-5 * ||A_pre||_inf.
"""
import numpy as np

EPS = np.finfo(np.float64).eps


def null_threshold_case(N, ks, block_scale=1.0, sweeps=3):
    """COO (rows, cols, vals) in Uno's layout plus the inertia MUMPS semantics give, and the threshold
    factor k* = 1e-5 * ||A_pre||_inf (k <= k* -> zero eigenvalue)."""
    n = 1 + N + 2 * len(ks)
    rows, cols, vals = [], [], []
    # hub 0, spokes 1..N
    rows.append(0); cols.append(0); vals.append(1.0)
    sp = np.arange(1, N + 1)
    rows += list(sp); cols += list(sp); vals += [2.0 ** -16] * N
    rows += list(sp); cols += [0] * N; vals += [2.0 ** -8] * N
    b = float(block_scale) ** 2
    for t, k in enumerate(ks):
        a = 1 + N + 2 * t
        rows += [a, a + 1, a + 1]
        cols += [a, a, a + 1]
        vals += [4.0 * b, 4.0 * b, (4.0 - 4.0 * k * EPS) * b]
    off = {1: 2.0 ** -4, 2: 2.0 ** -2, 3: 2.0 ** -1}[sweeps]
    anorm = max(1.0 + N * off, 2.0)
    kstar = 1e-5 * anorm
    nnull = sum(1 for k in ks if k * EPS <= EPS * kstar)
    inertia = (N + len(ks), 1 + len(ks) - nnull, nnull)
    return n, np.array(rows, np.int64), np.array(cols, np.int64), np.array(vals), inertia, kstar


def delay_case(N, eps_exp, d_hub=3.0, seed=0):
    """Fronts whose ONLY admissible pivots fail the threshold u = 0.01 (MUMPS CNTL(1), sym = 2): a hub (dense
    row: ordered last by both orderings, so it is never fully summed in a leaf front) joined with entries 1 to
    N spokes whose diagonals are +-10^e (e in eps_exp, cycled; signs random).  A leaf front's fully-summed
    block is then diagonal with |a_ii| = 10^e < u * 1 and has no off-diagonal for a 2x2 pivot, so MUMPS delays
    every column to the parent (the oracle does); delay_relaxed = 0 instead accepts them at a relaxed
    threshold (growth up to 10^-e).  Every spoke row has maximum 1 (its hub entry), so the equilibration
    leaves |a_ii| = 10^e below u; the inertia is analytic: Sylvester on [[D, e], [e^T, d]] gives inertia(D)
    plus the sign of the Schur complement d - sum 1/d_i, kept away from 0 (N must exceed 10 sqrt(N + 1),
    the dense-row cut of the analysis)."""
    rng = np.random.default_rng(seed)
    e = np.array([eps_exp[i % len(eps_exp)] for i in range(N)], dtype=float)
    d = rng.choice([-1.0, 1.0], N) * 10.0 ** e
    schur = d_hub - np.sum(1.0 / d)
    if abs(schur) < 1.0:  # keep the decision away from rounding
        d_hub += 10.0 * np.sign(schur if schur != 0 else 1.0)
        schur = d_hub - np.sum(1.0 / d)
    n = N + 1
    rows = [N] + list(range(N)) + [N] * N
    cols = [N] + list(range(N)) + list(range(N))
    vals = [d_hub] + list(d) + [1.0] * N
    pos = int((d > 0).sum()) + (1 if schur > 0 else 0)
    inertia = (pos, n - pos, 0)
    return n, np.array(rows, np.int64), np.array(cols, np.int64), np.array(vals), inertia
