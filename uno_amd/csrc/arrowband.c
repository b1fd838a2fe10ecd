/*
 * arrowband.c -- synthetic "arrowband" interior-point KKT generator.
 *
 * The reference ships no large KKT inputs, so the benchmark configurations C2/C3/C5 are defined
 * here.  The COO layout is exactly the one Uno's ipopt path hands to its linear solver
 * (Subproblem::assemble_augmented_matrix, uno/ingredients/subproblem/Subproblem.cpp:57-70, with the
 * regularization diagonal first as in COOFormat::initialize_regularization, COOFormat.hpp:120-125):
 *   [reg diag (0..N-1, value 0)] ++ [Hessian upper triangle, column-major, band half-width 12]
 *   ++ [barrier diagonal Sigma, every variable bounded] ++ [J^T entries (var, nv + j), row-major]
 * Variables nv = 3N/4, equality constraints m = N - nv.  Constraint j touches the 28 variables
 * starting at min(3j, nv - 34) plus the last 6 ("arrow") variables.  Values from splitmix64:
 *   H_ii ~ U[-1,3] (negative curvature -> inertia correction), H_ij ~ U[-0.5,0.5]/12,
 *   Sigma_ii = 10^U[-8,8], J entries +-U[0.5,1.5].
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

static uint64_t sm_next(uint64_t* s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
static double sm_unif(uint64_t* s) { return (double)(sm_next(s) >> 11) * (1.0 / 9007199254740992.0); }

#define AB_BAND 12
#define AB_WIN 28
#define AB_ARROW 6

/* sizes of the arrowband KKT of dimension N (N >= 64): returns nnz, writes nv and m */
int64_t arrowband_size(int64_t N, int64_t* nv_out, int64_t* m_out) {
    int64_t nv = (3 * N) / 4, m = N - nv;
    int64_t nh = 0;
    for (int64_t j = 0; j < nv; ++j) nh += (j < AB_BAND ? j : AB_BAND) + 1;
    if (nv_out) *nv_out = nv;
    if (m_out) *m_out = m;
    return N + nh + nv + m * (AB_WIN + AB_ARROW);
}

/* fill row/col/val (size nnz from arrowband_size); returns nnz or -1 if N too small */
int64_t arrowband_generate(int64_t N, uint64_t seed, int64_t* row, int64_t* col, double* val) {
    int64_t nv, m;
    int64_t nnz = arrowband_size(N, &nv, &m);
    if (nv < AB_WIN + AB_ARROW + 1 || m < 1) return -1;
    uint64_t s = seed;
    int64_t q = 0;
    for (int64_t i = 0; i < N; ++i) { row[q] = i; col[q] = i; val[q] = 0.0; ++q; }
    for (int64_t j = 0; j < nv; ++j) {
        int64_t i0 = j - AB_BAND < 0 ? 0 : j - AB_BAND;
        for (int64_t i = i0; i <= j; ++i) {
            double u = sm_unif(&s);
            row[q] = i; col[q] = j;
            val[q] = (i == j) ? -1.0 + 4.0 * u : (u - 0.5) / 12.0;
            ++q;
        }
    }
    for (int64_t v = 0; v < nv; ++v) {
        double u = sm_unif(&s);
        row[q] = v; col[q] = v; val[q] = pow(10.0, -8.0 + 16.0 * u);
        ++q;
    }
    for (int64_t j = 0; j < m; ++j) {
        int64_t start = 3 * j;
        if (start > nv - AB_ARROW - AB_WIN) start = nv - AB_ARROW - AB_WIN;
        for (int64_t t = 0; t < AB_WIN + AB_ARROW; ++t) {
            int64_t v = t < AB_WIN ? start + t : nv - AB_ARROW + (t - AB_WIN);
            double mag = 0.5 + sm_unif(&s);
            double sg = sm_unif(&s) < 0.5 ? -1.0 : 1.0;
            row[q] = v; col[q] = nv + j; val[q] = sg * mag;
            ++q;
        }
    }
    return q == nnz ? nnz : -1;
}

/* deterministic right-hand side U[-1,1] */
void arrowband_rhs(int64_t N, uint64_t seed, double* b) {
    uint64_t s = seed ^ 0xB0B0B0B0ULL;
    for (int64_t i = 0; i < N; ++i) b[i] = 2.0 * sm_unif(&s) - 1.0;
}

/* COO symmetric product y = K x (one triangle stored, duplicates summed): SymmetricMatrix::product,
 * uno/linear_algebra/SymmetricMatrix.hpp:100-109 (used for residual checks). */
void coo_symv(int64_t n, int64_t nnz, const int64_t* row, const int64_t* col, const double* val, const double* x,
              double* y) {
    memset(y, 0, sizeof(double) * (size_t)n);
    for (int64_t k = 0; k < nnz; ++k) {
        y[row[k]] += val[k] * x[col[k]];
        if (row[k] != col[k]) y[col[k]] += val[k] * x[row[k]];
    }
}
