/*
 * kkt_oracle.h -- TEST INFRASTRUCTURE ONLY (the parity checker, never the product).
 *
 * CPU restatement of the symmetric-indefinite factor/solve/inertia semantics that Uno obtains from
 * MUMPS 5.8.0 through uno/ingredients/subproblem_solvers/MUMPS/MUMPSSolver.cpp (reference snapshot
 * 2025-08-08).  MUMPS itself is a third-party dependency that is not vendored in /root/reference
 * (pinned as MUMPS_static_jll 5.8.0 in .github/julia/build_tarballs_release.jl:13) and is not
 * installable offline, so its published algorithm is restated here:
 *
 *   - sym=2 (general symmetric), LDL^T with 1x1 and 2x2 pivots     MUMPSSolver.cpp:17
 *   - threshold partial pivoting, u = CNTL(1) = 0.01 (MUMPS default for sym=2), delayed pivots
 *     passed to the parent front when no pivot of the fully-summed block passes the test
 *   - ICNTL(8)=8 iterative row/column scaling before every factorization  MUMPSSolver.cpp:82
 *     (restated as SCALE_ITERS sweeps of symmetric infinity-norm equilibration)
 *   - ICNTL(24)=1 null-pivot-row detection with CNTL(3)=0 => thres = eps*1e-5*||A_pre||_inf
 *     (MUMPSSolver.cpp:36); a null pivot counts in INFOG(28) and contributes 0 to the solution
 *   - inertia: INFOG(12) negatives, INFOG(28) zeros, positives = n - neg - zero
 *     (MUMPSSolver.cpp:124-139)
 *   - solve: nrhs = 1, rhs copied into result (MUMPSSolver.cpp:91-96)
 *
 * Input contract: 0-based COO (row, col) pairs, either triangle, duplicates summed
 * (MUMPS sym=2 semantics), the pattern fixed between analysis and every factorization.
 *
 * The ordering here is deliberately different from the GPU product's (reverse Cuthill-McKee with
 * dense nodes last, versus the product's nested dissection), so agreement of inertia and solution is
 * evidence about the factorization, not about shared code.
 */
#ifndef UNO_KKT_ORACLE_H
#define UNO_KKT_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_kkt* oracle_kkt_t;

oracle_kkt_t oracle_kkt_create(void);
void oracle_kkt_destroy(oracle_kkt_t h);
/* options: "pivot_threshold" (u, default 0.01), "scale_iters" (default 3), "null_tol_factor" (1e-5) */
int oracle_kkt_set_option(oracle_kkt_t h, const char* name, double value);
int oracle_kkt_analyze(oracle_kkt_t h, int64_t n, int64_t nnz, const int64_t* row, const int64_t* col);
int oracle_kkt_factorize(oracle_kkt_t h, const double* values);
int oracle_kkt_inertia(oracle_kkt_t h, int64_t* pos, int64_t* neg, int64_t* zero);
int oracle_kkt_solve(oracle_kkt_t h, const double* rhs, double* x);
/* counters: [0] nnz_L, [1] supernodes, [2] 2x2 pivots, [3] delayed pivots, [4] null pivots,
 *           [5] factor flops, [6] max front order */
int oracle_kkt_stats(oracle_kkt_t h, double* out7);
/* equilibration of the last factorization: scaling by original index, null-pivot threshold */
int oracle_kkt_scaling(oracle_kkt_t h, double* scale, double* thres);
const char* oracle_kkt_last_error(oracle_kkt_t h);

#ifdef __cplusplus
}
#endif
#endif
