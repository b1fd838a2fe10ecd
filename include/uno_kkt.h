/*
 * uno_kkt.h -- C ABI of the MI355X-native sparse symmetric-indefinite KKT backend.
 *
 * Drop-in boundary for Uno's linear-solver plugin surface (reference snapshot 2025-08-08):
 *   uno/ingredients/subproblem_solvers/DirectSymmetricIndefiniteLinearSolver.hpp:11-25
 *   uno/ingredients/subproblem_solvers/SymmetricIndefiniteLinearSolver.hpp:20-33
 * The entry points below are exactly what the MUMPS adapter binds today
 * (uno/ingredients/subproblem_solvers/MUMPS/MUMPSSolver.cpp); each one names the call it replaces.
 * The C++ adapter that implements the Uno class on top of this ABI is in integration/ and
 * INTEGRATION.md.  Plain pointers and sizes only; no torch or HIP types cross this boundary.
 *
 * Matrix contract: 0-based COO (row, col, value) triplets, either triangle, duplicates
 * summed (MUMPS sym=2); the pattern is fixed between uno_kkt_analyze and every later factorization,
 * only values change.  All arithmetic is IEEE binary64.
 */
#ifndef UNO_KKT_H
#define UNO_KKT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes */
#define UNO_KKT_OK 0
#define UNO_KKT_ERR_ARG (-1)      /* bad argument (size, index out of range, unknown option) */
#define UNO_KKT_ERR_STATE (-2)    /* call out of order (factorize before analyze, ...) */
#define UNO_KKT_ERR_HIP (-3)      /* HIP runtime error (message in uno_kkt_last_error) */
#define UNO_KKT_ERR_PIVOT (-4)    /* a fully-summed column admits no pivot in its front */
#define UNO_KKT_ERR_NOMEM (-5)    /* device allocation failed */
#define UNO_KKT_ERR_NODEVICE (-6) /* no HIP device / extension not usable */

typedef struct uno_kkt* uno_kkt_t;

typedef struct {
    int64_t n;              /* KKT dimension */
    int64_t nnz;            /* COO entries (with duplicates) */
    int64_t nnz_unique;     /* canonical lower-triangle entries */
    int64_t nnz_L;          /* strictly-lower nonzeros of L as stored by the fronts (unpadded) */
    int64_t n_fronts;       /* supernodes / frontal matrices */
    int64_t n_levels;       /* assembly-tree levels (launch waves) */
    int64_t max_front;      /* largest front order */
    int64_t n_dense;        /* dense (arrow) nodes ordered last */
    int64_t pivots_2x2;     /* last factorization */
    int64_t pivots_null;    /* last factorization: null pivots (= zero eigenvalues) */
    int64_t pivots_relaxed; /* last factorization: pivots accepted below the threshold u */
    int64_t factorizations; /* counters since analysis */
    int64_t solves;
    double flops;           /* factorization flops (sum over fronts) */
    double analysis_seconds;/* host wall time of the last uno_kkt_analyze */
    double bytes_L;         /* 8 * stored factor entries (L + D) */
    double bytes_cb;        /* 8 * contribution-block entries written per factorization */
    int64_t fronts_merged;  /* fronts amalgamated into their parent since analysis (delayed pivots) */
    int64_t solve_grid;     /* dataflow solve: resident one-wave blocks per direction (0 = level-scheduled) */
    int64_t solve_aborts;   /* dataflow solves abandoned at the dependency-wait limit (then level-scheduled) */
    int64_t factor_df_fronts; /* fronts factored by the one-launch dataflow kernel (upper tree; 0 = none) */
    int64_t factor_df_aborts; /* dataflow factorizations redone level by level after a wait limit */
    int64_t refinements;    /* refinement steps applied since analysis (option "refine") */
    int64_t refinements_skipped; /* refinement steps skipped: componentwise backward error <= "refine_tol" */
    double last_backward_error;  /* componentwise backward error max_i |b - A x|_i / (|A| |x| + |b|)_i of the last
                                    checked solve (before its refinement step; -1 = not checked) */
} uno_kkt_stats_t;

/* Create a solver bound to HIP device `device_id`.  Replaces MUMPS JOB=-1 (MUMPSSolver.cpp:16-37). */
int uno_kkt_create(uno_kkt_t* handle, int device_id);

/* Release all host and device memory.  Replaces MUMPS JOB=-2 (MUMPSSolver.cpp:46-49). */
void uno_kkt_destroy(uno_kkt_t handle);

/* Options: "pivot_threshold" (u, default 0.01 = MUMPS CNTL(1) for sym=2),
 * "null_tol_factor" (default 1e-5: thres = eps*1e-5*||A_pre||_inf, ICNTL(24)=1 with CNTL(3)=0),
 * "scale_iters" (default 3, ICNTL(8)=8 restated as symmetric
 * infinity-norm sweeps; the oracle uses the same default), "leaf_size" (ND leaf, default 32),
 * "max_block" (max supernode width, default 64), "wide_group" / "wide_block" (a separator or dense-row
 * group longer than wide_group = 128 columns is cut into supernodes of up to wide_block = 4096 columns,
 * factored as large fronts), "timing" (1 = per-kernel HIP event timing),
 * "dist_dataflow_solve" (distributed runs: -1 = auto, on with the RCCL transport (one GPU per rank);
 * 1 = each rank solves its own subtrees with the one-launch dataflow solve; 0 = level-scheduled),
 * "delay_relaxed" (default 1: a front whose fully-summed block has no pivot passing u is amalgamated
 * into its parent and refactored -- the delayed-pivot rule of MUMPS; 0 = accept relaxed pivots). */
int uno_kkt_set_option(uno_kkt_t handle, const char* name, double value);

/* Symbolic analysis on a COO pattern (0-based, any triangle, duplicates allowed).  Host pointers.
 * Replaces do_symbolic_analysis / JOB=1 (MUMPSSolver.cpp:72-83, save_sparsity_to_local_format :149-157). */
int uno_kkt_analyze(uno_kkt_t handle, int64_t n, int64_t nnz, const int64_t* row, const int64_t* col);

/* Numerical LDL^T factorization of the values in COO order (same order as the analysed pattern).
 * values_on_device = 0: host pointer (copied H2D), 1: device pointer, and values == NULL reuses the
 * device-resident values of the previous call (after uno_kkt_set_values / uno_kkt_fill_values).
 * Asynchronous for patterns whose fronts all fit the LDS kernels (m <= 128): the call returns once the work
 * is queued and uno_kkt_inertia / uno_kkt_solve synchronise.  A pattern with larger fronts blocks the host
 * inside this call while those fronts factor (their panel steps are driven from the host, one stream sync
 * per batch of steps).
 * Replaces do_numerical_factorization / JOB=2 (MUMPSSolver.cpp:85-89). */
int uno_kkt_factorize(uno_kkt_t handle, const double* values, int values_on_device);

/* Refactorization after a host-side edit of positions [first, first + count) only: `values` is the whole
 * host COO array of the previous host-pointer factorization, of which only that range is copied.  The
 * inertia-correction loop (PrimalDualRegularization.hpp:178-179, 210-211) rewrites only the regularization
 * diagonal, which COOFormat stores first (COOFormat.hpp:102-110), so each retry moves reg_size doubles
 * instead of nnz.  Options: "pin_host_values" (1: the host buffer is page-locked once with hipHostRegister,
 * so uploads are direct DMA; a registration is keyed by pointer and length, and the buffer must stay
 * allocated until the caller passes another buffer to uno_kkt_factorize, re-analyses or destroys the handle,
 * each of which unregisters it). */
int uno_kkt_factorize_update(uno_kkt_t handle, const double* values, int64_t first, int64_t count);

/* Staged upload while the caller assembles: copies host values [first, first + count) of
 * the COO array (analysed order) to the solver's device copy on an upload stream, asynchronously, so
 * PCIe transfers overlap the caller's assembly of the later entries; the next uno_kkt_factorize(h, NULL, 0)
 * waits for every staged chunk on the device (no host sync) and factors the device copy.  Chunks of one
 * set of values may come in any order and may be re-staged (e.g. the regularization diagonal after
 * COOFormat::set_regularization).  The host buffer stays valid until that factorization has been queried
 * (uno_kkt_inertia); with option "pin_host_values" it is page-locked like uno_kkt_factorize's.  One-GPU
 * handles.  Used by the plugin's StagedCOOMatrix (integration/StagedCOOMatrix.hpp); it replaces the whole
 * upload at the start of MUMPS JOB=2 (MUMPSSolver.cpp:85-89). */
int uno_kkt_stage_values(uno_kkt_t handle, const double* values, int64_t first, int64_t count);

/* Device-side value edits between factorizations (the inertia-correction loop changes only the
 * regularization diagonal: COOFormat::set_regularization, COOFormat.hpp:102-110). */
int uno_kkt_set_values(uno_kkt_t handle, const int64_t* positions, const double* values, int64_t count);
int uno_kkt_fill_values(uno_kkt_t handle, int64_t first_position, int64_t count, double value);

/* Inertia of the last factorization.  Replaces get_inertia / INFOG(12) / INFOG(28)
 * (MUMPSSolver.cpp:124-139).  Singular <=> zero > 0 (:141-143); rank = n - zero (:145-147). */
int uno_kkt_inertia(uno_kkt_t handle, int64_t* positive, int64_t* negative, int64_t* zero);

/* Solve K x = rhs with the last factorization (nrhs = 1).  on_device = 0: host pointers, 1: device
 * pointers.  rhs and x may alias.  Replaces solve_indefinite_system / JOB=3 (MUMPSSolver.cpp:91-96). */
int uno_kkt_solve(uno_kkt_t handle, const double* rhs, double* x, int on_device);

/* Counters of the last analysis / factorization. */
int uno_kkt_stats(uno_kkt_t handle, uno_kkt_stats_t* stats);

/* Per-kernel-class device time accumulated while option "timing" is 1 (HIP events on the solver's
 * stream).  names: comma-separated list written into `names` (size `cap`), ms/launches per class. */
int uno_kkt_kernel_times(uno_kkt_t handle, char* names, int cap, double* ms, int64_t* launches, int max_classes);
int uno_kkt_reset_kernel_times(uno_kkt_t handle);

/* The hipStream_t the solver launches on (as void*), for callers that time or overlap work. */
void* uno_kkt_stream(uno_kkt_t handle);

/* Human-readable description of the last error on this handle ("" if none). */
const char* uno_kkt_last_error(uno_kkt_t handle);

/* ---- Device-side vector work around the solve ----
 * For a caller whose iterate lives in HBM: all vector arguments are DEVICE pointers, work is queued
 * on the solver's stream (uno_kkt_stream).
 *
 * Augmented right-hand side, Subproblem::assemble_augmented_rhs (uno/ingredients/subproblem/Subproblem.cpp:80-99):
 *   rhs[i] = -grad[i] + sum_j y[j] * J[j][i]  (i < n_vars; terms of y[j] == 0 skipped, constraint-ascending
 *   order as the reference), rhs[n_vars + j] = -cons[j].  uno_kkt_rhs_setup takes the Jacobian pattern once
 *   (host arrays: entry e is d cons[jac_con[e]] / d x[jac_var[e]]); jac_values are in that entry order. */
int uno_kkt_rhs_setup(uno_kkt_t handle, int64_t n_vars, int64_t n_cons, int64_t nnz_jac, const int64_t* jac_con,
                      const int64_t* jac_var);
int uno_kkt_assemble_rhs(uno_kkt_t handle, const double* grad, const double* cons, const double* y,
                         const double* jac_values, double* rhs);

/* Barrier diagonal Sigma on the device, PrimalDualInteriorPointProblem::evaluate_lagrangian_hessian
 * (PrimalDualInteriorPointProblem.cpp:56-78): uno_kkt_barrier_setup takes the variable bounds once (HOST
 * arrays, +-inf = unbounded) and lists the variables with a finite bound in ascending order (the order Uno
 * inserts their diagonal terms); uno_kkt_assemble_barrier writes, for the t-th of them,
 * values[t] = 0 + zl[i] / (x[i] - lb[i]) [finite lb] + zu[i] / (x[i] - ub[i]) [finite ub] (DEVICE pointers;
 * `values` points at the first barrier entry of the COO value array).  uno_kkt_barrier_count: how many. */
int uno_kkt_barrier_setup(uno_kkt_t handle, int64_t n_vars, const double* lb, const double* ub);
int64_t uno_kkt_barrier_count(uno_kkt_t handle);
int uno_kkt_assemble_barrier(uno_kkt_t handle, const double* x, const double* zl, const double* zu, double* values);

/* Augmented (KKT) values on the device, Subproblem::assemble_augmented_matrix (uno/ingredients/subproblem/
 * Subproblem.cpp:57-70) with PrimalDualInteriorPointProblem::evaluate_lagrangian_hessian (:56-78) and COOFormat's
 * regularization-first layout (COOFormat.hpp:78-99): the whole COO value array in Uno's insertion order,
 *   values[0, reg_size)                             = 0 (the regularization diagonal after COOFormat::reset)
 *   values[reg_size + k], k < nnz_hess               = hess_scale * hess[k]: the model's Lagrangian Hessian terms in
 *                                                      its insertion order (upper triangle, column-major for an
 *                                                      AMPL-like model); hess_scale = the objective multiplier for a
 *                                                      model with linear constraints (Hessian sigma * H), else 1
 *   values[reg_size + nnz_hess + t], t < barrier_count = Sigma_t as uno_kkt_assemble_barrier
 *   values[reg_size + nnz_hess + barrier_count + e]  = jac[e]: Jacobian entries constraint-major (Subproblem.cpp:64-69)
 * bit-identical to the host assembly.  uno_kkt_augmented_setup (after uno_kkt_barrier_setup) fixes the segment
 * lengths, checked against the analysed nnz.  DEVICE pointers; queued on the solver's stream, so a following
 * uno_kkt_factorize(h, values, 1) sees them: with the iterate in HBM no value crosses PCIe. */
int uno_kkt_augmented_setup(uno_kkt_t handle, int64_t reg_size, int64_t nnz_hess, int64_t nnz_jac);
int uno_kkt_assemble_augmented(uno_kkt_t handle, double hess_scale, const double* hess, const double* jac, const double* x,
                               const double* zl, const double* zu, double* values);

/* Primal-dual direction, PrimalDualInteriorPointProblem::assemble_primal_dual_direction
 * (PrimalDualInteriorPointProblem.cpp:173-194) with compute_bound_dual_direction (:262-278) and the
 * fraction-to-boundary rules (:281-325), tau = max(tau_min, 1 - barrier_parameter): dx = sol[0:n],
 * dy = -sol[n:n+m], bound-dual directions for variables with finite lb / ub (+-inf = unbounded), then
 * dx, dy scaled by the primal step length and dzl, dzu by the dual one.  step_lengths (HOST, 2 doubles)
 * receives {primal, dual}. */
int uno_kkt_assemble_direction(uno_kkt_t handle, int64_t n_vars, int64_t n_cons, const double* solution,
                               const double* x, const double* lb, const double* ub, const double* zl, const double* zu,
                               double barrier_parameter, double tau_min, double* dx, double* dy, double* dzl,
                               double* dzu, double* step_lengths);

/* y += A x with the analysed pattern and the values of the last factorization / value edit,
 * SymmetricMatrix::product (uno/linear_algebra/SymmetricMatrix.hpp:100-109); vectors in original numbering.
 * uno_kkt_quadratic_product: x^T A y into *result (HOST), SymmetricMatrix::quadratic_product (:112-130).
 * One-GPU handles only. */
int uno_kkt_symv(uno_kkt_t handle, const double* x, double* y);
int uno_kkt_quadratic_product(uno_kkt_t handle, const double* x, const double* y, double* result);

/* ---- Multi-GPU: one factorization partitioned over the GPUs of a node ----
 * The assembly tree is cut into independent subtrees, one set per rank, factored without any
 * communication; the subtree roots' contribution blocks go to rank 0 (RCCL point-to-point over xGMI),
 * which factors the top of the tree.  Inertia counters are all-reduced, so every rank returns the
 * inertia of the whole matrix.  The solve hands the subtree roots' update vectors to rank 0 and
 * broadcasts the top rows of the solution back; with option "gather_solution" (default 1) rank 0
 * returns the complete x (MUMPS ICNTL(21) = 0), other ranks their own rows.  Every rank calls the same
 * sequence (analyze / factorize / inertia / solve) with the same pattern, values and rhs.
 * The reference has no multi-process path (MUMPS par = 1, MUMPSSolver.cpp:17); this is an extension.
 * Attach before uno_kkt_analyze. */
int uno_kkt_comm_unique_id(unsigned char id[128]);                                     /* rank 0, shared out of band */
int uno_kkt_attach_rccl(uno_kkt_t handle, const unsigned char id[128], int rank, int world);
/* In-process group (several handles in one process, one host thread each; e.g. several ranks on one GPU). */
typedef struct uno_kkt_group* uno_kkt_group_t;
int uno_kkt_group_create(uno_kkt_group_t* group, int world);
void uno_kkt_group_destroy(uno_kkt_group_t group);
int uno_kkt_attach_local(uno_kkt_t handle, uno_kkt_group_t group, int rank);

/* Host-staged transport: the caller's own exchange on HOST buffers (e.g. MPI, or torch.distributed over
 * gloo), for one process per rank where RCCL is not available (several ranks on one GPU).  Device data
 * is staged through page-locked buffers.  send / recv post an operation on a host buffer that stays
 * valid until the next group_end call, which completes every operation posted since the previous one
 * (the library calls group_end after each batch, and right after a send / recv outside a batch).
 * allreduce reduces `count` 8-byte elements in place (op 0: sum u64, 1: max u64, 2: max f64, 3: sum
 * f64), broadcast copies `bytes` from `root` in place; both block.  Callbacks return 0 on success. */
typedef struct {
    void* ctx;
    int (*send)(void* ctx, const void* buf, size_t bytes, int peer);
    int (*recv)(void* ctx, void* buf, size_t bytes, int peer);
    int (*group_end)(void* ctx);
    int (*allreduce)(void* ctx, void* buf, size_t count, int op);
    int (*broadcast)(void* ctx, void* buf, size_t bytes, int root);
} uno_kkt_host_comm_t;
int uno_kkt_attach_host(uno_kkt_t handle, const uno_kkt_host_comm_t* comm, int rank, int world);

typedef struct {
    int64_t rank, world;
    int64_t subtrees;      /* independent subtrees of the partition */
    int64_t top_fronts;    /* fronts above the cut (factored by rank 0) */
    int64_t my_fronts;     /* fronts in this rank's subtrees */
    int64_t own_rows;      /* rows eliminated in this rank's subtrees */
    int64_t top_rows;      /* rows eliminated in top fronts */
    double my_flops, top_flops;
    double est_imbalance;  /* max rank work / mean rank work (analysis estimate) */
    int64_t partitioned;   /* 1: the factorization is split over the ranks; 0: the partition was declined
                              (fewer subtrees than ranks, or est_efficiency below option "dist_min_efficiency",
                              default 0.5; option "dist_force" = 1 overrides): every rank factors and solves
                              the whole matrix itself (replicas, no collective), so every rank's x is complete */
    double est_efficiency; /* total work / (world * (max rank work + top work)), analysis cost model */
} uno_kkt_dist_info_t;
int uno_kkt_dist_info(uno_kkt_t handle, uno_kkt_dist_info_t* info);

/* Library version string. */
const char* uno_kkt_version(void);

#ifdef __cplusplus
}
#endif
#endif /* UNO_KKT_H */
