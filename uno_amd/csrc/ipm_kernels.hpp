// ipm_kernels.hpp -- device vector kernels around the KKT solve (ipm_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace ukkt {

struct DirArgs {
    int64_t n, m;
    const double* sol;  // KKT solution, n + m
    const double* x;    // current primals
    const double* lb;   // variable bounds (+-inf = unbounded)
    const double* ub;
    const double* zl;   // bound multipliers
    const double* zu;
    double mu, tau;
    double* dx;
    double* dy;
    double* dzl;
    double* dzu;
    unsigned long long* alpha;  // [primal, dual] step length bits (device)
};

struct SymvArgs {
    int64_t n;
    const int32_t* perm;
    const int32_t* cptr;
    const int32_t* rptr;
    const int32_t* rslot;
    const int32_t* ent_r;
    const int32_t* ent_c;
    const double* uval;
    const double* x;      // by original index
    double* y;            // y += A x, by original index
    const double* dot_w;  // optional: w^T A x partials (quadratic_product), by original index
    double* dot_part;     // per row (new numbering)
    // rows with more than long_len entries (the dense "arrow" rows: 2.5e5 entries each at C3), reduced by
    // chunks of kSymvChunk over a 2-D grid instead of 16 lanes (14 ms -> microseconds)
    int64_t long_len = INT64_MAX;
    const int32_t* long_rows = nullptr;  // new numbering
    int32_t n_long = 0, long_chunks = 0;
    double* long_part = nullptr;         // n_long * long_chunks chunk partials (summed in chunk order)
    int absval = 0;                      // y += |A| |x| (the denominator of the componentwise backward error)
};
constexpr int kSymvChunk = 4096;
constexpr int kSumParts = 1024;  // quadratic_product: block partials of the deterministic two-pass sum

// Subproblem::assemble_augmented_matrix on the device (ipm_kernels.hip k_assemble_augmented)
struct AugArgs {
    int64_t reg, nh, nb, nj;    // segment lengths: regularization diagonal, Hessian terms, barrier terms, Jacobian
    double hscale;              // objective multiplier applied to the Hessian terms
    const double* hess;         // nh Hessian terms (the model's insertion order)
    const double* jac;          // nj Jacobian entries (constraint-major)
    const int32_t* bvar;        // barrier: bounded variables (ascending), nb
    const int8_t* bwhich;       //          1: finite lower, 2: finite upper bound
    const double* lb;
    const double* ub;
    const double* x;
    const double* zl;
    const double* zu;
    double* values;             // reg + nh + nb + nj COO values
};
hipError_t launch_assemble_augmented(const AugArgs& A, hipStream_t s);

// variables with more than long_len entries (long_vars, n_long of them) are summed by k_rhs_long (same order)
hipError_t launch_rhs(const double* grad, const double* cons, const double* y, const double* jval, const int64_t* vptr,
                      const int32_t* vent, const int32_t* jcon, int64_t n, int64_t m, double* rhs, hipStream_t s,
                      const int32_t* long_vars, int32_t n_long, int64_t long_len);
constexpr int64_t kRhsLong = 1024;
hipError_t launch_direction(const DirArgs& A, hipStream_t s);
hipError_t launch_barrier(const int32_t* var, const int8_t* which, const double* lb, const double* ub, const double* x,
                          const double* zl, const double* zu, int64_t count, double* values, hipStream_t s);
// dot_out (only with A.dot_w): 1 + kSumParts doubles, the result first
// out_bits[0] = bits of max_i |r_i| / (t_i + |b_i|) (0 where the denominator is 0 and r_i = 0, +inf where only
// the denominator is 0): the componentwise backward error of x with r = A x - b, t = |A| |x|
hipError_t launch_backward_error(const double* r, const double* t, const double* b, int64_t n, unsigned long long* out_bits,
                                 hipStream_t s);
hipError_t launch_symv(const SymvArgs& A, double* dot_out, hipStream_t s);

}  // namespace ukkt
