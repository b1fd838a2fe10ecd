// ipm_kernels.hip -- device-side vector work around the KKT solve of Uno's ipopt preset (SURVEY.md 8(a)
// rows A10, A11, A15), so an iterate that lives in HBM never round-trips to the host:
//   k_rhs_*      Subproblem::assemble_augmented_rhs            (uno/ingredients/subproblem/Subproblem.cpp:80-99)
//   k_direction  PrimalDualInteriorPointProblem::assemble_primal_dual_direction + compute_bound_dual_direction
//                + primal/dual_fraction_to_boundary  (PrimalDualInteriorPointProblem.cpp:173-194, 262-325)
//   k_symv       SymmetricMatrix::product / quadratic_product  (uno/linear_algebra/SymmetricMatrix.hpp:100-130)
// All HBM-bound streaming kernels: grid-stride loops, coalesced loads, no same-address atomics except one
// per workgroup for the step-length minima.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "ipm_kernels.hpp"

// no FMA contraction: the reference's host arithmetic (g++, x86-64 baseline) rounds every product and
// sum separately, and the right-hand side and the direction are compared bit for bit with it
#pragma clang fp contract(off)

namespace ukkt {

namespace {
constexpr int kT = 256;

int grid_of(int64_t n) {
    int64_t g = (n + kT - 1) / kT;
    return (int)(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}

__device__ __forceinline__ unsigned long long bits(double d) { return (unsigned long long)__double_as_longlong(d); }
}  // namespace

// rhs[i] = -g[i] + sum_{e in column i of J^T, ascending constraint} y[c_e] * d_e  (i < n)
// rhs[n + j] = -c[j].  The per-variable entry lists are sorted by constraint index, the order in which
// the reference accumulates (it loops constraints in order), so the sums are bit-identical; entries
// of constraints with y_j == 0 are skipped as in the reference (Subproblem.cpp:89).
__global__ void k_rhs(const double* __restrict__ grad, const double* __restrict__ cons, const double* __restrict__ y,
                      const double* __restrict__ jval, const int64_t* __restrict__ vptr, const int32_t* __restrict__ vent,
                      const int32_t* __restrict__ jcon, int64_t n, int64_t m, double* __restrict__ rhs, int64_t long_len) {
    for (int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x; i < n + m; i += (int64_t)gridDim.x * kT) {
        if (i < n) {
            if (vptr[i + 1] - vptr[i] > long_len) continue;  // k_rhs_long
            double r = -grad[i];
            for (int64_t q = vptr[i]; q < vptr[i + 1]; ++q) {
                const int32_t e = vent[q];
                const double yj = y[jcon[e]];
                if (yj != 0.0) r += yj * jval[e];
            }
            rhs[i] = r;
        } else {
            rhs[i] = -cons[i - n];
        }
    }
}

// Variables in more than long_len constraints (C3: six linking variables in all 250 000): one thread summing
// such a list one dependent gather after the other took 163 ms.  One wave per such variable now gathers 64
// entries at a time (the next 512 in flight), stages the products in LDS and lane 0 adds them in list order,
// so the sum is the reference's, bit for bit (gathers with a branch per entry, 64 or 256 per chunk: 5.7 / 6.2 ms
// for 250 000 entries, every gather a round trip of its own; a readlane per term: 15 ms).
__global__ __launch_bounds__(64) void k_rhs_long(const double* __restrict__ grad, const double* __restrict__ y,
                                                 const double* __restrict__ jval, const int64_t* __restrict__ vptr,
                                                 const int32_t* __restrict__ vent, const int32_t* __restrict__ jcon,
                                                 const int32_t* __restrict__ long_vars, double* __restrict__ rhs) {
    constexpr int U = 8;  // entries per lane and chunk: 512 per chunk
    const int lane = threadIdx.x;
    const int32_t i = long_vars[blockIdx.x];
    const int64_t q0 = vptr[i], q1 = vptr[i + 1];
    // y_c * d_e of the chunk's entries, branch-free (indices clamped into the list) so the U gathers of each
    // dependent step are in flight together; -0.0 where skipped (y_c = 0, or past the list): -0.0 is the exact
    // identity of the addition (x + -0.0 = x for every x, the sign of a zero sum included), so lane 0 adds
    // every slot
    auto chunk = [&](int64_t q, double (&t)[U]) {
        int32_t e[U], c[U];
        double yv[U], dv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) e[u] = vent[min(q + 64 * u + lane, q1 - 1)];
#pragma unroll
        for (int u = 0; u < U; ++u) c[u] = jcon[e[u]];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            yv[u] = y[c[u]];
            dv[u] = jval[e[u]];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) t[u] = (q + 64 * u + lane < q1 && yv[u] != 0.0) ? yv[u] * dv[u] : -0.0;
    };
    __shared__ double buf[64 * U];
    double r = -grad[i];
    double t[U];
    chunk(q0, t);
    for (int64_t q = q0; q < q1; q += 64 * U) {
#pragma unroll
        for (int u = 0; u < U; ++u) buf[64 * u + lane] = t[u];
        __syncthreads();
        if (q + 64 * U < q1) chunk(q + 64 * U, t);  // the next chunk's gathers under this chunk's sum
        if (lane == 0) {
#pragma unroll 64
            for (int l = 0; l < 64 * U; ++l) r += buf[l];  // list order
        }
        __syncthreads();
    }
    if (lane == 0) rhs[i] = r;
}

// direction + fraction-to-boundary step lengths; alpha[0] / alpha[1] hold the bit patterns of the
// primal / dual step lengths (positive doubles order like their bits: one atomicMin per workgroup)
__global__ void k_direction(DirArgs A) {
    __shared__ unsigned long long red[2][kT / 64];
    double ap = 1.0, ad = 1.0;
    const int64_t n = A.n;
    for (int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x; i < n + A.m; i += (int64_t)gridDim.x * kT) {
        if (i >= n) {  // constraint multipliers: dy = -solution (PrimalDualInteriorPointProblem.cpp:178)
            A.dy[i - n] = -A.sol[i];
            continue;
        }
        const double dx = A.sol[i];
        const double x = A.x[i];
        A.dx[i] = dx;
        double dzl = 0.0, dzu = 0.0;
        const double lb = A.lb[i], ub = A.ub[i];
        if (isfinite(lb)) {  // lower-bounded variable (:266-271, :285-291, :307-313)
            const double zl = A.zl[i];
            const double dist = x - lb;
            dzl = (A.mu - dx * zl) / dist - zl;
            if (dx < 0.0) {
                const double d = -A.tau * dist / dx;
                if (0.0 < d) ap = fmin(ap, d);
            }
            if (dzl < 0.0) {
                const double d = -A.tau * zl / dzl;
                if (0.0 < d) ad = fmin(ad, d);
            }
        }
        if (isfinite(ub)) {  // upper-bounded variable (:272-277, :292-299, :314-320)
            const double zu = A.zu[i];
            const double dist = x - ub;
            dzu = (A.mu - dx * zu) / dist - zu;
            if (0.0 < dx) {
                const double d = -A.tau * dist / dx;
                if (0.0 < d) ap = fmin(ap, d);
            }
            if (0.0 < dzu) {
                const double d = -A.tau * zu / dzu;
                if (0.0 < d) ad = fmin(ad, d);
            }
        }
        A.dzl[i] = dzl;
        A.dzu[i] = dzu;
    }
    unsigned long long bp = bits(ap), bd = bits(ad);
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long op = __shfl_xor(bp, off), od = __shfl_xor(bd, off);
        bp = op < bp ? op : bp;
        bd = od < bd ? od : bd;
    }
    if ((threadIdx.x & 63) == 0) { red[0][threadIdx.x >> 6] = bp; red[1][threadIdx.x >> 6] = bd; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kT / 64; ++w) {
            bp = red[0][w] < bp ? red[0][w] : bp;
            bd = red[1][w] < bd ? red[1][w] : bd;
        }
        atomicMin(A.alpha, bp);
        atomicMin(A.alpha + 1, bd);
    }
}

// scaling by the step lengths (PrimalDualInteriorPointProblem.cpp:190-193)
__global__ void k_direction_scale(DirArgs A) {
    const double ap = __longlong_as_double((long long)A.alpha[0]);
    const double ad = __longlong_as_double((long long)A.alpha[1]);
    for (int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x; i < A.n + A.m; i += (int64_t)gridDim.x * kT) {
        if (i < A.n) {
            A.dx[i] *= ap;
            A.dzl[i] *= ad;
            A.dzu[i] *= ad;
        } else {
            A.dy[i - A.n] *= ap;
        }
    }
}

// y += A x for the symmetric matrix held as unique lower-triangle slots, row by row (atomic-free):
// row i = its column part (slots cptr[i] .. cptr[i+1], partner = later row) + its row part (rslot)
__global__ void k_symv(SymvArgs A) {
    const int64_t g = ((int64_t)blockIdx.x * kT + threadIdx.x) / 16;
    const int lane = threadIdx.x & 15;
    if (g >= A.n) return;
    const int32_t i = (int32_t)g;
    if ((int64_t)(A.cptr[i + 1] - A.cptr[i]) + (A.rptr[i + 1] - A.rptr[i]) > A.long_len) return;  // k_symv_long
    const int32_t oi = A.perm[i];
    double acc = 0.0;
    if (A.absval) {
        for (int32_t q = A.cptr[i] + lane; q < A.cptr[i + 1]; q += 16) acc += fabs(A.uval[q]) * fabs(A.x[A.ent_r[q]]);
        for (int32_t t = A.rptr[i] + lane; t < A.rptr[i + 1]; t += 16) {
            const int32_t q = A.rslot[t];
            acc += fabs(A.uval[q]) * fabs(A.x[A.ent_c[q]]);
        }
    } else {
        for (int32_t q = A.cptr[i] + lane; q < A.cptr[i + 1]; q += 16) acc += A.uval[q] * A.x[A.ent_r[q]];
        for (int32_t t = A.rptr[i] + lane; t < A.rptr[i + 1]; t += 16) {
            const int32_t q = A.rslot[t];
            acc += A.uval[q] * A.x[A.ent_c[q]];
        }
    }
    for (int off = 8; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 16);
    if (lane == 0) {
        A.y[oi] += acc;
        if (A.dot_w) A.dot_part[i] = A.dot_w[oi] * acc;
    }
}

// long rows: block (chunk c, long row k) sums the row's entries [c, c + 1) * kSymvChunk (column part,
// then row part, as k_symv walks them) in a fixed tree order into long_part[k * long_chunks + c]
__global__ void k_symv_long(SymvArgs A) {
    __shared__ double red[kT / 64];
    const int k = blockIdx.y;
    const int32_t i = A.long_rows[k];
    const int32_t c0 = A.cptr[i], nc = A.cptr[i + 1] - c0;
    const int32_t r0 = A.rptr[i], len = nc + (A.rptr[i + 1] - r0);
    const int32_t b = blockIdx.x * kSymvChunk, e = min(len, b + kSymvChunk);
    double acc = 0.0;
    for (int32_t t = b + threadIdx.x; t < e; t += kT) {
        const int32_t q = t < nc ? c0 + t : A.rslot[r0 + (t - nc)];
        const double xv = A.x[t < nc ? A.ent_r[q] : A.ent_c[q]];
        acc += A.absval ? fabs(A.uval[q]) * fabs(xv) : A.uval[q] * xv;
    }
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        double s = red[0];
        for (int w = 1; w < kT / 64; ++w) s += red[w];
        A.long_part[(int64_t)k * A.long_chunks + blockIdx.x] = s;  // 0 for chunks past the row's end
    }
}

__global__ void k_symv_long_fin(SymvArgs A) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= A.n_long) return;
    const int32_t i = A.long_rows[k];
    const int32_t oi = A.perm[i];
    double acc = 0.0;
    for (int c = 0; c < A.long_chunks; ++c) acc += A.long_part[(int64_t)k * A.long_chunks + c];
    A.y[oi] += acc;
    if (A.dot_w) A.dot_part[i] = A.dot_w[oi] * acc;
}

// sum of per-row partials (quadratic_product), deterministic: pass 1 writes one block-sum per workgroup
// (fixed grid, fixed tree order inside the block), pass 2 (one block) sums them in block order
__global__ void k_sum(const double* __restrict__ v, int64_t n, double* __restrict__ part) {
    __shared__ double red[kT / 64];
    double s = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x; i < n; i += (int64_t)gridDim.x * kT) s += v[i];
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kT / 64; ++w) s += red[w];
        part[blockIdx.x] = s;
    }
}

__global__ void k_sum_fin(const double* __restrict__ part, int nparts, double* __restrict__ out) {
    __shared__ double red[kT / 64];
    double s = 0.0;
    for (int i = threadIdx.x; i < nparts; i += kT) s += part[i];
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kT / 64; ++w) s += red[w];
        *out = s;
    }
}

// Barrier diagonal, PrimalDualInteriorPointProblem::evaluate_lagrangian_hessian
// (PrimalDualInteriorPointProblem.cpp:56-78): for the t-th variable with a finite bound (ascending, the order
// Uno inserts them), Sigma = 0 + zl / (x - lb) [finite lb] + zu / (x - ub) [finite ub], written into the COO
// value array at values[first + t] -- the same operations in the same order as the host, so bit-identical.
__global__ void k_barrier(const int32_t* __restrict__ var, const int8_t* __restrict__ which, const double* __restrict__ lb,
                          const double* __restrict__ ub, const double* __restrict__ x, const double* __restrict__ zl,
                          const double* __restrict__ zu, int64_t count, double* __restrict__ values) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < count; t += (int64_t)gridDim.x * blockDim.x) {
        const int32_t i = var[t];
        const int8_t w = which[t];
        double d = 0.;
        if (w & 1) d += zl[i] / (x[i] - lb[i]);
        if (w & 2) d += zu[i] / (x[i] - ub[i]);
        values[t] = d;
    }
}

// The whole augmented (KKT) value array in Uno's insertion order, Subproblem::assemble_augmented_matrix
// (Subproblem.cpp:57-70) after COOFormat::reset (COOFormat.hpp:78-89, the regularization diagonal first, zeros):
//   [0, reg)                 0
//   [reg, reg + nh)          hscale * hess[k]      the Lagrangian Hessian terms as the model inserts them (for a
//                                                  model with linear constraints: sigma * H, ArrowbandModel.hpp)
//   [.., + nb)               Sigma_t               PrimalDualInteriorPointProblem.cpp:62-77 (k_barrier's arithmetic)
//   [.., + nj)               jac[e]                Subproblem.cpp:64-69, constraint-major
// One streaming pass (every value written once, coalesced; the segments meet in at most 3 waves), the same IEEE
// operations in the same order as the host code, so bit-identical to it.
__global__ void k_assemble_augmented(AugArgs A) {
    const int64_t e1 = A.reg, e2 = e1 + A.nh, e3 = e2 + A.nb, total = e3 + A.nj;
    for (int64_t q = (int64_t)blockIdx.x * kT + threadIdx.x; q < total; q += (int64_t)gridDim.x * kT) {
        double v;
        if (q < e1) {
            v = 0.0;
        } else if (q < e2) {
            v = A.hscale * A.hess[q - e1];
        } else if (q < e3) {
            const int64_t t = q - e2;
            const int32_t i = A.bvar[t];
            const int8_t w = A.bwhich[t];
            v = 0.;
            if (w & 1) v += A.zl[i] / (A.x[i] - A.lb[i]);
            if (w & 2) v += A.zu[i] / (A.x[i] - A.ub[i]);
        } else {
            v = A.jac[q - e3];
        }
        A.values[q] = v;
    }
}

hipError_t launch_assemble_augmented(const AugArgs& A, hipStream_t s) {
    const int64_t total = A.reg + A.nh + A.nb + A.nj;
    if (total <= 0) return hipSuccess;
    // grid-stride over at most 8192 blocks of 256 threads (32 blocks per CU)
    hipLaunchKernelGGL(k_assemble_augmented, dim3(grid_of(total)), dim3(kT), 0, s, A);
    return hipGetLastError();
}

hipError_t launch_barrier(const int32_t* var, const int8_t* which, const double* lb, const double* ub, const double* x,
                          const double* zl, const double* zu, int64_t count, double* values, hipStream_t s) {
    if (count <= 0) return hipSuccess;
    int64_t g = (count + 255) / 256;
    hipLaunchKernelGGL(k_barrier, dim3((unsigned)(g > 4096 ? 4096 : g)), dim3(256), 0, s, var, which, lb, ub, x, zl, zu,
                       count, values);
    return hipGetLastError();
}

hipError_t launch_rhs(const double* grad, const double* cons, const double* y, const double* jval, const int64_t* vptr,
                      const int32_t* vent, const int32_t* jcon, int64_t n, int64_t m, double* rhs, hipStream_t s,
                      const int32_t* long_vars, int32_t n_long, int64_t long_len) {
    if (n + m == 0) return hipSuccess;
    if (n_long == 0) long_len = INT64_MAX;
    hipLaunchKernelGGL(k_rhs, dim3(grid_of(n + m)), dim3(kT), 0, s, grad, cons, y, jval, vptr, vent, jcon, n, m, rhs, long_len);
    if (n_long > 0)
        hipLaunchKernelGGL(k_rhs_long, dim3((unsigned)n_long), dim3(64), 0, s, grad, y, jval, vptr, vent, jcon, long_vars, rhs);
    return hipGetLastError();
}

__global__ void k_alpha_init(unsigned long long* alpha) {
    if (threadIdx.x < 2) alpha[threadIdx.x] = 0x3ff0000000000000ull;  // 1.0
}

hipError_t launch_direction(const DirArgs& A, hipStream_t s) {
    hipLaunchKernelGGL(k_alpha_init, dim3(1), dim3(64), 0, s, A.alpha);
    if (A.n + A.m == 0) return hipGetLastError();
    hipLaunchKernelGGL(k_direction, dim3(grid_of(A.n + A.m)), dim3(kT), 0, s, A);
    hipLaunchKernelGGL(k_direction_scale, dim3(grid_of(A.n + A.m)), dim3(kT), 0, s, A);
    return hipGetLastError();
}

__global__ void k_backward_error(const double* __restrict__ r, const double* __restrict__ t, const double* __restrict__ b,
                                 int64_t n, unsigned long long* __restrict__ out_bits) {
    double mx = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x; i < n; i += (int64_t)gridDim.x * kT) {
        const double num = fabs(r[i]), den = t[i] + fabs(b[i]);
        double w = den > 0.0 ? num / den : (num > 0.0 ? INFINITY : 0.0);
        if (!(num <= INFINITY) || !(den <= INFINITY) || !(w <= INFINITY)) w = INFINITY;  // NaN in x, r or b (or
                                                                                          // inf / inf): forces the refinement step
        mx = fmax(mx, w);
    }
    for (int off = 32; off > 0; off >>= 1) mx = fmax(mx, __shfl_xor(mx, off));
    if ((threadIdx.x & 63) == 0 && mx > 0.0) atomicMax(out_bits, (unsigned long long)__double_as_longlong(mx));
}

hipError_t launch_backward_error(const double* r, const double* t, const double* b, int64_t n, unsigned long long* out_bits,
                                 hipStream_t s) {
    hipError_t e = hipMemsetAsync(out_bits, 0, sizeof(unsigned long long), s);
    if (e != hipSuccess || n == 0) return e;
    const int64_t g = grid_of(n);
    hipLaunchKernelGGL(k_backward_error, dim3((unsigned)(g > 1024 ? 1024 : g)), dim3(kT), 0, s, r, t, b, n, out_bits);
    return hipGetLastError();
}

hipError_t launch_symv(const SymvArgs& A, double* dot_out, hipStream_t s) {
    if (A.n == 0) return hipSuccess;
    const int64_t threads = A.n * 16;
    hipLaunchKernelGGL(k_symv, dim3((unsigned)((threads + kT - 1) / kT)), dim3(kT), 0, s, A);
    if (A.n_long > 0) {
        hipLaunchKernelGGL(k_symv_long, dim3((unsigned)A.long_chunks, (unsigned)A.n_long), dim3(kT), 0, s, A);
        hipLaunchKernelGGL(k_symv_long_fin, dim3((unsigned)((A.n_long + 63) / 64)), dim3(64), 0, s, A);
    }
    if (A.dot_w) {  // dot_out: 1 + kSumParts doubles (result, then the block partials)
        const int g = (int)(grid_of(A.n) > kSumParts ? kSumParts : grid_of(A.n));
        hipLaunchKernelGGL(k_sum, dim3(g), dim3(kT), 0, s, A.dot_part, A.n, dot_out + 1);
        hipLaunchKernelGGL(k_sum_fin, dim3(1), dim3(kT), 0, s, dot_out + 1, g, dot_out);
    }
    return hipGetLastError();
}

}  // namespace ukkt
