// kkt_kernels.hip -- hand-written CDNA4 (gfx950) kernels of the sparse KKT LDL^T backend.
//
// Numerical phase that Uno delegates to MUMPS JOB=2 / JOB=3
// (uno/ingredients/subproblem_solvers/MUMPS/MUMPSSolver.cpp:85-96):
//   k_pack          COO values -> packed per-front slots (duplicates summed, MUMPS sym=2), row maxima
//   k_scale*        symmetric infinity-norm equilibration (ICNTL(8)=8 restated), ||A_pre||_inf
//   k_factor_lds<MR> one workgroup per front: assemble + extend-add + threshold 1x1/2x2 LDL^T in LDS
//   k_big_*          blocked LDL^T of fronts too large for LDS (HBM scratch, MFMA f64 trailing updates)
//   k_solve_fwd / k_solve_bwd  level-scheduled multifrontal triangular solves (nrhs = 1)
// Every front is processed by one 256-thread workgroup (4 waves of 64); pivot search runs in wave 0
// with butterfly shuffles, the rank-1/rank-2 Schur updates are spread over a 16x16 thread grid.
#include <hip/hip_runtime.h>

#include <atomic>

#include <algorithm>
#include <cfloat>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <type_traits>
#include <utility>

#include "kkt_kernels.hpp"

namespace ukkt {

constexpr int kThreads = 256;
template <int NT> constexpr int kGrid = NT == 64 ? 8 : 16;  // side of the Schur-update thread grid

typedef double dbl4 __attribute__((ext_vector_type(4)));  // v_mfma_f64_16x16x4f64 accumulator

enum : int8_t { PIV_NULL = 0, PIV_1X1 = 1, PIV_2X2_A = 2, PIV_2X2_B = 3, PIV_STUCK = 4 };

__device__ __forceinline__ double as_double(unsigned long long b) { return __longlong_as_double((long long)b); }
__device__ __forceinline__ unsigned long long as_bits(double d) { return (unsigned long long)__double_as_longlong(d); }

// ------------------------------------------------------------------------------------------------
// pack + scaling
// ------------------------------------------------------------------------------------------------

// slot_src (duplicates present): the slot's single COO position, or < 0 for a slot with several, which
// k_pack_multi writes from its list (dup_ptr range summed in ascending COO position): the slots of one
// COO position take two dependent loads, and no wave waits for the duplicates' longer chain
__global__ void k_pack(const double* __restrict__ values, const int32_t* __restrict__ dup_ptr,
                       const int32_t* __restrict__ dup_pos, const int32_t* __restrict__ slot_src, int64_t begin,
                       int64_t end, double* __restrict__ uval) {
    for (int64_t s = begin + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < end; s += (int64_t)gridDim.x * blockDim.x) {
        if (dup_ptr == nullptr) {
            uval[s] = values[dup_pos[s]];
        } else if (slot_src != nullptr) {
            const int32_t src = slot_src[s];
            if (src >= 0) uval[s] = 0.0 + values[src];  // as the summed form: -0.0 packs as +0.0
        } else {
            double v = 0.0;  // duplicates summed in ascending COO position (oracle order)
            for (int32_t q = dup_ptr[s]; q < dup_ptr[s + 1]; ++q) v += values[dup_pos[q]];
            uval[s] = v;
        }
    }
}

// multi: per slot {slot, p0, p1, p2} (COO positions ascending, -1 padded) or {slot, -2 - q0, count, 0}
__global__ void k_pack_multi(const double* __restrict__ values, const int32_t* __restrict__ dup_ptr,
                             const int32_t* __restrict__ dup_pos, const int32_t* __restrict__ multi, int64_t count,
                             double* __restrict__ uval) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < count; t += (int64_t)gridDim.x * blockDim.x) {
        const int4 d = reinterpret_cast<const int4*>(multi)[t];
        double v = 0.0;  // duplicates summed in ascending COO position (oracle order)
        if (d.y >= -1) {
            const double a = values[d.y], b = d.z >= 0 ? values[d.z] : 0.0, c = d.w >= 0 ? values[d.w] : 0.0;
            v += a;
            if (d.z >= 0) v += b;
            if (d.w >= 0) v += c;
        } else {
            for (int32_t q = -2 - d.y; q < -2 - d.y + d.z; ++q) v += values[dup_pos[q]];
        }
        uval[d.x] = v;
    }
}

// |s_a v s_b| evaluated as (s_a * v) * s_b with a the larger original index: the oracle's expression
// (oracle/kkt_oracle.c, sv[u] = s[ur] * uval[u] * s[uc], ur > uc), so the scaling vectors and the scaled
// entries are bit-identical to the oracle's whatever the row a scan visits the entry from
__device__ __forceinline__ double scaled_abs(int32_t i, double si, int32_t j, double v, const double* __restrict__ scale) {
    const double sj = scale[j];
    return i > j ? fabs(si * v * sj) : fabs(sj * v * si);
}

// Row-wise scans of the packed matrix (new numbering), atomic-free:
//   MODE 0: rmax_i = max_j |a_ij|               (first equilibration sweep, s = 1)
//   MODE 1: rmax_i = max_j |s_i a_ij s_j|       (later sweeps)
//   MODE 2: rsum_i = sum_j |s_i a_ij s_j|, and max_i rsum_i -> anorm (||A_pre||_inf)
// LPR lanes cooperate on one row; long (dense, "arrow") rows use LPR = 256 via a row list.
template <int LPR, int MODE>
__device__ __forceinline__ void row_scan(int32_t i, int lane, const ScanArgs& A, double* red) {
    const int32_t orig = A.perm[i];
    const double si = MODE > 0 ? A.scale[orig] : 1.0;
    double acc = 0.0;
    for (int32_t q = A.cptr[i] + lane; q < A.cptr[i + 1]; q += LPR) {
        double w = MODE == 0 ? fabs(A.uval[q]) : scaled_abs(orig, si, A.ent_r[q], A.uval[q], A.scale);
        acc = MODE == 2 ? acc + w : fmax(acc, w);
    }
    for (int32_t t = A.rptr[i] + lane; t < A.rptr[i + 1]; t += LPR) {
        const int32_t q = A.rslot[t];
        double w = MODE == 0 ? fabs(A.uval[q]) : scaled_abs(orig, si, A.ent_c[q], A.uval[q], A.scale);
        acc = MODE == 2 ? acc + w : fmax(acc, w);
    }
    const int wl = LPR < 64 ? LPR : 64;
    for (int off = wl / 2; off > 0; off >>= 1) {
        double o = __shfl_xor(acc, off);
        acc = MODE == 2 ? acc + o : fmax(acc, o);
    }
    if (LPR > 64) {
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
        __syncthreads();
        if (threadIdx.x == 0)
            for (int w = 1; w < LPR / 64; ++w) acc = MODE == 2 ? acc + red[w] : fmax(acc, red[w]);
        __syncthreads();
    }
    if (lane == 0) A.out[orig] = acc;
}

template <int MODE>
__global__ void k_rowscan(ScanArgs A) {
    // max scans (MODE 0/1) are order-free, so they use 8 lanes per row (more rows in flight); the sum
    // scan keeps 16 lanes so its summation order, and hence ||A_pre||_inf, is unchanged
    constexpr int LPR = MODE == 2 ? 16 : 8;
    const int64_t g = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / LPR;
    const int lane = threadIdx.x & (LPR - 1);
    if (g >= A.n) return;
    const int32_t i = A.list ? A.list[g] : (int32_t)g;
    if ((A.cptr[i + 1] - A.cptr[i]) + (A.rptr[i + 1] - A.rptr[i]) > kLongRow) {
        if (lane == 0) A.out[A.perm[i]] = 0.0;  // combined by k_rowscan_long
        return;
    }
    row_scan<LPR, MODE>(i, lane, A, nullptr);
}

// Long (dense) rows: each row is cut into chunks of kLongChunk entries, one workgroup per chunk; the
// chunk results go to A.part[row * A.long_chunks + chunk] and k_rowscan_long_fin combines them in chunk
// order (no atomics: the row sums, hence ||A_pre||_inf, are the same in every run).
template <int MODE>
__global__ void k_rowscan_long(ScanArgs A) {
    __shared__ double red[kThreads / 64];
    const int32_t i = A.long_rows[blockIdx.y];
    const int32_t orig = A.perm[i];
    const int32_t nc = A.cptr[i + 1] - A.cptr[i];
    const int32_t nr = A.rptr[i + 1] - A.rptr[i];
    const int64_t begin = (int64_t)blockIdx.x * kLongChunk;
    if (begin >= nc + nr) return;
    const int64_t end = begin + kLongChunk < nc + nr ? begin + kLongChunk : nc + nr;
    const double si = MODE > 0 ? A.scale[orig] : 1.0;
    double acc = 0.0;
    for (int64_t t = begin + threadIdx.x; t < end; t += kThreads) {
        int32_t q, partner;
        if (t < nc) { q = A.cptr[i] + (int32_t)t; partner = A.ent_r[q]; }
        else { q = A.rslot[A.rptr[i] + (int32_t)(t - nc)]; partner = A.ent_c[q]; }
        double w = MODE == 0 ? fabs(A.uval[q]) : scaled_abs(orig, si, partner, A.uval[q], A.scale);
        acc = MODE == 2 ? acc + w : fmax(acc, w);
    }
    for (int off = 32; off > 0; off >>= 1) {
        double o = __shfl_xor(acc, off);
        acc = MODE == 2 ? acc + o : fmax(acc, o);
    }
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kThreads / 64; ++w) acc = MODE == 2 ? acc + red[w] : fmax(acc, red[w]);
        A.part[(int64_t)blockIdx.y * A.long_chunks + blockIdx.x] = acc;
    }
}

// one lane per long row: its chunk results in chunk order
template <int MODE>
__global__ void k_rowscan_long_fin(ScanArgs A) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= A.n_long) return;
    const int32_t i = A.long_rows[r];
    const int64_t len = (A.cptr[i + 1] - A.cptr[i]) + (A.rptr[i + 1] - A.rptr[i]);
    const int64_t nch = (len + kLongChunk - 1) / kLongChunk;
    double acc = 0.0;
    for (int64_t c = 0; c < nch; ++c) {
        const double w = A.part[(int64_t)r * A.long_chunks + c];
        acc = MODE == 2 ? acc + w : fmax(acc, w);
    }
    A.out[A.perm[i]] = acc;
}

// Partial row scans of the separator ("top") rows on one rank of a distributed factorization: the
// rank's own slots of each top row, cut into chunks (one workgroup each, results in A.part), combined
// per row in chunk order by k_rowscan_part_fin; the ranks' partials are then all-reduced (max / sum)
// over the top rows.
template <int MODE>
__global__ void k_rowscan_part(PartArgs A) {
    __shared__ double red[kThreads / 64];
    const int64_t c = blockIdx.x;
    const int32_t t = A.chunk_row[c];
    const int32_t orig = A.trow_orig[t];
    const double si = MODE > 0 ? A.scale[orig] : 1.0;
    double acc = 0.0;
    for (int64_t q = A.chunk_begin[c] + threadIdx.x; q < A.chunk_begin[c + 1]; q += kThreads) {
        const int32_t slot = A.pslot[q];
        const double w = MODE == 0 ? fabs(A.uval[slot]) : scaled_abs(orig, si, A.ppartner[q], A.uval[slot], A.scale);
        acc = MODE == 2 ? acc + w : fmax(acc, w);
    }
    for (int off = 32; off > 0; off >>= 1) {
        double o = __shfl_xor(acc, off);
        acc = MODE == 2 ? acc + o : fmax(acc, o);
    }
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kThreads / 64; ++w) acc = MODE == 2 ? acc + red[w] : fmax(acc, red[w]);
        A.part[c] = acc;
    }
}

template <int MODE>
__global__ void k_rowscan_part_fin(PartArgs A) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < A.nrows; t += (int64_t)gridDim.x * blockDim.x) {
        double acc = 0.0;
        for (int64_t c = A.row_chunk[t]; c < A.row_chunk[t + 1]; ++c) acc = MODE == 2 ? acc + A.part[c] : fmax(acc, A.part[c]);
        A.outT[t] = acc;
    }
}

__global__ void k_scatter(const double* __restrict__ src, const int32_t* __restrict__ idx, double* __restrict__ dst,
                          int64_t k) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < k; t += (int64_t)gridDim.x * blockDim.x)
        dst[idx[t]] = src[t];
}

__global__ void k_fill_ones(double* __restrict__ x, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) x[i] = 1.0;
}

__global__ void k_scatter64(const double* __restrict__ src, const int64_t* __restrict__ idx, double* __restrict__ dst,
                            int64_t k) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < k; t += (int64_t)gridDim.x * blockDim.x)
        dst[idx[t]] = src[t];
}

__global__ void k_gather(const double* __restrict__ src, const int32_t* __restrict__ idx, double* __restrict__ dst,
                         int64_t k) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < k; t += (int64_t)gridDim.x * blockDim.x)
        dst[t] = src[idx[t]];
}

// ||A_pre||_inf = max_i rowsum_i: grid-stride block maxima, one atomic per workgroup
__global__ void k_normmax(const double* __restrict__ rowsum, const int32_t* __restrict__ list, int64_t n,
                          unsigned long long* __restrict__ anorm) {
    __shared__ double red[kThreads / 64];
    double mx = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        mx = fmax(mx, rowsum[list ? list[i] : i]);
    for (int off = 32; off > 0; off >>= 1) mx = fmax(mx, __shfl_xor(mx, off));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kThreads / 64; ++w) mx = fmax(mx, red[w]);
        atomicMax(anorm, as_bits(mx));
    }
}

__global__ void k_scale_update(const double* __restrict__ rmax, double* __restrict__ scale, const int32_t* __restrict__ list,
                               int64_t n, int first) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = list ? list[t] : t;
        double r = rmax[i];
        double s = first ? 1.0 : scale[i];
        if (r > 0.0) s = s / sqrt(r);
        scale[i] = s;
    }
}

// row-major packed lower triangle: t -> (r, c), t = r(r+1)/2 + c, 0 <= c <= r (t < 2^31)
__device__ __forceinline__ void tri_rc(int t, int& r, int& c) {
    int rr = (int)((sqrtf(8.0f * (float)t + 1.0f) - 1.0f) * 0.5f);
    int s0 = (int)(((long long)rr * (rr + 1)) >> 1);
    if (s0 > t) { s0 -= rr; --rr; }
    else if (s0 + rr + 1 <= t) { s0 += rr + 1; ++rr; }
    r = rr;
    c = t - s0;
}

// ------------------------------------------------------------------------------------------------
// inter-workgroup hand-offs of the dataflow schedules (factor: contribution blocks; solve: update
// vectors and solution values): sc1 (write-through) stores, sc1 loads, one signalling lane after the
// storing wave's vmcnt(0) (MI355X_MICROARCH.md, inter-workgroup visibility, first hand-off row)
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ double ld_sc1(const double* p) {
    return as_double(__hip_atomic_load((const unsigned long long*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void st_sc1(double* p, double v) {
    __hip_atomic_store((unsigned long long*)p, as_bits(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_sc1_u32(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr int kDfSpinLimit = 1 << 22;  // polls (each behind s_sleep 2): about a second

// Poll *addr (sc1) until it reaches `target` (wrap-safe); false on abort / limit.  Wave-uniform.
__device__ __forceinline__ bool df_wait(const uint32_t* addr, uint32_t target, uint32_t* abort_flag) {
    uint32_t v = ld_sc1_u32(addr);
    int it = 0;
    while ((int32_t)(v - target) < 0) {
        __builtin_amdgcn_s_sleep(2);
        v = ld_sc1_u32(addr);
        if ((++it & 63) == 0) {
            if (ld_sc1_u32(abort_flag)) return false;
            if (it >= kDfSpinLimit) {
                __hip_atomic_store(abort_flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                return false;
            }
        }
    }
    return true;
}

// every store of this wave has completed (sc1 stores: written through) before the signal below
__device__ __forceinline__ void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// ---- single-GPU equilibration on a row-major copy of |A| ----
// Row i (new numbering) of the symmetric matrix = its column part (slots cptr[i] .. cptr[i+1]) followed by
// its row part (slots rslot[rptr[i] .. rptr[i+1]]); the copy uvalR keeps |a| in that order at
// [cptr[i] + rptr[i], cptr[i+1] + rptr[i+1]).  rowpartner holds (partner's new index << 1) | (the row's
// original id > the partner's), so the scalings are kept in the NEW numbering (a row's partners are its
// nested-dissection neighbours: the gathers stay in cache) and the product is still formed in the oracle's
// order (s of the larger original id first).  MODE 0 (first sweep) gathers the packed values once and
// writes the copy; MODE 1 (later sweeps) and MODE 2 (row sums for ||A_pre||_inf) stream it.  A sweep reads
// one scaling buffer and writes another (s_out = s_in / sqrt(r), s_in = 1 in the first sweep).  Rows longer
// than kLongRow are cut into chunks handled by the first blocks of the same launch; the last chunk block
// of a row to finish (arrival counter) combines the chunk results in chunk order (deterministic).
template <int MODE>
__device__ __forceinline__ double rowR_term(const ScanArgs& A, int64_t t, int32_t i, int32_t c0, int32_t nc,
                                            int32_t r0, double si, const double* __restrict__ sc) {
    if (MODE == 0) {
        const int32_t q = t < nc ? c0 + (int32_t)t : A.rslot[r0 + (int32_t)(t - nc)];
        const double w = fabs(A.uval[q]);
        A.uvalR[(int64_t)c0 + r0 + t] = w;
        return w;
    }
    const int64_t e = (int64_t)c0 + r0 + t;
    const int32_t pc = A.rowpartner[e];
    const double v = A.uvalR[e], sj = sc[pc >> 1];
    return (pc & 1) ? si * v * sj : sj * v * si;  // |v| >= 0: no fabs needed
}

template <int MODE>
__device__ __forceinline__ void rowR_write(const ScanArgs& A, int32_t i, double acc, double si) {
    if (MODE == 2) A.out[i] = acc;
    else A.scale_out[i] = acc > 0.0 ? si / sqrt(acc) : si;
}

template <int MODE>
__global__ __launch_bounds__(256) void k_rowscanR(ScanArgs A) {
    const double* sc = MODE == 1 ? A.scale_in : A.scale_out;  // MODE 2: the final scaling (new numbering)
    const int64_t nlb = (int64_t)A.n_long * A.long_chunks;
    if ((int64_t)blockIdx.x < nlb) {  // chunk of a long row
        __shared__ double red[4];
        __shared__ int last;
        const int r = (int)(blockIdx.x / A.long_chunks), ch = (int)(blockIdx.x % A.long_chunks);
        const int32_t i = A.long_rows[r];
        const int32_t c0 = A.cptr[i], nc = A.cptr[i + 1] - c0, r0 = A.rptr[i];
        const int64_t len = nc + (A.rptr[i + 1] - r0);
        const int64_t nch = (len + kLongChunk - 1) / kLongChunk;
        if (ch >= nch) return;
        const double si = MODE == 0 ? 1.0 : sc[i];
        const int64_t end = (int64_t)(ch + 1) * kLongChunk < len ? (int64_t)(ch + 1) * kLongChunk : len;
        double acc = 0.0;
        for (int64_t t = (int64_t)ch * kLongChunk + threadIdx.x; t < end; t += 256) {
            const double w = rowR_term<MODE>(A, t, i, c0, nc, r0, si, sc);
            acc = MODE == 2 ? acc + w : fmax(acc, w);
        }
        for (int off = 32; off > 0; off >>= 1) {
            const double o = __shfl_xor(acc, off);
            acc = MODE == 2 ? acc + o : fmax(acc, o);
        }
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
        __syncthreads();
        if (threadIdx.x == 0) {
            acc = MODE == 2 ? (red[0] + red[1]) + (red[2] + red[3]) : fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
            st_sc1(A.part + (int64_t)r * A.long_chunks + ch, acc);
            drain_stores();
            last = __hip_atomic_fetch_add(A.long_cnt + r, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (uint32_t)(nch - 1);
        }
        __syncthreads();
        if (last && threadIdx.x == 0) {
            double tot = 0.0;
            for (int64_t c = 0; c < nch; ++c) {
                const double w = ld_sc1(A.part + (int64_t)r * A.long_chunks + c);
                tot = MODE == 2 ? tot + w : fmax(tot, w);
            }
            rowR_write<MODE>(A, i, tot, si);
            __hip_atomic_store(A.long_cnt + r, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch
        }
        return;
    }
    constexpr int LPR = MODE == 2 ? 16 : 8;
    constexpr int U = 64 / LPR;  // entries per lane per batch: a row of <= 64 entries takes one batch, whose
                                 // loads are all issued before the first use (two dependent round trips)
    const int64_t g = ((int64_t)(blockIdx.x - nlb) * blockDim.x + threadIdx.x) / LPR;
    const int lane = threadIdx.x & (LPR - 1);
    if (g >= A.n) return;
    const int32_t i = (int32_t)g;
    const int32_t c0 = A.cptr[i], nc = A.cptr[i + 1] - c0;
    const int32_t r0 = A.rptr[i], len = nc + (A.rptr[i + 1] - r0);
    if (len > kLongRow) return;  // chunk blocks above
    const double si = MODE == 0 ? 1.0 : sc[i];
    const int64_t e0 = (int64_t)c0 + r0;
    double acc = 0.0;
    for (int32_t b = 0; b < len; b += LPR * U) {
        int32_t key[U];
        double v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int32_t t = b + lane + LPR * u;
            const bool ok = t < len;
            if (MODE == 0) key[u] = !ok ? c0 : (t < nc ? c0 + t : A.rslot[r0 + (t - nc)]);  // packed slot
            else { key[u] = ok ? A.rowpartner[e0 + t] : 0; v[u] = ok ? A.uvalR[e0 + t] : 0.0; }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int32_t t = b + lane + LPR * u;
            double w;
            if (MODE == 0) {
                w = fabs(A.uval[key[u]]);
                if (t < len) A.uvalR[e0 + t] = w;
                else w = 0.0;
            } else {
                const double sj = sc[key[u] >> 1];
                w = (key[u] & 1) ? si * v[u] * sj : sj * v[u] * si;  // v = 0 beyond the row
            }
            acc = MODE == 2 ? acc + w : fmax(acc, w);
        }
    }
#pragma unroll
    for (int off = LPR / 2; off > 0; off >>= 1) {
        const double o = __shfl_xor(acc, off);
        acc = MODE == 2 ? acc + o : fmax(acc, o);
    }
    if (lane == 0) rowR_write<MODE>(A, i, acc, si);
}

template <int CTRL>
__device__ __forceinline__ unsigned long long dpp64(unsigned long long x) {
    unsigned lo = (unsigned)x, hi = (unsigned)(x >> 32);
    lo = (unsigned)__builtin_amdgcn_mov_dpp((int)lo, CTRL, 0xf, 0xf, false);
    hi = (unsigned)__builtin_amdgcn_mov_dpp((int)hi, CTRL, 0xf, 0xf, false);
    return ((unsigned long long)hi << 32) | lo;
}
__device__ __forceinline__ unsigned long long umax64(unsigned long long a, unsigned long long b) { return a > b ? a : b; }

// ---- single-GPU equilibration on the fronts' slots (SweepArgs) ----
// Every entry of the lower triangle is one packed slot of exactly one front, and both its rows are in
// that front's row list, so a row's maximum is the maximum over the fronts holding it of the front's
// partial.  One wave per front: the entries' |s_r a s_c| (the oracle's multiplication order, s of the
// larger original id first: bit-identical to oracle/kkt_oracle.c) reduce into the front's rows in LDS
// (64-bit max on the bit patterns: order-free), then one atomic max per (front, row) into rmax.  The
// first sweep (FIRST: s = 1) runs right after k_pack.
// BIG: fronts of more than kSweepBigSlots slots (the large fronts), which one wave would sweep for
// milliseconds: grid (big fronts x slices) of 256-thread blocks, each reducing a slice of the slots into
// its LDS row maxima, one atomic max per (block, row) straight into rmax (long rows included: there are
// few such blocks).  The one-wave launch skips those fronts (their long-row partials stay 0).
// a slot with several COO positions (k_pack_multi's record): duplicates summed in ascending COO position
__device__ __forceinline__ double pack_multi_value(const double* __restrict__ values, const int32_t* __restrict__ dup_pos,
                                                   int4 d) {
    double v = 0.0;
    if (d.y >= -1) {
        const double a = values[d.y], b = d.z >= 0 ? values[d.z] : 0.0, c = d.w >= 0 ? values[d.w] : 0.0;
        v += a;
        if (d.z >= 0) v += b;
        if (d.w >= 0) v += c;
    } else {
        for (int32_t q = -2 - d.y; q < -2 - d.y + d.z; ++q) v += values[dup_pos[q]];
    }
    return v;
}

// the scaling of row r before sweep A.iter: s = 1, then s <- s / sqrt(rmax_j(r)) for every earlier sweep j
// with rmax_j(r) > 0 (k_sweep_final's expression, so every sweep and the final scaling agree to the bit).
// The sweeps' row maxima stay in separate buffers until k_sweep_final: no update kernel between sweeps.
__device__ __forceinline__ double sweep_row_scale(const SweepArgs& A, int32_t r) {
    double x[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) x[j] = j < A.iter ? as_double(A.rmax_all[(int64_t)j * A.n + r]) : 0.0;
    double s = 1.0;
#pragma unroll
    for (int j = 0; j < 3; ++j)
        if (x[j] > 0.0) s = s / sqrt(x[j]);
    for (int j = 3; j < A.iter; ++j) {
        const double y = as_double(A.rmax_all[(int64_t)j * A.n + r]);
        if (y > 0.0) s = s / sqrt(y);
    }
    return s;
}

// 8 waves per SIMD (<= 64 VGPRs): the one-wave fronts are latency-bound, occupancy pays (76 VGPRs, 6 waves:
// 0.360 ms scale phase at C3; 54 VGPRs, 8 waves: 0.337 ms)
template <bool FIRST, bool BIG>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void k_sweep_front(SweepArgs A) {
    extern __shared__ __attribute__((aligned(16))) double swm[];
    const int f = BIG ? A.big_list[blockIdx.x] : blockIdx.x;
    const int m = A.fm[f];
    const int lane = threadIdx.x;  // thread of the block (one wave unless BIG)
    const int NT = BIG ? 256 : 64;
    double* sl = swm;                                                         // m: the front rows' scaling
    unsigned long long* rm = reinterpret_cast<unsigned long long*>(swm + m);  // m: row maxima (bits)
    const int64_t ro = A.rows_off[f];
    int64_t e0 = A.ent_off[f], e1 = A.ent_off[f + 1];
    if (FIRST && !BIG && A.counters && blockIdx.x == 0 && lane < kCounterSlots) A.counters[lane] = lane == 8 ? ~0ull : 0ull;
    if (!BIG && e1 - e0 > kSweepBigSlots) return;
    if (BIG) {
        const int64_t chunk = ((e1 - e0 + gridDim.y - 1) / gridDim.y + 7) & ~(int64_t)7;
        e0 += chunk * blockIdx.y;
        e1 = e0 + chunk < e1 ? e0 + chunk : e1;
    }
    // A batch is EB x NT consecutive slots: load u of lane l reads slot base + u NT + l, so a wave's load
    // instruction covers 256 / 512 contiguous bytes, and every slot does one LDS atomic max for its row and
    // one for its column.  (Each lane taking EB consecutive slots, keeping its column maximum in a register,
    // measured slower: every load instruction then spans NT strided cache lines.)
    constexpr int EB = 8;
    uint32_t lp[EB];
    double v[EB];
    auto load = [&](int64_t base) {
        if (FIRST) {
            // the pack (k_pack / k_pack_multi semantics) fused into the first sweep: each slot's value from
            // the caller's COO array, written to uval here
            int32_t src[EB];
#pragma unroll
            for (int u = 0; u < EB; ++u) {
                const int64_t e = base + (int64_t)u * NT + lane;
                const bool ok = e < e1;
                lp[u] = ok ? A.ent_lpos[e] : 0xffffffffu;
                src[u] = ok ? (A.slot_src != nullptr ? A.slot_src[e] : A.dup_pos[e]) : 0;
            }
#pragma unroll
            for (int u = 0; u < EB; ++u) {
                if (lp[u] == 0xffffffffu) { v[u] = 0.0; continue; }
                const int64_t e = base + (int64_t)u * NT + lane;
                double x;
                if (A.dup_ptr == nullptr) {
                    x = A.values[src[u]];
                } else if (src[u] >= 0) {
                    x = 0.0 + A.values[src[u]];  // as the summed form: -0.0 packs as +0.0
                } else {
                    x = pack_multi_value(A.values, A.dup_pos, reinterpret_cast<const int4*>(A.multi)[-1 - src[u]]);
                }
                v[u] = x;
                A.uval[e] = x;
            }
            return;
        }
#pragma unroll
        for (int u = 0; u < EB; ++u) {
            const int64_t e = base + (int64_t)u * NT + lane;
            const bool ok = e < e1;
            lp[u] = ok ? A.ent_lpos[e] : 0xffffffffu;
            v[u] = ok ? A.uval[e] : 0.0;
        }
    };
    load(e0);  // the first batch is in flight while the rows' scalings are gathered
    // one-wave fronts of <= 128 rows keep their row ids and long-row indices (per-front-row copy flong: no
    // rows -> longpos chain) in registers for the final flush; the rows' scalings come from the earlier
    // sweeps' row maxima (sweep_row_scale)
    constexpr int RQ = 2;
    const bool regrows = !BIG && m <= 64 * RQ;
    int32_t rr[RQ];
    int lk[RQ];
    if (regrows) {
        double sv[RQ];
#pragma unroll
        for (int u = 0; u < RQ; ++u) {
            const int q = lane + 64 * u;
            const bool ok = q < m;
            rr[u] = ok ? A.rows[ro + q] : 0;
            lk[u] = ok && A.flong ? (int)A.flong[ro + q] : -1;
            sv[u] = 1.0;
            if (!FIRST && ok) sv[u] = sweep_row_scale(A, rr[u]);
        }
#pragma unroll
        for (int u = 0; u < RQ; ++u) {
            const int q = lane + 64 * u;
            if (q < m) {
                rm[q] = 0ull;
                if (!FIRST) sl[q] = sv[u];
            }
        }
    } else {
        for (int q = lane; q < m; q += NT) {
            rm[q] = 0ull;
            if (!FIRST) sl[q] = sweep_row_scale(A, A.rows[ro + q]);
        }
    }
    __syncthreads();
    for (int64_t base = e0;;) {
#pragma unroll
        for (int u = 0; u < EB; ++u) {
            // slots are column-major, so runs of lanes share a column: an aligned quad whose four slots are in
            // one column reduces its maximum across the quad (DPP) and its first lane does the column's
            // atomic -- a quarter of the same-address LDS atomics (max is order-free: same result)
            const bool ok = lp[u] != 0xffffffffu;  // beyond the slot range: no atomics
            const int lr = (int)(lp[u] >> 16), lc = ok ? (int)(lp[u] & 0x7fffu) : -1;
            double w = ok ? fabs(v[u]) : 0.0;
            if (!FIRST && ok) {
                const double sr = sl[lr], sc = sl[lc];
                w = (lp[u] & 0x8000u) ? sc * w * sr : sr * w * sc;
            }
            const unsigned long long bw = as_bits(w);
            // every DPP read in all lanes (a short-circuit && would evaluate the last one under a partial EXEC)
            const int s1 = lc == __builtin_amdgcn_mov_dpp(lc, 0xB1, 0xF, 0xF, false) ? 1 : 0;  // quad_perm [1,0,3,2]
            const int s2 = lc == __builtin_amdgcn_mov_dpp(lc, 0x4E, 0xF, 0xF, false) ? 1 : 0;  // quad_perm [2,3,0,1]
            const int s3 = __builtin_amdgcn_mov_dpp(s1, 0x4E, 0xF, 0xF, false);               // the other pair
            const bool same = (s1 & s2 & s3) != 0;
            unsigned long long qm = umax64(bw, dpp64<0xB1>(bw));
            qm = umax64(qm, dpp64<0x4E>(qm));
            if (ok) atomicMax(rm + lr, bw);
            if (same) {
                if ((lane & 3) == 0 && lc >= 0) atomicMax(rm + lc, qm);
            } else if (ok) {
                atomicMax(rm + lc, bw);
            }
        }
        base += (int64_t)EB * NT;
        if (base >= e1) break;  // uniform
        load(base);
    }
    __syncthreads();
    if (regrows) {
#pragma unroll
        for (int u = 0; u < RQ; ++u) {
            const int q = lane + 64 * u;
            if (q >= m) continue;
            const unsigned long long bw = rm[q];
            if (lk[u] >= 0) A.part_long[(int64_t)f * A.n_long + lk[u]] = as_double(bw);  // every front writes its slot
            else if (bw != 0ull) atomicMax(A.rmax + rr[u], bw);
        }
        return;
    }
    for (int q = lane; q < m; q += NT) {
        const int32_t r = A.rows[ro + q];
        const unsigned long long bw = rm[q];
        if (BIG) {
            if (bw != 0ull) atomicMax(A.rmax + r, bw);
            continue;
        }
        const int k = A.n_long > 0 ? (int)A.longpos[r] : -1;
        if (k >= 0) A.part_long[(int64_t)f * A.n_long + k] = as_double(bw);  // every front writes its slot
        else if (bw != 0ull) atomicMax(A.rmax + r, bw);
    }
}

// long (dense) rows: thread t of the grid reduces fronts t, t + grid, ... (their n_long partials are
// contiguous) into the block's LDS maxima, then one atomic max per (block, long row) -- max is
// order-free, so the result is the same in every run
__global__ __launch_bounds__(256) void k_sweep_long_fin(SweepArgs A) {
    extern __shared__ unsigned long long lred[];
    for (int k = threadIdx.x; k < A.n_long; k += 256) lred[k] = 0ull;
    __syncthreads();
    const int64_t stride = (int64_t)gridDim.x * 256;
    constexpr int KB = 8;  // long rows per pass: their partial loads in flight together
    for (int k0 = 0; k0 < A.n_long; k0 += KB) {
        double mx[KB];
#pragma unroll
        for (int u = 0; u < KB; ++u) mx[u] = 0.0;
        for (int64_t f = (int64_t)blockIdx.x * 256 + threadIdx.x; f < A.nf; f += stride) {
#pragma unroll
            for (int u = 0; u < KB; ++u)
                if (k0 + u < A.n_long) mx[u] = fmax(mx[u], A.part_long[f * A.n_long + k0 + u]);
        }
#pragma unroll
        for (int u = 0; u < KB; ++u) {
            for (int off = 32; off > 0; off >>= 1) mx[u] = fmax(mx[u], __shfl_xor(mx[u], off));
            if ((threadIdx.x & 63) == 0 && k0 + u < A.n_long && mx[u] > 0.0) atomicMax(lred + k0 + u, as_bits(mx[u]));
        }
    }
    __syncthreads();
    for (int k = threadIdx.x; k < A.n_long; k += 256)
        if (lred[k] != 0ull) atomicMax(A.rmax + A.long_orig[k], lred[k]);
}

// ---- refinement residual over the fronts' slots (ResidArgs) ----
__global__ __launch_bounds__(64) void k_resid_front(ResidArgs A) {
    extern __shared__ __attribute__((aligned(16))) double rsm[];
    const int f = blockIdx.x;
    const int lane = threadIdx.x;
    const int64_t e0 = A.ent_off[f], e1 = A.ent_off[f + 1];
    if (e1 == e0) return;  // no slot: none of its rows has a partial here
    const int m = A.fm[f];
    const int64_t ro = A.rows_off[f];
    double* xl = rsm;      // m: x of the front rows
    double* yl = rsm + m;  // m: the front's partial A x
    for (int q = lane; q < m; q += 64) {
        xl[q] = A.x[A.rows[ro + q]];
        yl[q] = 0.0;
    }
    __syncthreads();
    constexpr int EB = 8;  // load u of lane l reads slot base + 64 u + l (coalesced), as the sweeps
    for (int64_t base = e0; base < e1; base += EB * 64) {
        uint32_t lp[EB];
        double v[EB];
#pragma unroll
        for (int u = 0; u < EB; ++u) {
            const int64_t e = base + (int64_t)u * 64 + lane;
            const bool ok = e < e1;
            lp[u] = ok ? A.ent_lpos[e] : 0xffffffffu;
            v[u] = ok ? A.uval[e] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < EB; ++u) {
            if (lp[u] == 0xffffffffu) continue;
            const int lr = (int)(lp[u] >> 16), lc = (int)(lp[u] & 0x7fffu);
            atomicAdd(yl + lr, v[u] * xl[lc]);
            if (lr != lc) atomicAdd(yl + lc, v[u] * xl[lr]);
        }
    }
    __syncthreads();
    for (int q = lane; q < m; q += 64) A.part[ro + q] = yl[q];
}

// waves [0, n_chunks): chunk q of the chunked rows (4 partials per lane, fixed tree) -> chunk_part[q]; then
// 4 lanes per row (up to 8 partials per lane, summed in order, fixed tree) -> r
__global__ __launch_bounds__(256) void k_resid_rows(ResidArgs A) {
    const int64_t wave = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    if (wave < A.n_chunks) {
        const int k = A.chunk_row[wave];
        const int32_t i = A.long_rows[k];
        const int32_t b = A.rz_ptr[i] + (int32_t)(wave - A.chunk_off[k]) * kResidChunk;
        const int32_t e = min(A.rz_ptr[i + 1], b + kResidChunk);
        int32_t pos[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int32_t t = b + u * 64 + lane;
            pos[u] = t < e ? A.rz_pos[t] : -1;
        }
        double acc = 0.0;
#pragma unroll
        for (int u = 0; u < 4; ++u) acc += pos[u] >= 0 ? A.part[pos[u]] : 0.0;
        for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
        if (lane == 0) A.chunk_part[wave] = acc;
        return;
    }
    const int64_t g = (((int64_t)blockIdx.x * 256 + threadIdx.x) - A.n_chunks * 64) >> 2;
    const int q = threadIdx.x & 3;
    if (g >= A.n) return;
    const int32_t p0 = A.rz_ptr[g], p1 = A.rz_ptr[g + 1];
    if (p1 - p0 > A.short_len) return;  // chunked
    int32_t pos[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        const int32_t t = p0 + u * 4 + q;
        pos[u] = t < p1 ? A.rz_pos[t] : -1;
    }
    double acc = 0.0;
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += pos[u] >= 0 ? A.part[pos[u]] : 0.0;
    acc += __shfl_xor(acc, 2, 4);
    acc += __shfl_xor(acc, 1, 4);
    if (q == 0) A.r[g] = acc - A.b[g];
}

__global__ void k_resid_long_fin(ResidArgs A) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= A.n_long) return;
    const int32_t i = A.long_rows[k];
    double acc = 0.0;
    for (int32_t c = A.chunk_off[k]; c < A.chunk_off[k + 1]; ++c) acc += A.chunk_part[c];
    A.r[i] = acc - A.b[i];
}

// after the front sweeps: scale (by original id perm[i]) = sweep_row_scale of new index i over all `iters`
// sweeps, and every sweep's row maxima back to 0 for the next factorization (`passes` buffers: iters == 0
// still ran the packing pass)
__global__ void k_sweep_final(unsigned long long* __restrict__ rmax_all, double* __restrict__ scale,
                              const int32_t* __restrict__ perm, int64_t n, int iters, int passes) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        double s = 1.0;
        for (int j = 0; j < passes; ++j) {
            const double r = as_double(rmax_all[(int64_t)j * n + i]);
            if (j < iters && r > 0.0) s = s / sqrt(r);
            rmax_all[(int64_t)j * n + i] = 0ull;
        }
        scale[perm[i]] = s;
    }
}

// s <- s / sqrt(r) (s = 1 before the first sweep; rows without entries keep s), and r <- 0 for the next sweep
__global__ void k_sweep_update(unsigned long long* __restrict__ rmax, double* __restrict__ scale, int64_t n, int first) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const double r = as_double(rmax[i]);
        double sc = first ? 1.0 : scale[i];
        if (r > 0.0) sc = sc / sqrt(r);
        scale[i] = sc;
        rmax[i] = 0ull;
    }
}

// scaling by original id for the factorization / solve kernels: scale[perm[i]] = scaleN[i]
__global__ void k_scale_to_orig(const double* __restrict__ sn, const int32_t* __restrict__ perm, double* __restrict__ scale,
                                int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        scale[perm[i]] = sn[i];
}

// ------------------------------------------------------------------------------------------------
// dense front factorization
// ------------------------------------------------------------------------------------------------
// Front storage: only the lower triangle A(i,j), j <= i, is kept.
//   PackedStore: row-packed lower triangle in LDS, m(m+1)/2 doubles (row i starts at i(i+1)/2)
//   FullStore:   m x ld square (fronts too large for LDS live in HBM scratch)
// doubles of a front's packed lower triangle in LDS, rounded up to even (16-byte alignment of what follows)
__device__ __forceinline__ int64_t packed_even(int m) { return (((int64_t)m * (m + 1) / 2) + 1) & ~1ll; }

struct PackedStore {
    double* F;
    __device__ __forceinline__ int idx(int i, int j) const { return ((i * (i + 1)) >> 1) + j; }
    __device__ __forceinline__ double& at(int i, int j) const { return F[idx(i, j)]; }
};
struct FullStore {
    double* F;
    int ld;
    __device__ __forceinline__ int idx(int i, int j) const { return i * ld + j; }
    __device__ __forceinline__ double& at(int i, int j) const { return F[idx(i, j)]; }
};

struct PivotDecision {
    int kind;  // PIV_*
    int c, r;  // candidate, 2x2 partner
    int relaxed;
};

// |A(i,c)| of the symmetric front from its lower triangle
template <class S>
__device__ __forceinline__ double absA(const S& st, int i, int c) {
    return fabs(i >= c ? st.at(i, c) : st.at(c, i));
}

// ---- wave-wide reductions: DPP within 16-lane rows, readlane across rows (result wave-uniform) ----
__device__ __forceinline__ unsigned long long readlane64(unsigned long long x, int l) {
    unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)x, l);
    unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(x >> 32), l);
    return ((unsigned long long)hi << 32) | lo;
}
__device__ __forceinline__ double readlane_d(double x, int l) { return as_double(readlane64(as_bits(x), l)); }
// Cross-lane hand-off through LDS inside ONE wave.  The hardware executes a wave's LDS operations in issue order,
// but the compiler reasons per lane: a plain LDS store by some lanes followed by plain loads of the same words in
// other lanes is a data race to it, so it may move a load above the store.  Round 5 hit exactly that (ISA diff in
// DESIGN.md §4 round 6): with the operand reads scheduled ahead of the ballot, LLVM forwarded the owner lanes' own
// stores into their loads and turned "if (owner) publish; read" into "if (!owner) read; else publish", running the
// non-owners' branch -- and their LDS reads -- BEFORE the owners' stores: stale operands, wrong inertia on the 5x5
// known answer.  A wavefront-scope release / wave barrier / acquire orders every LDS access before it against every
// one after it for all lanes of the wave, and costs no instruction on gfx950 (wavefront-scope fences emit nothing;
// the "local" address-space tag leaves global loads free to move across it).  Put it between a publish and its read-back, and before a buffer is rewritten.
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
}
// x of lane `src` (any lane pattern, one LDS-crossbar round trip, no LDS allocation, no barrier)
__device__ __forceinline__ double bperm_d(double x, int src) {
    const unsigned long long b = as_bits(x);
    const int lo = __builtin_amdgcn_ds_bpermute(src << 2, (int)(unsigned)b);
    const int hi = __builtin_amdgcn_ds_bpermute(src << 2, (int)(unsigned)(b >> 32));
    return as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
// max over the 64 lanes of a wave (every lane must be active)
__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long x) {
    x = umax64(x, dpp64<0xB1>(x));   // quad_perm [1,0,3,2]
    x = umax64(x, dpp64<0x4E>(x));   // quad_perm [2,3,0,1]
    x = umax64(x, dpp64<0x141>(x));  // row_half_mirror
    x = umax64(x, dpp64<0x140>(x));  // row_mirror
    return umax64(umax64(readlane64(x, 0), readlane64(x, 16)), umax64(readlane64(x, 32), readlane64(x, 48)));
}
__device__ __forceinline__ unsigned long long umin64(unsigned long long a, unsigned long long b) { return a < b ? a : b; }
// min over the 64 lanes of a wave (every lane must be active; result wave-uniform)
__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long x) {
    x = umin64(x, dpp64<0xB1>(x));
    x = umin64(x, dpp64<0x4E>(x));
    x = umin64(x, dpp64<0x141>(x));
    x = umin64(x, dpp64<0x140>(x));
    return umin64(umin64(readlane64(x, 0), readlane64(x, 16)), umin64(readlane64(x, 32), readlane64(x, 48)));
}
// non-negative doubles compare like their bit patterns
__device__ __forceinline__ double wave_max_abs(double v) { return as_double(wave_max_u64(as_bits(v))); }
// an upper bound of wave_max_abs within 2^-20 relative: the maximum of the high words, low word all ones (one
// 32-bit DPP chain instead of the 64-bit compare-and-select one)
__device__ __forceinline__ double wave_max_abs_ub(double v) {
    unsigned x = (unsigned)(as_bits(v) >> 32);
    x = max(x, (unsigned)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xf, 0xf, false));
    x = max(x, (unsigned)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xf, 0xf, false));
    x = max(x, (unsigned)__builtin_amdgcn_mov_dpp((int)x, 0x141, 0xf, 0xf, false));
    x = max(x, (unsigned)__builtin_amdgcn_mov_dpp((int)x, 0x140, 0xf, 0xf, false));
    const unsigned h = max(max((unsigned)__builtin_amdgcn_readlane((int)x, 0), (unsigned)__builtin_amdgcn_readlane((int)x, 16)),
                           max((unsigned)__builtin_amdgcn_readlane((int)x, 32), (unsigned)__builtin_amdgcn_readlane((int)x, 48)));
    return h >= 0x7ff00000u ? INFINITY : as_double(((unsigned long long)h << 32) | 0xffffffffull);  // inf / NaN: inf
}

template <class S> constexpr bool kFullStore = std::is_same<S, FullStore>::value;

// Threshold pivot search (MUMPS/Duff-Reid rule, u then relaxed); run by one full wave, result
// wave-uniform.  Mirrors test_pivot() of oracle/kkt_oracle.c; the relaxed ladder is only used at
// roots or when delays are disabled (otherwise the first relaxation reports the delayed columns).
template <class S>
__device__ PivotDecision search_pivot(const S& st, int m, int k, int p, double u, double thres, double& minpiv) {
    const int lane = threadIdx.x & 63;
    PivotDecision d{PIV_STUCK, k, -1, 0};
    for (int ul = 0; ul < 6; ++ul) {
        // relaxation ladder u, u/10, u/100, 1e-6, 1e-10, 0 (no array: avoids scratch)
        const double uu = ul == 0 ? u : ul == 1 ? u * 0.1 : ul == 2 ? u * 0.01 : ul == 3 ? 1e-6 : ul == 4 ? 1e-10 : 0.0;
        for (int c = k; c < p; ++c) {
            double g = 0.0;
            if constexpr (kFullStore<S>) {
                // front in HBM (large fronts): eight rows in flight per lane instead of one dependent load
                // after the other (~0.3 us each at m = 4096)
#pragma unroll 8
                for (int i = k + lane; i < m; i += 64) g = fmax(g, i == c ? 0.0 : absA(st, i, c));
            } else {
                for (int i = k + lane; i < m; i += 64) {
                    if (i == c) continue;
                    g = fmax(g, absA(st, i, c));
                }
            }
            g = wave_max_abs(g);
            const double acc = fabs(st.at(c, c));
            if (fmax(acc, g) <= thres) { d.kind = PIV_NULL; d.c = c; d.relaxed = ul > 0; return d; }
            minpiv = fmin(minpiv, fmax(acc, g));  // a larger null threshold would have stopped here
            if (acc != 0.0 && acc >= uu * g) { d.kind = PIV_1X1; d.c = c; d.relaxed = ul > 0; return d; }
            // 1x1 rejected: largest off-diagonal among the fully-summed rows is the 2x2 partner
            // exact argmax, ties to the smallest row (oracle test_pivot: first strict maximum)
            unsigned long long best = 0;
            int bi = 0x7fffffff;
            if constexpr (kFullStore<S>) {
#pragma unroll 8
                for (int i = k + lane; i < p; i += 64) {
                    const unsigned long long b = i == c ? 0ull : as_bits(absA(st, i, c));
                    if (b > best) { best = b; bi = i; }  // rows ascending per lane: a tie keeps the smaller row
                }
            } else {
                for (int i = k + lane; i < p; i += 64) {
                    if (i == c) continue;
                    const unsigned long long b = as_bits(absA(st, i, c));
                    if (b > best) { best = b; bi = i; }  // rows ascending per lane: a tie keeps the smaller row
                }
            }
            const unsigned long long mx = wave_max_u64(best);
            const unsigned long long ik = wave_max_u64(mx != 0 && best == mx ? 0xffffffffull - (unsigned)bi : 0ull);
            if (mx != 0) {
                const int r = (int)(0xffffffffull - ik);
                double gc = 0.0, gr = 0.0;
                if constexpr (kFullStore<S>) {
#pragma unroll 8
                    for (int i = k + lane; i < m; i += 64) {
                        const bool skip = i == c || i == r;
                        gc = fmax(gc, skip ? 0.0 : absA(st, i, c));
                        gr = fmax(gr, skip ? 0.0 : absA(st, i, r));
                    }
                } else {
                    for (int i = k + lane; i < m; i += 64) {
                        if (i == c || i == r) continue;
                        gc = fmax(gc, absA(st, i, c));
                        gr = fmax(gr, absA(st, i, r));
                    }
                }
                gc = wave_max_abs(gc);
                gr = wave_max_abs(gr);
                const double a = st.at(c, c);
                const double b = r > c ? st.at(r, c) : st.at(c, r);
                const double e = st.at(r, r);
                const double det = a * e - b * b;
                if (det != 0.0) {
                    const double lim = uu > 0.0 ? fabs(det) / uu : INFINITY;
                    if (fabs(e) * gc + fabs(b) * gr <= lim && fabs(b) * gc + fabs(a) * gr <= lim) {
                        d.kind = PIV_2X2_A; d.c = c; d.r = r; d.relaxed = ul > 0;
                        return d;
                    }
                }
            }
        }
    }
    return d;
}

// search_pivot for a front in LDS (PackedStore): the same decisions, with the relaxation ladder's later rungs
// evaluated candidate-parallel.  The first rung (u) runs exactly as search_pivot (its decision usually comes at
// the first or second candidate).  When every candidate fails it -- the pivot needs a relaxed threshold --
// search_pivot would rescan every candidate for each of the five remaining rungs, one after the other (the
// slowest fronts of a level, in the plugin's relaxed mode); here lane c - c0 evaluates candidate c (chunks of
// 64) once -- its column maximum g, its 2x2 partner r (the first strict maximum among the fully-summed rows,
// on the bit patterns), the partner test's maxima gc / gr, with search_pivot's expressions -- and tests it on
// every rung, and the decision is the first (rung, candidate) that passes: search_pivot's visiting order.
// The values are those the first rung saw, so minpiv is already complete (no null candidate either: the
// first rung would have taken it).
template <class S>
__device__ PivotDecision search_pivot_par(const S& st, int m, int k, int p, double u, double thres, double& minpiv) {
    const int lane = threadIdx.x & 63;
    for (int c = k; c < p; ++c) {  // the first rung (search_pivot with ul = 0)
        double g = 0.0;
        unsigned long long best = 0;
        int bi = 0x7fffffff;
        for (int i = k + lane; i < m; i += 64) {
            const double v = i == c ? 0.0 : absA(st, i, c);
            g = fmax(g, v);
            const unsigned long long bv = as_bits(v);
            if (i < p && bv > best) { best = bv; bi = i; }
        }
        g = wave_max_abs(g);
        const double acc = fabs(st.at(c, c));
        if (fmax(acc, g) <= thres) return PivotDecision{PIV_NULL, c, -1, 0};
        minpiv = fmin(minpiv, fmax(acc, g));
        if (acc != 0.0 && acc >= u * g) return PivotDecision{PIV_1X1, c, -1, 0};
        const unsigned long long mx = wave_max_u64(best);
        const unsigned long long ik = wave_max_u64(mx != 0 && best == mx ? 0xffffffffull - (unsigned)bi : 0ull);
        if (mx != 0) {
            const int r = (int)(0xffffffffull - ik);
            double gc = 0.0, gr = 0.0;
            for (int i = k + lane; i < m; i += 64) {
                const bool skip = i == c || i == r;
                gc = fmax(gc, skip ? 0.0 : absA(st, i, c));
                gr = fmax(gr, skip ? 0.0 : absA(st, i, r));
            }
            gc = wave_max_abs(gc);
            gr = wave_max_abs(gr);
            const double a = st.at(c, c);
            const double b = r > c ? st.at(r, c) : st.at(c, r);
            const double e = st.at(r, r);
            const double det = a * e - b * b;
            if (det != 0.0) {
                const double lim = u > 0.0 ? fabs(det) / u : INFINITY;
                if (fabs(e) * gc + fabs(b) * gr <= lim && fabs(b) * gc + fabs(a) * gr <= lim)
                    return PivotDecision{PIV_2X2_A, c, r, 0};
            }
        }
    }
    // rungs 1..5: every candidate at once
    constexpr int NCH = 2;  // up to 128 candidates (LDS fronts: p <= m <= 128)
    unsigned ok[NCH];       // bit ul: a 1x1 (low 8 bits) / 2x2 (high 8 bits) pivot passes rung ul
    int rr[NCH];
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
        const int c = k + 64 * ch + lane;
        ok[ch] = 0u;
        rr[ch] = -1;
        if (k + 64 * ch >= p) continue;  // uniform
        const int cc = c < p ? c : k;
        double g = 0.0;
        unsigned long long best = 0;
        int bi = 0x7fffffff;
        for (int i = k; i < m; ++i) {
            const double v = i == cc ? 0.0 : absA(st, i, cc);
            g = fmax(g, v);
            const unsigned long long bv = as_bits(v);
            if (i < p && bv > best) { best = bv; bi = i; }  // rows ascending: a tie keeps the smaller row
        }
        const double acc = fabs(st.at(cc, cc));
        double gc = 0.0, gr = 0.0, a = 0.0, b = 0.0, e = 0.0, det = 0.0;
        const bool two = best != 0;
        if (two) {
            const int r = bi;
            rr[ch] = r;
            for (int i = k; i < m; ++i) {
                const bool skip = i == cc || i == r;
                gc = fmax(gc, skip ? 0.0 : absA(st, i, cc));
                gr = fmax(gr, skip ? 0.0 : absA(st, i, r));
            }
            a = st.at(cc, cc);
            b = r > cc ? st.at(r, cc) : st.at(cc, r);
            e = st.at(r, r);
            det = a * e - b * b;
        }
#pragma unroll
        for (int ul = 1; ul < 6; ++ul) {
            const double uu = ul == 1 ? u * 0.1 : ul == 2 ? u * 0.01 : ul == 3 ? 1e-6 : ul == 4 ? 1e-10 : 0.0;
            if (acc != 0.0 && acc >= uu * g) ok[ch] |= 1u << ul;
            if (two && det != 0.0) {
                const double lim = uu > 0.0 ? fabs(det) / uu : INFINITY;
                if (fabs(e) * gc + fabs(b) * gr <= lim && fabs(b) * gc + fabs(a) * gr <= lim) ok[ch] |= 0x100u << ul;
            }
        }
        if (c >= p) ok[ch] = 0u;
    }
    for (int ul = 1; ul < 6; ++ul) {
#pragma unroll
        for (int ch = 0; ch < NCH; ++ch) {
            const unsigned long long msk = __ballot(((ok[ch] | (ok[ch] >> 8)) >> ul) & 1u);
            if (msk == 0ull) continue;  // uniform
            const int w = __ffsll((long long)msk) - 1;
            const unsigned okw = (unsigned)__builtin_amdgcn_readlane((int)ok[ch], w);
            const bool is1 = (okw >> ul) & 1u;
            return PivotDecision{is1 ? PIV_1X1 : PIV_2X2_A, k + 64 * ch + w, is1 ? -1 : __builtin_amdgcn_readlane(rr[ch], w), 1};
        }
    }
    return PivotDecision{PIV_STUCK, k, -1, 0};
}

// search_pivot for the large fronts in HBM (k_big_panel_reg): the same rule and the same decisions, every
// thread of the block scanning rows (the one-wave scans cost ~15 us per column at m = 4096)
template <int T>
__device__ PivotDecision search_pivot_blk(const FullStore& st, int m, int k, int p, double u, double thres,
                                          double& minpiv, unsigned long long* red) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    auto bmax = [&](unsigned long long v) __attribute__((always_inline)) -> unsigned long long {
        v = wave_max_u64(v);
        if (lane == 0) red[wv] = v;
        __syncthreads();
        unsigned long long r = red[0];
#pragma unroll
        for (int w = 1; w < T / 64; ++w) r = umax64(r, red[w]);
        __syncthreads();
        return r;
    };
    PivotDecision d{PIV_STUCK, k, -1, 0};
    for (int ul = 0; ul < 6; ++ul) {
        const double uu = ul == 0 ? u : ul == 1 ? u * 0.1 : ul == 2 ? u * 0.01 : ul == 3 ? 1e-6 : ul == 4 ? 1e-10 : 0.0;
        for (int c = k; c < p; ++c) {
            double g = 0.0;
#pragma unroll 4
            for (int i = k + tid; i < m; i += T) g = fmax(g, i == c ? 0.0 : absA(st, i, c));
            g = as_double(bmax(as_bits(g)));
            const double acc = fabs(st.at(c, c));
            if (fmax(acc, g) <= thres) { d.kind = PIV_NULL; d.c = c; d.relaxed = ul > 0; return d; }
            minpiv = fmin(minpiv, fmax(acc, g));
            if (acc != 0.0 && acc >= uu * g) { d.kind = PIV_1X1; d.c = c; d.relaxed = ul > 0; return d; }
            unsigned long long best = 0;
            int bi = 0x7fffffff;
#pragma unroll 4
            for (int i = k + tid; i < p; i += T) {
                const unsigned long long b = i == c ? 0ull : as_bits(absA(st, i, c));
                if (b > best) { best = b; bi = i; }  // rows ascending per thread: a tie keeps the smaller row
            }
            const unsigned long long mx = bmax(best);
            const unsigned long long ik = bmax(mx != 0 && best == mx ? 0xffffffffull - (unsigned)bi : 0ull);
            if (mx != 0) {
                const int r = (int)(0xffffffffull - ik);
                double gc = 0.0, gr = 0.0;
#pragma unroll 4
                for (int i = k + tid; i < m; i += T) {
                    const bool skip = i == c || i == r;
                    gc = fmax(gc, skip ? 0.0 : absA(st, i, c));
                    gr = fmax(gr, skip ? 0.0 : absA(st, i, r));
                }
                gc = as_double(bmax(as_bits(gc)));
                gr = as_double(bmax(as_bits(gr)));
                const double a = st.at(c, c);
                const double b = r > c ? st.at(r, c) : st.at(c, r);
                const double e = st.at(r, r);
                const double det = a * e - b * b;
                if (det != 0.0) {
                    const double lim = uu > 0.0 ? fabs(det) / uu : INFINITY;
                    if (fabs(e) * gc + fabs(b) * gr <= lim && fabs(b) * gc + fabs(a) * gr <= lim) {
                        d.kind = PIV_2X2_A; d.c = c; d.r = r; d.relaxed = ul > 0;
                        return d;
                    }
                }
            }
        }
    }
    return d;
}

// sym_swap for a front in HBM: eight positions per thread loaded before any is stored (the positions are
// distinct), instead of one dependent load/store round trip after the other
template <int NT>
__device__ void sym_swap_batched(const FullStore& st, int m, int a, int b, int32_t* lrow, int32_t* lorig) {
    for (int t0 = threadIdx.x; t0 < m; t0 += 8 * NT) {
        int p1[8], p2[8];
        double v1[8], v2[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int t = t0 + q * NT;
            p1[q] = -1; p2[q] = -1;
            if (t >= m || t == b) continue;
            if (t < a) { p1[q] = st.idx(a, t); p2[q] = st.idx(b, t); }
            else if (t == a) { p1[q] = st.idx(a, a); p2[q] = st.idx(b, b); }
            else if (t < b) { p1[q] = st.idx(t, a); p2[q] = st.idx(b, t); }
            else { p1[q] = st.idx(t, a); p2[q] = st.idx(t, b); }
        }
#pragma unroll
        for (int q = 0; q < 8; ++q)
            if (p1[q] >= 0) { v1[q] = st.F[p1[q]]; v2[q] = st.F[p2[q]]; }
#pragma unroll
        for (int q = 0; q < 8; ++q)
            if (p1[q] >= 0) { st.F[p1[q]] = v2[q]; st.F[p2[q]] = v1[q]; }
    }
    if (threadIdx.x == 0) {
        int32_t y = lrow[a]; lrow[a] = lrow[b]; lrow[b] = y;
        y = lorig[a]; lorig[a] = lorig[b]; lorig[b] = y;
    }
}

// Fast path of the same rule for the first candidate (c = k): every lane tests its own entries
// u*|a_ik| <= |a_kk| and one ballot decides; equivalent to search_pivot's first 1x1 acceptance
// (|a_kk| > thres excludes the null case, so fmax(|a_kk|, g) > thres).  Run by one full wave.
template <class S>
__device__ __forceinline__ bool quick_1x1(const S& st, int m, int k, double u, double thres) {
    const int lane = threadIdx.x & 63;
    const double akk = fabs(st.at(k, k));
    bool bad = !(akk > thres);
    for (int i = k + 1 + lane; i < m; i += 64) bad |= u * fabs(st.at(i, k)) > akk;
    return __ballot(bad) == 0;
}

// symmetric interchange of positions a < b (lower-triangle storage), all threads
template <int NT, class S>
__device__ void sym_swap(const S& st, int m, int a, int b, int32_t* lrow, int32_t* lorig) {
    for (int t = threadIdx.x; t < m; t += NT) {
        if (t < a) {
            double x = st.at(a, t); st.at(a, t) = st.at(b, t); st.at(b, t) = x;
        } else if (t == a) {
            double x = st.at(a, a); st.at(a, a) = st.at(b, b); st.at(b, b) = x;
            int32_t y = lrow[a]; lrow[a] = lrow[b]; lrow[b] = y;
            y = lorig[a]; lorig[a] = lorig[b]; lorig[b] = y;
        } else if (t < b) {
            double x = st.at(t, a); st.at(t, a) = st.at(b, t); st.at(b, t) = x;
        } else if (t > b) {
            double x = st.at(t, a); st.at(t, a) = st.at(t, b); st.at(t, b) = x;
        }
    }
}

// Schur update of the trailing lower triangle after a 1x1 (TWO=false) or 2x2 pivot at k.
// G x G thread grid, MR row/column blocks per thread, operand columns cached in registers.
template <int G, int MR, bool TWO, class S>
__device__ __forceinline__ void schur_update_tile(const S& st, int m, int k, double d0, double d1, double d2) {
    const int ty = threadIdx.x / G, tx = threadIdx.x % G;
    const int r0 = k + (TWO ? 2 : 1);
    // number of G-row blocks of the trailing triangle: wave-uniform, so the unrolled loops below
    // branch out (s_cbranch) instead of issuing masked-off work for empty blocks
    const int nb = (m - r0 + G - 1) / G;
    // Branch-free element access: a lane outside the triangle reads/writes the trash slot st.F[-1]
    // (reserved in the LDS layout); guarded accesses would compile to one divergent branch per
    // element and serialise every LDS access with its full latency.
    double ci0[MR], ci1[MR], lj0[MR], lj1[MR];
    int rb[MR];  // offset of A(i, 0) for this thread's rows (one multiply per row, not per element)
#pragma unroll
    for (int a = 0; a < MR; ++a) {
        if (a >= nb) break;
        const int i = r0 + ty + G * a;
        const int j = r0 + tx + G * a;
        rb[a] = st.idx(i, 0);
        const int ai = i < m ? rb[a] + k : -1;
        const int aj = j < m ? st.idx(j, k) : -1;
        ci0[a] = st.F[ai];
        const double x0 = st.F[aj];
        double x1 = 0.0;
        if (TWO) {
            ci1[a] = st.F[i < m ? ai + 1 : -1];
            x1 = st.F[j < m ? aj + 1 : -1];
        }
        if (TWO) {  // [l0 l1] = [x0 x1] * inv([[d0 d1][d1 d2]]) with d pre-divided by det
            lj0[a] = d2 * x0 - d1 * x1;
            lj1[a] = d0 * x1 - d1 * x0;
        } else {
            lj0[a] = x0 * d0;  // d0 = 1/pivot
            lj1[a] = 0.0;
        }
    }
    // per row block: all reads, then FMAs, then writes (reads issue back to back)
#pragma unroll
    for (int a = 0; a < MR; ++a) {
        if (a >= nb) break;
        const int i = r0 + ty + G * a;
        int addr[MR];
        double acc[MR];
#pragma unroll
        for (int b = 0; b <= a; ++b) {
            const int j = r0 + tx + G * b;
            addr[b] = (i < m && j <= i) ? rb[a] + j : -1;
            acc[b] = st.F[addr[b]];
        }
#pragma unroll
        for (int b = 0; b <= a; ++b) {
            double upd = ci0[a] * lj0[b];
            if (TWO) upd += ci1[a] * lj1[b];
            acc[b] -= upd;
        }
#pragma unroll
        for (int b = 0; b <= a; ++b) st.F[addr[b]] = acc[b];
    }
}

// generic Schur update, any m (fronts in HBM scratch)
template <int G, bool TWO, class S>
__device__ void schur_update_generic(const S& st, int m, int k, double d0, double d1, double d2) {
    const int ty = threadIdx.x / G, tx = threadIdx.x % G;
    const int r0 = k + (TWO ? 2 : 1);
    for (int i = r0 + ty; i < m; i += G) {
        const double a0 = st.at(i, k);
        const double a1 = TWO ? st.at(i, k + 1) : 0.0;
        for (int j = r0 + tx; j <= i; j += G) {
            const double x0 = st.at(j, k);
            double upd;
            if (TWO) {
                const double x1 = st.at(j, k + 1);
                upd = a0 * (d2 * x0 - d1 * x1) + a1 * (d0 * x1 - d1 * x0);
            } else {
                upd = a0 * (x0 * d0);
            }
            st.at(i, j) -= upd;
        }
    }
}


// ---- register-resident Schur complement (LDS fronts, m <= G*MR) ----
// Thread (ty, tx) of a G x G grid owns A(i, j), i = ty + G a, j = tx + G b, b <= a < MR.  A pivot
// step publishes column k to an LDS vector, tests the pivot (one ballot per wave) and applies the
// rank-1 update in registers: two LDS round trips per step instead of one per row block.  Steps
// that need the full search (swaps, 2x2, null pivots) spill to the packed LDS front, run the
// LDS code path, and reload; both paths do the same arithmetic on the same values.
template <int G, int MR, class S>
__device__ __forceinline__ void reg_load(const S& st, int m, double (&R)[MR][MR]) {
    int ty = threadIdx.x / G, tx = threadIdx.x % G;
    // opaque coordinates: keeps the 36 element addresses from being hoisted into live registers
    // across the whole pivot loop (this runs once per front plus once per fallback step)
    asm volatile("" : "+v"(ty), "+v"(tx));
#pragma unroll
    for (int a = 0; a < MR; ++a) {
        const int i = ty + G * a;
#pragma unroll
        for (int b = 0; b <= a; ++b) {
            const int j = tx + G * b;
            const bool in = i < m && j <= i;
            const double v = st.F[in ? st.idx(i, j) : -1];
            // padding rows (i >= m) and the upper-triangle slots of diagonal blocks hold 0: the one-wave
            // pivot step then needs no row-validity masks (a zero row never fails the test, publishes 0
            // and is updated by 0)
            R[a][b] = in ? v : 0.0;
        }
    }
}

template <int G, int MR, class S>
__device__ __forceinline__ void reg_store(const S& st, int m, const double (&R)[MR][MR]) {
    int ty = threadIdx.x / G, tx = threadIdx.x % G;
    // opaque coordinates: keeps the 36 element addresses from being hoisted into live registers
    // across the whole pivot loop (this runs once per front plus once per fallback step)
    asm volatile("" : "+v"(ty), "+v"(tx));
#pragma unroll
    for (int a = 0; a < MR; ++a) {
        const int i = ty + G * a;
#pragma unroll
        for (int b = 0; b <= a; ++b) {
            const int j = tx + G * b;
            st.F[(i < m && j <= i) ? st.idx(i, j) : -1] = R[a][b];
        }
    }
}

// contribution block of a register-path front straight from the registers: element (i, j), p <= j <= i < m,
// row-major packed lower triangle of order m - p (SC1: write-through stores for the dataflow hand-off)
template <int G, int RM, bool SC1>
__device__ __forceinline__ void write_cb_regs(const double (&R)[RM][RM], int m, int p, double* cb) {
    if (m - p <= 0) return;
    const int ty = threadIdx.x / G, tx = threadIdx.x % G;
#pragma unroll
    for (int a = 0; a < RM; ++a) {
        const int i = ty + G * a;
        if (G * (a + 1) <= p) continue;  // uniform: block entirely in the pivot rows
#pragma unroll
        for (int b = 0; b <= a; ++b) {
            const int j = tx + G * b;
            if (i < m && j >= p && j <= i) {
                double* dst = cb + ((i - p) * (i - p + 1)) / 2 + (j - p);
                if (SC1) st_sc1(dst, R[a][b]);
                else *dst = R[a][b];
            }
        }
    }
}

// null-pivot threshold eps * null_fac * ||A_pre||_inf.  With anorm_bits == nullptr the norm is still being computed
// on a second stream: the front is factored with threshold 0 and records the smallest pivot magnitude it accepted
// (minpiv), which the host checks against the exact threshold.  The kernels load it at their start: read inside
// factor_front (behind the assembly's barriers) it put one global round trip before every front's first pivot.
__device__ __forceinline__ double front_thres(const FactorArgs& A) {
    return A.anorm_bits ? DBL_EPSILON * A.null_fac * as_double(*A.anorm_bits) : 0.0;
}

struct FrontShared {
    PivotDecision dec;
    int stuck;
    int failk;  // register path, several waves: last step whose quick pivot test failed in some wave
};

// Factor one front (lower triangle in st), fully-summed columns 0..p-1.
// Writes L (packed trapezoid), pivot kinds, permuted row ids, CB, inertia counters.
// thres: the null-pivot threshold eps * null_fac * ||A_pre||_inf (front_thres), loaded by the caller at kernel start
template <int NT, int MR, bool DF, class S>
__device__ void factor_front(const S& st, int m, int p, int32_t* lrow, int32_t* lorig, int8_t* piv,
                             double* coefA, double* coefB, const FactorArgs& A, int f, FrontShared* sh, const double thres) {
    const int tid = threadIdx.x;
    for (int i = tid; i < m; i += NT) lorig[i] = i;  // local position before pivoting
    __syncthreads();
    double minpiv = INFINITY;
    long long npos = 0, nneg = 0, nzero = 0, n2 = 0, nrel = 0, nstuck = 0;
    int nlds = 0;  // steps through the LDS path (search / interchanges / 2x2 / null)
    bool delays_recorded = false;
    // diagnostics (stamps build path only): shader-clock cycles spent in search / update / rest
    unsigned long long cyc_search = 0, cyc_update = 0, cyc_rest = 0, t_mark = 0;
    // per-step cycle counters only in a build with UKKT_STEP_STAMPS (a runtime flag costs VALU / SALU in every
    // pivot step); the phase stamps (assembly / loop / write-out) need no flag here
#ifdef UKKT_STEP_STAMPS
    const bool stamping = A.stamps != nullptr && A.stamp_mode != 7 && A.stamp_mode != 9;  // MODE 9: phases only
    const bool st8 = A.stamps != nullptr && A.stamp_mode == 8;  // LDS-path steps by phase (stamps.py MODE=8)
#else
    constexpr bool stamping = false;
    constexpr bool st8 = false;
#endif
    unsigned long long ls_spill = 0, ls_search = 0, ls_upd = 0, ls_reload = 0, t8 = 0;
#ifdef UKKT_STEP_STAMPS
    // MODE=9 (stamps build): shader cycles of reg_load, the pivot loop, the early contribution block + drain, and
    // the bookkeeping + L write after it
    const bool st9 = A.stamps != nullptr && A.stamp_mode == 9;
#else
    constexpr bool st9 = false;
#endif
    unsigned long long t9[5] = {0, 0, 0, 0, 0};
    if (st9) t9[0] = __builtin_amdgcn_s_memtime();
    // MODE 10 (any build): the same phase boundaries on the 100 MHz real-time clock, no per-step code
    const bool st10 = A.stamps != nullptr && A.stamp_mode == 10;
    unsigned long long r10[4] = {0, 0, 0, 0};
    int k = 0;
    constexpr bool REG = MR > 0;
    constexpr int RM = MR > 0 ? MR : 1;
    constexpr int G = kGrid<NT>;
    constexpr int W = NT / 64;
    // register-resident path (see reg_load): the loop over column blocks is unrolled so the owner
    // registers of column k (block k/G) are static; a step that fails the quick test spills, runs
    // the LDS step below (search, interchanges, 1x1/2x2/null, Schur update) and reloads
    double R[RM][RM];
    double* colv = coefB;  // free until the write-out
    // one-wave register path: the published column gets its own G * RM doubles after the piv bytes (the
    // slack factor_lds_bytes reserves), so padding rows can be stored unmasked
    double* colw = coefB + 2 * m + (m + 7) / 8 + 1;
    // one-wave register path: columns whose L was written during the pivot loop (wave-uniform);
    // cleared by any later symmetric interchange (their rows moved: rewritten from LDS at the end)
    unsigned long long fastmask = 0;
    // one-wave register path: the steps it took (never cleared) and which of them had a negative pivot --
    // their pivot kinds and inertia counts are written once after the loop instead of per step
    unsigned long long fastpiv = 0, fastneg = 0;  // columns < 64 (one-wave fronts pivot at most 72 columns)
    bool spilled = false;  // some step ran the LDS path: the LDS front is current after the loop
    double* Lf = A.L + A.L_off[f];
    if constexpr (REG) {
        if (W > 1 && tid == 0) sh->failk = -1;
        reg_load<G, RM>(st, m, R);
    }
    if (st9) { __builtin_amdgcn_s_waitcnt(0); t9[1] = __builtin_amdgcn_s_memtime(); }
    if (st10) { __builtin_amdgcn_s_waitcnt(0); r10[0] = __builtin_amdgcn_s_memrealtime(); }
    // one-wave register path: the front is current in LDS only -- the step after an LDS step failed the same test
    // (quick_1x1 on the LDS front, the register path's test restated), so it runs in LDS without the reload and the
    // spill between (~3 300 shader cycles per step on the delayed-column fronts, whose LDS steps come in runs)
    bool in_lds = false;
    while (k < p) {
        if constexpr (REG && W == 1) {
          if (!in_lds) {
            // One wave owns the whole front (m <= G * RM): column k lives in register R[.][k / G] of
            // the lanes with tx = k % G.  Those lanes test it in place (one compare per row block,
            // one ballot) and publish it to an LDS vector (one store per block) that every lane reads
            // back as its row / column operands (wave_lds_sync between: no workgroup barrier); the rank-1 update
            // stays in registers.  Rows <= k of column k are never read back (upper-triangle register
            // slots are scratch) and column k itself is left untouched, so L is written from the
            // registers after the loop.
            const int ty = tid / G, tx = tid % G;
            bool need = false;
#pragma unroll
            for (int bk = 0; bk < RM; ++bk) {
                while (!need && k < p && k / G == bk) {
                    if (stamping) t_mark = __builtin_amdgcn_s_memtime();
                    const int kk = k - G * bk;
                    const bool owner = tx == kk;
                    const double akk = readlane_d(R[bk][bk], kk * G + kk);
                    const double aak = fabs(akk);
                    // the owners (tx == kk) publish column k (padding rows are 0: stored as is); every lane then
                    // reads back its row / column operands and tests ONE candidate row of the column (lane i: row i,
                    // and row i + 64 in the 72-row kernels): "some u |a_ik| > |a_kk|, i > k" with the same products
                    // and compares as the oracle's test, one ballot.  The test costs two VALU instructions instead of
                    // a multiply, a compare and a count per row block in the owner lanes, and the division above
                    // runs under the LDS round trip instead of after the ballot.
                    wave_lds_sync();  // the previous step's reads of colw are done before it is rewritten
                    if (owner) {
#pragma unroll
                        for (int a = bk; a < RM; ++a) colw[ty + G * a] = R[a][bk];
                    }
                    // publish -> read-back across lanes: explicit (see wave_lds_sync; without it the compiler may
                    // legally run the non-owners' reads before the owners' stores)
                    wave_lds_sync();
                    // rows < G * bk of colw are stale (earlier steps) but <= k: excluded by the row test.  The test's
                    // reads go first and are unconditional (no branch, no wait for the operand reads behind them)
                    constexpr int NR = G * RM;
                    const double t0 = colw[NR >= 64 ? tid : (tid < NR ? tid : 0)];
                    const double t1 = NR > 64 ? colw[64 + (tid < NR - 64 ? tid : 0)] : 0.0;
                    double lv[RM], cw[RM];
#pragma unroll
                    for (int a = bk; a < RM; ++a) {
                        lv[a] = colw[ty + G * a];
                        cw[a] = colw[tx + G * a];
                    }
                    // the division is computed before the ballot (not sunk into the pivot branch): it runs under the
                    // LDS round trip
                    double dinv = 1.0 / akk;
                    asm volatile("" : "+v"(dinv));
                    // the candidate's product, 0 for rows that are not candidates (0 > aak never holds): one DP compare
                    // feeds the ballot directly
                    double tv = ((tid > k) & (tid < NR)) ? A.u * fabs(t0) : 0.0;
                    if constexpr (NR > 64) {
                        const double tv1 = ((tid < NR - 64) & (tid + 64 > k)) ? A.u * fabs(t1) : 0.0;
                        tv = fmax(tv, tv1);  // max: "either exceeds aak" (tv1 is never NaN-vs-number ambiguous: |x| * u)
                    }
                    need = (__ballot(tv > aak) != 0) || !(aak > thres);
                    if (stamping) { unsigned long long t = __builtin_amdgcn_s_memtime(); cyc_search += t - t_mark; t_mark = t; }
                    if (!need) {  // 1x1 pivot at k without interchange (k < 64: its |a_kk| enters minpiv after the loop)
                        double cv[RM];
#pragma unroll
                        for (int a = bk; a < RM; ++a) cv[a] = cw[a] * dinv;
                        if (tx <= kk) cv[bk] = 0.0;  // columns <= k keep their values
#pragma unroll
                        for (int a = bk; a < RM; ++a)
#pragma unroll
                            for (int b = bk; b <= a; ++b) R[a][b] -= lv[a] * cv[b];
                        if (k < 64) {  // uniform
                            fastpiv |= 1ull << k;
                            // an accepted pivot is nonzero (|a_kk| > thres >= 0), so "not positive" is its sign bit: a
                            // scalar shift of the uniform akk (no VALU compare -> readfirstlane -> SALU hop in the step)
                            fastneg |= (as_bits(akk) >> 63) << k;
                        } else {  // columns beyond the masks (fronts of 65..72 columns after delays): per step
                            minpiv = fmin(minpiv, aak);
                            if (tid == 0) { piv[k] = PIV_1X1; if (akk > 0.0) npos++; else nneg++; }
                        }
                        fastmask |= 1ull << k;
                        if (stamping) { unsigned long long t = __builtin_amdgcn_s_memtime(); cyc_update += t - t_mark; }
                        k += 1;
                    }
                }
            }
            if (!need) break;
            spilled = true;
            if (st8) t8 = __builtin_amdgcn_s_memtime();
            reg_store<G, RM>(st, m, R);
            __syncthreads();
            if (st8) { const unsigned long long t = __builtin_amdgcn_s_memtime(); ls_spill += t - t8; t8 = t; }
          }
        } else if constexpr (REG) {
            const int ty = tid / G, tx = tid % G;
            bool need = false;
#pragma unroll
            for (int bk = 0; bk < RM; ++bk) {
                while (!need && k < p && k / G == bk) {
                    if (stamping) t_mark = __builtin_amdgcn_s_memtime();
                    const bool mine = tx == k % G;
#pragma unroll
                    for (int a = bk; a < RM; ++a) {
                        const int i = ty + G * a;
                        double* dst = (mine && i >= k && i < m) ? colv + i : st.F - 1;
                        *dst = R[a][bk];
                    }
                    __syncthreads();
                    const double akk = colv[k];
                    const int q = k + 1 + tid;
                    // unclamped reads: colv has G*RM readable entries (factor_lds_bytes slack), so
                    // each read is one base register plus an immediate offset
                    double x = colv[q < m ? q : m - 1];
                    double lv[RM], cv[RM];
#pragma unroll
                    for (int a = bk; a < RM; ++a) {
                        lv[a] = colv[ty + G * a];
                        cv[a] = colv[tx + G * a];
                    }
                    // keep the reads unconditional (all issued before the first wait): sunk under
                    // the masks below they become one divergent branch + LDS wait per element
                    asm volatile("" : "+v"(x));
#pragma unroll
                    for (int a = bk; a < RM; ++a) asm volatile("" : "+v"(lv[a]), "+v"(cv[a]));
#pragma unroll
                    for (int a = bk; a < RM; ++a) {
                        const int i = ty + G * a, j = tx + G * a;
                        lv[a] = (i > k && i < m) ? lv[a] : 0.0;
                        cv[a] = (j > k && j < m) ? cv[a] : 0.0;
                    }
                    const double aak = fabs(akk);
                    const bool bad = !(aak > thres) || (q < m && A.u * fabs(x) > aak);
                    if constexpr (W == 1) {
                        need = __ballot(bad) != 0;
                    } else {
                        // every wave tests its rows; a failing wave marks the step, a second
                        // barrier publishes the verdict (and frees colv for the next step)
                        if (__ballot(bad) != 0 && (tid & 63) == 0) sh->failk = k;
                        __syncthreads();
                        need = sh->failk == k;
                    }
                    if (stamping) { unsigned long long t = __builtin_amdgcn_s_memtime(); cyc_search += t - t_mark; t_mark = t; }
                    if (!need) {  // 1x1 pivot at k without interchange: rank-1 update in registers
                        minpiv = fmin(minpiv, aak);
                        const double dinv = 1.0 / akk;
#pragma unroll
                        for (int b = bk; b < RM; ++b) cv[b] *= dinv;
#pragma unroll
                        for (int a = bk; a < RM; ++a)
#pragma unroll
                            for (int b = bk; b <= a; ++b) R[a][b] -= lv[a] * cv[b];
                        if (tid == 0) { piv[k] = PIV_1X1; if (akk > 0.0) npos++; else nneg++; }
                        if (stamping) { unsigned long long t = __builtin_amdgcn_s_memtime(); cyc_update += t - t_mark; }
                        k += 1;
                    }
                }
            }
            if (!need) break;
            reg_store<G, RM>(st, m, R);
            __syncthreads();
        }
        if (stamping) t_mark = __builtin_amdgcn_s_memtime();
        nlds++;
        if (tid < 64) {
            PivotDecision d;
            if (!REG && quick_1x1(st, m, k, A.u, thres)) {
                d = PivotDecision{PIV_1X1, k, -1, 0};
                minpiv = fmin(minpiv, fabs(st.at(k, k)));
            } else {
                if constexpr (!kFullStore<S>) {
                    d = search_pivot_par(st, m, k, p, A.u, thres, minpiv);  // LDS fronts: p - k <= m <= 128
                } else {
                    d = search_pivot(st, m, k, p, A.u, thres, minpiv);
                }
            }
            if (tid == 0) sh->dec = d;
        }
        __syncthreads();
        if (stamping) { unsigned long long t = __builtin_amdgcn_s_memtime(); cyc_search += t - t_mark; t_mark = t; }
        if (st8) { const unsigned long long t = __builtin_amdgcn_s_memtime(); ls_search += t - t8; t8 = t; }
        PivotDecision d = sh->dec;
        if (d.kind == PIV_STUCK) { d.kind = PIV_NULL; d.c = k; }
        if (d.c != k) {
            sym_swap<NT>(st, m, k, d.c, lrow, lorig);
            __syncthreads();
            fastmask = 0;
        }
        if (d.kind == PIV_2X2_A) {
            int r = d.r == k ? d.c : d.r;
            if (r != k + 1) {
                sym_swap<NT>(st, m, k + 1, r, lrow, lorig);
                __syncthreads();
                fastmask = 0;
            }
        }
        if (tid == 0) {
            if (sh->dec.kind == PIV_STUCK) nstuck++;
            nrel += d.relaxed;
            // first pivot that needed a relaxed threshold: the columns still fully summed would be
            // delayed by MUMPS; report them (except at roots) so the host moves them to the parent
            if (d.relaxed && !delays_recorded && A.record_delays && A.fparent[f] >= 0) {
                delays_recorded = true;
                unsigned long long base = atomicAdd(&A.counters[6], (unsigned long long)(p - k));
                for (int q = k; q < p; ++q) A.delayed[base + (q - k)] = lrow[q];
            }
        }
        if (d.kind == PIV_NULL) {
            for (int i = k + 1 + tid; i < m; i += NT) st.at(i, k) = 0.0;
            if (tid == 0) { piv[k] = PIV_NULL; nzero++; }
            __syncthreads();
            k += 1;
        } else if (d.kind == PIV_1X1) {
            const double dk = st.at(k, k);
            const double dinv = 1.0 / dk;
            if (stamping) { unsigned long long t = __builtin_amdgcn_s_memtime(); cyc_rest += t - t_mark; t_mark = t; }
            // register path: the register front is dead here (reloaded after the step), so the tiled update (reads
            // batched per row block, no per-element LDS round trip) fits the fast path's VGPR budget; round 6:
            // ~9 000 shader cycles per LDS step in the generic loop, and the dataflow chain's slowest fronts are
            // the ones with ~10 such steps (delayed columns).  Same products and order: bit-identical.  (MR = 9:
            // the tile's 9 row blocks spill the 2-wave budget; generic there)
            if constexpr (REG && RM <= 8) schur_update_tile<G, RM, false>(st, m, k, dinv, 0.0, 0.0);
            else schur_update_generic<kGrid<NT>, false>(st, m, k, dinv, 0.0, 0.0);
            if (tid == 0) { piv[k] = PIV_1X1; if (dk > 0.0) npos++; else nneg++; }
            __syncthreads();
            if (stamping) { unsigned long long t = __builtin_amdgcn_s_memtime(); cyc_update += t - t_mark; t_mark = t; }
            k += 1;
        } else {  // 2x2
            const double a = st.at(k, k), b = st.at(k + 1, k), e = st.at(k + 1, k + 1);
            const double det = a * e - b * b;
            const double idet = 1.0 / det;
            if constexpr (REG && RM <= 8) schur_update_tile<G, RM, true>(st, m, k, a * idet, b * idet, e * idet);
            else schur_update_generic<kGrid<NT>, true>(st, m, k, a * idet, b * idet, e * idet);
            if (tid == 0) {
                piv[k] = PIV_2X2_A; piv[k + 1] = PIV_2X2_B; n2++;
                if (det < 0.0) { npos++; nneg++; }
                else if (a + e > 0.0) npos += 2;
                else nneg += 2;
            }
            __syncthreads();
            k += 2;
        }
        if (st8) { const unsigned long long t = __builtin_amdgcn_s_memtime(); ls_upd += t - t8; t8 = t; }
        if constexpr (REG && W == 1) {
            in_lds = k < p && !quick_1x1(st, m, k, A.u, thres);  // uniform (ballot)
            if (!in_lds) {
                reg_load<G, RM>(st, m, R);
            } else {
                // the registers are stale until the reload: tell the compiler (no value to keep across the LDS steps)
#pragma unroll
                for (int a = 0; a < RM; ++a)
#pragma unroll
                    for (int b = 0; b < RM; ++b) R[a][b] = __builtin_nondeterministic_value(R[a][b]);
            }
        } else if constexpr (REG) {
            reg_load<G, RM>(st, m, R);
        }
        if (st8) { const unsigned long long t = __builtin_amdgcn_s_memtime(); ls_reload += t - t8; t8 = t; }
    }
    // dataflow kernel, one wave: the contribution block -- all the parent waits for -- is stored first, straight
    // from the registers, and the parent signalled after ITS stores drain; L, the row maps and the counters follow
    // (nothing in this launch reads them), so their stores (and the pivot bookkeeping below) no longer delay the hand-off up the tree
    constexpr bool kEarlyCb = DF && REG && W == 1;
    if (st9) t9[2] = __builtin_amdgcn_s_memtime();
    if (st10) r10[1] = __builtin_amdgcn_s_memrealtime();
    if constexpr (kEarlyCb) {
        write_cb_regs<G, RM, true>(R, m, p, A.cb + A.cb_off[f]);
        drain_stores();
        if (tid == 0 && A.fparent[f] >= 0)
            __hip_atomic_fetch_add(A.df_cnt + A.fparent[f], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (A.stamps && A.stamp_mode == 11 && tid == 0) A.stamps[8 * f + 5] = __builtin_amdgcn_s_memrealtime();  // signalled
    }
    if (st9) t9[3] = __builtin_amdgcn_s_memtime();
    if (st10) r10[2] = __builtin_amdgcn_s_memrealtime();
    if constexpr (REG && W == 1) {
        // pivot kinds and inertia counts of the register path's 1x1 steps (recorded as bit masks in the loop)
        if ((fastpiv >> (tid & 63)) & 1) piv[tid & 63] = PIV_1X1;
        if (tid == 0) {
            npos += __popcll(fastpiv & ~fastneg);
            nneg += __popcll(fastneg);
        }
        // and the smallest of their |a_kk|: a pivoted column is never updated again, so its diagonal is still the
        // pivot (R[b][b] of the lanes tx == ty); one wave minimum instead of one fmin per step
        if (fastpiv) {
            const int ty = tid / G, tx = tid % G;
            unsigned long long mn = ~0ull;
#pragma unroll
            for (int b = 0; b < RM; ++b) {
                const int j = tx + G * b;
                if (ty == tx && j < 64 && ((fastpiv >> j) & 1)) mn = umin64(mn, as_bits(fabs(R[b][b])));
            }
            mn = wave_min_u64(mn);
            if (mn != ~0ull) minpiv = fmin(minpiv, as_double(mn));
        }
    }
    if constexpr (REG) {
        if (W > 1 || spilled) {  // the write-out below reads the LDS front
            reg_store<G, RM>(st, m, R);
            __syncthreads();
        }
    }
    if constexpr (REG && W == 1) {
        // L of the columns pivoted by the register path: column j (< p) still holds A(i, j) as it
        // was at step j, so L(i, j) = A(i, j) / d_j and L(j, j) = d_j, stored straight from the
        // registers (for a fixed register, the 8 lanes of a column group write 8 consecutive rows)
        if (fastmask) {
            const int ty = tid / G, tx = tid % G;
#pragma unroll
            for (int b = 0; b < RM; ++b) {
                if (G * b >= p) break;  // uniform
                const int j = tx + G * b;
                const double dj = bperm_d(R[b][b], tx * (G + 1));  // A(j, j): lane (tx, tx)
                const bool colok = j < p && ((fastmask >> (j & 63)) & 1);
                const double djinv = 1.0 / dj;
                double* Lj = Lf + (int64_t)j * m - (int64_t)j * (j - 1) / 2 - j;  // L(i, j) = Lj[i]
#pragma unroll
                for (int a = b; a < RM; ++a) {
                    const int i = ty + G * a;
                    if (colok && i >= j && i < m) Lj[i] = i == j ? dj : R[a][b] * djinv;
                }
            }
        }
    }
    // columns still to be written from the LDS front (all when no register path ran)
    const bool lds_L = !(REG && W == 1) || fastmask != (p >= 64 ? ~0ull : ((1ull << p) - 1));
    const bool sub = A.stamps && A.stamp_mode == 2 && tid == 0;
    if (st9) { __builtin_amdgcn_s_waitcnt(0); t9[4] = __builtin_amdgcn_s_memtime(); }
    if (A.stamps && tid == 0) {
        A.stamps[8 * f + 2] = __builtin_amdgcn_s_memrealtime();
        if (st9) {
            for (int q = 0; q < 4; ++q) A.stamps[8 * f + 4 + q] = t9[q + 1] - t9[q];
        } else if (A.stamp_mode == 11) {
            // [4], [5], [6] written above
        } else if (st10) {
            A.stamps[8 * f + 4] = r10[0];
            A.stamps[8 * f + 5] = r10[1];
            A.stamps[8 * f + 6] = r10[2];
            A.stamps[8 * f + 7] = (unsigned long long)p;
        } else if (st8) {
            A.stamps[8 * f + 4] = ls_spill;
            A.stamps[8 * f + 5] = ls_search;
            A.stamps[8 * f + 6] = ls_upd;
            A.stamps[8 * f + 7] = ((unsigned long long)nlds << 40) | (ls_reload & 0xffffffffffull);
        } else if (!sub && A.stamp_mode != 4) {
            A.stamps[8 * f + 4] = cyc_search;
            A.stamps[8 * f + 5] = cyc_update;
            A.stamps[8 * f + 6] = cyc_rest;
            A.stamps[8 * f + 7] = (unsigned long long)p;
        }
    }
    // ---- write L: packed lower trapezoid, column j rows j..m-1 ----
    // per-column coefficients first (one division per column, not per entry):
    // L(i,j) = cA[j] * A(i,base) + cB[j] * A(i,base+1), base = j (1x1, 2x2 first) or j-1 (2x2 second)
    for (int j = tid; j < p && lds_L; j += NT) {
        const int8_t kind = piv[j];
        double ca = 0.0, cbv = 0.0;
        if (kind == PIV_1X1) {
            ca = 1.0 / st.at(j, j);
        } else if (kind == PIV_2X2_A || kind == PIV_2X2_B) {
            const int k0 = kind == PIV_2X2_A ? j : j - 1;
            const double a = st.at(k0, k0), b = st.at(k0 + 1, k0), e = st.at(k0 + 1, k0 + 1);
            const double idet = 1.0 / (a * e - b * b);
            if (kind == PIV_2X2_A) { ca = e * idet; cbv = -b * idet; }
            else { ca = -b * idet; cbv = a * idet; }
        }
        coefA[j] = ca;
        coefB[j] = cbv;
    }
    __syncthreads();
    if (sub) A.stamps[8 * f + 4] = __builtin_amdgcn_s_memrealtime();
    double* L = Lf;
    if (!lds_L) {
        // every column was written by the register path
    } else if (NT == 64 && m <= 64) {
        // one wave, m <= 64: column j is one coalesced store, lane = row offset from the diagonal.
        // Per-column data lives in lane j and is broadcast with readlane (scalar, uniform control).
        const int mykind = tid < p ? (int)piv[tid] : 0;
        const double myca = tid < p ? coefA[tid] : 0.0, mycb = tid < p ? coefB[tid] : 0.0;
        int64_t cs = 0;  // start of column j
        for (int j0 = 0; j0 < p; j0 += 4) {
            double v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int j = j0 + u < p ? j0 + u : p - 1;
                const int kind = __builtin_amdgcn_readlane(mykind, j);
                const double ca = readlane_d(myca, j), cb2 = readlane_d(mycb, j);
                const int base = kind == PIV_2X2_B ? j - 1 : j;
                const int i = j + tid;
                const int ii = i < m ? i : m - 1;
                const int rs = (ii * (ii + 1)) >> 1;
                const double x0 = st.F[rs + base];
                const double x1 = st.F[rs + (base + 1 <= ii ? base + 1 : base)];
                const double dj = st.F[((j * (j + 1)) >> 1) + j];
                double w = ca * x0;
                if (kind >= PIV_2X2_A) w += cb2 * x1;  // uniform
                if (i == j) w = kind == PIV_NULL ? 0.0 : dj;
                else if (kind == PIV_2X2_A && i == j + 1) w = x0;  // D off-diagonal A(j+1, j)
                v[u] = w;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int j = j0 + u;
                if (j < p) {  // uniform
                    if (j + tid < m && !((fastmask >> j) & 1)) L[cs + tid] = v[u];
                    cs += m - j;
                }
            }
        }
    } else {
        const int64_t total = (int64_t)p * m - (int64_t)p * (p - 1) / 2;
        int j = 0;
        int64_t cs = 0;  // start of column j
#pragma unroll 4
        for (int64_t t = tid; t < total; t += NT) {
            while (t >= cs + (m - j)) { cs += m - j; ++j; }
            const int i = j + (int)(t - cs);
            const int8_t kind = piv[j];
            double v;
            if (i == j) {
                v = kind == PIV_NULL ? 0.0 : st.at(j, j);
            } else if (kind == PIV_2X2_A && i == j + 1) {
                v = st.at(j + 1, j);  // D off-diagonal
            } else {
                const int base = kind == PIV_2X2_B ? j - 1 : j;
                v = coefA[j] * st.at(i, base);
                if (kind >= PIV_2X2_A) v += coefB[j] * st.at(i, base + 1);
            }
            L[t] = v;
        }
    }
    if (sub) A.stamps[8 * f + 5] = __builtin_amdgcn_s_memrealtime();
    // ---- permuted row ids and pivot kinds ----
    for (int i = tid; i < m; i += NT) {
        A.frow[A.rows_off[f] + i] = lrow[i];
        A.fpos[A.rows_off[f] + lorig[i]] = i;  // analysis-order local row -> pivoted position
        if (i < p) A.piv[A.rows_off[f] + i] = piv[i];
        // one GPU, dataflow solve: the pivot's solution slot (k_xpos pass 0, written here instead)
        if (i < p && A.xpos) A.xpos[lrow[i]] = (int32_t)(A.xs_off[f] + i);
    }
    if (sub) A.stamps[8 * f + 6] = __builtin_amdgcn_s_memrealtime();
    // ---- contribution block: row-major packed lower triangle of order cm = m - p ----
    const int cm = m - p;
    if constexpr (kEarlyCb) {
        // stored above
    } else if constexpr (REG && W == 1) {
        write_cb_regs<G, RM, DF>(R, m, p, A.cb + A.cb_off[f]);
    } else if (cm > 0) {
        double* cb = A.cb + A.cb_off[f];
        const int ctot = cm * (cm + 1) / 2;
        constexpr int WB = 4;  // batch: all LDS reads, then all stores (one LDS wait per batch)
        for (int t0 = tid; t0 < ctot; t0 += WB * NT) {
            double v[WB];
#pragma unroll
            for (int u = 0; u < WB; ++u) {
                const int t = t0 + u * NT;
                int r, c;
                tri_rc(t < ctot ? t : ctot - 1, r, c);
                v[u] = st.at(p + r, p + c);
            }
#pragma unroll
            for (int u = 0; u < WB; ++u)
                if (t0 + u * NT < ctot) {
                    if (DF) st_sc1(cb + t0 + u * NT, v[u]);
                    else cb[t0 + u * NT] = v[u];
                }
        }
    }
    if (sub) A.stamps[8 * f + 7] = __builtin_amdgcn_s_memrealtime();
    if (tid == 0) {
        A.fstat[f] = (int32_t)((nstuck > 0xffff ? 0xffff : nstuck) | ((nrel > 0x7fff ? 0x7fff : nrel) << 16));
        if (A.fslow) A.fslow[f] = nlds;
        // per-front record instead of global atomics: thousands of fronts finishing together would
        // serialize on the counters' cache line and stall every access routed to that L2 channel
        A.fcnt[f] = (unsigned long long)npos | (unsigned long long)nneg << 16 | (unsigned long long)nzero << 32 |
                    (unsigned long long)n2 << 48;
        A.fmin[f] = minpiv;
    }
}

// assemble original entries and children contribution blocks into the (zeroed) front.
// Latency-bound (a few KB per front), so the loads are grouped into as few dependent round trips as
// possible: {rows, first entry batch, children's edge metadata} -> {scales} -> {per child: CB values
// and both relmap entries of each element together}.
// A front's offsets (scalar), and the first round trip of its assembly held in registers: the row ids and their
// scalings (rows < 2 NT: every front of the LDS kernels), the first batch of its original entries and its
// children's edge records.  asm_issue issues those loads, assemble_front_pre consumes them.  (Issuing them for the
// next front under the current front's pivot loop, in a resident-grid kernel, measured slower at C3: 1.36 / 1.25 ms
// vs 1.18 ms, 255-256 VGPRs with spills; round 3.)
struct FrontMeta {
    int m, p, c0, c1;
    int64_t ro, e0, e1;
};
__device__ __forceinline__ FrontMeta front_meta(const FactorArgs& A, int f) {
    FrontMeta r;
    r.m = A.fm[f]; r.p = A.fp[f];
    r.ro = A.rows_off[f];
    r.e0 = A.ent_off[f]; r.e1 = A.ent_off[f + 1];
    r.c0 = A.child_off[f]; r.c1 = A.child_off[f + 1];
    return r;
}
constexpr int kAsmEB = 8;
struct AsmPre {
    uint32_t lp[kAsmEB];
    double uv[kAsmEB];
    int my_cm;
    unsigned long long my_rmo, my_cbo;
    int32_t r0, r1;
    double s0, s1;
};
template <int NT>
__device__ __forceinline__ void asm_issue_entries(AsmPre& q, const FactorArgs& A, const FrontMeta& M) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int u = 0; u < kAsmEB; ++u) {
        const int64_t e = M.e0 + tid + (int64_t)u * NT;
        q.lp[u] = e < M.e1 ? A.ent_lpos[e] : 0u;
        q.uv[u] = e < M.e1 ? A.uval[e] : 0.0;
    }
}
template <int NT>
__device__ __forceinline__ void asm_issue(AsmPre& q, const FactorArgs& A, const FrontMeta& M, bool with_scale) {
    const int tid = threadIdx.x, lane = tid & 63;
    asm_issue_entries<NT>(q, A, M);
    q.my_cm = 0;
    q.my_rmo = q.my_cbo = 0;
    if (lane < M.c1 - M.c0) {
        q.my_cm = A.ch_cm[M.c0 + lane];
        q.my_rmo = (unsigned long long)A.ch_relmap_off[M.c0 + lane];
        q.my_cbo = (unsigned long long)A.ch_cb_off[M.c0 + lane];
    }
    q.r0 = tid < M.m ? A.rows[M.ro + tid] : 0;
    q.r1 = tid + NT < M.m ? A.rows[M.ro + tid + NT] : 0;
    if (with_scale) {  // per-front-row scalings (A.fscale): same round trip as the row ids
        q.s0 = tid < M.m ? A.fscale[M.ro + tid] : 0.0;
        q.s1 = tid + NT < M.m ? A.fscale[M.ro + tid + NT] : 0.0;
    }
}

template <int NT, bool DF, class S>
__device__ void assemble_front_pre(const S& st, int64_t fsize, const FrontMeta& M, int32_t* lrow, double* sloc,
                                   AsmPre& q, const FactorArgs& A, int f);

template <int NT, bool DF, class S>
__device__ void assemble_front(const S& st, int64_t fsize, int m, int p, int32_t* lrow, double* sloc, int32_t* rstage,
                               const FactorArgs& A, int f) {
    const FrontMeta M = front_meta(A, f);
    AsmPre q;
    asm_issue<NT>(q, A, M, A.fscale != nullptr);
    assemble_front_pre<NT, DF>(st, fsize, M, lrow, sloc, q, A, f);
}

template <int NT, bool DF, class S>
__device__ void assemble_front_pre(const S& st, int64_t fsize, const FrontMeta& M, int32_t* lrow, double* sloc,
                                   AsmPre& q, const FactorArgs& A, int f) {
    const int tid = threadIdx.x, lane = tid & 63;
    const int m = M.m;
    const int64_t e0 = M.e0, e1 = M.e1;
    const int c0 = M.c0, c1 = M.c1;
    constexpr int EB = kAsmEB;
    uint32_t (&lp)[EB] = q.lp;
    double (&uv)[EB] = q.uv;
    int my_cm = q.my_cm;
    unsigned long long my_rmo = q.my_rmo, my_cbo = q.my_cbo;
    if (tid < m) {
        lrow[tid] = q.r0;
        sloc[tid] = A.fscale ? q.s0 : A.scale[q.r0];
    }
    if (tid + NT < m) {
        lrow[tid + NT] = q.r1;
        sloc[tid + NT] = A.fscale ? q.s1 : A.scale[q.r1];
    }
    for (int64_t t = tid; t < fsize; t += NT) st.F[t] = 0.0;
    __syncthreads();
    const bool asm_st = A.stamps && A.stamp_mode == 4 && tid == 0;  // diagnostics: assembly sub-phases
    if (asm_st) A.stamps[8 * f + 4] = __builtin_amdgcn_s_memrealtime();
    // original entries (distinct positions, summed duplicates already packed by k_pack)
    for (int64_t eb = e0 + tid;; eb += (int64_t)EB * NT) {
#pragma unroll
        for (int q = 0; q < EB; ++q) {
            const int64_t e = eb + (int64_t)q * NT;
            const int lr = (int)(lp[q] >> 16), lc = (int)(lp[q] & 0x7fffu);
            // the oracle's multiplication order (s of the larger original id first): bit-identical entries
            const double sr = sloc[lr], sc = sloc[lc];
            const double v = (lp[q] & 0x8000u) ? sc * uv[q] * sr : sr * uv[q] * sc;
            st.F[e < e1 ? st.idx(lr, lc) : -1] = v;
        }
        const int64_t nb = eb + (int64_t)EB * NT;
        if (nb - tid >= e1) break;  // uniform
#pragma unroll
        for (int q = 0; q < EB; ++q) {
            const int64_t e = nb + (int64_t)q * NT;
            lp[q] = e < e1 ? A.ent_lpos[e] : 0u;
            uv[q] = e < e1 ? A.uval[e] : 0.0;
        }
    }
    if (asm_st) { __builtin_amdgcn_s_waitcnt(0); A.stamps[8 * f + 5] = __builtin_amdgcn_s_memrealtime(); }
    // dataflow schedule: children factored in this launch have published their contribution blocks
    if (DF && A.df_nch[f] > 0) df_wait(A.df_cnt + f, A.df_epoch * (uint32_t)A.df_nch[f], A.df_abort);
    // MODE 11 (dataflow hand-off): [4] the children's arrival seen, [6] the children assembled (below)
    if (DF && A.stamps && A.stamp_mode == 11 && tid == 0) A.stamps[8 * f + 4] = __builtin_amdgcn_s_memrealtime();
    // children: contribution blocks are row-major packed lower triangles (row r: columns 0..r);
    // relmap maps child CB rows to ascending parent rows, so (rm[r], rm[c]) is in the lower triangle.
    // Children are taken in pairs whose first batches are loaded together (the loads of a child are
    // one global round trip, mostly TLB / HBM latency at the upper levels); the additions are applied
    // child by child in a fixed order (deterministic sums).
    constexpr int CB = 8;  // entries per lane per batch (8: the one-wave kernels stay within 168 VGPRs, 3 waves per SIMD)
    struct Batch {
        double v[CB];
        int pos[CB];
    };
    // the entries' positions in this front, precomputed (FactorArgs::cbpos): no relmap gathers
    auto load_batch_pos = [&](const double* cb, const uint16_t* cp, int ctot, int t0, Batch& b) {
#pragma unroll
        for (int u = 0; u < CB; ++u) {
            const int t = t0 + u * NT;
            b.v[u] = t < ctot ? (DF ? ld_sc1(cb + t) : cb[t]) : 0.0;
            b.pos[u] = t < ctot ? (int)cp[t] : -1;
        }
    };
    auto load_batch = [&](const double* cb, const int32_t* rm, const uint16_t* cp, int ctot, int t0, Batch& b) {
        if (cp) {
            load_batch_pos(cb, cp, ctot, t0, b);
            return;
        }
        int32_t gi[CB], gj[CB];
#pragma unroll
        for (int u = 0; u < CB; ++u) {
            const int t = t0 + u * NT;
            int r = 0, c = 0;
            if (t < ctot) tri_rc(t, r, c);
            b.v[u] = t < ctot ? (DF ? ld_sc1(cb + t) : cb[t]) : 0.0;
            gi[u] = rm[r];
            gj[u] = rm[c];
        }
#pragma unroll
        for (int u = 0; u < CB; ++u) b.pos[u] = t0 + u * NT < ctot ? st.idx(gi[u], gj[u]) : -1;
    };
    auto add_batch = [&](const Batch& b) {
        double old[CB];
#pragma unroll
        for (int u = 0; u < CB; ++u) old[u] = st.F[b.pos[u]];
#pragma unroll
        for (int u = 0; u < CB; ++u) st.F[b.pos[u]] = old[u] + b.v[u];
    };
    for (int cb0 = c0; cb0 < c1; cb0 += 64) {
        if (cb0 != c0 && lane < c1 - cb0) {
            my_cm = A.ch_cm[cb0 + lane];
            my_rmo = (unsigned long long)A.ch_relmap_off[cb0 + lane];
            my_cbo = (unsigned long long)A.ch_cb_off[cb0 + lane];
        }
        const int nc = c1 - cb0 < 64 ? c1 - cb0 : 64;
        for (int q = 0; q < nc; q += 2) {
            const bool two = q + 1 < nc;  // uniform
            const int cma = __builtin_amdgcn_readlane(my_cm, q);
            const int cmb = two ? __builtin_amdgcn_readlane(my_cm, q + 1) : 0;
            const int32_t* rma = A.relmap + (int64_t)readlane64(my_rmo, q);
            const double* cba = A.cb + (int64_t)readlane64(my_cbo, q);
            const int32_t* rmb = A.relmap + (two ? (int64_t)readlane64(my_rmo, q + 1) : 0);
            const double* cbb = A.cb + (two ? (int64_t)readlane64(my_cbo, q + 1) : 0);
            const uint16_t* cpa = A.cbpos ? A.cbpos + (int64_t)readlane64(my_cbo, q) : nullptr;
            const uint16_t* cpb = A.cbpos && two ? A.cbpos + (int64_t)readlane64(my_cbo, q + 1) : nullptr;
            const int ta = cma > 0 ? cma * (cma + 1) / 2 : 0, tb = cmb > 0 ? cmb * (cmb + 1) / 2 : 0;
            Batch ba, bb, ba2;
            load_batch(cba, rma, cpa, ta, tid, ba);
            load_batch(cbb, rmb, cpb, tb, tid, bb);
            // the second batch of child a in flight with the first batches, and child b's second batch issued before
            // b's first is added (into a's registers, free by then): contribution blocks of up to 2 NT CB entries (63
            // rows at one wave: every one-wave front's children) no longer cost three round trips in sequence (round
            // 6: 3.0 - 3.8 us of children assembly per level of the upper-tree chain).  Three batches live at most:
            // a fourth spills the 168-VGPR kernels.
            // (the precomputed-position path only: the relmap path's loop-invariant row/column decodes of a second
            // batch, hoisted out of the children loop by the compiler, would spill)
            // (the dataflow kernel only, where the hand-off chain waits on it: the level kernels keep 4 waves per SIMD
            // at MR = 4 without the third batch)
            const bool a2 = DF && cpa && ta > NT * CB, b2 = DF && cpb && tb > NT * CB;  // uniform
            if (a2) load_batch_pos(cba, cpa, ta, NT * CB + tid, ba2);
            add_batch(ba);
            if (a2) add_batch(ba2);
            // rest of a / b: uniform loops, so the barrier below is reached by every wave; the additions stay child by
            // child, batch by batch (the same order as before)
            for (int base = (a2 ? 2 : 1) * NT * CB; base < ta; base += NT * CB) {
                load_batch(cba, rma, cpa, ta, base + tid, ba);
                add_batch(ba);
            }
            __builtin_amdgcn_sched_barrier(0);  // keep b's second batch after a's additions (a fourth live batch spills)
            if (b2) load_batch_pos(cbb, cpb, tb, NT * CB + tid, ba);
            if (NT > 64) __syncthreads();  // children may overlap: one child at a time
            add_batch(bb);
            if (b2) add_batch(ba);
            for (int base = (b2 ? 2 : 1) * NT * CB; base < tb; base += NT * CB) {
                load_batch(cbb, rmb, cpb, tb, base + tid, bb);
                add_batch(bb);
            }
            if (NT > 64) __syncthreads();
        }
    }
    __syncthreads();
    if (asm_st || (DF && A.stamps && A.stamp_mode == 11 && tid == 0)) A.stamps[8 * f + 6] = __builtin_amdgcn_s_memrealtime();
}

// LDS layout of one front: [FrontShared 32 B][packed lower m(m+1)/2, even][sloc m][coefB m]
// [lrow m][rstage/lorig m][piv m]

template <int NT, int MR, int WPE = (MR > 8 ? 2 : 3)>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(WPE))) void k_factor_lds(FactorArgs A, const int32_t* __restrict__ fronts) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    FrontShared* sh = reinterpret_cast<FrontShared*>(smem);  // first 32 B of the dynamic region
    const double thres = front_thres(A);  // issued first: in flight during the assembly
    const int f = fronts[blockIdx.x];
    const int m = A.fm[f], p = A.fp[f];
    const PackedStore st{smem + 4};
    const int64_t fsize = packed_even(m);
    double* sloc = smem + 4 + fsize;
    double* coefB = sloc + m;
    int32_t* lrow = (int32_t*)(coefB + m);
    int32_t* rstage = lrow + m;
    int8_t* pk = (int8_t*)(rstage + m);
    if (A.stamps && threadIdx.x == 0) A.stamps[8 * f + 0] = __builtin_amdgcn_s_memrealtime();
    assemble_front<NT, false>(st, fsize, m, p, lrow, sloc, rstage, A, f);
    if (A.stamps && threadIdx.x == 0) A.stamps[8 * f + 1] = __builtin_amdgcn_s_memrealtime();
    factor_front<NT, MR, false>(st, m, p, lrow, rstage, pk, sloc, coefB, A, f, sh, thres);
    if (A.stamps && threadIdx.x == 0) A.stamps[8 * f + 3] = __builtin_amdgcn_s_memrealtime();
}

// Dataflow factorization of the upper part of the assembly tree (every front one-wave, m <= 64):
// ONE launch of one block per front.  A block draws a ticket (atomic counter) when it starts and takes
// front A.df_order[ticket] (children before parents), so it only ever waits for fronts taken by blocks
// that started before it: no residency assumption, no deadlock whatever the dispatch order.  A front
// assembles its original entries, waits for its children of this launch (arrival counter, sc1 poll),
// reads their contribution blocks with sc1 loads, factors, writes its own contribution block with sc1
// stores and, after the wave's vmcnt(0), adds one to its parent's counter.  Children factored by the
// earlier level launches are complete before the launch.
template <int MR, int WPE = 3>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE))) void k_factor_df(FactorArgs A) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    FrontShared* sh = reinterpret_cast<FrontShared*>(smem);
    uint32_t tk = 0;
    if (threadIdx.x == 0) tk = __hip_atomic_fetch_add(A.df_ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    tk = (uint32_t)__builtin_amdgcn_readfirstlane((int)tk);  // lane 0 is the first active lane
    const int t = (int)(tk - (A.df_epoch - 1u) * (uint32_t)A.df_nf);  // tickets are cumulative over launches
    if (t < 0 || t >= A.df_nf) return;  // cannot happen with one block per front
    const int f = A.df_order[t];
    const double thres = front_thres(A);  // issued before the assembly: in flight under it
    const int m = A.fm[f], p = A.fp[f];
    const PackedStore st{smem + 4};
    const int64_t fsize = packed_even(m);
    double* sloc = smem + 4 + fsize;
    double* coefB = sloc + m;
    int32_t* lrow = (int32_t*)(coefB + m);
    int32_t* rstage = lrow + m;
    int8_t* pk = (int8_t*)(rstage + m);
    if (A.stamps && threadIdx.x == 0) A.stamps[8 * f + 0] = __builtin_amdgcn_s_memrealtime();
    assemble_front<64, true>(st, fsize, m, p, lrow, sloc, rstage, A, f);
    if (A.stamps && threadIdx.x == 0) A.stamps[8 * f + 1] = __builtin_amdgcn_s_memrealtime();
    factor_front<64, MR, true>(st, m, p, lrow, rstage, pk, sloc, coefB, A, f, sh, thres);  // signals the parent itself
    if (A.stamps && threadIdx.x == 0) A.stamps[8 * f + 3] = __builtin_amdgcn_s_memrealtime();
    static_assert(MR > 0, "k_factor_df runs the one-wave register path (factor_front signals the parent early)");
}

// ------------------------------------------------------------------------------------------------
// triangular solves (multifrontal, level by level)
// ------------------------------------------------------------------------------------------------

__device__ __forceinline__ int64_t colptr(int64_t L_off, int m, int k) {
    return L_off + (int64_t)k * m - (int64_t)k * (k - 1) / 2 - k;  // L(i,k) = L[colptr + i], i >= k
}

__global__ void k_rhs_scale(const double* __restrict__ b, const double* __restrict__ scale, double* __restrict__ w,
                            int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        w[i] = scale[i] * b[i];
}

__global__ void k_unscale(const double* __restrict__ w, const double* __restrict__ scale, double* __restrict__ x,
                          int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        x[i] = scale[i] * w[i];
}


// wave-wide sum (all lanes active); result wave-uniform
__device__ __forceinline__ double wave_sum(double x) {
    x += as_double(dpp64<0xB1>(as_bits(x)));
    x += as_double(dpp64<0x4E>(as_bits(x)));
    x += as_double(dpp64<0x141>(as_bits(x)));
    x += as_double(dpp64<0x140>(as_bits(x)));
    return (readlane_d(x, 0) + readlane_d(x, 16)) + (readlane_d(x, 32) + readlane_d(x, 48));
}

// stage the p x p lower triangle of the front's L panel into LDS (T[i*ldt + k] = L(i,k), k <= i < p)
__device__ __forceinline__ void stage_triangle(const double* __restrict__ L, int64_t Lo, int m, int p, double* T, int ldt) {
    for (int k = 0; k < p; ++k) {
        const double* Lk = L + colptr(Lo, m, k);
        for (int i = k + (int)threadIdx.x; i < p; i += kThreads) T[i * ldt + k] = Lk[i];
    }
}

// Forward solve of one front: y <- L^{-1} y on the front rows, z = D^{-1} y on its pivots,
// update vector of the contribution rows handed to the parent (multifrontal solve).
__global__ __launch_bounds__(kThreads) void k_solve_fwd(SolveArgs A, const int32_t* __restrict__ fronts) {
    extern __shared__ __attribute__((aligned(16))) double y[];
    const int f = fronts[blockIdx.x];
    const int m = A.fm[f], p = A.fp[f];
    const int tid = threadIdx.x;
    const int64_t ro = A.rows_off[f];
    const int8_t* piv = A.piv + ro;
    const int64_t Lo = A.L_off[f];
    const bool small = p <= 64;
    const int ldt = p | 1;
    double* T = y + ((m + 1) & ~1);
    for (int i = tid; i < m; i += kThreads) y[i] = i < p ? A.w[A.frow[ro + i]] : 0.0;
    if (small) stage_triangle(A.L, Lo, m, p, T, ldt);
    for (int ci = A.child_off[f]; ci < A.child_off[f + 1]; ++ci) {
        const int c = A.child[ci];
        const int cm = A.fm[c] - A.fp[c];
        __syncthreads();
        const int32_t* rm = A.relmap + A.relmap_off[c];
        const double* cv = A.cvec + A.relmap_off[c];
        const int32_t* fpos = A.fpos + ro;  // this front's rows were permuted by pivoting
        for (int t = tid; t < cm; t += kThreads) y[fpos[rm[t]]] += cv[t];
    }
    __syncthreads();
    if (small) {
        // triangle: one wave, lane i owns y_i, pivots broadcast by readlane (no barriers)
        if (tid < 64) {
            double yi = tid < p ? y[tid] : 0.0;
            for (int k = 0; k < p; ++k) {
                const int8_t kind = piv[k];
                if (kind == PIV_1X1) {
                    const double yk = readlane_d(yi, k);
                    if (tid > k && tid < p) yi -= T[tid * ldt + k] * yk;
                } else if (kind == PIV_2X2_A) {
                    const double y0 = readlane_d(yi, k), y1 = readlane_d(yi, k + 1);
                    if (tid > k + 1 && tid < p) yi -= T[tid * ldt + k] * y0 + T[tid * ldt + k + 1] * y1;
                    ++k;
                }
            }
            if (tid < p) y[tid] = yi;
        }
        __syncthreads();
        // rectangle: contribution rows, independent dot products
        for (int i = p + tid; i < m; i += kThreads) {
            double acc = y[i];
#pragma unroll 8
            for (int k = 0; k < p; ++k) acc -= A.L[colptr(Lo, m, k) + i] * y[k];
            y[i] = acc;
        }
    } else {
        for (int k = 0; k < p; ++k) {
            const int8_t kind = piv[k];
            if (kind == PIV_1X1) {
                const double yk = y[k];
                const double* Lk = A.L + colptr(Lo, m, k);
                for (int i = k + 1 + tid; i < m; i += kThreads) y[i] -= Lk[i] * yk;
            } else if (kind == PIV_2X2_A) {
                const double y0 = y[k], y1 = y[k + 1];
                const double* L0 = A.L + colptr(Lo, m, k);
                const double* L1 = A.L + colptr(Lo, m, k + 1);
                for (int i = k + 2 + tid; i < m; i += kThreads) y[i] -= L0[i] * y0 + L1[i] * y1;
                ++k;
            }
            __syncthreads();
        }
    }
    __syncthreads();
    // block diagonal
    for (int k = tid; k < p; k += kThreads) {
        const int8_t kind = piv[k];
        if (kind == PIV_1X1) {
            A.w[A.frow[ro + k]] = y[k] / A.L[colptr(Lo, m, k) + k];
        } else if (kind == PIV_2X2_A) {
            const double a = A.L[colptr(Lo, m, k) + k], b = A.L[colptr(Lo, m, k) + k + 1];
            const double e = A.L[colptr(Lo, m, k + 1) + k + 1];
            const double det = a * e - b * b;
            const double y0 = y[k], y1 = y[k + 1];
            A.w[A.frow[ro + k]] = (e * y0 - b * y1) / det;
            A.w[A.frow[ro + k + 1]] = (a * y1 - b * y0) / det;
        } else if (kind != PIV_2X2_B) {
            A.w[A.frow[ro + k]] = 0.0;  // null pivot contributes 0
        }
    }
    double* cv = A.cvec + A.relmap_off[f];
    for (int i = p + tid; i < m; i += kThreads) cv[i - p] = y[i];
}

// Backward solve of one front: x_k = z_k - sum_{i>k} L(i,k) x_i (struct rows are final, from ancestors).
__global__ __launch_bounds__(kThreads) void k_solve_bwd(SolveArgs A, const int32_t* __restrict__ fronts) {
    extern __shared__ __attribute__((aligned(16))) double x[];
    const int f = fronts[blockIdx.x];
    const int m = A.fm[f], p = A.fp[f];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t ro = A.rows_off[f];
    const int8_t* piv = A.piv + ro;
    const int64_t Lo = A.L_off[f];
    const bool small = p <= 64;
    const int ldt = p | 1;
    double* T = x + ((m + 1) & ~1);
    for (int i = tid; i < m; i += kThreads) x[i] = A.w[A.frow[ro + i]];
    if (small) stage_triangle(A.L, Lo, m, p, T, ldt);
    __syncthreads();
    // rectangular part: x_k -= sum_{i>=p} L(i,k) x_i, one wave per column
    for (int k = wave; k < p; k += kThreads / 64) {
        const double* Lk = A.L + colptr(Lo, m, k);
        double sum = 0.0;
        for (int i = p + lane; i < m; i += 64) sum += Lk[i] * x[i];
        sum = wave_sum(sum);
        if (lane == 0 && piv[k] != PIV_NULL) x[k] -= sum;
    }
    __syncthreads();
    if (small) {
        if (tid < 64) {
            double xj = tid < p ? x[tid] : 0.0;
            for (int k = p - 1; k >= 0; --k) {
                const int8_t kind = piv[k];
                if (kind == PIV_NULL) continue;
                const double xk = readlane_d(xj, k);
                const int skip = kind == PIV_2X2_B ? k - 1 : -1;
                if (tid < k && tid != skip && piv[tid] != PIV_NULL) xj -= T[k * ldt + tid] * xk;
            }
            if (tid < p) A.w[A.frow[ro + tid]] = xj;
        }
    } else {
        for (int k = p - 1; k >= 0; --k) {
            const int8_t kind = piv[k];
            if (kind != PIV_NULL) {
                const double xk = x[k];
                const int skip = kind == PIV_2X2_B ? k - 1 : -1;
                for (int j = tid; j < k; j += kThreads)
                    if (j != skip && piv[j] != PIV_NULL) x[j] -= A.L[colptr(Lo, m, j) + k] * xk;
            }
            __syncthreads();
        }
        for (int k = tid; k < p; k += kThreads) A.w[A.frow[ro + k]] = x[k];
    }
}

// One-wave solves for fronts with p <= 64 and m <= kMaxLdsFront (all but the rare dense fronts).
// The front's packed L panel (column k rows k..m-1, SolveArgs::L_off) is copied into LDS in one flat
// coalesced pass -- every load of the panel in flight at once instead of one round trip per column --
// and the triangle, rectangle and diagonal then run from LDS: lane i owns row i of the triangle,
// pivots are broadcast with readlane, no barriers beyond the staging one.
//
// Two schedules share the per-front bodies below:
//   level-synchronous (DF = false): one launch per level and LDS class, a block per front;
//   dataflow (DF = true): ONE launch per direction, a resident grid of one-wave blocks walking the
//     fronts in a topological order (block b takes positions b, b + grid, ...).  A front waits only
//     for fronts earlier in that order, so with every block resident (grid sized from the occupancy
//     query) the earliest unfinished front can always proceed.  Hand-offs inside the launch
//     (forward: children's update vectors; backward: ancestors' solution values) are written with
//     sc1 (write-through) stores into 128-byte-aligned per-front slots, read with sc1 loads, and
//     signalled after the storing wave's vmcnt(0) by one lane: an agent-scope add on the parent's
//     arrival counter (forward) or an sc1 epoch store (backward), polled with sc1 loads
//     (MI355X_MICROARCH.md, inter-workgroup visibility, first row of the hand-off table).
//     Every wait is bounded: past the limit the wave raises abort_flag and every waiter returns, the
//     host reports the abort and falls back to the level schedule.
__device__ __forceinline__ int pcol(int m, int k) { return k * m - k * (k - 1) / 2 - k; }  // P[pcol + i] = L(i,k)

// Panel -> LDS: 16-byte loads (after one leading double when the panel starts on an odd double), up
// to 16 per lane issued before the first LDS write.
template <int B = 16>
__device__ __forceinline__ void stage_panel(const double* __restrict__ L, int64_t Lo, int sz, double* P) {
    const int lane = threadIdx.x;
    const int head = (int)(Lo & 1) < sz ? (int)(Lo & 1) : sz;
    if (head && lane == 0) P[0] = L[Lo];
    const int npair = (sz - head) >> 1;
    if (((sz - head) & 1) && lane == 0) P[sz - 1] = L[Lo + sz - 1];
    if (npair <= 0) return;
    const double2* L2 = reinterpret_cast<const double2*>(L + Lo + head);
    
    for (int t0 = 0; t0 < npair; t0 += B * 64) {
        double2 v[B];
#pragma unroll
        for (int q = 0; q < B; ++q) {
            const int t = t0 + q * 64 + lane;
            v[q] = L2[t < npair ? t : npair - 1];  // clamped: branch-free, every load in flight
        }
#pragma unroll
        for (int q = 0; q < B; ++q) {
            const int t = t0 + q * 64 + lane;
            if (t < npair) {
                P[head + 2 * t] = v[q].x;
                P[head + 2 * t + 1] = v[q].y;
            }
        }
    }
}



// ---- per-front pieces shared by both schedules ----

// children's update vectors -> y (LDS rows, permuted by fpl); CH children's loads in flight at once
template <bool DF>
__device__ __forceinline__ void fwd_extend_add(const SolveArgs& A, const DfArgs& D, int c0, int c1, int my_cm,
                                               long long my_rmo, long long my_cxo, double* y, const int32_t* fpl) {
    const int lane = threadIdx.x;
    constexpr int CH = 4;
    for (int cb = c0; cb < c1; cb += CH) {
        if (cb != c0 && (cb - c0) % 64 == 0 && lane < c1 - cb) {  // more than 64 children: next records
            my_cm = A.ch_cm[cb + lane];
            my_rmo = A.ch_relmap_off[cb + lane];
            if (DF) my_cxo = D.ch_cvx_off[cb + lane];
        }
        double v[CH][2];
        int32_t r[CH][2];
#pragma unroll
        for (int u = 0; u < CH; ++u) {
            const int q = (cb - c0) % 64 + u;
            const bool have = cb + u < c1;  // uniform
            const int cm = have ? __builtin_amdgcn_readlane(my_cm, q) : 0;
            const int64_t off = have ? (int64_t)readlane64((unsigned long long)my_rmo, q) : 0;
            const int64_t offx = DF && have ? (int64_t)readlane64((unsigned long long)my_cxo, q) : 0;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int t = lane + 64 * h;
                if (DF) v[u][h] = t < cm ? ld_sc1(D.cvx + offx + t) : 0.0;
                else v[u][h] = t < cm ? A.cvec[off + t] : 0.0;
                r[u][h] = t < cm ? A.relmap[off + t] : -1;
            }
        }
#pragma unroll
        for (int u = 0; u < CH; ++u)  // children in order (rows of one child are distinct)
#pragma unroll
            for (int h = 0; h < 2; ++h)
                if (r[u][h] >= 0) y[fpl[r[u][h]]] += v[u][h];
    }
}

// LDS readable beyond a front's panel + rows by the unclamped operand reads of fwd/bwd_compute
constexpr int kSolveSlack = 192;  // doubles (>= p + 128 for p <= 64)

// Forward elimination of one front from LDS (panel P = packed columns, rows y), one pass over the
// pivot columns: y_k is final when step k starts, so each step updates the triangle rows (lane i owns
// y_i, i < p) AND the contribution rows (lane i owns rows p + i and p + 64 + i): one readlane
// broadcast of y_k, two or three LDS operand reads (unclamped, see kSolveSlack), two or three FMAs.
// A 2x2 pivot (k, k+1) acts as two column steps on the rows below it; a null pivot adds nothing.
template <bool DF>
__device__ __forceinline__ void fwd_compute(int m, int p, const double* P, double* y, int mypiv, double* zdst,
                                            double* cvo) {
    const int lane = threadIdx.x;
    const bool tri = lane < p;
    const bool two = m - p > 64;  // uniform
    double yi = tri ? y[lane] : 0.0;
    double a0 = p + lane < m ? y[p + lane] : 0.0;
    double a1 = two && p + 64 + lane < m ? y[p + 64 + lane] : 0.0;
    const double* pt = P + lane;      // pt[pc] = L(lane, k), pc = start of column k
    const double* pr = P + p + lane;  // pr[pc] = L(p + lane, k), pr[pc + 64] = L(p + 64 + lane, k)
    int pc = 0;
    for (int k = 0; k < p; ++k) {
        const double lt = pt[pc], l0 = pr[pc];
        const double l1 = two ? pr[pc + 64] : 0.0;
        const int kind = __builtin_amdgcn_readlane(mypiv, k);
        const bool live = kind == PIV_1X1 || kind == PIV_2X2_A || kind == PIV_2X2_B;
        const double yk = live ? readlane_d(yi, k) : 0.0;
        const int lim = kind == PIV_2X2_A ? k + 1 : k;
        const double t = yi - lt * yk;
        yi = (tri && lane > lim) ? t : yi;
        a0 -= l0 * yk;
        a1 -= l1 * yk;
        pc += m - k - 1;
    }
    if (p + lane < m) {
        if (DF) st_sc1(cvo + lane, a0);
        else cvo[lane] = a0;
    }
    if (two && p + 64 + lane < m) {
        if (DF) st_sc1(cvo + 64 + lane, a1);
        else cvo[64 + lane] = a1;
    }
    if (tri) y[lane] = yi;
    __syncthreads();  // y of the 2x2 partners below
    if (tri) {
        const int kind = mypiv;
        double out = 0.0;  // null pivot contributes 0
        if (kind == PIV_1X1) {
            out = yi / P[pcol(m, lane) + lane];
        } else if (kind == PIV_2X2_A || kind == PIV_2X2_B) {
            const int k0 = kind == PIV_2X2_A ? lane : lane - 1;
            const double a = P[pcol(m, k0) + k0], b = P[pcol(m, k0) + k0 + 1];
            const double e = P[pcol(m, k0 + 1) + k0 + 1];
            const double det = a * e - b * b;
            const double y0 = y[k0], y1 = y[k0 + 1];
            out = kind == PIV_2X2_A ? (e * y0 - b * y1) / det : (a * y1 - b * y0) / det;
        }
        *zdst = out;
    }
}

// Backward substitution of one front from LDS (panel P, x: own pivots z, contribution rows final):
// returns x_j in lane j < p.  Rectangle: lane k dots column k with the broadcast contribution rows;
// triangle: steps k = p-1 .. 0, x_k broadcast by readlane, operand L(k, lane) read unclamped.
__device__ __forceinline__ double bwd_compute(int m, int p, const double* P, const double* x, int mypiv) {
    const int lane = threadIdx.x;
    const bool tri = lane < p;
    const double* pk = P + pcol(m, tri ? lane : 0);  // pk[i] = L(i, lane), i >= lane
    double s0 = 0.0, s1 = 0.0;
    int i = p;
    for (; i + 1 < m; i += 2) {
        s0 += pk[i] * x[i];
        s1 += pk[i + 1] * x[i + 1];
    }
    if (i < m) s0 += pk[i] * x[i];
    const bool live = tri && mypiv != PIV_NULL;
    double xj = tri ? x[lane] : 0.0;
    if (live) xj -= s0 + s1;
    for (int k = p - 1; k >= 0; --k) {
        const double l = pk[k];  // L(k, lane) for lane < k (other lanes read in-bounds garbage)
        const int kind = __builtin_amdgcn_readlane(mypiv, k);
        const double xk = kind != PIV_NULL ? readlane_d(xj, k) : 0.0;
        const int skip = kind == PIV_2X2_B ? k - 1 : -1;
        const double t = xj - l * xk;
        xj = (live && lane < k && lane != skip) ? t : xj;
    }
    return xj;
}

// ---- level-synchronous schedule: one block per front ----
__global__ __launch_bounds__(64) void k_solve_fwd_w(SolveArgs A, const int32_t* __restrict__ fronts) {
    // Latency-bound per front: the global loads are grouped into three dependent round trips
    // {front record} -> {row ids, pivoted positions, pivot kinds, children's edge records, L panel}
    // -> {w at the pivot rows, children's update vectors and maps}; the rest runs from LDS/registers.
    extern __shared__ __attribute__((aligned(16))) double smem_s[];
    const int f = fronts[blockIdx.x];
    const int m = A.fm[f], p = A.fp[f];
    const int lane = threadIdx.x;
    const int64_t ro = A.rows_off[f];
    const int c0 = A.child_off[f], c1 = A.child_off[f + 1];
    const int sz = p * m - p * (p - 1) / 2;
    double* P = smem_s;
    double* y = smem_s + ((sz + 1) & ~1);
    int32_t* fpl = (int32_t*)(y + ((m + 1) & ~1));  // this front's rows were permuted by pivoting
    const int mypiv = lane < p ? (int)A.piv[ro + lane] : 0;
    int32_t fr0 = 0, fr1 = 0;
    if (lane < p) fr0 = A.frow[ro + lane];
    if (lane + 64 < p) fr1 = A.frow[ro + lane + 64];
    const int32_t fp0 = lane < m ? A.fpos[ro + lane] : 0;
    const int32_t fp1 = lane + 64 < m ? A.fpos[ro + lane + 64] : 0;
    int my_cm = 0;
    long long my_rmo = 0;
    if (lane < c1 - c0) {
        my_cm = A.ch_cm[c0 + lane];
        my_rmo = A.ch_relmap_off[c0 + lane];
    }
    stage_panel(A.L, A.L_off[f], sz, P);
    if (lane < m) { y[lane] = lane < p ? A.w[fr0] : 0.0; fpl[lane] = fp0; }
    if (lane + 64 < m) { y[lane + 64] = lane + 64 < p ? A.w[fr1] : 0.0; fpl[lane + 64] = fp1; }
    __syncthreads();
    fwd_extend_add<false>(A, DfArgs{}, c0, c1, my_cm, my_rmo, 0, y, fpl);
    __syncthreads();
    fwd_compute<false>(m, p, P, y, mypiv, A.w + fr0, A.cvec + A.relmap_off[f]);
}

__global__ __launch_bounds__(64) void k_solve_bwd_w(SolveArgs A, const int32_t* __restrict__ fronts) {
    extern __shared__ __attribute__((aligned(16))) double smem_s[];
    const int f = fronts[blockIdx.x];
    const int m = A.fm[f], p = A.fp[f];
    const int lane = threadIdx.x;
    const int64_t ro = A.rows_off[f];
    const int sz = p * m - p * (p - 1) / 2;
    double* P = smem_s;
    double* x = smem_s + ((sz + 1) & ~1);
    const int mypiv = lane < p ? (int)A.piv[ro + lane] : PIV_NULL;
    for (int i = lane; i < m; i += 64) x[i] = A.w[A.frow[ro + i]];
    stage_panel(A.L, A.L_off[f], sz, P);
    __syncthreads();
    const double xj = bwd_compute(m, p, P, x, mypiv);
    if (lane < p) A.w[A.frow[ro + lane]] = xj;
}

// ---- dataflow schedule: a resident grid walks the topological order, software-pipelined ----
// Per block, fronts t, t + grid, ...: while front t computes, the next front's record (scalar),
// row data, dependency word and (up to kPre * 128 doubles of) L panel are in flight into registers,
// including its own-pivot values: the dataflow solve works on xs, the solution vector in elimination
// order (each front's pivots contiguous in a 128-byte-aligned slot; right-hand side scattered in and
// solution gathered out by k_xs_in / k_xs_out), so a front's own values need no row-id round trip.
// A front then costs one dependent round trip (its children's / ancestors' values), its arithmetic
// and the store drain before its signal.
__device__ __forceinline__ int cstart(int m, int k) { return k * m - ((k * (k - 1)) >> 1); }  // flat index of L(k, k)
__device__ __forceinline__ int col_start(int m, int k) { return k * m - k * (k - 1) / 2; }  // flat index of L(k, k)
__device__ __forceinline__ int fwd_chunk_end(int m, int p, int k0, int win) {
    int k1 = k0, used = 0;
    while (k1 < p && used + (m - k1) <= win) { used += m - k1; ++k1; }
    return k1 > k0 ? k1 : k0 + 1;
}
__device__ __forceinline__ int bwd_chunk_begin(int m, int p, int c1, int win) {
    const int e1 = col_start(m, c1);
    int c0 = c1;
    while (c0 > 0 && e1 - col_start(m, c0 - 1) <= win) --c0;
    return c0 < c1 ? c0 : c1 - 1;
}

constexpr int kPre = 8;  // 1 024 doubles: the default panel window (solve_window) fits
struct FrontRec {
    int f, m, p, sz, par, c0, c1;
    int nw;  // children the forward walk waits for (kDescNW)
    int64_t ro, Lo;
    int64_t xoff;  // forward: cvx slot
    int64_t woff;  // xs slot (the front's pivots in elimination order)
};
struct FrontPre {
    FrontRec r;
    int w0, wlen;      // the prefetched window: flat panel range [w0, w0 + wlen), its first column window
    int kw;            // forward: end column of that window; backward: its first column
    int head, npair;
    int mypiv;
    int32_t a0, a1;    // backward: xs index (rxpos) of the contribution rows lane, lane + 64 (>= p)
    int32_t fp0, fp1;  // forward: pivoted positions of the analysis-order rows
    int my_cm;
    long long my_rmo, my_cxo;
    uint32_t dep;      // dependency word as loaded at prefetch time (sc1)
    double e0;         // xs at the own pivots (forward: scaled right-hand side; backward: z)
    double hv, tv;     // panel elements outside the 16-byte pairs (leading / trailing double)
    double2 v[kPre];
};

// A front's record lives in DfArgs::desc (16 words per walk position, kDesc* fields): one dword per
// lane, loaded a whole phase before the fields are extracted with readlane, so the load is never
// waited for alone (a uniform load consumed at once would stall the wave for a full round trip).
__device__ __forceinline__ int df_desc_load(const DfArgs& D, int pos) { return D.desc[pos * 16 + (threadIdx.x & 15)]; }
__device__ __forceinline__ FrontRec df_record(int dv) {
    auto w = [&](int k) { return __builtin_amdgcn_readlane(dv, k); };
    auto w64 = [&](int k) { return (int64_t)(((uint64_t)(uint32_t)w(k + 1) << 32) | (uint32_t)w(k)); };
    FrontRec r;
    r.f = w(kDescF);
    r.m = w(kDescM);
    r.p = w(kDescP);
    r.par = w(kDescPar);
    r.c0 = w(kDescC0);
    r.c1 = w(kDescC1);
    r.nw = w(kDescNW);
    r.ro = w64(kDescRo);
    r.Lo = w64(kDescLo);
    r.xoff = w64(kDescCvx);
    r.woff = w64(kDescXs);
    r.sz = r.p * r.m - r.p * (r.p - 1) / 2;
    return r;
}

template <bool FWD>
__device__ __forceinline__ void df_issue(const SolveArgs& A, const DfArgs& D, FrontPre& q) {
    const int lane = threadIdx.x;
    const int m = q.r.m, p = q.r.p;
    const int64_t ro = q.r.ro;
    q.mypiv = lane < p ? (int)A.piv[ro + lane] : (FWD ? 0 : (int)PIV_NULL);
    q.my_cm = 0;
    q.my_rmo = q.my_cxo = 0;
    q.fp0 = q.fp1 = 0;
    q.e0 = lane < p ? D.xs[q.r.woff + lane] : 0.0;
    if (FWD) {
        q.a0 = q.a1 = 0;
        q.fp0 = lane < m ? A.fpos[ro + lane] : 0;
        q.fp1 = lane + 64 < m ? A.fpos[ro + lane + 64] : 0;
        if (lane < q.r.c1 - q.r.c0) {
            q.my_cm = A.ch_cm[q.r.c0 + lane];
            q.my_rmo = A.ch_relmap_off[q.r.c0 + lane];
            q.my_cxo = D.ch_cvx_off[q.r.c0 + lane];
        }
        q.dep = q.r.c1 > q.r.c0 ? ld_sc1_u32(D.cnt + q.r.f) : 0u;
    } else {
        q.a0 = lane < m && lane >= p ? D.rxpos[ro + lane] : 0;
        q.a1 = lane + 64 < m && lane + 64 >= p ? D.rxpos[ro + lane + 64] : 0;
        q.dep = q.r.par >= 0 ? ld_sc1_u32(D.done + q.r.par) : 0u;
    }
    // first column window of the walk: forward columns [0, kw), backward columns [kw, p)
    if (FWD) {
        q.kw = fwd_chunk_end(m, p, 0, D.win);
        q.w0 = 0;
        q.wlen = col_start(m, q.kw);
    } else {
        q.kw = bwd_chunk_begin(m, p, p, D.win);
        q.w0 = col_start(m, q.kw);
        q.wlen = q.r.sz - q.w0;
    }
    const int64_t Lw = q.r.Lo + q.w0;
    q.head = (int)(Lw & 1) < q.wlen ? (int)(Lw & 1) : q.wlen;
    q.npair = (q.wlen - q.head) >> 1;
    const double2* L2 = reinterpret_cast<const double2*>(A.L + Lw + q.head);
    const int last = q.npair > 0 ? q.npair - 1 : 0;
    q.hv = q.head ? A.L[Lw] : 0.0;
    q.tv = ((q.wlen - q.head) & 1) ? A.L[Lw + q.wlen - 1] : 0.0;
#pragma unroll
    for (int u = 0; u < kPre; ++u) {
        const int t = u * 64 + lane;
        q.v[u] = q.npair > 0 ? L2[t < q.npair ? t : last] : make_double2(0.0, 0.0);
    }
}

// ---- panel window (DfArgs::win doubles of LDS) ----
// A front's packed panel is staged in column windows of at most `win` doubles, so the LDS per block
// is sized for the window, not for the largest panel, and more blocks fit a CU (the dataflow solve is
// bound by the number of fronts in flight).  Most panels fit one window; a larger one is processed in
// column chunks (forward: first to last, backward: last to first), its later chunks loaded from L.
// The arithmetic per lane is the same sequence of operations as fwd_compute / bwd_compute, so the
// windowed solve is bit-identical to the level schedule.
// the prefetched first window -> P[0 .. wlen) (plus the remainder beyond the prefetch, loaded here)
__device__ __forceinline__ void df_stage_window(const SolveArgs& A, const FrontPre& q, double* P) {
    const int lane = threadIdx.x;
    if (q.head && lane == 0) P[0] = q.hv;
    if (((q.wlen - q.head) & 1) && lane == 0) P[q.wlen - 1] = q.tv;
#pragma unroll
    for (int u = 0; u < kPre; ++u) {
        const int t = u * 64 + lane;
        if (t < q.npair) {
            P[q.head + 2 * t] = q.v[u].x;
            P[q.head + 2 * t + 1] = q.v[u].y;
        }
    }
    if (q.npair > kPre * 64) {
        const double2* L2 = reinterpret_cast<const double2*>(A.L + q.r.Lo + q.w0 + q.head);
        for (int t = kPre * 64 + lane; t < q.npair; t += 64) {
            const double2 v = L2[t];
            P[q.head + 2 * t] = v.x;
            P[q.head + 2 * t + 1] = v.y;
        }
    }
}

// fwd_compute over column windows: columns [0, k1) are staged at P on entry.  The diagonal blocks are
// captured from the operand reads (lane k at step k: L(k,k); lane k+1: L(k+1,k)) instead of being
// re-read from the panel after the loop.
__device__ __forceinline__ void fwd_compute_win(const double* __restrict__ L, int64_t Lo, int m, int p, double* P, int win,
                                                int k1, double* y, int mypiv, double* zdst, double* cvo) {
    const int lane = threadIdx.x;
    const bool tri = lane < p;
    const bool two = m - p > 64;  // uniform
    double yi = tri ? y[lane] : 0.0;
    double a0 = p + lane < m ? y[p + lane] : 0.0;
    double a1 = two && p + 64 + lane < m ? y[p + 64 + lane] : 0.0;
    double dg = 0.0, sb = 0.0;
    int pc = 0, base = 0, k = 0;
    for (;;) {
        for (; k < k1; ++k) {
            const int o = pc - base;
            const double lt = P[max(o + lane, 0)], l0 = P[o + p + lane];
            const double l1 = two ? P[o + p + 64 + lane] : 0.0;
            const int kind = __builtin_amdgcn_readlane(mypiv, k);
            const bool live = kind == PIV_1X1 || kind == PIV_2X2_A || kind == PIV_2X2_B;
            const double yk = live ? readlane_d(yi, k) : 0.0;
            const int lim = kind == PIV_2X2_A ? k + 1 : k;
            const double t = yi - lt * yk;
            yi = (tri && lane > lim) ? t : yi;
            a0 -= l0 * yk;
            a1 -= l1 * yk;
            dg = lane == k ? lt : dg;
            sb = lane == k + 1 ? lt : sb;
            pc += m - k - 1;
        }
        if (k >= p) break;
        base = col_start(m, k);
        k1 = fwd_chunk_end(m, p, k, win);
        __syncthreads();
        stage_panel<4>(L, Lo + base, col_start(m, k1) - base, P);
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the window's loads are all consumed here, so the
                                              // operand loop below carries no pending global load
        __syncthreads();
    }
    if (p + lane < m) st_sc1(cvo + lane, a0);
    if (two && p + 64 + lane < m) st_sc1(cvo + 64 + lane, a1);
    if (tri) y[lane] = yi;
    const double dgn = __shfl(dg, lane < 63 ? lane + 1 : lane), sbn = __shfl(sb, lane < 63 ? lane + 1 : lane);
    const double dgp = __shfl(dg, lane > 0 ? lane - 1 : 0);
    __syncthreads();  // y of the 2x2 partners below
    if (tri) {
        const int kind = mypiv;
        double out = 0.0;  // null pivot contributes 0
        if (kind == PIV_1X1) {
            out = yi / dg;
        } else if (kind == PIV_2X2_A || kind == PIV_2X2_B) {
            const bool first = kind == PIV_2X2_A;
            const int k0 = first ? lane : lane - 1;
            const double a = first ? dg : dgp, b = first ? sbn : sb, e = first ? dgn : dg;
            const double det = a * e - b * b;
            const double y0 = y[k0], y1 = y[k0 + 1];
            out = first ? (e * y0 - b * y1) / det : (a * y1 - b * y0) / det;
        }
        *zdst = out;
    }
}

// bwd_compute over column windows, last window first: columns [c0, p) are staged at P on entry.  A
// lane's updates keep their order (rectangle, then k = p-1 .. lane+1): in window [c0, c1) the lanes of
// the window take the steps k >= c1 with the final x_k of the later windows' lanes, then their own.
__device__ __forceinline__ double bwd_compute_win(const double* __restrict__ L, int64_t Lo, int m, int p, double* P, int win,
                                                  int c0, const double* x, int mypiv) {
    const int lane = threadIdx.x;
    const bool tri = lane < p;
    const bool live = tri && mypiv != PIV_NULL;
    double xj = tri ? x[lane] : 0.0;
    int c1 = p, base = col_start(m, c0);
    for (;;) {
        const bool mine = lane >= c0 && lane < c1;
        const double* pk = P + (pcol(m, mine ? lane : c0) - base);  // pk[i] = L(i, lane), i >= lane
        double s0 = 0.0, s1 = 0.0;
        int i = p;
        // four pairs' operands read before their products (one LDS wait per 8 rows instead of per 2); the
        // products accumulate in the same order as the pairwise loop below (s0: rows p, p+2, ...; s1: odd)
        for (; i + 7 < m; i += 8) {
            double a[8], b[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) { a[u] = pk[i + u]; b[u] = x[i + u]; }
#pragma unroll
            for (int u = 0; u < 8; u += 2) {
                s0 += a[u] * b[u];
                s1 += a[u + 1] * b[u + 1];
            }
        }
        for (; i + 1 < m; i += 2) {
            s0 += pk[i] * x[i];
            s1 += pk[i + 1] * x[i + 1];
        }
        if (i < m) s0 += pk[i] * x[i];
        if (live && mine) xj -= s0 + s1;
        auto step = [&](int k, double l) {
            const int kind = __builtin_amdgcn_readlane(mypiv, k);
            const double xk = kind != PIV_NULL ? readlane_d(xj, k) : 0.0;
            const int skip = kind == PIV_2X2_B ? k - 1 : -1;
            const double t = xj - l * xk;
            xj = (live && mine && lane < k && lane != skip) ? t : xj;
        };
        int k = p - 1;
        for (; k - 3 >= c0; k -= 4) {  // four steps' operands read first (the chain runs through xj only)
            double l4[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) l4[u] = pk[k - u];
#pragma unroll
            for (int u = 0; u < 4; ++u) step(k - u, l4[u]);
        }
        for (; k >= c0; --k) step(k, pk[k]);
        if (c0 == 0) break;
        c1 = c0;
        c0 = bwd_chunk_begin(m, p, c1, win);
        base = col_start(m, c0);
        __syncthreads();
        stage_panel<4>(L, Lo + base, col_start(m, c1) - base, P);
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the window's loads are all consumed here, so the
                                              // operand loop below carries no pending global load
        __syncthreads();
    }
    return xj;
}

// Round 4: the pivot-step loops of fwd_compute_win / bwd_compute_win, unrolled by 8 with the 8 steps' LDS
// operands read before the first step (no LDS latency on the dependency chain), pivot kinds as wave-uniform
// ballot masks (scalar bit tests, no branch per step), and lane = row in the forward (rows < 64 in y0,
// rows >= 64 in a1).  The per-row / per-column sequence of operations is unchanged: bit-identical results.
__device__ __forceinline__ void fwd_compute_win2(const double* __restrict__ L, int64_t Lo, int m, int p, double* P, int win,
                                                 int k1, double* y, int mypiv, double* zdst, double* cvo) {
    const int lane = threadIdx.x;
    const bool two = m > 64;  // uniform
    const unsigned long long liveM = __ballot(lane < p && mypiv != PIV_NULL);
    const unsigned long long twoAM = __ballot(lane < p && mypiv == PIV_2X2_A);
    double y0 = y[lane];
    double a1 = two && lane + 64 < m ? y[lane + 64] : 0.0;
    double dg = 0.0, sb = 0.0;
    const int csl = cstart(m, lane);                      // lane's own column start (pivot lanes)
    const int csp = lane > 0 ? cstart(m, lane - 1) : 0;   // and its predecessor's
    int base = 0, k = 0, cs = 0;                          // cs = cstart(m, k)
    for (;;) {
        while (k < k1) {
            const int kend = min(k + 8, k1);
            double l0[8], l1[8];
            int c = cs;
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int kk = k + u;
                if (kk < kend) {  // uniform
                    const int o = c - base - kk;  // P[o + i] = L(i, kk)
                    l0[u] = P[max(o + lane, 0)];
                    l1[u] = two ? P[o + 64 + lane] : 0.0;
                    c += m - kk;
                }
            }
            if (lane >= k && lane < kend) dg = P[csl - base];           // D(k, k) of the chunk's pivots
            if (lane > k && lane <= kend && lane - 1 < p) sb = P[csp - base + 1];  // L(k + 1, k)
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int kk = k + u;
                if (kk < kend) {  // uniform
                    const double yb = readlane_d(y0, kk);
                    const double yk = (liveM >> kk) & 1 ? yb : 0.0;
                    const int lim = (twoAM >> kk) & 1 ? kk + 1 : kk;
                    const double t = y0 - l0[u] * yk;
                    y0 = lane > lim ? t : y0;
                    a1 -= l1[u] * yk;
                }
            }
            k = kend;
            cs = c;
        }
        if (k >= p) break;
        base = cs;
        k1 = fwd_chunk_end(m, p, k, win);
        __syncthreads();
        stage_panel<4>(L, Lo + base, cstart(m, k1) - base, P);
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the window's loads are all consumed here
        __syncthreads();
    }
    if (lane >= p && lane < m) st_sc1(cvo + (lane - p), y0);
    if (two && lane + 64 < m) st_sc1(cvo + (lane + 64 - p), a1);
    const double dgn = __shfl(dg, lane < 63 ? lane + 1 : lane), sbn = __shfl(sb, lane < 63 ? lane + 1 : lane);
    const double dgp = __shfl(dg, lane > 0 ? lane - 1 : 0);
    const double yn = __shfl(y0, lane < 63 ? lane + 1 : lane), yp = __shfl(y0, lane > 0 ? lane - 1 : 0);
    if (lane < p) {
        const int kind = mypiv;
        double out = 0.0;  // null pivot contributes 0
        if (kind == PIV_1X1) {
            out = y0 / dg;
        } else if (kind == PIV_2X2_A || kind == PIV_2X2_B) {
            const bool first = kind == PIV_2X2_A;
            const double a = first ? dg : dgp, b = first ? sbn : sb, e = first ? dgn : dg;
            const double det = a * e - b * b;
            const double yA = first ? y0 : yp, yB = first ? yn : y0;
            out = first ? (e * yA - b * yB) / det : (a * yB - b * yA) / det;
        }
        *zdst = out;
    }
}

__device__ __forceinline__ double bwd_compute_win2(const double* __restrict__ L, int64_t Lo, int m, int p, double* P, int win,
                                                   int c0, const double* x, int mypiv) {
    const int lane = threadIdx.x;
    const bool tri = lane < p;
    const bool live = tri && mypiv != PIV_NULL;
    const unsigned long long liveM = __ballot(live);
    const unsigned long long twoBM = __ballot(tri && mypiv == PIV_2X2_B);
    double xj = tri ? x[lane] : 0.0;
    int c1 = p, base = cstart(m, c0);
    for (;;) {
        const bool mine = lane >= c0 && lane < c1;
        const double* pk = P + (pcol(m, mine ? lane : c0) - base);  // pk[i] = L(i, lane), i >= lane
        double s0 = 0.0, s1 = 0.0;
        for (int i0 = p; i0 < m; i0 += 8) {  // rectangle rows, 8 per chunk (pairs: s0 even, s1 odd offsets)
            double lv[8], xv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                lv[u] = pk[i0 + u];  // rows >= m read in-bounds garbage (kSolveSlack), unused
                xv[u] = x[i0 + u];
            }
#pragma unroll
            for (int u = 0; u < 8; u += 2) {
                if (i0 + u < m) s0 += lv[u] * xv[u];  // uniform
                if (i0 + u + 1 < m) s1 += lv[u + 1] * xv[u + 1];
            }
        }
        if (live && mine) xj -= s0 + s1;
        for (int kh = p - 1; kh >= c0; kh -= 8) {  // triangle steps k = kh .. kh - 7 (>= c0)
            double lv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) lv[u] = pk[max(kh - u, 0)];  // L(k, lane) for lane < k
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int k = kh - u;
                if (k >= c0) {  // uniform
                    const double xb = readlane_d(xj, k);
                    const double xk = (liveM >> k) & 1 ? xb : 0.0;
                    const int skip = (twoBM >> k) & 1 ? k - 1 : -1;
                    const double t = xj - lv[u] * xk;
                    xj = (live && mine && lane < k && lane != skip) ? t : xj;
                }
            }
        }
        if (c0 == 0) break;
        c1 = c0;
        c0 = bwd_chunk_begin(m, p, c1, win);
        base = cstart(m, c0);
        __syncthreads();
        stage_panel<4>(L, Lo + base, cstart(m, c1) - base, P);
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the window's loads are all consumed here
        __syncthreads();
    }
    return xj;
}

// The walk keeps ONE FrontPre: once a front's prefetched data is consumed (staged into LDS, its
// scalars copied), the next front's loads are issued into the same registers, so no register copy of
// an in-flight load (which would wait for it) is needed across iterations.
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4))) void k_solve_fwd_df(SolveArgs A, DfArgs D) {
    extern __shared__ __attribute__((aligned(16))) double smem_s[];
    const int lane = threadIdx.x;
    int t = blockIdx.x;
    if (t >= D.nf) return;
    FrontPre q;
    q.r = df_record(df_desc_load(D, t));
    df_issue<true>(A, D, q);
    // The previous front's signal is deferred past this front's first dependent loads, so its store
    // drain overlaps them; it is sent before any wait (this front may be that front's parent).
    int pend = -1;
    auto signal = [&]() {
        drain_stores();
        if (pend >= 0 && lane == 0) __hip_atomic_fetch_add(D.cnt + pend, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        pend = -1;
    };
    for (; t < D.nf; t += gridDim.x) {
        // next position (clamped: the last front re-prefetches itself, branch-free loop-carried loads)
        const int tn = min(t + (int)gridDim.x, D.nf - 1);
        const int dn = df_desc_load(D, tn);  // next record: extracted after the children's loads
        const int m = q.r.m, p = q.r.p, f = q.r.f, par = q.r.par;
        const int64_t xoff = q.r.xoff, woff = q.r.woff;
        unsigned long long* st = D.stamps ? D.stamps + 8 * (int64_t)f : nullptr;
        if (st && lane == 0) st[0] = __builtin_amdgcn_s_memrealtime();
        double* P = smem_s;
        double* y = smem_s + D.win;
        int32_t* fpl = (int32_t*)(y + ((m + 1) & ~1));  // this front's rows were permuted by pivoting
        const int k1 = q.kw;
        const int64_t Lo = q.r.Lo;
        // pivot kinds through LDS: a register copy of q.mypiv (reloaded by df_issue below) would make the
        // loop back-edge wait for the next front's prefetch
        int32_t* ipl = (int32_t*)(smem_s + D.piv_off);
        ipl[lane] = q.mypiv;
        if (lane < m) { y[lane] = q.e0; fpl[lane] = q.fp0; }
        if (lane + 64 < m) { y[lane + 64] = 0.0; fpl[lane + 64] = q.fp1; }
        const uint32_t target = D.epoch * (uint32_t)(q.r.c1 - q.r.c0);
        if ((int32_t)(q.dep - target) < 0) {
            signal();
            df_wait(D.cnt + f, target, D.abort_flag);
        }
        df_stage_window(A, q, P);
        __syncthreads();
        fwd_extend_add<true>(A, D, q.r.c0, q.r.c1, q.my_cm, q.my_rmo, q.my_cxo, y, fpl);
        __syncthreads();
        signal();
        if (st && lane == 0) st[1] = __builtin_amdgcn_s_memrealtime();
        q.r = df_record(dn);
        df_issue<true>(A, D, q);
        if (st && lane == 0) st[2] = __builtin_amdgcn_s_memrealtime();
        const int mypiv = ipl[lane];
        fwd_compute_win(A.L, Lo, m, p, P, D.win, k1, y, mypiv, D.xs + woff + lane, D.cvx + xoff);
        if (st && lane == 0) st[3] = __builtin_amdgcn_s_memrealtime();
        pend = par;
        __syncthreads();  // LDS reused by the next front
    }
    signal();
}

__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4))) void k_solve_bwd_df(SolveArgs A, DfArgs D) {
    extern __shared__ __attribute__((aligned(16))) double smem_s[];
    const int lane = threadIdx.x;
    int t = blockIdx.x;
    // the backward walk: the walk without its flat levels (k_solve_bwd_flat solves those after it)
    D.desc = D.bdesc;
    D.nf = D.bnf;
    if (t >= D.nf) return;
    FrontPre q;
    q.r = df_record(df_desc_load(D, D.nf - 1 - t));
    df_issue<false>(A, D, q);
    int pend = -1;  // deferred publication of the previous front (see k_solve_fwd_df)
    auto signal = [&]() {
        drain_stores();
        if (pend >= 0 && lane == 0) __hip_atomic_store(D.done + pend, D.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        pend = -1;
    };
    for (; t < D.nf; t += gridDim.x) {
        const int tn = min(t + (int)gridDim.x, D.nf - 1);
        const int dn = df_desc_load(D, D.nf - 1 - tn);
        const int m = q.r.m, p = q.r.p, f = q.r.f;
        const int64_t woff = q.r.woff;
        unsigned long long* st = D.stamps ? D.stamps + 8 * (int64_t)f + 4 : nullptr;
        if (st && lane == 0) st[0] = __builtin_amdgcn_s_memrealtime();
        double* P = smem_s;
        double* x = smem_s + D.win;
        const int c0 = q.kw;
        const int64_t Lo = q.r.Lo;
        // own pivots: z of the forward solve; contribution rows: the ancestors' published solution
        // values (this launch), through the per-row slot index rxpos, once the parent has published
        if (q.r.par >= 0 && (int32_t)(q.dep - D.epoch) < 0) {
            signal();
            df_wait(D.done + q.r.par, D.epoch, D.abort_flag);
        }
        int32_t* ipl = (int32_t*)(smem_s + D.piv_off);  // pivot kinds through LDS (see k_solve_fwd_df)
        ipl[lane] = q.mypiv;
        if (lane < m) x[lane] = lane < p ? q.e0 : ld_sc1(D.xs + q.a0);
        if (lane + 64 < m) x[lane + 64] = ld_sc1(D.xs + q.a1);
        df_stage_window(A, q, P);
        __syncthreads();
        signal();
        if (st && lane == 0) st[1] = __builtin_amdgcn_s_memrealtime();
        q.r = df_record(dn);
        df_issue<false>(A, D, q);
        if (st && lane == 0) st[2] = __builtin_amdgcn_s_memrealtime();
        const int mypiv = ipl[lane];
        const double xj = bwd_compute_win(A.L, Lo, m, p, P, D.win, c0, x, mypiv);
        if (st && lane == 0) st[3] = __builtin_amdgcn_s_memrealtime();
        if (lane < p) st_sc1(D.xs + woff + lane, xj);
        pend = f;
        __syncthreads();
    }
    signal();
}

// Backward of the flat levels (the forward's k_solve_fwd_flat fronts), one launch per level after the backward
// walk, top level first, one wave per front: no dependency waits (the launch boundary orders a level after the
// walk / the level above) and no done flags (a flat front's children are flat).  The walk's per-front code
// (df_issue, df_stage_window, bwd_compute_win): bit-identical.
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4))) void k_solve_bwd_flat(SolveArgs A, DfArgs D, int begin,
                                                                                                 int count) {
    extern __shared__ __attribute__((aligned(16))) double smem_s[];
    const int lane = threadIdx.x;
    const int t = blockIdx.x;
    if (t >= count) return;
    FrontPre q;
    q.r = df_record(D.flat_desc[(int64_t)(begin + t) * 16 + (lane & 15)]);
    df_issue<false>(A, D, q);
    const int m = q.r.m, p = q.r.p;
    unsigned long long* st = D.stamps ? D.stamps + 8 * (int64_t)q.r.f + 4 : nullptr;
    if (st && lane == 0) st[0] = st[1] = __builtin_amdgcn_s_memrealtime();
    double* P = smem_s;
    double* x = smem_s + D.win;
    int32_t* ipl = (int32_t*)(smem_s + D.piv_off);
    ipl[lane] = q.mypiv;
    if (lane < m) x[lane] = lane < p ? q.e0 : ld_sc1(D.xs + q.a0);
    if (lane + 64 < m) x[lane + 64] = ld_sc1(D.xs + q.a1);
    df_stage_window(A, q, P);
    __syncthreads();
    if (st && lane == 0) st[2] = __builtin_amdgcn_s_memrealtime();
    const int mypiv = ipl[lane];
    const double xj = bwd_compute_win(A.L, q.r.Lo, m, p, P, D.win, q.kw, x, mypiv);
    if (lane < p) st_sc1(D.xs + q.r.woff + lane, xj);
    if (st && lane == 0) st[3] = __builtin_amdgcn_s_memrealtime();
}

// ---- register-resident dataflow solve (round 4): the default dataflow kernels ----
// Same walk, hand-offs (sc1 update vectors / solution values, arrival counters / done epochs) and per-lane
// arithmetic as k_solve_{fwd,bwd}_df, with the pivot-step loops taken off LDS:
//  forward (lane = row i): column k of L arrives by one coalesced load straight into register B[k - k0]
//    (rows k..m-1 of the column are consecutive in the packed trapezoid), the pivot loop is unrolled over
//    the registers, pivot kinds are wave-uniform ballot masks (scalar bit tests, no branch per step) and
//    y_k is broadcast by readlane: a step is one readlane pair, one FMA and one select, no memory access.
//    Rows >= 64 (m > 64) take the same column updates afterwards from the broadcast values (same order).
//  backward (lane = column j): the panel is read in 8-row windows (rectangle rows ascending, then the
//    triangle's rows descending), eight lanes per 64-byte column piece, all windows of the front in flight
//    in registers at once; each window is written to an LDS tile T[r * ld + c] (ld = 2 mod 32: the
//    writes of a 16-lane group hit 32 distinct banks, a row read by the 64 lanes is contiguous) and
//    consumed as rows of L, the operands of the column-oriented dot products / updates of bwd_compute.
//  Both walks issue the next front's loads before draining the finished front's stores, so a front in
//  the bulk of the tree costs one memory round trip (plus one for its children's / ancestors' values).
constexpr int kRgCols = 32;   // forward: columns of L per register round

// base[rel] with rel clamped into [0, n): a uniform 64-bit base plus a 32-bit byte offset (one VGPR per
// address: the loads use the scalar-base addressing form)
__device__ __forceinline__ double ld_clamped(const double* base, int rel, int n) {
    const uint32_t off = (uint32_t)min(max(rel, 0), n - 1) * 8u;
    return *reinterpret_cast<const double*>(reinterpret_cast<const char*>(base) + off);
}


// Fronts outside the register kernels' class (p > 32 or m > 72: in practice a few parents enlarged by delayed
// columns) form a second walk (DfArgs::ov_*, the same topological order) that the last ov_grid blocks of the
// launch process with the LDS-panel per-front code of k_solve_{fwd,bwd}_df (same arithmetic) in a window of
// kRgWin doubles; the hand-offs are the per-front counters, so the two walks wait on each other as any two
// blocks do.  The roles split at the top of the kernel: the register fast path keeps its own budget.
constexpr int kRgWin = 512;                         // doubles (> one column of a front of <= 128 rows)
constexpr int kRgRegion = kRgWin + kSolveSlack;     // the window and its read slack
__device__ __forceinline__ bool rg_fits(int m, int p) { return p <= 32 && m <= 72; }

// forward of one oversized front (over role): y (128) and fpl (128 words) at smem, window P after them
__device__ void rg_fwd_over(const SolveArgs& A, const DfArgs& D, const FrontRec& r, double* y, int32_t* fpl, double* P) {
    const int lane = threadIdx.x;
    const int m = r.m, p = r.p, f = r.f;
    const int64_t ro = r.ro;
    const int mypiv = lane < p ? (int)A.piv[ro + lane] : 0;
    const double e0 = lane < p ? D.xs[r.woff + lane] : 0.0;
    int my_cm = 0;
    long long my_rmo = 0, my_cxo = 0;
    if (lane < r.c1 - r.c0) {
        my_cm = A.ch_cm[r.c0 + lane];
        my_rmo = A.ch_relmap_off[r.c0 + lane];
        my_cxo = D.ch_cvx_off[r.c0 + lane];
    }
    y[lane] = e0;
    y[lane + 64] = 0.0;
    fpl[lane] = lane < m ? A.fpos[ro + lane] : 0;
    fpl[lane + 64] = lane + 64 < m ? A.fpos[ro + lane + 64] : 0;
    if (r.c1 > r.c0) {
        if (r.nw > 0) df_wait(D.cnt + f, D.epoch * (uint32_t)r.nw, D.abort_flag);
        __syncthreads();
        fwd_extend_add<true>(A, D, r.c0, r.c1, my_cm, my_rmo, my_cxo, y, fpl);
    }
    __syncthreads();
    const int k1 = fwd_chunk_end(m, p, 0, kRgWin);
    stage_panel<4>(A.L, r.Lo, cstart(m, k1), P);
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    __syncthreads();
    fwd_compute_win2(A.L, r.Lo, m, p, P, kRgWin, k1, y, mypiv, D.xs + r.woff + lane, D.cvx + r.xoff);
    drain_stores();
    if (r.par >= 0 && lane == 0) __hip_atomic_fetch_add(D.cnt + r.par, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();  // LDS reused by the next front
}

// the backward arithmetic of an oversized front (bwd_compute_win2 from the last window), x in X (LDS)
__device__ __forceinline__ double rg_bwd_over_core(const double* __restrict__ L, int64_t Lo, int m, int p, double* P,
                                                   const double* X, int mypiv) {
    const int c0 = bwd_chunk_begin(m, p, p, kRgWin);
    const int base = cstart(m, c0);
    stage_panel<4>(L, Lo + base, cstart(m, p) - base, P);
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    __syncthreads();
    return bwd_compute_win2(L, Lo, m, p, P, kRgWin, c0, X, mypiv);
}

// backward of one oversized front (over role): X (128 doubles: the rows' values) at smem, window P after it
__device__ void rg_bwd_over(const SolveArgs& A, const DfArgs& D, const FrontRec& r, double* X, double* P) {
    const int lane = threadIdx.x;
    const int m = r.m, p = r.p;
    const int64_t ro = r.ro;
    const int mypiv = lane < p ? (int)A.piv[ro + lane] : (int)PIV_NULL;
    if (r.par >= 0) df_wait(D.done + r.par, D.epoch, D.abort_flag);
    for (int i = lane; i < m; i += 64) X[i] = i < p ? D.xs[r.woff + i] : ld_sc1(D.xs + D.rxpos[ro + i]);
    const double xj = rg_bwd_over_core(A.L, r.Lo, m, p, P, X, mypiv);
    if (lane < p) st_sc1(D.xs + r.woff + lane, xj);
    drain_stores();
    if (lane == 0) __hip_atomic_store(D.done + r.f, D.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();  // LDS reused by the next front
}

// per-front loads of the forward walk other than the panel columns
struct RgFwdMeta {
    int piv;                    // lane < p: pivot kind
    double e0;                  // lane < p: right-hand side at the own pivots (xs)
    int32_t fp0, fp1;           // pivoted positions of the analysis-order rows lane, lane + 64
    int my_cm;
    long long my_rmo, my_cxo;   // children's edge records (lane < children)
    uint32_t dep;               // arrival counter as seen at issue time (sc1)
    double dgl, sbl;            // L(lane, lane), L(lane, lane - 1): the diagonal blocks of D
    double H[4];                // rows 64..71: H[c] = L(64 + (lane & 7), 8c + (lane >> 3))
};

// L(row0 + lane, k0 + u) -> B[u] for the front's columns k0 + u < p (uniform guards: only those are loaded;
// row indices clamped into the panel: rows outside it read a harmless in-panel value that no step uses)
__device__ __forceinline__ void rg_load_cols(const double* __restrict__ L, int64_t Lo, int m, int p, int k0, int row0,
                                             double (&B)[kRgCols]) {
    const int lane = threadIdx.x;
    const int sz = p * m - ((p * (p - 1)) >> 1);
    int cs = cstart(m, k0);
#pragma unroll
    for (int u = 0; u < kRgCols; ++u) {
        const int k = k0 + u;
        if (k < p) B[u] = ld_clamped(L + Lo, cs + row0 + lane - k, sz);
        cs += m - k;
    }
}

// rows 64..71 of the panel (m <= 72, p <= 32), compact: H[c] = L(64 + (lane & 7), 8c + (lane >> 3))
__device__ __forceinline__ void rg_load_high(const double* __restrict__ L, int64_t Lo, int m, int p, double (&H)[4]) {
    const int lane = threadIdx.x;
    const int sz = p * m - ((p * (p - 1)) >> 1);
    const int rr = lane & 7, kk = lane >> 3;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int col = 8 * c + kk;
        if (8 * c < p) H[c] = ld_clamped(L + Lo, cstart(m, col) + 64 + rr - col, sz);
    }
}

__device__ __forceinline__ void rg_fwd_meta(const SolveArgs& A, const DfArgs& D, const FrontRec& r, RgFwdMeta& q) {
    const int lane = threadIdx.x;
    const int m = r.m, p = r.p;
    const int64_t ro = r.ro;
    q.piv = lane < p ? (int)A.piv[ro + lane] : 0;
    q.e0 = lane < p ? D.xs[r.woff + lane] : 0.0;
    q.fp0 = lane < m ? A.fpos[ro + lane] : 0;
    q.fp1 = lane + 64 < m ? A.fpos[ro + lane + 64] : 0;
    q.my_cm = 0;
    q.my_rmo = q.my_cxo = 0;
    if (lane < r.c1 - r.c0) {
        q.my_cm = A.ch_cm[r.c0 + lane];
        q.my_rmo = A.ch_relmap_off[r.c0 + lane];
        q.my_cxo = D.ch_cvx_off[r.c0 + lane];
    }
    q.dep = r.c1 > r.c0 ? ld_sc1_u32(D.cnt + r.f) : 0u;
    const int lc = lane < p ? lane : 0;
    q.dgl = A.L[r.Lo + cstart(m, lc)];
    q.sbl = lane > 0 && lane < p ? A.L[r.Lo + cstart(m, lane - 1) + 1] : 0.0;
    if (m > 64) rg_load_high(A.L, r.Lo, m, p, q.H);  // uniform (walk precondition: m <= 72, p <= 32)
}

// children's update vectors -> y (LDS rows, permuted by fpl), two children's loads in flight at a time
// (the register-resident forward keeps its panel registers live here); rows 64.. of a child only when
// the child has them.  Same additions, same order as fwd_extend_add.
__device__ __forceinline__ void rg_extend_add(const SolveArgs& A, const DfArgs& D, int c0, int c1, int my_cm,
                                              long long my_rmo, long long my_cxo, double* y, const int32_t* fpl) {
    const int lane = threadIdx.x;
    constexpr int CH = 2;
    for (int cb = c0; cb < c1; cb += CH) {
        if (cb != c0 && (cb - c0) % 64 == 0 && lane < c1 - cb) {  // more than 64 children: next records
            my_cm = A.ch_cm[cb + lane];
            my_rmo = A.ch_relmap_off[cb + lane];
            my_cxo = D.ch_cvx_off[cb + lane];
        }
        double v[CH];
        int32_t rw[CH];
        int cms[CH];
#pragma unroll
        for (int u = 0; u < CH; ++u) {
            const int q = (cb - c0) % 64 + u;
            const bool have = cb + u < c1;  // uniform
            const int cm = have ? __builtin_amdgcn_readlane(my_cm, q) : 0;
            cms[u] = cm;
            const int32_t* rmp = A.relmap + (have ? (int64_t)readlane64((unsigned long long)my_rmo, q) : 0);
            const double* cvp = D.cvx + (have ? (int64_t)readlane64((unsigned long long)my_cxo, q) : 0);
            v[u] = lane < cm ? ld_sc1(cvp + lane) : 0.0;
            rw[u] = lane < cm ? rmp[lane] : -1;
        }
#pragma unroll
        for (int u = 0; u < CH; ++u) {  // children in order (rows of one child are distinct)
            wave_lds_sync();  // the previous child's (or the caller's) LDS writes before these cross-lane reads
            if (rw[u] >= 0) y[fpl[rw[u]]] += v[u];
            if (cms[u] > 64) {  // uniform: the child's rows 64..
                const int q = (cb - c0) % 64 + u;
                const int32_t* rmp = A.relmap + (int64_t)readlane64((unsigned long long)my_rmo, q);
                const double* cvp = D.cvx + (int64_t)readlane64((unsigned long long)my_cxo, q);
                const int t = lane + 64;
                if (t < cms[u]) y[fpl[rmp[t]]] += ld_sc1(cvp + t);
            }
        }
    }
}

// The walk issues the next front's loads under the current front's work: its metadata right after the
// current front's children are assembled, and its panel column u into register B[u] as soon as step u of
// the current front has consumed B[u] (rolling prefetch).  Walk precondition (setup_dataflow): every front
// has p <= 32 and m <= 72 (rows 64..71 go through a small LDS tile, Th); other walks use k_solve_fwd_df.
template <int WPE>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE))) void k_solve_fwd_rg(SolveArgs A, DfArgs D) {
    extern __shared__ __attribute__((aligned(16))) double smem_s[];
    const int lane = threadIdx.x;
    double* y = smem_s;                          // 128 doubles: the front's rows (pivoted order)
    int32_t* fpl = (int32_t*)(smem_s + 128);     // 128 words
    const int G = (int)gridDim.x - D.ov_grid;
    if ((int)blockIdx.x >= G) {  // over role: the oversized fronts' walk
        for (int t = blockIdx.x - G; t < D.ov_nf; t += D.ov_grid) {
            const FrontRec r = df_record(D.ov_desc[t * 16 + (lane & 15)]);
            unsigned long long* st = D.stamps ? D.stamps + 8 * (int64_t)r.f : nullptr;
            if (st && lane == 0) st[0] = st[1] = __builtin_amdgcn_s_memrealtime();
            rg_fwd_over(A, D, r, y, fpl, smem_s + 192);
            if (st && lane == 0) st[2] = st[3] = __builtin_amdgcn_s_memrealtime();
        }
        return;
    }
    int t = blockIdx.x;
    if (t >= D.rgf_nf) return;
    double* Th = smem_s + 192;                   // 8 x 33 doubles: rows 64..71 of the panel
    const int* desc = D.rgf_desc;
    FrontRec r = df_record(desc[t * 16 + (lane & 15)]);
    RgFwdMeta q;
    double B[kRgCols];
    rg_fwd_meta(A, D, r, q);
    rg_load_cols(A.L, r.Lo, r.m, r.p, 0, 0, B);
    int dn = desc[min(t + G, D.rgf_nf - 1) * 16 + (lane & 15)];
    for (;;) {
        const int m = r.m, p = r.p, f = r.f, par = r.par;
        const int64_t xoff = r.xoff, woff = r.woff;
        unsigned long long* st = D.stamps ? D.stamps + 8 * (int64_t)f : nullptr;
        if (st && lane == 0) st[0] = __builtin_amdgcn_s_memrealtime();
        const unsigned long long liveM = __ballot(lane < p && q.piv != PIV_NULL);
        const unsigned long long twoAM = __ballot(lane < p && q.piv == PIV_2X2_A);
        const int piv_c = q.piv;
        const double dgl = q.dgl, sbl = q.sbl;
        wave_lds_sync();  // the previous front's reads of y, fpl and Th are done before they are rewritten
        if (m > 64) {  // uniform
#pragma unroll
            for (int c = 0; c < 4; ++c)
                if (8 * c < p) Th[(lane & 7) * 33 + 8 * c + (lane >> 3)] = q.H[c];
        }
        y[lane] = q.e0;
        y[lane + 64] = 0.0;
        fpl[lane] = q.fp0;
        fpl[lane + 64] = q.fp1;
        if (r.c1 > r.c0) {
            const uint32_t target = D.epoch * (uint32_t)r.nw;  // leaves solved before the walk are not waited for
            if (r.nw > 0 && (int32_t)(q.dep - target) < 0) df_wait(D.cnt + f, target, D.abort_flag);
            rg_extend_add(A, D, r.c0, r.c1, q.my_cm, q.my_rmo, q.my_cxo, y, fpl);
        }
        wave_lds_sync();  // y, fpl and Th were written by other lanes
        double y0 = y[lane];
        double a1 = m > 64 ? y[lane + 64] : 0.0;
        if (st && lane == 0) st[1] = __builtin_amdgcn_s_memrealtime();
        const int tn = t + G;
        const bool more = tn < D.rgf_nf;
        FrontRec rn = r;
        asm volatile("" ::: "memory");  // the next front's loads stay below this front's assembly
        if (more) {
            rn = df_record(dn);
            dn = desc[min(tn + G, D.rgf_nf - 1) * 16 + (lane & 15)];
            rg_fwd_meta(A, D, rn, q);
        } else {
            rn.p = 0;
        }
        // the pivot steps on the rows < 64; the next front's column u goes into B[u] once step u has used it
        {
            const int sz_n = rn.p * rn.m - ((rn.p * (rn.p - 1)) >> 1);
            int cs_n = 0;  // cstart(rn.m, u)
#pragma unroll
            for (int u = 0; u < kRgCols; ++u) {
                if (u < p) {  // uniform
                    const double yb = readlane_d(y0, u);
                    const double yk = (liveM >> u) & 1 ? yb : 0.0;
                    const int lim = (twoAM >> u) & 1 ? u + 1 : u;
                    const double tv = y0 - B[u] * yk;
                    y0 = lane > lim ? tv : y0;
                }
                if (u < rn.p) {  // uniform
                    B[u] = ld_clamped(A.L + rn.Lo, cs_n + lane - u, sz_n);
                    cs_n += rn.m - u;
                }
                __builtin_amdgcn_sched_barrier(0);  // keep the load behind the step that frees its register
            }
        }
        // rows 64..71: the same column updates with the values the steps broadcast (y_k, 0 for a null pivot),
        // from the LDS tile, lane = row - 64
        if (m > 64) {
            const double ybv = lane < p && ((liveM >> lane) & 1) ? y0 : 0.0;
            const int rw = lane < 8 ? lane : 0;
#pragma unroll
            for (int k = 0; k < kRgCols; ++k)
                if (k < p) a1 -= Th[rw * 33 + k] * readlane_d(ybv, k);
        }
        // update vector (rows >= p) and the own pivots' z = D^-1 y
        double* cvo = D.cvx + xoff;
        if (lane >= p && lane < m) st_sc1(cvo + (lane - p), y0);
        if (lane + 64 < m) st_sc1(cvo + (lane + 64 - p), a1);
        {
            const double dg = dgl, sb = sbl;
            const double dgn = __shfl(dg, lane < 63 ? lane + 1 : lane), sbn = __shfl(sb, lane < 63 ? lane + 1 : lane);
            const double dgp = __shfl(dg, lane > 0 ? lane - 1 : 0);
            const double yn = __shfl(y0, lane < 63 ? lane + 1 : lane), yp = __shfl(y0, lane > 0 ? lane - 1 : 0);
            const int kind = piv_c;
            double out = 0.0;  // null pivot contributes 0
            if (kind == PIV_1X1) {
                out = y0 / dg;
            } else if (kind == PIV_2X2_A || kind == PIV_2X2_B) {
                const bool first = kind == PIV_2X2_A;
                const double a = first ? dg : dgp, b = first ? sbn : sb, e = first ? dgn : dg;
                const double det = a * e - b * b;
                const double yA = first ? y0 : yp, yB = first ? yn : y0;
                out = first ? (e * yA - b * yB) / det : (a * yB - b * yA) / det;
            }
            if (lane < p) D.xs[woff + lane] = out;
        }
        if (st && lane == 0) st[2] = __builtin_amdgcn_s_memrealtime();
        drain_stores();
        if (par >= 0 && lane == 0) __hip_atomic_fetch_add(D.cnt + par, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (st && lane == 0) st[3] = __builtin_amdgcn_s_memrealtime();
        if (!more) break;
        r = rn;
        t = tn;
    }
}

// Forward of the bottom levels of the register walk (option solve_flat_levels, default 2: levels 0 and 1), one
// flat launch per level before the walk, one wave per front.  The walk spends most of such a front's time issuing
// and draining loads one front after the other (its drain before the parent's counter also waits for the next
// front's prefetch: one vmcnt for loads and stores); here the hardware keeps as many independent fronts in flight
// as fit, with no counters at all: the launch boundary orders a level after the one below, and the walk's
// fronts wait only for their walk children (kDescNW).  The per-lane arithmetic is the walk's (same extend-add,
// same steps, same order): bit-identical.  (A resident grid looping over the fronts measured slower, 72.6 vs
// 49.3 us for the leaves at C3: its wait for the next record also waited for the finished front's stores.)
template <int WPE>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE))) void k_solve_fwd_flat(SolveArgs A, DfArgs D, int begin,
                                                                                                   int count) {
    extern __shared__ __attribute__((aligned(16))) double smem_s[];
    const int lane = threadIdx.x;
    const int t = blockIdx.x;
    if (t >= count) return;
    double* y = smem_s;                       // 128 doubles: the front's rows (pivoted order)
    int32_t* fpl = (int32_t*)(smem_s + 128);  // 128 words
    double* Th = smem_s + 192;                // 8 x 33 doubles: rows 64..71 of the panel
    const FrontRec r = df_record(D.flat_desc[(int64_t)(begin + t) * 16 + (lane & 15)]);
    const int m = r.m, p = r.p;
    unsigned long long* st = D.stamps ? D.stamps + 8 * (int64_t)r.f : nullptr;
    if (st && lane == 0) st[0] = st[1] = __builtin_amdgcn_s_memrealtime();
    RgFwdMeta q;
    double B[kRgCols];
    rg_fwd_meta(A, D, r, q);
    rg_load_cols(A.L, r.Lo, m, p, 0, 0, B);
    const unsigned long long liveM = __ballot(lane < p && q.piv != PIV_NULL);
    const unsigned long long twoAM = __ballot(lane < p && q.piv == PIV_2X2_A);
    if (m > 64) {  // uniform
#pragma unroll
        for (int c = 0; c < 4; ++c)
            if (8 * c < p) Th[(lane & 7) * 33 + 8 * c + (lane >> 3)] = q.H[c];
    }
    double y0, a1;
    if (r.c1 > r.c0) {  // children (a lower flat level, complete): their update vectors into y, as the walk
        y[lane] = q.e0;
        y[lane + 64] = 0.0;
        fpl[lane] = q.fp0;
        fpl[lane + 64] = q.fp1;
        rg_extend_add(A, D, r.c0, r.c1, q.my_cm, q.my_rmo, q.my_cxo, y, fpl);
        wave_lds_sync();  // y, fpl and Th were written by other lanes
        y0 = y[lane];
        a1 = m > 64 ? y[lane + 64] : 0.0;
    } else {  // a leaf: y = the right-hand side at the pivots, 0 on the contribution rows
        wave_lds_sync();  // Th was written by other lanes
        y0 = q.e0;
        a1 = 0.0;
    }
#pragma unroll
    for (int u = 0; u < kRgCols; ++u) {
        if (u < p) {  // uniform
            const double yb = readlane_d(y0, u);
            const double yk = (liveM >> u) & 1 ? yb : 0.0;
            const int lim = (twoAM >> u) & 1 ? u + 1 : u;
            const double tv = y0 - B[u] * yk;
            y0 = lane > lim ? tv : y0;
        }
    }
    if (m > 64) {
        const double ybv = lane < p && ((liveM >> lane) & 1) ? y0 : 0.0;
        const int rw = lane < 8 ? lane : 0;
#pragma unroll
        for (int k = 0; k < kRgCols; ++k)
            if (k < p) a1 -= Th[rw * 33 + k] * readlane_d(ybv, k);
    }
    double* cvo = D.cvx + r.xoff;
    if (lane >= p && lane < m) st_sc1(cvo + (lane - p), y0);
    if (lane + 64 < m) st_sc1(cvo + (lane + 64 - p), a1);
    {
        const double dg = q.dgl, sb = q.sbl;
        const double dgn = __shfl(dg, lane < 63 ? lane + 1 : lane), sbn = __shfl(sb, lane < 63 ? lane + 1 : lane);
        const double dgp = __shfl(dg, lane > 0 ? lane - 1 : 0);
        const double yn = __shfl(y0, lane < 63 ? lane + 1 : lane), yp = __shfl(y0, lane > 0 ? lane - 1 : 0);
        const int kind = q.piv;
        double out = 0.0;  // null pivot contributes 0
        if (kind == PIV_1X1) {
            out = y0 / dg;
        } else if (kind == PIV_2X2_A || kind == PIV_2X2_B) {
            const bool first = kind == PIV_2X2_A;
            const double a = first ? dg : dgp, b = first ? sbn : sb, e = first ? dgn : dg;
            const double det = a * e - b * b;
            const double yA = first ? y0 : yp, yB = first ? yn : y0;
            out = first ? (e * yA - b * yB) / det : (a * yB - b * yA) / det;
        }
        if (lane < p) D.xs[r.woff + lane] = out;
    }
    if (st && lane == 0) st[2] = st[3] = __builtin_amdgcn_s_memrealtime();
}

// ---- register-resident backward (fronts with p <= 32, m <= 72) ----
// Lane = row, as the forward: B[j] = L(lane, j) (j < p), H the rows 64..71.  The rectangle's column sums
// s_j = sum_{i >= p} L(i, j) x_i are one transpose-reduction across the wave: the 32 per-lane products
// are halved by v_permlane32_swap / v_permlane16_swap exchanges (lane bits 5, 4) and shuffles (bits 3, 2,
// 1), so lane 2c ends with column c's sum, summed in a fixed tree order; rows 64..71 add their column sums
// (8-lane reductions) after it.  The triangle goes through an LDS tile T[i * 33 + j] = L(i, j) (stride 33:
// conflict-free writes down a column, contiguous reads along a row) and runs lane = column, steps
// k = p-1 .. 0 as bwd_compute.  The level-scheduled solve of such fronts (k_solve_bwd_w2) calls the same
// core, so both schedules stay bit-identical; handles whose one-wave fronts all fit use it (new_bwd).
__device__ __forceinline__ void dswap32(double& a, double& b) {  // a: vdst, b: vsrc of v_permlane32_swap
    const unsigned long long ua = as_bits(a), ub = as_bits(b);
    const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)ua, (unsigned)ub, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(ua >> 32), (unsigned)(ub >> 32), false, false);
    a = as_double(((unsigned long long)(unsigned)hi[0] << 32) | (unsigned)lo[0]);
    b = as_double(((unsigned long long)(unsigned)hi[1] << 32) | (unsigned)lo[1]);
}
__device__ __forceinline__ void dswap16(double& a, double& b) {  // v_permlane16_swap: odd rows of a <-> even rows of b
    const unsigned long long ua = as_bits(a), ub = as_bits(b);
    const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)ua, (unsigned)ub, false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(ua >> 32), (unsigned)(ub >> 32), false, false);
    a = as_double(((unsigned long long)(unsigned)hi[0] << 32) | (unsigned)lo[0]);
    b = as_double(((unsigned long long)(unsigned)hi[1] << 32) | (unsigned)lo[1]);
}
__device__ __forceinline__ double shfl_xor_d(double v, int mask) { return bperm_d(v, (int)(threadIdx.x ^ mask)); }

// The backward of one front (see above).  After B has been consumed (T written, products formed and halved
// three times), next() is called: the walk issues the next front's loads into B there.  Returns x_j in lane j < p.
template <class Next>
__device__ __forceinline__ double rg_bwd_core(double (&B)[kRgCols], const double (&H)[4], double xr0, double xh, int m,
                                              int p, int piv, double* T, Next next) {
    const int lane = threadIdx.x;
    constexpr int ld = 33;
    const bool live = lane < p && piv != PIV_NULL;
    const unsigned long long liveM = __ballot(live);
    const unsigned long long twoBM = __ballot(lane < p && piv == PIV_2X2_B);
    // triangle tile: row lane (< p), columns j < p
#pragma unroll
    for (int j = 0; j < kRgCols; ++j)
        if (j < p && lane < p) T[lane * ld + j] = B[j];  // j: uniform
    // rectangle products (rows p <= lane < m), first halving: lanes < 32 keep columns 0..15, lanes >= 32 16..31.
    // Each product's rounding error e = fma(l, x, -l x) is carried through the first two halvings in its own
    // tree and added back there, so the products enter the sum exactly (as in bwd_compute's FMA accumulation)
    const bool rowok = lane >= p && lane < m;
    double r2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {  // columns j, j + 8, j + 16, j + 24: two halvings (lane bits 5, 4)
        double r1[2], e1[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int c = j + 8 * h;
            const double la = rowok && c < p ? B[c] : 0.0, lb = rowok && c + 16 < p ? B[c + 16] : 0.0;
            double a = la * xr0, b = lb * xr0;
            double ea = fma(la, xr0, -a), eb = fma(lb, xr0, -b);
            dswap32(a, b);
            dswap32(ea, eb);
            r1[h] = a + b;
            e1[h] = ea + eb;
        }
        double a = r1[0], b = r1[1], ea = e1[0], eb = e1[1];
        dswap16(a, b);
        dswap16(ea, eb);
        r2[j] = (a + b) + (ea + eb);
    }
    const bool b3 = (lane >> 3) & 1, b2 = (lane >> 2) & 1, b1 = (lane >> 1) & 1;
    double r3[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const double keep = b3 ? r2[j + 4] : r2[j], send = b3 ? r2[j] : r2[j + 4];
        r3[j] = keep + shfl_xor_d(send, 8);
    }
    __builtin_amdgcn_sched_barrier(0);
    next();  // B is free and the products are down to four registers per lane
    double r4[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const double keep = b2 ? r3[j + 2] : r3[j], send = b2 ? r3[j] : r3[j + 2];
        r4[j] = keep + shfl_xor_d(send, 4);
    }
    const double keep5 = b1 ? r4[1] : r4[0], send5 = b1 ? r4[0] : r4[1];
    const double r5 = keep5 + shfl_xor_d(send5, 2);
    const double r6 = r5 + shfl_xor_d(r5, 1);          // lane 2c, 2c + 1: column c
    double sj = bperm_d(r6, (2 * lane) & 63);          // lane j < 32: column j
    if (m > 64) {  // uniform: rows 64..71, 8-lane groups of one column (lane >> 3) per H[c]
        const int rr = lane & 7;
        double hs[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            double v = 8 * c < p && 64 + rr < m ? H[c] * xh : 0.0;
            v += shfl_xor_d(v, 1);
            v += shfl_xor_d(v, 2);
            v += shfl_xor_d(v, 4);
            hs[c] = v;  // column 8c + (lane >> 3)
        }
        const int src = 8 * (lane & 7);  // lane j reads column j = 8c + g from lane 8g, c = j >> 3
        double h = 0.0;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const double v = bperm_d(hs[c], src);
            h = (lane >> 3) == c ? v : h;
        }
        sj += h;
    }
    double xj = lane < p ? xr0 : 0.0;
    if (live) xj -= sj;
    // triangle: steps k = p-1 .. 0, eight LDS rows read ahead
    for (int kh = p - 1; kh >= 0; kh -= 8) {
        double lv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) lv[u] = T[max(kh - u, 0) * ld + lane];  // L(k, lane), lane < k
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int k = kh - u;
            if (k >= 0) {  // uniform
                const double xb = readlane_d(xj, k);
                const double xk = (liveM >> k) & 1 ? xb : 0.0;
                const int skip = (twoBM >> k) & 1 ? k - 1 : -1;
                const double tv = xj - lv[u] * xk;
                xj = (live && lane < k && lane != skip) ? tv : xj;
            }
        }
    }
    return xj;
}

struct RgBwdMeta {
    int piv;          // lane < p: pivot kind
    double e0;        // lane < p: z (forward result)
    int32_t a0;       // p <= lane < m: xs index of row lane (an ancestor's published solution value)
    int32_t ah;       // m > 64: xs index of row 64 + (lane & 7)
    uint32_t dep;     // parent's done word as seen at issue time (sc1)
    double H[4];      // rows 64..71 (compact, see rg_load_high)
};
__device__ __forceinline__ void rg_bwd_meta(const SolveArgs& A, const DfArgs& D, const FrontRec& r, RgBwdMeta& q) {
    const int lane = threadIdx.x;
    const int m = r.m, p = r.p;
    const int64_t ro = r.ro;
    q.piv = lane < p ? (int)A.piv[ro + lane] : (int)PIV_NULL;
    q.e0 = lane < p ? D.xs[r.woff + lane] : 0.0;
    q.a0 = lane >= p && lane < m ? D.rxpos[ro + lane] : 0;
    q.ah = 64 + (lane & 7) < m ? D.rxpos[ro + 64 + (lane & 7)] : 0;
    q.dep = r.par >= 0 ? ld_sc1_u32(D.done + r.par) : 0u;
    if (m > 64) rg_load_high(A.L, r.Lo, m, p, q.H);
}

template <int WPE>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE))) void k_solve_bwd_rg(SolveArgs A, DfArgs D) {
    extern __shared__ __attribute__((aligned(16))) double smem_s[];
    const int lane = threadIdx.x;
    const int G = (int)gridDim.x - D.ov_grid;
    if ((int)blockIdx.x >= G) {  // over role: the oversized fronts' walk, last to first
        for (int t = blockIdx.x - G; t < D.ov_nf; t += D.ov_grid) {
            const FrontRec r = df_record(D.ov_desc[(D.ov_nf - 1 - t) * 16 + (lane & 15)]);
            unsigned long long* st = D.stamps ? D.stamps + 8 * (int64_t)r.f + 4 : nullptr;
            if (st && lane == 0) st[0] = st[1] = __builtin_amdgcn_s_memrealtime();
            rg_bwd_over(A, D, r, smem_s, smem_s + 128);
            if (st && lane == 0) st[2] = st[3] = __builtin_amdgcn_s_memrealtime();
        }
        return;
    }
    int t = blockIdx.x;
    if (t >= D.rg_nf) return;
    double* T = smem_s;  // 32 x 33 doubles
    const int* desc = D.rg_desc;
    const int nf = D.rg_nf;
    FrontRec r = df_record(desc[(nf - 1 - t) * 16 + (lane & 15)]);
    RgBwdMeta q;
    double B[kRgCols];
    rg_bwd_meta(A, D, r, q);
    rg_load_cols(A.L, r.Lo, r.m, r.p, 0, 0, B);
    int dn = desc[(nf - 1 - min(t + G, nf - 1)) * 16 + (lane & 15)];
    for (;;) {
        const int m = r.m, p = r.p, f = r.f;
        const int64_t woff = r.woff;
        unsigned long long* st = D.stamps ? D.stamps + 8 * (int64_t)f + 4 : nullptr;
        if (st && lane == 0) st[0] = __builtin_amdgcn_s_memrealtime();
        if (r.par >= 0 && (int32_t)(q.dep - D.epoch) < 0) df_wait(D.done + r.par, D.epoch, D.abort_flag);
        // the rows' values, lane = row: own z (lane < p), the ancestors' published solution values
        const double xr0 = lane < p ? q.e0 : (lane < m ? ld_sc1(D.xs + q.a0) : 0.0);
        const double xh = 64 + (lane & 7) < m ? ld_sc1(D.xs + q.ah) : 0.0;
        const int piv = q.piv;
        double H[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) H[c] = q.H[c];
        if (st && lane == 0) st[1] = __builtin_amdgcn_s_memrealtime();
        const int tn = t + G;
        const bool more = tn < nf;
        FrontRec rn = r;
        auto next = [&]() {  // the next front's loads, issued as soon as B is free
            if (more) {
                rn = df_record(dn);
                dn = desc[(nf - 1 - min(tn + G, nf - 1)) * 16 + (lane & 15)];
                rg_bwd_meta(A, D, rn, q);
                rg_load_cols(A.L, rn.Lo, rn.m, rn.p, 0, 0, B);
            }
        };
        const double xj = rg_bwd_core(B, H, xr0, xh, m, p, piv, T, next);
        if (lane < p) st_sc1(D.xs + woff + lane, xj);
        if (st && lane == 0) st[2] = __builtin_amdgcn_s_memrealtime();
        drain_stores();
        if (lane == 0) __hip_atomic_store(D.done + f, D.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (st && lane == 0) st[3] = __builtin_amdgcn_s_memrealtime();
        if (!more) break;
        r = rn;
        t = tn;
    }
}

// level-scheduled backward of one-wave fronts with the arithmetic of k_solve_bwd_rg (w by original index):
// rg_bwd_core for fronts with p <= 32, m <= 72, the oversized fronts' LDS-panel code otherwise
__global__ __launch_bounds__(64) void k_solve_bwd_w2(SolveArgs A, const int32_t* __restrict__ fronts) {
    extern __shared__ __attribute__((aligned(16))) double smem_s[];
    const int lane = threadIdx.x;
    const int f = fronts[blockIdx.x];
    const int m = A.fm[f], p = A.fp[f];
    const int64_t ro = A.rows_off[f], Lo = A.L_off[f];
    const int piv = lane < p ? (int)A.piv[ro + lane] : (int)PIV_NULL;
    double xj;
    if (rg_fits(m, p)) {
        double B[kRgCols], H[4];
        rg_load_cols(A.L, Lo, m, p, 0, 0, B);
        if (m > 64) rg_load_high(A.L, Lo, m, p, H);
        const double xr0 = lane < m ? A.w[A.frow[ro + lane]] : 0.0;
        const double xh = 64 + (lane & 7) < m ? A.w[A.frow[ro + 64 + (lane & 7)]] : 0.0;
        xj = rg_bwd_core(B, H, xr0, xh, m, p, piv, smem_s, [] {});
    } else {
        double* X = smem_s;
        for (int i = lane; i < m; i += 64) X[i] = A.w[A.frow[ro + i]];
        xj = rg_bwd_over_core(A.L, Lo, m, p, smem_s + 128, X, piv);
    }
    if (lane < p) A.w[A.frow[ro + lane]] = xj;
}

// right-hand side into elimination order (xs[xpos[i]] = s_i b_i) and the solution back (x_i = s_i xs[xpos[i]])
__global__ void k_xs_in(const double* __restrict__ b, const double* __restrict__ scale, const int32_t* __restrict__ xpos,
                        double* __restrict__ xs, int64_t n, const int32_t* __restrict__ list) {
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = list ? list[t] : t;
        xs[xpos[i]] = scale[i] * b[i];
    }
}
__global__ void k_xs_out(const double* __restrict__ xs, const double* __restrict__ scale, const int32_t* __restrict__ xpos,
                         const uint32_t* __restrict__ abort_flag, double* __restrict__ x, int64_t n, const int32_t* __restrict__ list,
                         int sub) {
    if (*abort_flag) return;  // aborted dataflow solve: x (possibly aliasing the rhs) is left untouched
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = list ? list[t] : t;
        const double d = __dmul_rn(scale[i], xs[xpos[i]]);  // no contraction into the subtraction
        x[i] = sub ? x[i] - d : d;
    }
}
__global__ void k_xpos_top(const int32_t* __restrict__ top_orig, int64_t n_top, int64_t top_base, int32_t* __restrict__ xpos) {
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n_top; t += (int64_t)gridDim.x * blockDim.x)
        xpos[top_orig[t]] = (int32_t)(top_base + t);
}
__global__ __launch_bounds__(64) void k_cvx_to_cvec(DfArgs D, SolveArgs A, const int32_t* __restrict__ roots, int count,
                                                    double* __restrict__ cvec) {
    for (int r = blockIdx.x; r < count; r += gridDim.x) {
        const int f = roots[r];
        const int cm = A.fm[f] - A.fp[f];
        const double* src = D.cvx + D.cvx_off[f];
        double* dst = cvec + A.relmap_off[f];
        for (int t = threadIdx.x; t < cm; t += 64) dst[t] = src[t];
    }
}
__global__ void k_set_done(uint32_t* __restrict__ done, const int32_t* __restrict__ list, int count, uint32_t epoch) {
    for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < count; t += gridDim.x * blockDim.x)
        __hip_atomic_store(done + list[t], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Per-factorization map for the dataflow backward solve: rxpos[row slot] = xs index of the row's
// solution value (pass 0: xpos[original id] of every pivot; pass 1: rows >= p of every front).  Flat over
// the front rows (coalesced): rowx (per analysis) holds each walk front's pivot-position xs slot, or -2 for its
// contribution rows; frow (per factorization) the row now at that position.  One block per front left both
// passes dispatch-bound (2 x 15 us at C3), one thread per front gather-bound (2 x 25 us).
__global__ void k_xpos(DfArgs D, const int32_t* __restrict__ frow, int32_t* __restrict__ xpos,
                       int32_t* __restrict__ rxpos, int pass) {
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < D.rows_total; t += (int64_t)gridDim.x * blockDim.x) {
        const int32_t v = D.rowx[t];
        if (pass == 0) {
            if (v >= 0) xpos[frow[t]] = v;
        } else if (v == -2) {
            rxpos[t] = xpos[frow[t]];
        }
    }
}

// ------------------------------------------------------------------------------------------------
// large fronts (m > kMaxLdsFront): blocked LDL^T in HBM scratch, trailing updates on MFMA f64
// ------------------------------------------------------------------------------------------------
// The front lives in its FullStore (row-major, lower triangle used) and is factored in panels of at most
// kBigNB pivots by a sequence of batched launches over the large fronts of one level:
//   k_big_init / k_big_entries / k_big_child   zero, original entries, children's contribution blocks
//                   (the additions of assemble_front, same order), row ids -- 2-D grids (slices x fronts)
//   k_big_panel_reg one block per front (m <= 4096): the next panel's pivots with the panel in registers
//                   (below); k_big_panel for larger fronts: column k is brought up to date
//                   left-looking (minus the panel's earlier pivots, L(i,q) W(k,q)), then tested with the
//                   threshold rule; a pass is a 1x1 pivot.  On a failure with pivots pending the panel
//                   ends (the trailing update must land first); on a failure at the panel's start every
//                   column is current and the exact full search of the small-front kernels runs
//                   (search_pivot: interchanges, 2x2, null pivots, relaxed ladder) -- so the pivot
//                   sequence follows the same rule as factor_front / the oracle.
//   k_big_update    C -= L21 W21^T over the trailing lower triangle, W = the unnormalised pivot columns
//                   (= L D), on v_mfma_f64_16x16x4f64: 64 x 64 macro tiles, one 16-row strip per wave.
//   k_big_finish    L (packed trapezoid), pivoted row maps, contribution block, pivot counters.
// The host repeats panel + update until every front of the launch is done (one check per batch).
constexpr int kBigNB = 32;


// L(i, q) = ca * W(i, base) + cb * W(i, base + 1): the write-out coefficients of factor_front
template <class S>
__device__ __forceinline__ void piv_coefs(const S& st, const int8_t* piv, int q, double& ca, double& cb, int& base) {
    const int8_t kind = piv[q];
    ca = 0.0; cb = 0.0; base = q;
    if (kind == PIV_1X1) {
        ca = 1.0 / st.at(q, q);
    } else if (kind == PIV_2X2_A || kind == PIV_2X2_B) {
        const int k0 = kind == PIV_2X2_A ? q : q - 1;
        const double a = st.at(k0, k0), b = st.at(k0 + 1, k0), e = st.at(k0 + 1, k0 + 1);
        const double idet = 1.0 / (a * e - b * b);
        if (kind == PIV_2X2_A) { ca = e * idet; cb = -b * idet; }
        else { ca = -b * idet; cb = a * idet; }
        base = k0;
    }
}

__device__ __forceinline__ double block_max256(double v, double* red) {
    v = wave_max_abs(v);  // non-negative values
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    const double r = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
    __syncthreads();
    return r;
}

// Assembly of the large fronts, spread over a 2-D grid (x: slices of the front, y: fronts) so an order-m
// front is not assembled by one workgroup (m^2 stores plus the children's (m - p)^2 / 2 additions at one
// CU's bandwidth was ~1 ms per front at m = 2048).  Three passes with the additions of assemble_front
// in the same order per element: zero (+ row ids, state), original entries (distinct positions,
// stored), then child 0, 1, ... (one launch each; a child's elements map to distinct parent positions).
__global__ __launch_bounds__(kThreads) void k_big_init(FactorArgs A, const int32_t* __restrict__ fronts) {
    const int f = fronts[blockIdx.y];
    const int m = A.fm[f], p = A.fp[f];
    double* F = A.gscratch + A.gscratch_off[f];
    const int64_t tot = (int64_t)m * m;
    for (int64_t t = (int64_t)blockIdx.x * kThreads + threadIdx.x; t < tot; t += (int64_t)gridDim.x * kThreads) F[t] = 0.0;
    if (blockIdx.x == 0) {
        const int64_t ro = A.rows_off[f];
        for (int i = threadIdx.x; i < m; i += kThreads) {
            A.frow[ro + i] = A.rows[ro + i];  // row ids, permuted in place by the interchanges
            A.fpos[ro + i] = i;               // analysis-order local row of position i (inverted by k_big_finish)
        }
        if (threadIdx.x == 0) {
            BigFrontState z{};
            z.done = p == 0;
            z.minpiv = INFINITY;
            A.big[f] = z;
        }
    }
}

__global__ __launch_bounds__(kThreads) void k_big_entries(FactorArgs A, const int32_t* __restrict__ fronts) {
    const int f = fronts[blockIdx.y];
    const int m = A.fm[f];
    const FullStore st{A.gscratch + A.gscratch_off[f], m};
    const int64_t ro = A.rows_off[f];
    const int64_t e0 = A.ent_off[f], e1 = A.ent_off[f + 1];
    for (int64_t e = e0 + (int64_t)blockIdx.x * kThreads + threadIdx.x; e < e1; e += (int64_t)gridDim.x * kThreads) {
        const uint32_t lp = A.ent_lpos[e];
        const int lr = (int)(lp >> 16), lc = (int)(lp & 0x7fffu);
        const double sr = A.scale[A.rows[ro + lr]], sc = A.scale[A.rows[ro + lc]];
        const double uv = A.uval[e];
        st.at(lr, lc) = (lp & 0x8000u) ? sc * uv * sr : sr * uv * sc;  // assemble_front's multiplication order
    }
}

__global__ __launch_bounds__(kThreads) void k_big_child(FactorArgs A, const int32_t* __restrict__ fronts, int ci) {
    const int f = fronts[blockIdx.y];
    const int c = A.child_off[f] + ci;
    if (c >= A.child_off[f + 1]) return;
    const int m = A.fm[f];
    const FullStore st{A.gscratch + A.gscratch_off[f], m};
    const int cm = A.ch_cm[c];
    const int32_t* rm = A.relmap + A.ch_relmap_off[c];
    const double* cb = A.cb + A.ch_cb_off[c];
    const int ctot = cm * (cm + 1) / 2;
    for (int t = blockIdx.x * kThreads + threadIdx.x; t < ctot; t += gridDim.x * kThreads) {
        int r, cc;
        tri_rc(t, r, cc);
        st.at(rm[r], rm[cc]) += cb[t];
    }
}

// Trailing update of the pending panel [k0, k1): rows / columns [k1, m), lower triangle.  Block = one
// 64 x 64 macro tile (blockIdx.x, lower-triangular order) of front fronts[blockIdx.y]; wave w owns rows
// 16w .. 16w+15 of it and four 16 x 16 MFMA accumulators along the columns.
__global__ __launch_bounds__(kThreads) void k_big_update(FactorArgs A, const int32_t* __restrict__ fronts) {
    __shared__ double cA[kBigNB + 2], cB[kBigNB + 2];
    __shared__ int bq[kBigNB + 2];
    const int f = fronts[blockIdx.y];
    const BigFrontState S = A.big[f];
    const int k0 = S.k0, k1 = S.k1;
    if (k1 <= k0) return;
    const int m = A.fm[f];
    const int u0 = S.pad > k1 ? S.pad : k1;  // k_big_panel_reg writes its whole panel back: the update starts after it
    const int nt = (m - u0 + 63) / 64;
    if ((int)blockIdx.x >= nt * (nt + 1) / 2) return;
    int ti, tj;
    tri_rc((int)blockIdx.x, ti, tj);
    const FullStore st{A.gscratch + A.gscratch_off[f], m};
    const int8_t* piv = A.piv + A.rows_off[f];
    const int np = k1 - k0;
    for (int q = threadIdx.x; q < np; q += kThreads) {
        double ca, cb;
        int b;
        piv_coefs(st, piv, k0 + q, ca, cb, b);
        cA[q] = ca; cB[q] = cb; bq[q] = b;
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int i0 = u0 + 64 * ti + 16 * w;
    const int lr = lane & 15, lk = lane >> 4;
    dbl4 acc[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int j0 = u0 + 64 * tj + 16 * c;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = i0 + lk + 4 * r, j = j0 + lr;
            acc[c][r] = (i < m && j < m && j <= i) ? st.at(i, j) : 0.0;
        }
    }
    const bool diag = ti == tj;
    const int ia = i0 + lr;  // A-operand row of this lane
    for (int q = 0; q < np; q += 4) {
        const int qq = q + lk;
        double a = 0.0;
        if (qq < np && ia < m) {
            a = cA[qq] * st.at(ia, bq[qq]);
            if (cB[qq] != 0.0) a += cB[qq] * st.at(ia, bq[qq] + 1);
            a = -a;
        }
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            if (diag && c > w) continue;  // wave-uniform: strip entirely above the diagonal
            const int jb = u0 + 64 * tj + 16 * c + lr;  // B-operand column of this lane
            const double b = (qq < np && jb < m) ? st.at(jb, k0 + qq) : 0.0;
            acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[c], 0, 0, 0);
        }
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        if (diag && c > w) continue;
        const int j0 = u0 + 64 * tj + 16 * c;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = i0 + lk + 4 * r, j = j0 + lr;
            if (i < m && j < m && j <= i) st.at(i, j) = acc[c][r];
        }
    }
}

// ---- a-posteriori blocked steps of the large fronts ----
// One step takes the next kAppNB columns of every unfinished large front in three launches, so the trailing
// matrix is read and written once per kAppNB pivots (one rank-kAppNB MFMA update) instead of once per
// register panel of 8 or 16:
//   k_app_diag   one wave per front: the diagonal block right-looking in registers (lane = row), each column's quick Duff-Reid 1x1 test, else the 2x2 test with the next column,
//                over the block's rows; the first failure ends the block (nbt columns pass).  W (un-normalised columns) into the step's panel, pivots into AppSlot.
//   k_app_rows   the rows below, one per lane: W(i, c) = A(i, c) - sum_{q < c} L(i, q) W(c, q), L = W / d
//                (k_big_panel_reg's products, pivots ascending), into the panel; per-column max |W(i, c)|
//                by atomic max of the bits.  The last block to arrive applies the complete quick test
//                u max_i |W(i, c)| <= |d_c| a posteriori: the first failing column ends the accepted run
//                (nacc) -- the later columns' W used a rejected pivot and are discarded (column c of W
//                depends on pivots <= c only) -- and commits pivots, counters and the front state.
//   k_app_update C -= L W^T of the nacc accepted pivots over the trailing lower triangle from column k0 + nacc
//                (A / B tiles staged in LDS, v_mfma_f64_16x16x4f64), plus the accepted columns (W form,
//                diagonal = d) copied into the front.
// The accepted pivots are the ones the register panel's quick test would accept on the same column values
// (up to the rounding of the MFMA update order).  A failure leaves the front current at the failing column
// with BigFrontState::exact set: the register panel then runs its exact search there (interchanges, 2x2,
// null pivots, relaxation, delays) and k_big_update applies its pivots, in the same step.
__device__ __forceinline__ double* app_panel(const FactorArgs& A, int f, int m) {
    return A.gscratch + A.gscratch_off[f] + (int64_t)m * m;
}
__device__ __forceinline__ AppSlot* app_slot(const FactorArgs& A, int f, int m) {
    return reinterpret_cast<AppSlot*>(app_panel(A, f, m) + (int64_t)m * kAppNB);
}

template <class F, int... I>
__device__ __forceinline__ void each_index(F& f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}

// One wave (lane = row).  Pivot c's d, block-local column maximum, off-diagonal and kind stay in lane c's
// registers until the loop ends: a global store per step would make every step's barrier wait for its
// completion.  One wave, every lane publishes and reads: the column broadcast needs compiler ordering only (a memory
// clobber: the LDS operations of one wave complete in issue order).
// The 64 steps are expanded at compile time (each_index): a[] indices stay constants, i.e. registers (the plain
// unrolled loop with the 2x2 branch passes the full-unroll limit, and the rolled one indexes a[] from scratch).
// The tests run on upper bounds of the column maxima (wave_max_abs_ub), recorded as such: conservative by 2^-20
// at most, so every accepted pivot passes the exact test, and a borderline one is left to k_app_exact's exact rule.
__global__ __launch_bounds__(64) void k_app_diag(FactorArgs A, const int32_t* __restrict__ fronts) {
    __shared__ double colc[kAppNB], colc1[kAppNB];
    const int lane = threadIdx.x;
    const int f = fronts[blockIdx.x];
    const int m = A.fm[f], p = A.fp[f];
    BigFrontState* Sg = A.big + f;
    const int k = Sg->k;
    AppSlot* sl = app_slot(A, f, m);
    const int nb = Sg->done ? 0 : min(kAppNB, p - k);
    if (nb <= 0) {
        if (lane == 0) { sl->nbt = 0; sl->nacc = 0; Sg->k0 = Sg->k1; }
        return;
    }
    const FullStore st{A.gscratch + A.gscratch_off[f], m};
    const double thres = A.anorm_bits ? DBL_EPSILON * A.null_fac * as_double(*A.anorm_bits) : 0.0;
    const double* row = st.F + (int64_t)(k + (lane < nb ? lane : 0)) * m + k;
    double a[kAppNB];
#pragma unroll
    for (int c = 0; c < kAppNB; ++c) a[c] = (lane < nb && c <= lane) ? row[c] : 0.0;
    int nbt = nb;
    double dmine = 0.0, gmine = 0.0, omine = 0.0;
    int kmine = PIV_1X1;
    bool second = false;  // column c is the second of an accepted 2x2 pair (uniform)
    auto step = [&](auto cc) {
        constexpr int c = decltype(cc)::value;
        if (c >= nbt) return;  // uniform
        if (second) { second = false; return; }
        const double akk = readlane_d(a[c], c);
        const double g = wave_max_abs_ub((lane > c && lane < nb) ? fabs(a[c]) : 0.0);
        const double aak = fabs(akk);
        if (aak > thres && !(A.u * g > aak)) {  // 1x1 (uniform)
            dmine = lane == c ? akk : dmine;
            gmine = lane == c ? g : gmine;
            const double l = lane > c ? a[c] * (1.0 / akk) : 0.0;
            colc[lane] = a[c];  // W(k + lane, c): every lane writes, every lane reads (no conditional publish)
            // compiler ordering only: a memory clobber keeps the reads after the write and before the next step's
            // write (wave_lds_sync's fences cost this 256-VGPR kernel its batched reads: 36.7 -> 46.4 us per launch)
            __asm__ volatile("" ::: "memory");
#pragma unroll
            for (int j = c + 1; j < kAppNB; ++j) a[j] -= l * colc[j];
            __asm__ volatile("" ::: "memory");
            return;
        }
        // 2x2 with the next column, no interchange: Duff-Reid's 2x2 test (oracle test_pivot's inequalities) on the
        // block's rows below the pair now, on every row below it a posteriori (k_app_rows).  A valid threshold
        // pivot -- not always the partner MUMPS would pick (the argmax row): large fronts are checked by inertia
        // and residual, not bit for bit.
        constexpr int cn = c + 1 < kAppNB ? c + 1 : c;
        if (c + 1 < nb) {  // uniform
            const double b = readlane_d(a[c], cn), dd = readlane_d(a[cn], cn);
            const double gc = wave_max_abs_ub((lane > c + 1 && lane < nb) ? fabs(a[c]) : 0.0);
            const double gr = wave_max_abs_ub((lane > c + 1 && lane < nb) ? fabs(a[cn]) : 0.0);
            const double det = akk * dd - b * b;
            const double lim = fabs(det) / A.u;
            if (det != 0.0 && fmax(aak, fabs(b)) > thres && fabs(dd) > 0.0 && fabs(dd) * gc + fabs(b) * gr <= lim &&
                fabs(b) * gc + aak * gr <= lim) {
                dmine = lane == c ? akk : (lane == c + 1 ? dd : dmine);
                gmine = lane == c ? gc : (lane == c + 1 ? gr : gmine);
                omine = lane == c || lane == c + 1 ? b : omine;
                kmine = lane == c ? PIV_2X2_A : (lane == c + 1 ? PIV_2X2_B : kmine);
                const double inv = 1.0 / det;
                const double l0 = lane > c + 1 ? (dd * a[c] - b * a[cn]) * inv : 0.0;
                const double l1 = lane > c + 1 ? (akk * a[cn] - b * a[c]) * inv : 0.0;
                colc[lane] = a[c];
                colc1[lane] = a[cn];
                __asm__ volatile("" ::: "memory");
#pragma unroll
                for (int j = c + 2; j < kAppNB; ++j) a[j] -= l0 * colc[j] + l1 * colc1[j];
                __asm__ volatile("" ::: "memory");
                second = true;
                return;
            }
        }
        nbt = c;  // uniform
    };
    each_index(step, std::make_integer_sequence<int, kAppNB>{});
    if (lane < nbt) {
        sl->d[lane] = dmine;
        sl->cmax[lane] = as_bits(gmine);
        sl->offd[lane] = omine;
        sl->kind[lane] = (int8_t)kmine;
        double* pr = app_panel(A, f, m) + (int64_t)lane * kAppNB;
#pragma unroll
        for (int c = 0; c < kAppNB; ++c)
            if (c <= lane) pr[c] = a[c];
    }
    if (lane == 0) {
        sl->k0 = k; sl->nbt = nbt; sl->nb = nb; sl->nacc = 0; sl->arrive = 0u;
        if (nbt == 0) Sg->exact = 1;  // the first column fails already within the block
        Sg->k0 = Sg->k1;              // nothing pending for k_big_update unless the register panel runs
    }
}

// L(i, c) = cself[c] W(i, c) + coth[c] W(i, partner(c)) for the accepted pivot columns of an a-posteriori step:
// 1x1: 1 / d; 2x2 pair (a, b; b, e) = the columns (c, c + 1): L(i, c) = (e W_c - b W_c+1) / det, L(i, c + 1) =
// (a W_c+1 - b W_c) / det (the oracle's elim_2x2 with the inverse precomputed)
__device__ __forceinline__ void app_coefs(const AppSlot* sl, int c, int nbt, double& cself, double& coth, int& partner) {
    cself = 0.0;
    coth = 0.0;
    partner = c;
    if (c >= nbt) return;
    const int kind = sl->kind[c];
    if (kind == PIV_2X2_A || kind == PIV_2X2_B) {
        const int c0 = kind == PIV_2X2_A ? c : c - 1;
        const double a = sl->d[c0], e = sl->d[c0 + 1], b = sl->offd[c0];
        const double inv = 1.0 / (a * e - b * b);
        cself = (kind == PIV_2X2_A ? e : a) * inv;
        coth = -b * inv;
        partner = kind == PIV_2X2_A ? c + 1 : c - 1;
    } else {
        cself = 1.0 / sl->d[c];
    }
}

// quad_perm broadcast of lane s of each quad (s a constant once the caller's loop is unrolled)
__device__ __forceinline__ double quad_bcast(double v, int s) {
    switch (s & 3) {
        case 0: return as_double(dpp64<0x00>(as_bits(v)));
        case 1: return as_double(dpp64<0x55>(as_bits(v)));
        case 2: return as_double(dpp64<0xAA>(as_bits(v)));
        default: return as_double(dpp64<0xFF>(as_bits(v)));
    }
}

// 64 rows per block, four lanes per row: lane q of a quad owns the row's columns q, q + 4, ... (balanced
// over the triangle); column c's multiplier comes from its owner by a quad broadcast
__global__ __launch_bounds__(256) void k_app_rows(FactorArgs A, const int32_t* __restrict__ fronts) {
    __shared__ __attribute__((aligned(16))) double WdS[kAppNB][4][kAppNB / 4];  // W(k0 + 4jj + q, c) at [c][q][jj]
    __shared__ double amax[kAppNB][kAppNB + 1];                              // |W| of the block's rows, [col][row]
    __shared__ double cself[kAppNB], coth[kAppNB];                           // app_coefs
    __shared__ int kindS[kAppNB];
    __shared__ int last;
    const int tid = threadIdx.x, q = tid & 3, rl = tid >> 2;
    const int lane = tid & 63;
    const int f = fronts[blockIdx.y];
    const int m = A.fm[f];
    AppSlot* sl = app_slot(A, f, m);
    const int nbt = sl->nbt;
    if (nbt == 0) return;  // no step for this front (done, or the register panel's exact search is next)
    const int k0 = sl->k0;
    double* P = app_panel(A, f, m);
    // the pair's second row (W(c + 1, c) = its off-diagonal) is not an update operand of the pair's columns
    // thread t stages column c = t % 64 of rows t / 64 + 4 u: every load issued before the first LDS write
    {
        const int c = tid & 63, j0 = tid >> 6;
        const bool pairc = c < nbt && sl->kind[c] == PIV_2X2_A;
        double v[kAppNB / 4];
#pragma unroll
        for (int u = 0; u < kAppNB / 4; ++u) v[u] = P[(int64_t)(j0 + 4 * u) * kAppNB + c];
#pragma unroll
        for (int u = 0; u < kAppNB / 4; ++u) {
            const int j = j0 + 4 * u;
            WdS[c][j & 3][j >> 2] = (c < j && j < nbt && !(pairc && j == c + 1)) ? v[u] : 0.0;
        }
    }
    if (tid < kAppNB) {
        int pt;
        app_coefs(sl, tid, nbt, cself[tid], coth[tid], pt);
        kindS[tid] = tid < nbt ? (int)sl->kind[tid] : PIV_1X1;
    }
    __syncthreads();
    const FullStore st{A.gscratch + A.gscratch_off[f], m};
    const int i = k0 + nbt + (int)blockIdx.x * 64 + rl;
    const bool valid = i < m;
    const double* row = st.F + (int64_t)(valid ? i : k0) * m + k0;
    double w[kAppNB / 4];
#pragma unroll
    for (int jj = 0; jj < kAppNB / 4; ++jj) w[jj] = (valid && 4 * jj + q < nbt) ? row[4 * jj + q] : 0.0;
    // one update body per column (the code stays within the instruction cache): L(i, c) = cself W(i, c) +
    // coth W(i, partner).  A pair's columns are applied one after the other: column c's update does not touch
    // W(i, c + 1) (the pair row is zero in WdS[c]) and no update touches columns <= c, so both L(i, .) of the
    // pair see the W values of the pair's start.
#pragma unroll
    for (int c = 0; c < kAppNB; ++c) {
        const int kc = kindS[c];  // uniform
        const double wc = quad_bcast(w[c >> 2], c & 3);
        const double wa = quad_bcast(w[(c + 1 < kAppNB ? c + 1 : c) >> 2], (c + 1) & 3);
        const double wb = quad_bcast(w[(c > 0 ? c - 1 : c) >> 2], (c + 3) & 3);
        const double wp = kc == PIV_2X2_A ? wa : (kc == PIV_2X2_B ? wb : 0.0);
        const double l = cself[c] * wc + coth[c] * wp;  // 0 from column nbt on
        const double* wd = &WdS[c][q][0];
#pragma unroll
        for (int jj = c >> 2; jj < kAppNB / 4; ++jj) w[jj] -= l * wd[jj];  // W(., c) = 0 at columns <= c
        __asm__ volatile("" ::: "memory");  // the next column's LDS operands are not hoisted above this one
    }
    if (valid) {
        double* pw = P + (int64_t)(i - k0) * kAppNB;
#pragma unroll
        for (int jj = 0; jj < kAppNB / 4; ++jj)
            if (4 * jj + q < nbt) pw[4 * jj + q] = w[jj];
    }
#pragma unroll
    for (int jj = 0; jj < kAppNB / 4; ++jj) amax[4 * jj + q][rl] = fabs(w[jj]);  // invalid rows hold 0
    __syncthreads();
    if (tid < kAppNB) {
        double g = 0.0;
        for (int r = 0; r < 64; ++r) g = fmax(g, amax[tid][r]);
        if (tid < nbt && g > 0.0) atomicMax(&sl->cmax[tid], as_bits(g));
    }
    __threadfence();
    __syncthreads();
    if (tid == 0) last = atomicAdd(&sl->arrive, 1u) == gridDim.x - 1;
    __syncthreads();
    if (!last || tid >= 64) return;
    __threadfence();
    // every block's maxima are in: the a-posteriori test and the commit
    const unsigned long long cm = lane < nbt ? __hip_atomic_load(&sl->cmax[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
    const double dd = lane < nbt ? sl->d[lane] : 0.0;
    const int kind = lane < nbt ? (int)sl->kind[lane] : PIV_1X1;
    const double off = lane < nbt ? sl->offd[lane] : 0.0;
    // 2x2 pairs: the test of k_app_diag again with the maxima over every row below the pair
    const double g = as_double(cm), gn = __shfl(g, lane < 63 ? lane + 1 : lane), dn = __shfl(dd, lane < 63 ? lane + 1 : lane);
    const double det = dd * dn - off * off;
    const double lim = fabs(det) / A.u;
    const bool badA = !(det != 0.0 && fabs(dn) * g + fabs(off) * gn <= lim && fabs(off) * g + fabs(dd) * gn <= lim);
    const bool badAprev = __shfl(badA, lane > 0 ? lane - 1 : 0);
    const bool bad1 = kind == PIV_2X2_A ? badA : kind == PIV_2X2_B ? badAprev : A.u * g > fabs(dd);
    const unsigned long long bad = __ballot(lane < nbt && bad1);
    const int nacc = bad ? (int)__builtin_ctzll(bad) : nbt;  // a failing pair fails at its first column
    const bool acc = lane < nacc;
    if (acc) A.piv[A.rows_off[f] + k0 + lane] = (int8_t)kind;
    // inertia: a 1x1 by its sign; a pair by det < 0 (one each) or the sign of its trace (both)
    const int npos = (int)__popcll(__ballot(acc && kind == PIV_1X1 && dd > 0.0)) +
                     (int)__popcll(__ballot(acc && kind == PIV_2X2_A && det < 0.0)) +
                     2 * (int)__popcll(__ballot(acc && kind == PIV_2X2_A && det > 0.0 && dd + dn > 0.0));
    const int n2 = (int)__popcll(__ballot(acc && kind == PIV_2X2_A));
    double mn = acc ? (kind == PIV_1X1 ? fabs(dd) : fmax(fabs(dd), fabs(off))) : INFINITY;
    for (int o = 32; o > 0; o >>= 1) mn = fmin(mn, __shfl_xor(mn, o));
    if (lane == 0) {
        BigFrontState S = A.big[f];
        S.npos += npos;
        S.nneg += nacc - npos;
        S.n2 += n2;
        S.minpiv = fmin(S.minpiv, mn);
        S.k = k0 + nacc;
        S.k0 = S.k;
        S.k1 = S.k;
        S.done = S.k >= A.fp[f];
        S.exact = (!S.done && nacc < sl->nb) ? 1 : 0;
        A.big[f] = S;
        sl->nacc = nacc;
    }
}

// The exact step of the a-posteriori path at a failing column (BigFrontState::exact): the exact search
// (search_pivot_blk: interchanges, 2x2, null pivots, relaxation ladder, delays) decides one or two pivots
// on the current front; their columns are already their W columns, so nothing else is computed here --
// k_big_update applies them to the trailing matrix and the next a-posteriori step continues after them.
// (The register panel k_big_panel_reg would also load and write back NB columns: ~35 us more per step
// at m = 4096.)
__global__ __launch_bounds__(512) void k_app_exact(FactorArgs A, const int32_t* __restrict__ fronts) {
    constexpr int T = 512;
    __shared__ unsigned long long ured[T / 64];
    __shared__ BigFrontState SF;
    const int tid = threadIdx.x;
    const int f = fronts[blockIdx.x];
    if (tid == 0) SF = A.big[f];
    __syncthreads();
    if (SF.done || !SF.exact) return;
    const int m = A.fm[f], p = A.fp[f];
    const int64_t ro = A.rows_off[f];
    const FullStore st{A.gscratch + A.gscratch_off[f], m};
    int32_t* lrow = A.frow + ro;
    int32_t* lorig = A.fpos + ro;
    int8_t* piv = A.piv + ro;
    const double thres = A.anorm_bits ? DBL_EPSILON * A.null_fac * as_double(*A.anorm_bits) : 0.0;
    double minpiv = SF.minpiv;
    const int k = SF.k;
    PivotDecision d = search_pivot_blk<T>(st, m, k, p, A.u, thres, minpiv, ured);
    const bool stuck = d.kind == PIV_STUCK;
    if (stuck) { d.kind = PIV_NULL; d.c = k; }
    if (d.c != k) {
        sym_swap_batched<T>(st, m, k, d.c, lrow, lorig);
        __syncthreads();
    }
    if (d.kind == PIV_2X2_A) {
        const int r = d.r == k ? d.c : d.r;
        if (r != k + 1) {
            sym_swap_batched<T>(st, m, k + 1, r, lrow, lorig);
            __syncthreads();
        }
    }
    int np = 1;
    if (d.kind == PIV_NULL) {
        for (int i = k + 1 + tid; i < m; i += T) st.at(i, k) = 0.0;
    } else if (d.kind == PIV_2X2_A) {
        np = 2;
    }
    if (tid == 0) {
        if (stuck) SF.nstuck++;
        SF.nrel += d.relaxed;
        if (d.relaxed && !SF.delays && A.record_delays && A.fparent[f] >= 0) {  // see factor_front
            SF.delays = 1;
            const unsigned long long base = atomicAdd(&A.counters[6], (unsigned long long)(p - k));
            for (int q = k; q < p; ++q) A.delayed[base + (q - k)] = lrow[q];
        }
        if (d.kind == PIV_NULL) {
            piv[k] = PIV_NULL;
            SF.nzero++;
        } else if (d.kind == PIV_1X1) {
            const double dk = st.at(k, k);
            piv[k] = PIV_1X1;
            if (dk > 0.0) SF.npos++; else SF.nneg++;
        } else {
            const double a = st.at(k, k), b = st.at(k + 1, k), e = st.at(k + 1, k + 1);
            const double det = a * e - b * b;
            piv[k] = PIV_2X2_A; piv[k + 1] = PIV_2X2_B; SF.n2++;
            if (det < 0.0) { SF.npos++; SF.nneg++; }
            else if (a + e > 0.0) SF.npos += 2;
            else SF.nneg += 2;
        }
        SF.minpiv = minpiv;
        SF.k0 = k;
        SF.k1 = k + np;
        SF.k = k + np;
        SF.pad = k + np;  // the trailing update starts right after the pivots
        SF.done = SF.k >= p;
        SF.exact = 0;
        A.big[f] = SF;
    }
}

// grid.x: tiles_max trailing tiles (lower-triangular order, 64 x 64, wave w owns rows 16w..16w+15 as in
// k_big_update), then ceil(mmax / 64) copy blocks of 64 panel rows each
__global__ __launch_bounds__(kThreads) void k_app_update(FactorArgs A, const int32_t* __restrict__ fronts, int tiles_max) {
    __shared__ __attribute__((aligned(16))) double As[kAppNB][64 + 2];  // -L(i0t + r, q) at [q][r]
    __shared__ __attribute__((aligned(16))) double Bs[kAppNB][64 + 2];  //  W(j0t + c, q) at [q][c]
    const int f = fronts[blockIdx.y];
    const int m = A.fm[f];
    const AppSlot* sl = app_slot(A, f, m);
    const int nacc = sl->nacc;
    if (nacc == 0) return;
    const int k0 = sl->k0, u0 = k0 + nacc;
    const double* P = app_panel(A, f, m);
    const FullStore st{A.gscratch + A.gscratch_off[f], m};
    const int tid = threadIdx.x;
    if ((int)blockIdx.x >= tiles_max) {  // the accepted columns into the front
        const int rb = (int)blockIdx.x - tiles_max;
        for (int t = tid; t < 64 * kAppNB; t += kThreads) {
            const int rr = 64 * rb + (t >> 6), q = t & 63;
            const int i = k0 + rr;
            if (i < m && q < nacc && q <= rr) st.at(i, k0 + q) = P[(int64_t)rr * kAppNB + q];
        }
        return;
    }
    const int nt = (m - u0 + 63) / 64;
    if ((int)blockIdx.x >= nt * (nt + 1) / 2) return;
    int ti, tj;
    tri_rc((int)blockIdx.x, ti, tj);
    const int i0t = u0 + 64 * ti, j0t = u0 + 64 * tj;
    // the panel staging: thread t stages column q = t % 64 of rows t / 64 + 4 u (its coefficients formed by
    // itself, no barrier before); every load is issued before the first LDS write (one memory round trip,
    // not one per row), and the C tile's loads go out with them
    static_assert(kThreads == 4 * kAppNB, "staging: 4 rows x 64 columns per pass");
    constexpr int SR = 64 / (kThreads / kAppNB);  // rows per thread
    const int q = tid & 63, r0 = tid >> 6;
    double cs, co;
    int pt;
    app_coefs(sl, q, nacc, cs, co, pt);
    double pa[SR], pb[SR], pc[SR];
#pragma unroll
    for (int u = 0; u < SR; ++u) {
        const int r = r0 + 4 * u;
        const int i = min(i0t + r, m - 1), j = min(j0t + r, m - 1);  // clamped: rows past m stage zeros below
        const double* Pi = P + (int64_t)(i - k0) * kAppNB;
        pa[u] = Pi[q];
        pb[u] = Pi[pt];
        pc[u] = P[(int64_t)(j - k0) * kAppNB + q];
    }
    const int lane = tid & 63, w = tid >> 6;
    const int lr = lane & 15, lk = lane >> 4;
    const int i0 = i0t + 16 * w;
    dbl4 acc[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int j0 = j0t + 16 * c;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = i0 + lk + 4 * r, j = j0 + lr;
            acc[c][r] = (i < m && j < m && j <= i) ? st.at(i, j) : 0.0;
        }
    }
#pragma unroll
    for (int u = 0; u < SR; ++u) {
        const int r = r0 + 4 * u;
        As[q][r] = (i0t + r < m && q < nacc) ? -(cs * pa[u] + co * pb[u]) : 0.0;
        Bs[q][r] = (j0t + r < m && q < nacc) ? pc[u] : 0.0;
    }
    __syncthreads();
    const bool diag = ti == tj;
    for (int qq = 0; qq < nacc; qq += 4) {
        const double a = As[qq + lk][16 * w + lr];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            if (diag && c > w) continue;  // wave-uniform: strip entirely above the diagonal
            const double b = Bs[qq + lk][16 * c + lr];
            acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[c], 0, 0, 0);
        }
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        if (diag && c > w) continue;
        const int j0 = j0t + 16 * c;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = i0 + lk + 4 * r, j = j0 + lr;
            if (i < m && j < m && j <= i) st.at(i, j) = acc[c][r];
        }
    }
}

// fronts of a launch still factoring (host loop condition)
__global__ void k_big_pending(const FactorArgs A, const int32_t* __restrict__ fronts, int count, int32_t* __restrict__ out) {
    int n = 0;
    for (int t = threadIdx.x; t < count; t += blockDim.x) n += A.big[fronts[t]].done ? 0 : 1;
    for (int off = 32; off > 0; off >>= 1) n += __shfl_xor(n, off);
    __shared__ int red[4];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = n;
    __syncthreads();
    if (threadIdx.x == 0) *out = red[0] + red[1] + red[2] + red[3];
}

// L, contribution block, row maps and counters of the large fronts: grid (x: slices, y: fronts); the
// columns of L and the rows of the contribution block are spread over every wave of the slices, the row
// map inversion and the counters are slice 0's.
__global__ __launch_bounds__(kThreads) void k_big_finish(FactorArgs A, const int32_t* __restrict__ fronts) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    int32_t* lorig = (int32_t*)smem;
    const int tid = threadIdx.x;
    const int f = fronts[blockIdx.y];
    const int m = A.fm[f], p = A.fp[f];
    const int64_t ro = A.rows_off[f];
    const FullStore st{A.gscratch + A.gscratch_off[f], m};
    const int8_t* piv = A.piv + ro;
    const int lane = tid & 63;
    const int gw = blockIdx.x * (kThreads / 64) + (tid >> 6), nw = gridDim.x * (kThreads / 64);
    // L: packed lower trapezoid, column j rows j..m-1; one wave per column (coalesced stores)
    double* L = A.L + A.L_off[f];
    for (int j = gw; j < p; j += nw) {
        double ca, cb;
        int base;
        piv_coefs(st, piv, j, ca, cb, base);
        const int8_t kind = piv[j];
        double* Lj = L + (int64_t)j * m - (int64_t)j * (j - 1) / 2 - j;  // L(i, j) = Lj[i]
        for (int i = j + lane; i < m; i += 64) {
            double v;
            if (i == j) v = kind == PIV_NULL ? 0.0 : st.at(j, j);
            else if (kind == PIV_2X2_A && i == j + 1) v = st.at(j + 1, j);  // D off-diagonal
            else {
                v = ca * st.at(i, base);
                if (kind >= PIV_2X2_A) v += cb * st.at(i, base + 1);
            }
            Lj[i] = v;
        }
    }
    // contribution block: row-major packed lower triangle of order m - p
    const int cm = m - p;
    if (cm > 0) {
        double* cbp = A.cb + A.cb_off[f];
        for (int r = gw; r < cm; r += nw)
            for (int c = lane; c <= r; c += 64) cbp[(int64_t)r * (r + 1) / 2 + c] = st.at(p + r, p + c);
    }
    if (blockIdx.x != 0) return;
    // analysis-order local row -> pivoted position
    for (int i = tid; i < m; i += kThreads) lorig[i] = A.fpos[ro + i];
    __syncthreads();
    for (int i = tid; i < m; i += kThreads) A.fpos[ro + lorig[i]] = i;
    if (A.xpos)  // see factor_front's row-id write-out
        for (int i = tid; i < p; i += kThreads) A.xpos[A.frow[ro + i]] = (int32_t)(A.xs_off[f] + i);
    if (tid == 0) {
        const BigFrontState S = A.big[f];
        A.fstat[f] = (int32_t)((S.nstuck > 0xffff ? 0xffff : S.nstuck) | ((S.nrel > 0x7fff ? 0x7fff : S.nrel) << 16));
        A.fcnt[f] = (unsigned long long)S.npos | (unsigned long long)S.nneg << 16 | (unsigned long long)S.nzero << 32 |
                    (unsigned long long)S.n2 << 48;
        A.fmin[f] = S.minpiv;
    }
}

// ------------------------------------------------------------------------------------------------
// host-side launch helpers
// ------------------------------------------------------------------------------------------------

static int grid_for(int64_t n, int block) {
    int64_t g = (n + block - 1) / block;
    if (g > 4096) g = 4096;
    if (g < 1) g = 1;
    return (int)g;
}

hipError_t launch_pack(const double* values, const int32_t* dup_ptr, const int32_t* dup_pos, const int32_t* slot_src,
                       int64_t begin, int64_t end, double* uval, hipStream_t s) {
    if (end <= begin) return hipSuccess;
    hipLaunchKernelGGL(k_pack, dim3(grid_for(end - begin, 256)), dim3(256), 0, s, values, dup_ptr, dup_pos, slot_src, begin, end, uval);
    return hipGetLastError();
}

hipError_t launch_pack_multi(const double* values, const int32_t* dup_ptr, const int32_t* dup_pos, const int32_t* multi,
                             int64_t count, double* uval, hipStream_t s) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_pack_multi, dim3(grid_for(count, 256)), dim3(256), 0, s, values, dup_ptr, dup_pos, multi, count, uval);
    return hipGetLastError();
}

hipError_t launch_rowscan(const ScanArgs& A, int mode, hipStream_t s) {
    if (A.n > 0) {
        const int64_t threads = A.n * (mode == 2 ? 16 : 8);  // lanes per row, as in k_rowscan
        const dim3 g((unsigned)((threads + 255) / 256));
        if (mode == 0) hipLaunchKernelGGL(k_rowscan<0>, g, dim3(256), 0, s, A);
        else if (mode == 1) hipLaunchKernelGGL(k_rowscan<1>, g, dim3(256), 0, s, A);
        else hipLaunchKernelGGL(k_rowscan<2>, g, dim3(256), 0, s, A);
    }
    if (A.n_long > 0) {
        const dim3 g((unsigned)A.long_chunks, A.n_long);
        const dim3 gf((unsigned)((A.n_long + 63) / 64));
        if (mode == 0) {
            hipLaunchKernelGGL(k_rowscan_long<0>, g, dim3(kThreads), 0, s, A);
            hipLaunchKernelGGL(k_rowscan_long_fin<0>, gf, dim3(64), 0, s, A);
        } else if (mode == 1) {
            hipLaunchKernelGGL(k_rowscan_long<1>, g, dim3(kThreads), 0, s, A);
            hipLaunchKernelGGL(k_rowscan_long_fin<1>, gf, dim3(64), 0, s, A);
        } else {
            hipLaunchKernelGGL(k_rowscan_long<2>, g, dim3(kThreads), 0, s, A);
            hipLaunchKernelGGL(k_rowscan_long_fin<2>, gf, dim3(64), 0, s, A);
        }
    }
    return hipGetLastError();
}

hipError_t launch_rowscan_part(const PartArgs& A, int mode, hipStream_t s) {
    if (A.nrows <= 0) return hipSuccess;
    const dim3 g((unsigned)A.nchunks), gf((unsigned)grid_for(A.nrows, 256));
    if (mode == 0) {
        if (A.nchunks > 0) hipLaunchKernelGGL(k_rowscan_part<0>, g, dim3(kThreads), 0, s, A);
        hipLaunchKernelGGL(k_rowscan_part_fin<0>, gf, dim3(256), 0, s, A);
    } else if (mode == 1) {
        if (A.nchunks > 0) hipLaunchKernelGGL(k_rowscan_part<1>, g, dim3(kThreads), 0, s, A);
        hipLaunchKernelGGL(k_rowscan_part_fin<1>, gf, dim3(256), 0, s, A);
    } else {
        if (A.nchunks > 0) hipLaunchKernelGGL(k_rowscan_part<2>, g, dim3(kThreads), 0, s, A);
        hipLaunchKernelGGL(k_rowscan_part_fin<2>, gf, dim3(256), 0, s, A);
    }
    return hipGetLastError();
}

hipError_t launch_scale_update(const double* rmax, double* scale, const int32_t* list, int64_t n, int first, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_scale_update, dim3(grid_for(n, 256)), dim3(256), 0, s, rmax, scale, list, n, first);
    return hipGetLastError();
}

hipError_t launch_normmax(const double* rowsum, const int32_t* list, int64_t n, unsigned long long* anorm, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    int g = grid_for(n, kThreads);
    hipLaunchKernelGGL(k_normmax, dim3(g > 512 ? 512 : g), dim3(kThreads), 0, s, rowsum, list, n, anorm);
    return hipGetLastError();
}

hipError_t launch_scatter(const double* src, const int32_t* idx, double* dst, int64_t k, hipStream_t s) {
    if (k <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_scatter, dim3(grid_for(k, 256)), dim3(256), 0, s, src, idx, dst, k);
    return hipGetLastError();
}

__global__ void k_neg(const double* __restrict__ b, double* __restrict__ r, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) r[i] = -b[i];
}
__global__ void k_sub(double* __restrict__ x, const double* __restrict__ d, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) x[i] -= d[i];
}
hipError_t launch_neg(const double* b, double* r, int64_t n, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_neg, dim3(grid_for(n, 256)), dim3(256), 0, s, b, r, n);
    return hipGetLastError();
}
hipError_t launch_sub(double* x, const double* d, int64_t n, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_sub, dim3(grid_for(n, 256)), dim3(256), 0, s, x, d, n);
    return hipGetLastError();
}

hipError_t launch_scatter64(const double* src, const int64_t* idx, double* dst, int64_t k, hipStream_t s) {
    if (k <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_scatter64, dim3(grid_for(k, 256)), dim3(256), 0, s, src, idx, dst, k);
    return hipGetLastError();
}

hipError_t launch_gather(const double* src, const int32_t* idx, double* dst, int64_t k, hipStream_t s) {
    if (k <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_gather, dim3(grid_for(k, 256)), dim3(256), 0, s, src, idx, dst, k);
    return hipGetLastError();
}

template <int MODE>
static hipError_t launch_rowscanR(const ScanArgs& A, hipStream_t s) {
    const int64_t threads = A.n * (MODE == 2 ? 16 : 8);
    const int64_t blocks = (threads + 255) / 256 + (int64_t)A.n_long * A.long_chunks;
    hipLaunchKernelGGL(k_rowscanR<MODE>, dim3((unsigned)blocks), dim3(256), 0, s, A);
    return hipGetLastError();
}

// iters sweeps over the row-major copy.  The scalings live in the new numbering in A.scale_in / A.scale_out
// (two scratch buffers of n doubles, the last sweep writes A.scale_out); A.scale (by original id) receives
// the final one.
hipError_t launch_front_sweeps(const SweepArgs& A0, int iters, hipStream_t s, bool fused_pack) {
    if (A0.n == 0) return hipSuccess;
    SweepArgs A = A0;
    const size_t sh = 16 * (size_t)std::max(A.max_m, 1);
    const dim3 gn(grid_for(A.n, 256));
    const int passes = iters > 0 ? iters : 1;  // iters == 0: one pass packs the values (scaling 1)
    hipError_t e = A.rmax_zero ? hipSuccess : hipMemsetAsync(A.rmax_all, 0, sizeof(unsigned long long) * A.n * passes, s);
    if (e != hipSuccess) return e;
    // the COO values are packed into the slots by the first sweep (k_sweep_front<true, .>), or by k_pack before
    // (fused_pack false: the first sweep then reads the slots with the scaling 1 -- the same maxima, bit for bit)
    for (int it = 0; it < passes; ++it) {
        A.iter = it;
        A.rmax = A.rmax_all + (int64_t)it * A.n;
        const bool first = it == 0 && fused_pack;
        if (A.nf > 0) {
            if (first) hipLaunchKernelGGL((k_sweep_front<true, false>), dim3((unsigned)A.nf), dim3(64), sh, s, A);
            else hipLaunchKernelGGL((k_sweep_front<false, false>), dim3((unsigned)A.nf), dim3(64), sh, s, A);
        }
        if (A.n_big > 0) {
            const dim3 gb((unsigned)A.n_big, (unsigned)A.big_slices);
            if (first) hipLaunchKernelGGL((k_sweep_front<true, true>), gb, dim3(256), sh, s, A);
            else hipLaunchKernelGGL((k_sweep_front<false, true>), gb, dim3(256), sh, s, A);
        }
        if (A.n_long > 0) {
            const unsigned gl = (unsigned)std::min<int64_t>(256, (A.nf + 255) / 256);
            hipLaunchKernelGGL(k_sweep_long_fin, dim3(std::max(gl, 1u)), dim3(256), sizeof(unsigned long long) * A.n_long, s, A);
        }
    }
    hipLaunchKernelGGL(k_sweep_final, gn, dim3(256), 0, s, A.rmax_all, A.scale, A.perm, A.n, iters, passes);
    return hipGetLastError();
}

hipError_t launch_resid(const ResidArgs& A, hipStream_t s) {
    if (A.n == 0) return hipSuccess;
    if (A.nf > 0)
        hipLaunchKernelGGL(k_resid_front, dim3((unsigned)A.nf), dim3(64), 16 * (size_t)std::max(A.max_m, 1), s, A);
    const int64_t threads = A.n_chunks * 64 + A.n * 4;
    hipLaunchKernelGGL(k_resid_rows, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, A);
    if (A.n_long > 0) hipLaunchKernelGGL(k_resid_long_fin, dim3((unsigned)((A.n_long + 255) / 256)), dim3(256), 0, s, A);
    return hipGetLastError();
}

hipError_t launch_rowsum_norm_orig(ScanArgs A, double* rowsum, hipStream_t s) {
    if (A.n == 0) return hipSuccess;
    A.out = rowsum;
    A.list = nullptr;
    hipError_t e = launch_rowscan(A, 2, s);
    if (e != hipSuccess) return e;
    return launch_normmax(rowsum, nullptr, A.n, A.anorm, s);
}

hipError_t launch_scale_sweeps(ScanArgs A, int iters, double* rmax, hipStream_t s) {
    if (A.n == 0) return hipSuccess;
    (void)rmax;
    double* bufs[2] = {A.scale_out, const_cast<double*>(A.scale_in)};
    double* out = nullptr;
    for (int it = 0; it < (iters > 0 ? iters : 1); ++it) {
        out = bufs[(iters - 1 - it) % 2 == 0 ? 0 : 1];  // the last sweep writes bufs[0] (the final scaling)
        A.scale_in = it == 0 ? nullptr : (out == bufs[0] ? bufs[1] : bufs[0]);
        A.scale_out = out;
        hipError_t e = it == 0 ? launch_rowscanR<0>(A, s) : launch_rowscanR<1>(A, s);
        if (e != hipSuccess) return e;
    }
    if (iters == 0) {  // no scaling: s = 1 (the first pass above only built the copy of |A|)
        hipLaunchKernelGGL(k_fill_ones, dim3(grid_for(A.n, 256)), dim3(256), 0, s, bufs[0], A.n);
    }
    hipLaunchKernelGGL(k_scale_to_orig, dim3(grid_for(A.n, 256)), dim3(256), 0, s, bufs[0], A.perm, A.scale, A.n);
    return hipGetLastError();
}

// row sums of the equilibrated matrix and ||A_pre||_inf; A.scale_out = the final scaling (new numbering)
hipError_t launch_rowsum_norm(ScanArgs A, double* rowsum, hipStream_t s) {
    if (A.n == 0) return hipSuccess;
    A.out = rowsum;
    hipError_t e = launch_rowscanR<2>(A, s);
    if (e != hipSuccess) return e;
    return launch_normmax(rowsum, nullptr, A.n, A.anorm, s);
}

hipError_t launch_scale(ScanArgs A, int iters, double* rmax, double* rowsum, hipStream_t s) {
    hipError_t e = launch_scale_sweeps(A, iters, rmax, s);
    return e != hipSuccess ? e : launch_rowsum_norm(A, rowsum, s);
}

size_t factor_lds_bytes(int mmax) {
    const size_t packed = (((size_t)mmax * (mmax + 1) / 2) + 1) & ~(size_t)1;
    // + slack: the register path reads the column vector (coefB) unclamped up to 2*kThreads... entries
    // (the one-wave kernels publish the pivot column into G * RM doubles there: 64 for MR <= 8, also when
    // the dataflow kernel k_factor_df<8> runs fronts of <= 32 rows)
    const int grid_rows = mmax <= 64 ? 64 : (mmax <= kMaxWaveFront ? kMaxWaveFront : 2 * kThreads);
    return 32 + packed * sizeof(double) + 2 * (size_t)mmax * sizeof(double) + 2 * (size_t)mmax * sizeof(int32_t) +
           (size_t)((mmax + 15) & ~15) + (size_t)grid_rows * sizeof(double);
}

hipError_t launch_factor(const FactorArgs& A, const int32_t* fronts, int count, int mmax, bool global, hipStream_t s) {
    if (count <= 0) return hipSuccess;
    if (global) {
        return hipErrorInvalidValue;  // fronts beyond LDS: launch_big_* (host loop in kkt_api.cpp)
    } else {
        const size_t sh = factor_lds_bytes(mmax);
        // small fronts: one wave per front (no cross-wave barriers, more fronts per CU);
        // larger fronts: four waves on a 16x16 update grid
        if (mmax <= 32) hipLaunchKernelGGL((k_factor_lds<64, 4>), dim3(count), dim3(64), sh, s, A, fronts);
        else if (mmax <= 64) hipLaunchKernelGGL((k_factor_lds<64, 8>), dim3(count), dim3(64), sh, s, A, fronts);
        else if (mmax <= kMaxWaveFront) hipLaunchKernelGGL((k_factor_lds<64, 9>), dim3(count), dim3(64), sh, s, A, fronts);
        else hipLaunchKernelGGL((k_factor_lds<kThreads, 8>), dim3(count), dim3(kThreads), sh, s, A, fronts);
    }
    return hipGetLastError();
}

// host_out (one GPU): the last block to finish also writes counters [0..8] and the dataflow abort word (slot
// 11) straight into the page-locked host block -- the two device-to-host copies that followed are gone
__global__ void __launch_bounds__(256) k_count(const unsigned long long* __restrict__ fcnt,
                                               const int32_t* __restrict__ fstat, const double* __restrict__ fmin,
                                               int64_t nf, unsigned long long* __restrict__ counters,
                                               unsigned long long* __restrict__ minbits, const uint32_t* __restrict__ abort_word,
                                               unsigned long long* __restrict__ host_out, unsigned long long seq) {
    unsigned long long acc[6] = {0, 0, 0, 0, 0, 0};
    unsigned long long mn = ~0ull;
    // four fronts per thread and trip, their loads issued together (one memory round trip per four fronts, not
    // one per front: C3's 63 865 fronts over 64 x 256 threads are one trip)
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t f0 = blockIdx.x * 256 + threadIdx.x; f0 < nf; f0 += 4 * stride) {
        unsigned long long fm[4], c[4];
        uint32_t st[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t f = f0 + u * stride;
            const bool ok = f < nf;
            fm[u] = ok ? as_bits(fmin[f]) : ~0ull;  // non-negative doubles order like their bits
            c[u] = ok ? fcnt[f] : 0ull;
            st[u] = ok ? (uint32_t)fstat[f] : 0u;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            mn = fm[u] < mn ? fm[u] : mn;
            acc[0] += c[u] & 0xffff; acc[1] += (c[u] >> 16) & 0xffff; acc[2] += (c[u] >> 32) & 0xffff; acc[3] += c[u] >> 48;
            acc[4] += st[u] >> 16; acc[5] += st[u] & 0xffff;
        }
    }
    __shared__ unsigned long long red[6][4];
#pragma unroll
    for (int q = 0; q < 6; ++q) {
        unsigned long long v = acc[q];
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
        if ((threadIdx.x & 63) == 0) red[q][threadIdx.x >> 6] = v;
    }
    __shared__ unsigned long long rmin[4];
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long x = __shfl_xor(mn, o);
        mn = x < mn ? x : mn;
    }
    if ((threadIdx.x & 63) == 0) rmin[threadIdx.x >> 6] = mn;
    __syncthreads();
    if (threadIdx.x < 6) {
        const unsigned long long v = red[threadIdx.x][0] + red[threadIdx.x][1] + red[threadIdx.x][2] + red[threadIdx.x][3];
        if (v) atomicAdd(counters + threadIdx.x, v);
    }
    if (threadIdx.x == 6 && minbits) {
        unsigned long long v = rmin[0];
        for (int w = 1; w < 4; ++w) v = rmin[w] < v ? rmin[w] : v;
        atomicMin(minbits, v);
    }
    if (host_out == nullptr) return;
    __shared__ int last;
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) last = atomicAdd(reinterpret_cast<unsigned int*>(counters + 10), 1u) == gridDim.x - 1;
    __syncthreads();
    if (!last) return;
    __threadfence();
    // system-scope (write-through) stores, drained, then the sequence number in slot 10 that the host polls
    // (option host_flag): the host sees the counters without waiting for the kernel's end and its completion
    // signal (no event marker in the stream; no system-scope release either, which would write back the L2)
    if (threadIdx.x < 9)
        __hip_atomic_store(host_out + threadIdx.x, __hip_atomic_load(counters + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (threadIdx.x == 11)
        __hip_atomic_store(host_out + 11, abort_word ? (unsigned long long)__hip_atomic_load(abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    drain_stores();
    __syncthreads();
    if (threadIdx.x == 0 && seq) __hip_atomic_store(host_out + 10, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

hipError_t launch_count(const unsigned long long* fcnt, const int32_t* fstat, const double* fmin, int64_t nf,
                        unsigned long long* counters, unsigned long long* minbits, hipStream_t s, const uint32_t* abort_word,
                        unsigned long long* host_out, unsigned long long seq) {
    // (1024 blocks, one front per thread, measured no faster than 64: more same-address atomics; round 6)
    const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(64, (nf + 255) / 256));
    if (nf <= 0 && host_out == nullptr) return hipSuccess;
    hipLaunchKernelGGL(k_count, dim3(blocks), dim3(256), 0, s, fcnt, fstat, fmin, nf, counters, minbits, abort_word, host_out, seq);
    return hipGetLastError();
}

// one launch for the per-factorization resets: counters[0..7] = 0, minbits (slot 8) = all ones (the min
// is taken on the bit patterns), anorm (slot 9) = 0 -- three fill launches before
__global__ void k_reset_counters(unsigned long long* __restrict__ c) {
    const int t = threadIdx.x;
    if (t < kCounterSlots) c[t] = t == 8 ? ~0ull : 0ull;
}
__global__ void k_front_scale(const int32_t* __restrict__ rows, const double* __restrict__ scale, double* __restrict__ fscale,
                              int64_t total) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x)
        fscale[t] = scale[rows[t]];
}

hipError_t launch_front_scale(const int32_t* rows, const double* scale, double* fscale, int64_t total, hipStream_t s) {
    if (total <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_front_scale, dim3(grid_for(total, 256)), dim3(256), 0, s, rows, scale, fscale, total);
    return hipGetLastError();
}

hipError_t launch_reset_counters(unsigned long long* counters, hipStream_t s) {
    hipLaunchKernelGGL(k_reset_counters, dim3(1), dim3(64), 0, s, counters);
    return hipGetLastError();
}

hipError_t launch_rhs_scale(const double* b, const double* scale, double* w, int64_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_rhs_scale, dim3(grid_for(n, 256)), dim3(256), 0, s, b, scale, w, n);
    return hipGetLastError();
}

hipError_t launch_unscale(const double* w, const double* scale, double* x, int64_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_unscale, dim3(grid_for(n, 256)), dim3(256), 0, s, w, scale, x, n);
    return hipGetLastError();
}

hipError_t launch_solve(const SolveArgs& A, const int32_t* fronts, int count, int mmax, int pmax, bool forward,
                        hipStream_t s) {
    if (count <= 0) return hipSuccess;
    size_t tri = pmax <= 64 ? (size_t)pmax * (pmax | 1) * sizeof(double) : 0;
    size_t sh = (size_t)((mmax + 1) & ~1) * sizeof(double) + tri + 16;
    if (forward) hipLaunchKernelGGL(k_solve_fwd, dim3(count), dim3(kThreads), sh, s, A, fronts);
    else hipLaunchKernelGGL(k_solve_bwd, dim3(count), dim3(kThreads), sh, s, A, fronts);
    return hipGetLastError();
}

hipError_t launch_solve_wave(const SolveArgs& A, const int32_t* fronts, int count, int lds_doubles, bool forward,
                             hipStream_t s) {
    if (count <= 0) return hipSuccess;
    const size_t sh = (size_t)(lds_doubles + kSolveSlack) * sizeof(double) + 16;
    if (forward) hipLaunchKernelGGL(k_solve_fwd_w, dim3(count), dim3(64), sh, s, A, fronts);
    else hipLaunchKernelGGL(k_solve_bwd_w, dim3(count), dim3(64), sh, s, A, fronts);
    return hipGetLastError();
}

// slices per large front: ~32 K elements of an order-mmax front per workgroup, at most 512
static unsigned big_slices(int mmax) {
    const int64_t el = (int64_t)mmax * mmax;
    return (unsigned)std::max<int64_t>(1, std::min<int64_t>(512, el / 32768));
}

hipError_t launch_big_assemble(const FactorArgs& A, const int32_t* fronts, int count, int mmax, int maxch, hipStream_t s) {
    if (count <= 0) return hipSuccess;
    const dim3 g(big_slices(mmax), count);
    hipLaunchKernelGGL(k_big_init, g, dim3(kThreads), 0, s, A, fronts);
    hipLaunchKernelGGL(k_big_entries, g, dim3(kThreads), 0, s, A, fronts);
    for (int c = 0; c < maxch; ++c) hipLaunchKernelGGL(k_big_child, g, dim3(kThreads), 0, s, A, fronts, c);
    return hipGetLastError();
}

hipError_t launch_big_step(const FactorArgs& A, const int32_t* fronts, int count, int mmax, hipStream_t s) {
    if (count <= 0) return hipSuccess;
    const int rb = (mmax + 63) / 64;
    hipLaunchKernelGGL(k_app_diag, dim3(count), dim3(64), 0, s, A, fronts);
    hipLaunchKernelGGL(k_app_rows, dim3(rb, count), dim3(256), 0, s, A, fronts);
    hipLaunchKernelGGL(k_app_update, dim3(rb * (rb + 1) / 2 + rb, count), dim3(kThreads), 0, s, A, fronts, rb * (rb + 1) / 2);
    hipLaunchKernelGGL(k_app_exact, dim3(count), dim3(512), 0, s, A, fronts);
    hipLaunchKernelGGL(k_big_update, dim3(rb * (rb + 1) / 2, count), dim3(kThreads), 0, s, A, fronts);
    return hipGetLastError();
}

hipError_t launch_big_pending(const FactorArgs& A, const int32_t* fronts, int count, int32_t* out, hipStream_t s) {
    hipLaunchKernelGGL(k_big_pending, dim3(1), dim3(256), 0, s, A, fronts, count, out);
    return hipGetLastError();
}

hipError_t launch_big_finish(const FactorArgs& A, const int32_t* fronts, int count, int mmax, hipStream_t s) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_big_finish, dim3(big_slices(mmax), count), dim3(kThreads), (size_t)mmax * sizeof(int32_t) + 16, s, A, fronts);
    return hipGetLastError();
}

int big_panel_width() { return kAppNB; }

hipError_t launch_factor_df(const FactorArgs& A, int mmax, hipStream_t s) {
    if (A.df_nf <= 0) return hipSuccess;
    hipLaunchKernelGGL((k_factor_df<8>), dim3(A.df_nf), dim3(64), factor_lds_bytes(mmax), s, A);
    return hipGetLastError();
}

int solve_slack_doubles() { return kSolveSlack; }

int solve_df_grid(int lds_doubles, int nf) {
    const size_t sh = (size_t)(lds_doubles + kSolveSlack) * sizeof(double) + 16;
    int dev = 0, cus = 0, nf_blk = 0, nb_blk = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nf_blk, k_solve_fwd_df, 64, sh) != hipSuccess) return 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb_blk, k_solve_bwd_df, 64, sh) != hipSuccess) return 0;
    // one block per CU below the reported residency (the query can over-report by one)
    int per_cu = std::min(nf_blk, nb_blk) - 1;
    if (per_cu < 1) return 0;
    const int64_t g = (int64_t)per_cu * cus;
    return (int)std::min<int64_t>(g, std::max(nf, 1));
}

hipError_t launch_solve_df(const SolveArgs& A, const DfArgs& D, int grid, int lds_doubles, bool forward, hipStream_t s) {
    if (D.nf <= 0 || grid <= 0) return hipSuccess;
    const size_t sh = (size_t)(lds_doubles + kSolveSlack) * sizeof(double) + 16;
    if (forward) hipLaunchKernelGGL(k_solve_fwd_df, dim3(grid), dim3(64), sh, s, A, D);
    else hipLaunchKernelGGL(k_solve_bwd_df, dim3(grid), dim3(64), sh, s, A, D);
    return hipGetLastError();
}

// register-resident dataflow solve kernels (k_solve_{fwd,bwd}_rg): grid = resident blocks (one below the
// occupancy query's answer per CU, which can over-report by one), at most the walk length
static constexpr size_t kRgFwdLds = (192 + (kRgRegion > 8 * 33 ? kRgRegion : 8 * 33)) * sizeof(double);
static constexpr size_t kRgBwdLds = (32 * 33 > 128 + kRgRegion ? 32 * 33 : 128 + kRgRegion) * sizeof(double);
// wpe: waves per SIMD of the walk kernels' register budget (per-handle option "solve_rg_wpe": 3 or 4); the
// occupancy answers are per kernel variant, so the grid always matches the variant launch_solve_rg(wpe) runs
int solve_rg_grid(bool forward, int nf, int wpe) {
    // occupancy answers cached per variant; ranks of an in-process group query from their own threads, so the
    // cache is atomic (every thread computes the same value)
    static std::atomic<int> per_cu[4] = {{-1}, {-1}, {-1}, {-1}};
    int cus = 0;
    const int d = (forward ? 0 : 1) + (wpe == 4 ? 2 : 0);
    {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess) return 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    }
    if (per_cu[d].load() < 0) {
        int n = 0;
        hipError_t e = d == 0   ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_solve_fwd_rg<3>, 64, kRgFwdLds)
                       : d == 1 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_solve_bwd_rg<3>, 64, kRgBwdLds)
                       : d == 2 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_solve_fwd_rg<4>, 64, kRgFwdLds)
                                : hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_solve_bwd_rg<4>, 64, kRgBwdLds);
        if (e != hipSuccess) return 0;
        per_cu[d].store(n - 1);
    }
    const int pc = per_cu[d].load();
    if (pc < 1) return 0;
    return (int)std::min<int64_t>((int64_t)pc * cus, std::max(nf, 1));
}

hipError_t launch_solve_rg(const SolveArgs& A, const DfArgs& D, int grid, bool forward, int wpe, hipStream_t s) {
    if (D.nf <= 0 || grid <= 0) return hipSuccess;
    if (wpe == 4) {
        if (forward) hipLaunchKernelGGL(k_solve_fwd_rg<4>, dim3(grid), dim3(64), kRgFwdLds, s, A, D);
        else hipLaunchKernelGGL(k_solve_bwd_rg<4>, dim3(grid), dim3(64), kRgBwdLds, s, A, D);
    } else {
        if (forward) hipLaunchKernelGGL(k_solve_fwd_rg<3>, dim3(grid), dim3(64), kRgFwdLds, s, A, D);
        else hipLaunchKernelGGL(k_solve_bwd_rg<3>, dim3(grid), dim3(64), kRgBwdLds, s, A, D);
    }
    return hipGetLastError();
}

hipError_t launch_solve_bwd_flat(const SolveArgs& A, const DfArgs& D, int begin, int count, int lds_doubles, hipStream_t s) {
    if (count <= 0) return hipSuccess;
    const size_t sh = (size_t)(lds_doubles + kSolveSlack) * sizeof(double) + 16;  // as the walk (launch_solve_df)
    hipLaunchKernelGGL(k_solve_bwd_flat, dim3(count), dim3(64), sh, s, A, D, begin, count);
    return hipGetLastError();
}

hipError_t launch_solve_fwd_flat(const SolveArgs& A, const DfArgs& D, int begin, int count, hipStream_t s) {
    if (count <= 0) return hipSuccess;
    // one wave per front; 6 waves per SIMD fit its registers
    hipLaunchKernelGGL(k_solve_fwd_flat<6>, dim3(count), dim3(64), (192 + 8 * 33) * sizeof(double), s, A, D, begin, count);
    return hipGetLastError();
}

// level-scheduled backward of one-wave fronts through rg_bwd_core (handles whose fronts all have p <= 32,
// m <= 72: the arithmetic of k_solve_bwd_rg)
hipError_t launch_solve_bwd_w2(const SolveArgs& A, const int32_t* fronts, int count, hipStream_t s) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_solve_bwd_w2, dim3(count), dim3(64), kRgBwdLds, s, A, fronts);
    return hipGetLastError();
}

hipError_t launch_xs_in(const double* b, const double* scale, const int32_t* xpos, double* xs, int64_t n, hipStream_t s,
                        const int32_t* list) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_xs_in, dim3(grid_for(n, 256)), dim3(256), 0, s, b, scale, xpos, xs, n, list);
    return hipGetLastError();
}

hipError_t launch_xs_out(const double* xs, const double* scale, const int32_t* xpos, const uint32_t* abort_flag, double* x,
                         int64_t n, hipStream_t s, const int32_t* list, bool sub) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_xs_out, dim3(grid_for(n, 256)), dim3(256), 0, s, xs, scale, xpos, abort_flag, x, n, list, sub ? 1 : 0);
    return hipGetLastError();
}

hipError_t launch_xpos(const SolveArgs& A, const DfArgs& D, int32_t* xpos, int32_t* rxpos, const int32_t* top_orig,
                       int64_t n_top, int64_t top_base, hipStream_t s, bool pass0) {
    if (D.nf <= 0) return hipSuccess;
    // (one row per thread instead of the 4096-block cap measured no faster: round 6)
    const dim3 g(grid_for(D.rows_total, 256));
    if (pass0) hipLaunchKernelGGL(k_xpos, g, dim3(256), 0, s, D, A.frow, xpos, rxpos, 0);
    if (n_top > 0) hipLaunchKernelGGL(k_xpos_top, dim3(grid_for(n_top, 256)), dim3(256), 0, s, top_orig, n_top, top_base, xpos);
    hipLaunchKernelGGL(k_xpos, g, dim3(256), 0, s, D, A.frow, xpos, rxpos, 1);
    return hipGetLastError();
}

hipError_t launch_cvx_to_cvec(const DfArgs& D, const SolveArgs& A, const int32_t* roots, int count, double* cvec, hipStream_t s) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_cvx_to_cvec, dim3(std::min(count, 4096)), dim3(64), 0, s, D, A, roots, count, cvec);
    return hipGetLastError();
}

hipError_t launch_set_done(uint32_t* done, const int32_t* list, int count, uint32_t epoch, hipStream_t s) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_set_done, dim3(grid_for(count, 256)), dim3(256), 0, s, done, list, count, epoch);
    return hipGetLastError();
}

}  // namespace ukkt
