// cpu_mf.cpp -- TEST / BASELINE INFRASTRUCTURE ONLY (never linked into the product).
//
// Multi-threaded CPU multifrontal LDL^T on the product's own symbolic analysis (nested dissection,
// supernodes, assembly tree: uno_amd/csrc/analysis.cpp, compiled into this library): the CPU baseline of
// bench.py (BASELINE.md section 4 "Fallback": MUMPS 5.8.0 is not available offline, so the baseline is a
// multi-threaded CPU restatement timed on the host cores).  Same semantics as the GPU path and the oracle
// (MUMPSSolver.cpp:16-36,82): COO duplicates summed, 3 symmetric infinity-norm equilibration sweeps with the
// oracle's multiplication order, null pivots at eps * 1e-5 * ||A_pre||_inf, Duff-Reid 1x1 / 2x2 threshold
// pivoting with u = 0.01 inside each front.  A front whose fully-summed block admits no pivot at u relaxes
// the threshold (u/10, u/100, 1e-6, 1e-10, 0) instead of delaying (the product's delay_relaxed = 0 mode:
// no re-analysis inside a timed factorization).
//
// Parallelism: OpenMP over the independent fronts of each assembly-tree level (level by level, the
// schedule MUMPS' tree parallelism would use on a shared-memory node), for the factorization and both
// triangular solves.  Dense kernels are plain loops over row-major lower triangles (fronts have m <= ~100
// at the bench sizes; BLAS3 would not change the picture).
#include <omp.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "../uno_amd/csrc/analysis.hpp"

namespace {

enum : int8_t { P_NULL = 0, P_1X1 = 1, P_2X2_A = 2, P_2X2_B = 3 };

struct Handle {
    ukkt::Pattern P;
    ukkt::Symbolic S;
    double u = 0.01, null_fac = 1e-5;
    int scale_iters = 3;
    std::vector<double> uval, scale, L, cb, w, cvec;
    std::vector<int32_t> frow, fpos;
    std::vector<int8_t> piv;
    int64_t npos = 0, nneg = 0, nzero = 0;
    bool factored = false;
    std::string err;
};

inline double sabs(const std::vector<double>& s, int32_t a, int32_t b, double v) {  // oracle order
    return a > b ? std::fabs(s[a] * v * s[b]) : std::fabs(s[b] * v * s[a]);
}

// threshold pivot search of one candidate column c at step k (oracle test_pivot / kkt_kernels search_pivot)
int test_pivot(const double* F, int m, int k, int p, int c, double u, double thres, int& r_out) {
    auto at = [&](int i, int j) { return i >= j ? F[(int64_t)i * m + j] : F[(int64_t)j * m + i]; };
    const double acc = std::fabs(at(c, c));
    double gamma = 0.0, rmax = 0.0;
    int r = -1;
    for (int i = k; i < m; ++i) {
        if (i == c) continue;
        const double v = std::fabs(at(i, c));
        gamma = std::max(gamma, v);
        if (i < p && v > rmax) { rmax = v; r = i; }
    }
    if (std::max(acc, gamma) <= thres) return 1;
    if (acc != 0.0 && acc >= u * gamma) return 2;
    if (r >= 0 && rmax > 0.0) {
        double gc = 0.0, gr = 0.0;
        for (int i = k; i < m; ++i) {
            if (i == c || i == r) continue;
            gc = std::max(gc, std::fabs(at(i, c)));
            gr = std::max(gr, std::fabs(at(i, r)));
        }
        const double a = at(c, c), b = at(r, c), d = at(r, r);
        const double det = a * d - b * b;
        if (det != 0.0) {
            const double lim = u > 0.0 ? std::fabs(det) / u : INFINITY;
            if (std::fabs(d) * gc + std::fabs(b) * gr <= lim && std::fabs(b) * gc + std::fabs(a) * gr <= lim) {
                r_out = r;
                return 3;
            }
        }
    }
    return 0;
}

void sym_swap(double* F, int m, int a, int b, int32_t* rows, int32_t* lorig) {  // a < b, lower storage
    if (a == b) return;
    auto A = [&](int i, int j) -> double& { return F[(int64_t)i * m + j]; };
    for (int t = 0; t < a; ++t) std::swap(A(a, t), A(b, t));
    std::swap(A(a, a), A(b, b));
    for (int t = a + 1; t < b; ++t) std::swap(A(t, a), A(b, t));
    for (int t = b + 1; t < m; ++t) std::swap(A(t, a), A(t, b));
    std::swap(rows[a], rows[b]);
    std::swap(lorig[a], lorig[b]);
}

struct Counts { int64_t pos = 0, neg = 0, zero = 0; };

void factor_front(Handle& h, int32_t f, std::vector<double>& F, std::vector<int32_t>& lorig, double thres, Counts& cnt) {
    const ukkt::Symbolic& S = h.S;
    const int m = S.f_m[f], p = S.f_p[f];
    const int64_t ro = S.f_rows_off[f];
    F.assign((size_t)m * m, 0.0);
    auto A = [&](int i, int j) -> double& { return F[(int64_t)i * m + j]; };
    int32_t* rows = h.frow.data() + ro;
    for (int i = 0; i < m; ++i) { rows[i] = S.rows[ro + i]; lorig[i] = i; }
    // original entries (scaled in the oracle's multiplication order)
    for (int64_t e = S.f_ent_off[f]; e < S.f_ent_off[f + 1]; ++e) {
        const uint32_t lp = S.ent_lpos[e];
        const int lr = (int)(lp >> 16), lc = (int)(lp & 0x7fffu);
        const double sr = h.scale[rows[lr]], sc = h.scale[rows[lc]];
        A(lr, lc) = (lp & 0x8000u) ? sc * h.uval[e] * sr : sr * h.uval[e] * sc;
    }
    // children's contribution blocks (row-major packed lower triangles)
    for (int32_t q = S.f_child_off[f]; q < S.f_child_off[f + 1]; ++q) {
        const int32_t c = S.child[q];
        const int cm = S.f_m[c] - S.f_p[c];
        const int32_t* rm = S.relmap.data() + S.f_relmap_off[c];
        const double* cbv = h.cb.data() + S.f_cb_off[c];
        for (int r = 0; r < cm; ++r)
            for (int cc = 0; cc <= r; ++cc) A(rm[r], rm[cc]) += cbv[(int64_t)r * (r + 1) / 2 + cc];
    }
    int8_t* piv = h.piv.data() + ro;
    const double ulist[] = {h.u, h.u * 0.1, h.u * 0.01, 1e-6, 1e-10, 0.0};
    int k = 0;
    while (k < p) {
        // quick 1x1 test on column k
        const double akk = A(k, k);
        double g = 0.0;
        for (int i = k + 1; i < m; ++i) g = std::max(g, std::fabs(A(i, k)));
        int kind = 0, c = k, r = -1;
        if (std::fabs(akk) > thres && !(h.u * g > std::fabs(akk))) {
            kind = 2;
        } else {
            for (int ul = 0; ul < 6 && !kind; ++ul)
                for (c = k; c < p && !kind; ++c) {
                    kind = test_pivot(F.data(), m, k, p, c, ulist[ul], thres, r);
                    if (kind) break;
                }
            if (!kind) { kind = 1; c = k; }  // everything below the threshold: null pivot
        }
        sym_swap(F.data(), m, k, c, rows, lorig.data());
        if (kind == 1) {
            for (int i = k + 1; i < m; ++i) A(i, k) = 0.0;
            piv[k] = P_NULL;
            cnt.zero++;
            k += 1;
        } else if (kind == 2) {
            const double d = A(k, k), dinv = 1.0 / d;
            for (int i = k + 1; i < m; ++i) {
                const double li = A(i, k) * dinv;
                double* Fi = &A(i, 0);
                for (int j = k + 1; j <= i; ++j) Fi[j] -= li * A(j, k);
            }
            piv[k] = P_1X1;
            (d > 0.0 ? cnt.pos : cnt.neg)++;
            k += 1;
        } else {
            if (r == k) r = c;
            sym_swap(F.data(), m, k + 1, r, rows, lorig.data());
            const double a = A(k, k), b = A(k + 1, k), e = A(k + 1, k + 1);
            const double det = a * e - b * b, idet = 1.0 / det;
            const double d0 = a * idet, d1 = b * idet, d2 = e * idet;
            for (int i = k + 2; i < m; ++i) {
                const double a0 = A(i, k), a1 = A(i, k + 1);
                const double l0 = d2 * a0 - d1 * a1, l1 = d0 * a1 - d1 * a0;
                double* Fi = &A(i, 0);
                for (int j = k + 2; j <= i; ++j) Fi[j] -= l0 * A(j, k) + l1 * A(j, k + 1);
            }
            piv[k] = P_2X2_A;
            piv[k + 1] = P_2X2_B;
            if (det < 0.0) { cnt.pos++; cnt.neg++; }
            else if (a + e > 0.0) cnt.pos += 2;
            else cnt.neg += 2;
            k += 2;
        }
    }
    // L: packed lower trapezoid, column j rows j..m-1 (the GPU write-out formula)
    double* L = h.L.data() + S.f_L_off[f];
    int64_t cs = 0;
    for (int j = 0; j < p; ++j) {
        double ca = 0.0, cbv = 0.0;
        int base = j;
        if (piv[j] == P_1X1) ca = 1.0 / A(j, j);
        else if (piv[j] == P_2X2_A || piv[j] == P_2X2_B) {
            const int k0 = piv[j] == P_2X2_A ? j : j - 1;
            const double a = A(k0, k0), b = A(k0 + 1, k0), e = A(k0 + 1, k0 + 1);
            const double idet = 1.0 / (a * e - b * b);
            if (piv[j] == P_2X2_A) { ca = e * idet; cbv = -b * idet; }
            else { ca = -b * idet; cbv = a * idet; }
            base = k0;
        }
        for (int i = j; i < m; ++i) {
            double v;
            if (i == j) v = piv[j] == P_NULL ? 0.0 : A(j, j);
            else if (piv[j] == P_2X2_A && i == j + 1) v = A(j + 1, j);
            else v = ca * A(i, base) + (piv[j] >= P_2X2_A ? cbv * A(i, base + 1) : 0.0);
            L[cs + (i - j)] = v;
        }
        cs += m - j;
    }
    for (int i = 0; i < m; ++i) h.fpos[ro + lorig[i]] = i;
    const int cm = m - p;
    double* cbo = h.cb.data() + S.f_cb_off[f];
    for (int r2 = 0; r2 < cm; ++r2)
        for (int c2 = 0; c2 <= r2; ++c2) cbo[(int64_t)r2 * (r2 + 1) / 2 + c2] = A(p + r2, p + c2);
}

inline int64_t colptr(int64_t Lo, int m, int k) { return Lo + (int64_t)k * m - (int64_t)k * (k - 1) / 2 - k; }

}  // namespace

extern "C" {

void* cpu_mf_create() { return new Handle(); }
void cpu_mf_destroy(void* p) { delete static_cast<Handle*>(p); }
const char* cpu_mf_last_error(void* p) { return static_cast<Handle*>(p)->err.c_str(); }
int cpu_mf_threads() { return omp_get_max_threads(); }

int cpu_mf_analyze(void* ph, int64_t n, int64_t nnz, const int64_t* row, const int64_t* col) {
    Handle& h = *static_cast<Handle*>(ph);
    ukkt::AnalysisOptions opt;
    h.err = ukkt::analyze(n, nnz, row, col, opt, h.P, h.S);
    if (!h.err.empty()) return -1;
    const ukkt::Symbolic& S = h.S;
    h.uval.assign(S.nu, 0.0);
    h.scale.assign(n, 1.0);
    h.L.assign(S.L_size, 0.0);
    h.cb.assign(S.cb_size, 0.0);
    h.frow.assign(S.rows.size(), 0);
    h.fpos.assign(S.rows.size(), 0);
    h.piv.assign(S.rows.size(), 0);
    h.w.assign(n, 0.0);
    h.cvec.assign(S.f_relmap_off.empty() ? 0 : S.f_relmap_off.back(), 0.0);
    h.factored = false;
    return 0;
}

int cpu_mf_factorize(void* ph, const double* values) {
    Handle& h = *static_cast<Handle*>(ph);
    const ukkt::Symbolic& S = h.S;
    const int64_t n = S.n, nu = S.nu;
    // pack (duplicates summed in ascending COO position)
#pragma omp parallel for schedule(static)
    for (int64_t s = 0; s < nu; ++s) {
        if (S.identity_dups) { h.uval[s] = values[S.dup_pos[s]]; continue; }
        double v = 0.0;
        for (int32_t q = S.dup_ptr[s]; q < S.dup_ptr[s + 1]; ++q) v += values[S.dup_pos[q]];
        h.uval[s] = v;
    }
    // equilibration: row i (new numbering) = column part cptr[i].. + row part rslot[rptr[i]..]
    std::vector<double> snew(n, 1.0), rsum(n, 0.0);
    std::fill(h.scale.begin(), h.scale.end(), 1.0);
    for (int it = 0; it < h.scale_iters; ++it) {
#pragma omp parallel for schedule(static, 4096)
        for (int64_t i = 0; i < n; ++i) {
            const int32_t o = S.perm[i];
            double r = 0.0;
            for (int32_t q = S.cptr[i]; q < S.cptr[i + 1]; ++q) r = std::max(r, sabs(h.scale, o, S.ent_r[q], h.uval[q]));
            for (int32_t t = S.rptr[i]; t < S.rptr[i + 1]; ++t) {
                const int32_t q = S.rslot[t];
                r = std::max(r, sabs(h.scale, o, S.ent_c[q], h.uval[q]));
            }
            snew[o] = r > 0.0 ? h.scale[o] / std::sqrt(r) : h.scale[o];
        }
        std::swap(h.scale, snew);
    }
    double anorm = 0.0;
#pragma omp parallel for schedule(static, 4096) reduction(max : anorm)
    for (int64_t i = 0; i < n; ++i) {
        const int32_t o = S.perm[i];
        double r = 0.0;
        for (int32_t q = S.cptr[i]; q < S.cptr[i + 1]; ++q) r += sabs(h.scale, o, S.ent_r[q], h.uval[q]);
        for (int32_t t = S.rptr[i]; t < S.rptr[i + 1]; ++t) {
            const int32_t q = S.rslot[t];
            r += sabs(h.scale, o, S.ent_c[q], h.uval[q]);
        }
        anorm = std::max(anorm, r);
    }
    const double thres = DBL_EPSILON * h.null_fac * anorm;
    int64_t pos = 0, neg = 0, zero = 0;
    for (int l = 0; l < S.nlevels; ++l) {
#pragma omp parallel reduction(+ : pos, neg, zero)
        {
            std::vector<double> F;
            std::vector<int32_t> lorig(S.max_m + 1);
            Counts c;
#pragma omp for schedule(dynamic, 8)
            for (int32_t q = S.level_off[l]; q < S.level_off[l + 1]; ++q) factor_front(h, S.level_fronts[q], F, lorig, thres, c);
            pos += c.pos; neg += c.neg; zero += c.zero;
        }
    }
    h.npos = pos; h.nneg = neg; h.nzero = zero;
    h.factored = true;
    return 0;
}

int cpu_mf_inertia(void* ph, int64_t* pos, int64_t* neg, int64_t* zero) {
    Handle& h = *static_cast<Handle*>(ph);
    if (!h.factored) { h.err = "inertia before factorize"; return -1; }
    *pos = h.npos; *neg = h.nneg; *zero = h.nzero;
    return 0;
}

int cpu_mf_solve(void* ph, const double* rhs, double* x) {
    Handle& h = *static_cast<Handle*>(ph);
    if (!h.factored) { h.err = "solve before factorize"; return -1; }
    const ukkt::Symbolic& S = h.S;
    const int64_t n = S.n;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) h.w[i] = h.scale[i] * rhs[i];
    // forward (levels ascending): y = L^-1 on the front, z = D^-1 y at its pivots, update vector to the parent
    for (int l = 0; l < S.nlevels; ++l) {
#pragma omp parallel
        {
            std::vector<double> y;
#pragma omp for schedule(dynamic, 16)
            for (int32_t q = S.level_off[l]; q < S.level_off[l + 1]; ++q) {
                const int32_t f = S.level_fronts[q];
                const int m = S.f_m[f], p = S.f_p[f];
                const int64_t ro = S.f_rows_off[f], Lo = S.f_L_off[f];
                const int8_t* piv = h.piv.data() + ro;
                y.assign(m, 0.0);
                for (int i = 0; i < p; ++i) y[i] = h.w[h.frow[ro + i]];
                for (int32_t cq = S.f_child_off[f]; cq < S.f_child_off[f + 1]; ++cq) {
                    const int32_t c = S.child[cq];
                    const int cm = S.f_m[c] - S.f_p[c];
                    const int32_t* rm = S.relmap.data() + S.f_relmap_off[c];
                    const double* cv = h.cvec.data() + S.f_relmap_off[c];
                    for (int t = 0; t < cm; ++t) y[h.fpos[ro + rm[t]]] += cv[t];
                }
                for (int k = 0; k < p; ++k) {
                    if (piv[k] == P_1X1) {
                        const double* Lk = h.L.data() + colptr(Lo, m, k);
                        for (int i = k + 1; i < m; ++i) y[i] -= Lk[i] * y[k];
                    } else if (piv[k] == P_2X2_A) {
                        const double* L0 = h.L.data() + colptr(Lo, m, k);
                        const double* L1 = h.L.data() + colptr(Lo, m, k + 1);
                        for (int i = k + 2; i < m; ++i) y[i] -= L0[i] * y[k] + L1[i] * y[k + 1];
                        ++k;
                    }
                }
                for (int k = 0; k < p; ++k) {
                    double& out = h.w[h.frow[ro + k]];
                    if (piv[k] == P_1X1) out = y[k] / h.L[colptr(Lo, m, k) + k];
                    else if (piv[k] == P_2X2_A) {
                        const double a = h.L[colptr(Lo, m, k) + k], b = h.L[colptr(Lo, m, k) + k + 1];
                        const double e = h.L[colptr(Lo, m, k + 1) + k + 1], det = a * e - b * b;
                        out = (e * y[k] - b * y[k + 1]) / det;
                        h.w[h.frow[ro + k + 1]] = (a * y[k + 1] - b * y[k]) / det;
                        ++k;
                    } else out = 0.0;
                }
                double* cv = h.cvec.data() + S.f_relmap_off[f];
                for (int i = p; i < m; ++i) cv[i - p] = y[i];
            }
        }
    }
    // backward (levels descending): x_k = z_k - sum_{i > k} L(i, k) x_i
    for (int l = S.nlevels - 1; l >= 0; --l) {
#pragma omp parallel
        {
            std::vector<double> xl;
#pragma omp for schedule(dynamic, 16)
            for (int32_t q = S.level_off[l]; q < S.level_off[l + 1]; ++q) {
                const int32_t f = S.level_fronts[q];
                const int m = S.f_m[f], p = S.f_p[f];
                const int64_t ro = S.f_rows_off[f], Lo = S.f_L_off[f];
                const int8_t* piv = h.piv.data() + ro;
                xl.assign(m, 0.0);
                for (int i = 0; i < m; ++i) xl[i] = h.w[h.frow[ro + i]];
                for (int k = p - 1; k >= 0; --k) {
                    if (piv[k] == P_NULL) continue;
                    const double* Lk = h.L.data() + colptr(Lo, m, k);
                    const int skip = piv[k] == P_2X2_A ? k + 1 : -1;  // D off-diagonal entry of the block
                    double s = 0.0;
                    for (int i = k + 1; i < m; ++i)
                        if (i != skip) s += Lk[i] * xl[i];
                    xl[k] -= s;
                }
                for (int k = 0; k < p; ++k) h.w[h.frow[ro + k]] = xl[k];
            }
        }
    }
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) x[i] = h.scale[i] * h.w[i];
    return 0;
}

}  // extern "C"
