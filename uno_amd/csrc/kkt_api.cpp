// kkt_api.cpp -- implementation of the uno_kkt C ABI (include/uno_kkt.h).
//
// Host orchestration of one factor/solve handle: symbolic analysis on the host (analysis.cpp),
// device-resident layout, level-scheduled launches of the kernels in kkt_kernels.hip on one HIP
// stream.  Mirrors the call sequence of Uno's MUMPS adapter
// (uno/ingredients/subproblem_solvers/MUMPS/MUMPSSolver.cpp:72-147) but keeps the factor on the GPU.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/uno_kkt.h"
#include "../../include/uno_kkt_debug.h"
#include "analysis.hpp"
#include "kkt_kernels.hpp"

using namespace ukkt;

namespace {

template <class T>
struct DBuf {
    T* p = nullptr;
    size_t n = 0;
    hipError_t alloc(size_t count) {
        release();
        n = count;
        if (count == 0) return hipSuccess;
        return hipMalloc((void**)&p, count * sizeof(T));
    }
    hipError_t upload(const std::vector<T>& v, hipStream_t s) {
        hipError_t e = alloc(v.size());
        if (e != hipSuccess || v.empty()) return e;
        return hipMemcpyAsync(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s);
    }
    void release() {
        if (p) hipFree(p);
        p = nullptr;
        n = 0;
    }
    ~DBuf() { release(); }
};

enum KernelClass { KC_PACK = 0, KC_SCALE, KC_FACTOR_LDS, KC_FACTOR_GLOBAL, KC_SOLVE_FWD, KC_SOLVE_BWD, KC_RHS, KC_COUNT };
const char* kClassNames[KC_COUNT] = {"pack", "scale", "factor_lds", "factor_global", "solve_fwd", "solve_bwd", "rhs"};

struct Launch {
    int begin, count, mmax;
    bool global;
};

// one solve launch: fronts solve_fronts[begin, begin+count) of one level; wave kernels (p <= 64,
// m <= kMaxLdsFront) are grouped by the LDS their packed panel needs so small fronts keep occupancy
struct SolveLaunch {
    int level, begin, count, lds, mmax, pmax;
    bool wave;
};

}  // namespace

struct uno_kkt {
    int device = 0;
    hipStream_t stream = nullptr;
    AnalysisOptions aopt;
    double u = 0.01, null_fac = 1e-5;
    int scale_iters = 1;
    int timing = 0;
    Pattern P;
    Symbolic S;
    int delay_relaxed = 1;      // also amalgamate fronts whose pivots needed a relaxed threshold (MUMPS: delay)
    int max_merge_rounds = 64;
    int64_t merges_total = 0;
    bool analyzed = false, factor_enqueued = false, factored = false;
    const double* values_ptr = nullptr;  // device values used by the last factorization
    // device arrays
    DBuf<double> values, uval, scale, L, cb, gscratch, w, cvec, rowsum, rmax, bvec;
    DBuf<int32_t> dup_ptr, dup_pos, ent_r, ent_c, fm, fp, rows, frow, fpos, child_off, child, relmap, level_fronts, fstat;
    DBuf<uint32_t> ent_lpos;
    DBuf<int64_t> rows_off, ent_off, relmap_off, L_off, cb_off, gscratch_off, ch_relmap_off, ch_cb_off;
    DBuf<int32_t> ch_cm;
    DBuf<int8_t> piv;
    DBuf<unsigned long long> anorm, counters, stamps, fcnt;
    int want_stamps = 0;
    DBuf<int32_t> perm_d, cptr, rptr, rslot, long_rows, fparent, delayed;
    int32_t n_long = 0;
    int64_t max_long = 0;
    unsigned long long* h_counters = nullptr;
    std::vector<Launch> fac_launches;
    std::vector<SolveLaunch> sol_launches;  // ordered by level
    DBuf<int32_t> solve_fronts;
    uno_kkt_stats_t st{};
    std::string err;
    // timing
    struct Timed { int cls; hipEvent_t a, b; };
    std::vector<Timed> pending;
    std::vector<hipEvent_t> ev_pool;
    double t_ms[KC_COUNT] = {0};
    int64_t t_n[KC_COUNT] = {0};
};

namespace {

int set_err(uno_kkt_t h, int code, const std::string& msg) {
    if (h) h->err = msg;
    return code;
}

#define HIPCHK(h, expr)                                                                              \
    do {                                                                                             \
        hipError_t _e = (expr);                                                                      \
        if (_e != hipSuccess)                                                                        \
            return set_err(h, _e == hipErrorOutOfMemory ? UNO_KKT_ERR_NOMEM : UNO_KKT_ERR_HIP,       \
                           std::string(#expr) + ": " + hipGetErrorString(_e));                       \
    } while (0)

hipEvent_t get_event(uno_kkt_t h) {
    if (!h->ev_pool.empty()) {
        hipEvent_t e = h->ev_pool.back();
        h->ev_pool.pop_back();
        return e;
    }
    hipEvent_t e;
    hipEventCreate(&e);
    return e;
}

struct TimerScope {
    uno_kkt_t h;
    int cls;
    hipEvent_t a = nullptr;
    TimerScope(uno_kkt_t h_, int c) : h(h_), cls(c) {
        if (h->timing) {
            a = get_event(h);
            hipEventRecord(a, h->stream);
        }
    }
    ~TimerScope() {
        if (a) {
            hipEvent_t b = get_event(h);
            hipEventRecord(b, h->stream);
            h->pending.push_back({cls, a, b});
        }
    }
};

void flush_timing(uno_kkt_t h) {
    if (h->pending.empty()) return;
    hipStreamSynchronize(h->stream);
    for (auto& t : h->pending) {
        float ms = 0.f;
        hipEventElapsedTime(&ms, t.a, t.b);
        h->t_ms[t.cls] += ms;
        h->t_n[t.cls] += 1;
        h->ev_pool.push_back(t.a);
        h->ev_pool.push_back(t.b);
    }
    h->pending.clear();
}

int upload_structure(uno_kkt_t h);
int enqueue_factorization(uno_kkt_t h);

int finish_factorization(uno_kkt_t h) {
    if (!h->factor_enqueued) return h->factored ? UNO_KKT_OK : set_err(h, UNO_KKT_ERR_STATE, "no factorization");
    HIPCHK(h, hipStreamSynchronize(h->stream));
    flush_timing(h);
    h->factor_enqueued = false;
    // delayed pivots: a front that could not pivot a fully-summed column (or, optionally, needed a
    // relaxed threshold) is amalgamated into its parent and the factorization is redone.  The merge
    // is sticky for later factorizations of the same pattern.
    for (int round = 0; round < h->max_merge_rounds; ++round) {
        const unsigned long long* c = h->h_counters;
        int64_t nd = (int64_t)std::min<unsigned long long>(c[6], (unsigned long long)h->S.n);
        bool need = c[5] != 0 || (h->delay_relaxed && nd > 0);
        if (!need) break;
        std::vector<int32_t> dv(nd);
        if (nd > 0) HIPCHK(h, hipMemcpy(dv.data(), h->delayed.p, sizeof(int32_t) * nd, hipMemcpyDeviceToHost));
        int64_t moved = delay_columns(h->P, h->S, dv);
        if (moved == 0) {
            // fall back to whole-front amalgamation for stuck fronts (cannot happen at roots)
            std::vector<int32_t> fs(h->S.nf);
            HIPCHK(h, hipMemcpy(fs.data(), h->fstat.p, sizeof(int32_t) * fs.size(), hipMemcpyDeviceToHost));
            std::vector<char> merge(h->S.nf, 0);
            for (int64_t f = 0; f < h->S.nf; ++f) merge[f] = (fs[f] & 0xffff) != 0;
            moved = amalgamate(h->P, h->S, merge);
        }
        if (moved == 0) break;
        h->merges_total += moved;
        std::string msg = build_structure(h->P, h->S);
        if (!msg.empty()) return set_err(h, UNO_KKT_ERR_ARG, msg);
        int rc = upload_structure(h);
        if (rc != UNO_KKT_OK) return rc;
        rc = enqueue_factorization(h);
        if (rc != UNO_KKT_OK) return rc;
        HIPCHK(h, hipStreamSynchronize(h->stream));
        flush_timing(h);
        h->factor_enqueued = false;
    }
    const unsigned long long* c = h->h_counters;
    h->st.pivots_2x2 = (int64_t)c[3];
    h->st.pivots_null = (int64_t)c[2];
    h->st.pivots_relaxed = (int64_t)c[4];
    if (c[5] != 0) {
        h->factored = false;
        return set_err(h, UNO_KKT_ERR_PIVOT,
                       std::to_string(c[5]) + " fully-summed column(s) admit no pivot inside their front");
    }
    if ((int64_t)(c[0] + c[1] + c[2]) != h->S.n) {
        h->factored = false;
        return set_err(h, UNO_KKT_ERR_HIP, "internal: inertia does not sum to n");
    }
    h->factored = true;
    return UNO_KKT_OK;
}

int upload_structure(uno_kkt_t h) {
    Symbolic& S = h->S;
    if (S.max_m > kMaxGlobalFront)
        return set_err(h, UNO_KKT_ERR_ARG, "front of order " + std::to_string(S.max_m) + " exceeds " +
                                               std::to_string(kMaxGlobalFront));
    const int64_t n = S.n;
    // global scratch for fronts too large for LDS
    std::vector<int64_t> goff(S.nf + 1, 0);
    int64_t gtot = 8;  // leading pad: element -1 of the first front is the kernels' trash slot
    for (int64_t f = 0; f < S.nf; ++f) {
        goff[f] = gtot;
        if (S.f_m[f] > kMaxLdsFront) gtot += (int64_t)S.f_m[f] * S.f_m[f];
    }
    hipStream_t s = h->stream;
    HIPCHK(h, S.identity_dups ? (h->dup_ptr.release(), hipSuccess) : h->dup_ptr.upload(S.dup_ptr, s));
    HIPCHK(h, h->dup_pos.upload(S.dup_pos, s));
    HIPCHK(h, h->ent_r.upload(S.ent_r, s));
    HIPCHK(h, h->ent_c.upload(S.ent_c, s));
    HIPCHK(h, h->ent_lpos.upload(S.ent_lpos, s));
    HIPCHK(h, h->fm.upload(S.f_m, s));
    HIPCHK(h, h->fp.upload(S.f_p, s));
    HIPCHK(h, h->rows_off.upload(S.f_rows_off, s));
    HIPCHK(h, h->rows.upload(S.rows, s));
    HIPCHK(h, h->ent_off.upload(S.f_ent_off, s));
    HIPCHK(h, h->child_off.upload(S.f_child_off, s));
    HIPCHK(h, h->child.upload(S.child, s));
    {
        std::vector<int32_t> ccm(S.child.size());
        std::vector<int64_t> crel(S.child.size()), ccb(S.child.size());
        for (size_t q = 0; q < S.child.size(); ++q) {
            int32_t c = S.child[q];
            ccm[q] = S.f_m[c] - S.f_p[c];
            crel[q] = S.f_relmap_off[c];
            ccb[q] = S.f_cb_off[c];
        }
        HIPCHK(h, h->ch_cm.upload(ccm, s));
        HIPCHK(h, h->ch_relmap_off.upload(crel, s));
        HIPCHK(h, h->ch_cb_off.upload(ccb, s));
    }
    HIPCHK(h, h->relmap_off.upload(S.f_relmap_off, s));
    HIPCHK(h, h->relmap.upload(S.relmap, s));
    HIPCHK(h, h->L_off.upload(S.f_L_off, s));
    HIPCHK(h, h->cb_off.upload(S.f_cb_off, s));
    HIPCHK(h, h->gscratch_off.upload(goff, s));
    HIPCHK(h, h->level_fronts.upload(S.level_fronts, s));
    HIPCHK(h, h->fstat.alloc(S.nf));
    HIPCHK(h, h->fcnt.alloc(S.nf));
    HIPCHK(h, h->perm_d.upload(S.perm, s));
    HIPCHK(h, h->cptr.upload(S.cptr, s));
    HIPCHK(h, h->rptr.upload(S.rptr, s));
    HIPCHK(h, h->rslot.upload(S.rslot, s));
    HIPCHK(h, h->fparent.upload(S.f_parent, s));
    {
        std::vector<int32_t> lr;
        h->max_long = 0;
        for (int64_t i = 0; i < n; ++i) {
            int64_t len = (S.cptr[i + 1] - S.cptr[i]) + (S.rptr[i + 1] - S.rptr[i]);
            if (len > kLongRow) { lr.push_back((int32_t)i); h->max_long = std::max(h->max_long, len); }
        }
        h->n_long = (int32_t)lr.size();
        HIPCHK(h, h->long_rows.upload(lr, s));
    }
    if (h->delayed.n != (size_t)std::max<int64_t>(n, 1)) HIPCHK(h, h->delayed.alloc(std::max<int64_t>(n, 1)));
    if (h->uval.n != (size_t)S.nu) HIPCHK(h, h->uval.alloc(S.nu));
    if (h->scale.n != (size_t)n) {
        HIPCHK(h, h->scale.alloc(n));
        HIPCHK(h, h->rowsum.alloc(n));
        HIPCHK(h, h->rmax.alloc(n));
        HIPCHK(h, h->w.alloc(n));
        HIPCHK(h, h->bvec.alloc(n));
    }
    HIPCHK(h, h->L.alloc(S.L_size));
    HIPCHK(h, h->cb.alloc(S.cb_size));
    HIPCHK(h, h->cvec.alloc(S.f_relmap_off.empty() ? 0 : S.f_relmap_off.back()));
    HIPCHK(h, h->gscratch.alloc(gtot));
    HIPCHK(h, h->frow.alloc(S.rows.size()));
    HIPCHK(h, h->fpos.alloc(S.rows.size()));
    HIPCHK(h, h->piv.alloc(S.rows.size()));
    if (!h->anorm.p) {
        HIPCHK(h, h->anorm.alloc(1));
        HIPCHK(h, h->counters.alloc(8));
    }
    // launch plan: per level, fronts sorted by order (descending) -> size classes
    h->fac_launches.clear();
    h->sol_launches.clear();
    std::vector<int32_t> sfr;
    sfr.reserve(S.nf);
    for (int l = 0; l < S.nlevels; ++l) {
        int b = S.level_off[l], e = S.level_off[l + 1];
        {
            std::vector<std::pair<int, int32_t>> wv;  // (LDS doubles, front)
            std::vector<int32_t> big;
            for (int q = b; q < e; ++q) {
                const int32_t f = S.level_fronts[q];
                const int m = S.f_m[f], p = S.f_p[f];
                if (p <= 64 && m <= kMaxLdsFront) {
                    const int sz = p * m - p * (p - 1) / 2;
                    wv.push_back({((sz + 1) & ~1) + m, f});
                } else {
                    big.push_back(f);
                }
            }
            std::sort(wv.begin(), wv.end(), [](const auto& x, const auto& y) { return x.first > y.first; });
            size_t q = 0;
            while (q < wv.size()) {
                int cap = 256;
                while (cap < wv[q].first) cap *= 2;
                size_t r = q;
                while (r < wv.size() && (wv[r].first > cap / 2 || cap == 256)) ++r;
                SolveLaunch sl{l, (int)sfr.size(), (int)(r - q), wv[q].first, 0, 0, true};
                for (size_t t = q; t < r; ++t) sfr.push_back(wv[t].second);
                h->sol_launches.push_back(sl);
                q = r;
            }
            if (!big.empty()) {
                SolveLaunch sl{l, (int)sfr.size(), (int)big.size(), 0, 0, 0, false};
                for (int32_t f : big) {
                    sfr.push_back(f);
                    sl.mmax = std::max(sl.mmax, S.f_m[f]);
                    sl.pmax = std::max(sl.pmax, S.f_p[f]);
                }
                h->sol_launches.push_back(sl);
            }
        }
        int q = b;
        while (q < e) {
            int m0 = S.f_m[S.level_fronts[q]];
            bool global = m0 > kMaxLdsFront;
            int cap = global ? 1 << 30 : (m0 > 64 ? kMaxLdsFront : (m0 > 32 ? 64 : 32));
            int floor_ = global ? kMaxLdsFront : (cap == kMaxLdsFront ? 64 : (cap == 64 ? 32 : 0));
            int r = q;
            while (r < e && S.f_m[S.level_fronts[r]] > floor_ && S.f_m[S.level_fronts[r]] <= cap) ++r;
            h->fac_launches.push_back({q, r - q, m0, global});
            q = r;
        }
    }
    HIPCHK(h, h->solve_fronts.upload(sfr, s));
    HIPCHK(h, hipStreamSynchronize(s));
    double an = h->st.analysis_seconds;
    int64_t nfac = h->st.factorizations, nsol = h->st.solves;
    memset(&h->st, 0, sizeof(h->st));
    h->st.n = S.n;
    h->st.nnz = S.nnz;
    h->st.nnz_unique = S.nu;
    h->st.nnz_L = S.nnz_L;
    h->st.n_fronts = S.nf;
    h->st.n_levels = S.nlevels;
    h->st.max_front = S.max_m;
    h->st.n_dense = S.n_dense;
    h->st.flops = S.flops;
    h->st.analysis_seconds = an;
    h->st.factorizations = nfac;
    h->st.solves = nsol;
    h->st.bytes_L = 8.0 * (double)S.L_size;
    h->st.bytes_cb = 8.0 * (double)S.cb_size;
    return UNO_KKT_OK;
}

int enqueue_factorization(uno_kkt_t h) {
    Symbolic& S = h->S;
    hipStream_t s = h->stream;
    HIPCHK(h, hipMemsetAsync(h->counters.p, 0, 8 * sizeof(unsigned long long), s));
    HIPCHK(h, hipMemsetAsync(h->anorm.p, 0, sizeof(unsigned long long), s));
    {
        TimerScope t(h, KC_PACK);
        HIPCHK(h, launch_pack(h->values_ptr, h->dup_ptr.p, h->dup_pos.p, S.nu, h->uval.p, s));
    }
    {
        TimerScope t(h, KC_SCALE);
        ScanArgs SA;
        SA.n = S.n; SA.perm = h->perm_d.p; SA.cptr = h->cptr.p; SA.rptr = h->rptr.p; SA.rslot = h->rslot.p;
        SA.ent_r = h->ent_r.p; SA.ent_c = h->ent_c.p; SA.uval = h->uval.p; SA.scale = h->scale.p; SA.out = nullptr;
        SA.anorm = h->anorm.p; SA.long_rows = h->long_rows.p; SA.n_long = h->n_long;
        SA.max_long = h->max_long;
        HIPCHK(h, launch_scale(SA, h->scale_iters, h->rmax.p, h->rowsum.p, s));
    }
    FactorArgs A;
    A.fm = h->fm.p; A.fp = h->fp.p; A.rows_off = h->rows_off.p; A.rows = h->rows.p;
    A.ent_off = h->ent_off.p; A.ent_lpos = h->ent_lpos.p; A.uval = h->uval.p; A.scale = h->scale.p;
    A.child_off = h->child_off.p; A.child = h->child.p; A.relmap_off = h->relmap_off.p; A.relmap = h->relmap.p;
    A.ch_cm = h->ch_cm.p; A.ch_relmap_off = h->ch_relmap_off.p; A.ch_cb_off = h->ch_cb_off.p;
    A.L_off = h->L_off.p; A.cb_off = h->cb_off.p; A.gscratch_off = h->gscratch_off.p; A.anorm_bits = h->anorm.p;
    A.L = h->L.p; A.cb = h->cb.p; A.gscratch = h->gscratch.p; A.frow = h->frow.p; A.fpos = h->fpos.p; A.piv = h->piv.p;
    A.counters = h->counters.p; A.fstat = h->fstat.p; A.fcnt = h->fcnt.p; A.u = h->u; A.null_fac = h->null_fac;
    A.fparent = h->fparent.p; A.delayed = h->delayed.p; A.record_delays = h->delay_relaxed;
    A.stamps = nullptr;
    A.stamp_mode = h->want_stamps;
    if (h->want_stamps) {
        if (h->stamps.n != (size_t)(8 * S.nf)) HIPCHK(h, h->stamps.alloc(8 * S.nf));
        HIPCHK(h, hipMemsetAsync(h->stamps.p, 0, sizeof(unsigned long long) * 8 * S.nf, s));
        A.stamps = h->stamps.p;
    }
    for (const Launch& L : h->fac_launches) {
        TimerScope t(h, L.global ? KC_FACTOR_GLOBAL : KC_FACTOR_LDS);
        HIPCHK(h, launch_factor(A, h->level_fronts.p + L.begin, L.count, L.mmax, L.global, s));
    }
    HIPCHK(h, launch_count(h->fcnt.p, h->fstat.p, S.nf, h->counters.p, s));
    HIPCHK(h, hipMemcpyAsync(h->h_counters, h->counters.p, 8 * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    h->factor_enqueued = true;
    return UNO_KKT_OK;
}

}  // namespace

extern "C" {


const char* uno_kkt_version(void) { return "uno-kkt-mi355x 0.1.0 (gfx950)"; }

int uno_kkt_create(uno_kkt_t* handle, int device_id) {
    if (!handle) return UNO_KKT_ERR_ARG;
    *handle = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return UNO_KKT_ERR_NODEVICE;
    if (device_id < 0 || device_id >= ndev) return UNO_KKT_ERR_ARG;
    auto* h = new uno_kkt();
    h->device = device_id;
    if (hipSetDevice(device_id) != hipSuccess || hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess ||
        hipHostMalloc((void**)&h->h_counters, 8 * sizeof(unsigned long long)) != hipSuccess) {
        delete h;
        return UNO_KKT_ERR_HIP;
    }
    memset(h->h_counters, 0, 8 * sizeof(unsigned long long));
    *handle = h;
    return UNO_KKT_OK;
}

void uno_kkt_destroy(uno_kkt_t h) {
    if (!h) return;
    hipSetDevice(h->device);
    if (h->stream) hipStreamSynchronize(h->stream);
    for (auto& t : h->pending) { hipEventDestroy(t.a); hipEventDestroy(t.b); }
    for (auto e : h->ev_pool) hipEventDestroy(e);
    if (h->h_counters) hipHostFree(h->h_counters);
    if (h->stream) hipStreamDestroy(h->stream);
    delete h;
}

int uno_kkt_set_option(uno_kkt_t h, const char* name, double value) {
    if (!h || !name) return UNO_KKT_ERR_ARG;
    std::string n(name);
    if (n == "pivot_threshold") h->u = value;
    else if (n == "null_tol_factor") h->null_fac = value;
    else if (n == "scale_iters") h->scale_iters = std::max(0, (int)value);
    else if (n == "leaf_size") h->aopt.leaf_size = std::max(1, (int)value);
    else if (n == "max_block") h->aopt.max_block = std::max(1, std::min((int)value, 1024));
    else if (n == "dense_factor") h->aopt.dense_factor = value;
    else if (n == "timing") h->timing = value != 0.0;
    else if (n == "delay_relaxed") h->delay_relaxed = value != 0.0;
    else if (n == "stamps") h->want_stamps = (int)value;
    else if (n == "max_merge_rounds") h->max_merge_rounds = std::max(0, (int)value);
    else return set_err(h, UNO_KKT_ERR_ARG, "unknown option '" + n + "'");
    return UNO_KKT_OK;
}

int uno_kkt_analyze(uno_kkt_t h, int64_t n, int64_t nnz, const int64_t* row, const int64_t* col) {
    if (!h) return UNO_KKT_ERR_ARG;
    if (n < 0 || nnz < 0 || (nnz > 0 && (!row || !col))) return set_err(h, UNO_KKT_ERR_ARG, "bad pattern arguments");
    HIPCHK(h, hipSetDevice(h->device));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    h->analyzed = h->factored = h->factor_enqueued = false;
    h->values_ptr = nullptr;
    h->merges_total = 0;
    auto t0 = std::chrono::steady_clock::now();
    std::string msg = ukkt::analyze(n, nnz, row, col, h->aopt, h->P, h->S);
    if (!msg.empty()) return set_err(h, UNO_KKT_ERR_ARG, msg);
    HIPCHK(h, h->values.alloc(nnz));
    int rc = upload_structure(h);
    if (rc != UNO_KKT_OK) return rc;
    auto t1 = std::chrono::steady_clock::now();
    h->st.analysis_seconds = std::chrono::duration<double>(t1 - t0).count();
    h->st.factorizations = 0;
    h->st.solves = 0;
    h->analyzed = true;
    h->err.clear();
    return UNO_KKT_OK;
}

int uno_kkt_set_values(uno_kkt_t h, const int64_t* positions, const double* v, int64_t count) {
    if (!h) return UNO_KKT_ERR_ARG;
    if (!h->analyzed || !h->values_ptr) return set_err(h, UNO_KKT_ERR_STATE, "set_values before a factorization");
    if (count < 0 || (count > 0 && (!positions || !v))) return set_err(h, UNO_KKT_ERR_ARG, "bad arguments");
    HIPCHK(h, hipSetDevice(h->device));
    // small host-driven edit: positions are few (regularization diagonal), copy one by one in batches
    for (int64_t i = 0; i < count; ++i) {
        if (positions[i] < 0 || positions[i] >= h->S.nnz) return set_err(h, UNO_KKT_ERR_ARG, "position out of range");
        HIPCHK(h, hipMemcpyAsync(const_cast<double*>(h->values_ptr) + positions[i], v + i, sizeof(double),
                                 hipMemcpyHostToDevice, h->stream));
    }
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return UNO_KKT_OK;
}

}  // extern "C"

__global__ void k_fill(double* p, int64_t n, double v) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = v;
}

extern "C" {

int uno_kkt_fill_values(uno_kkt_t h, int64_t first, int64_t count, double value) {
    if (!h) return UNO_KKT_ERR_ARG;
    if (!h->analyzed || !h->values_ptr) return set_err(h, UNO_KKT_ERR_STATE, "fill_values before a factorization");
    if (first < 0 || count < 0 || first + count > h->S.nnz) return set_err(h, UNO_KKT_ERR_ARG, "range out of bounds");
    if (count == 0) return UNO_KKT_OK;
    HIPCHK(h, hipSetDevice(h->device));
    int grid = (int)std::min<int64_t>((count + 255) / 256, 4096);
    hipLaunchKernelGGL(k_fill, dim3(grid), dim3(256), 0, h->stream, const_cast<double*>(h->values_ptr) + first, count, value);
    HIPCHK(h, hipGetLastError());
    return UNO_KKT_OK;
}

int uno_kkt_factorize(uno_kkt_t h, const double* values, int values_on_device) {
    if (!h) return UNO_KKT_ERR_ARG;
    if (!h->analyzed) return set_err(h, UNO_KKT_ERR_STATE, "factorize before analyze");
    HIPCHK(h, hipSetDevice(h->device));
    Symbolic& S = h->S;
    if (h->factor_enqueued) {  // previous factorization never queried: drain it first
        int rc = finish_factorization(h);
        (void)rc;
    }
    h->factored = false;
    if (values == nullptr) {
        if (!h->values_ptr && S.nnz > 0) return set_err(h, UNO_KKT_ERR_STATE, "no device values to reuse");
    } else if (values_on_device) {
        h->values_ptr = values;
    } else {
        if (S.nnz > 0)
            HIPCHK(h, hipMemcpyAsync(h->values.p, values, S.nnz * sizeof(double), hipMemcpyHostToDevice, h->stream));
        h->values_ptr = h->values.p;
    }
    int rc = enqueue_factorization(h);
    if (rc != UNO_KKT_OK) return rc;
    h->st.factorizations++;
    return UNO_KKT_OK;
}

int uno_kkt_inertia(uno_kkt_t h, int64_t* positive, int64_t* negative, int64_t* zero) {
    if (!h || !positive || !negative || !zero) return UNO_KKT_ERR_ARG;
    HIPCHK(h, hipSetDevice(h->device));
    int rc = finish_factorization(h);
    if (rc != UNO_KKT_OK) return rc;
    *positive = (int64_t)h->h_counters[0];
    *negative = (int64_t)h->h_counters[1];
    *zero = (int64_t)h->h_counters[2];
    return UNO_KKT_OK;
}

int uno_kkt_solve(uno_kkt_t h, const double* rhs, double* x, int on_device) {
    if (!h || !rhs || !x) return UNO_KKT_ERR_ARG;
    if (!h->analyzed || (!h->factored && !h->factor_enqueued))
        return set_err(h, UNO_KKT_ERR_STATE, "solve before factorize");
    HIPCHK(h, hipSetDevice(h->device));
    Symbolic& S = h->S;
    hipStream_t s = h->stream;
    const double* b = rhs;
    if (!on_device) {
        if (S.n > 0) HIPCHK(h, hipMemcpyAsync(h->bvec.p, rhs, S.n * sizeof(double), hipMemcpyHostToDevice, s));
        b = h->bvec.p;
    }
    {
        TimerScope t(h, KC_RHS);
        HIPCHK(h, launch_rhs_scale(b, h->scale.p, h->w.p, S.n, s));
    }
    SolveArgs A;
    A.fm = h->fm.p; A.fp = h->fp.p; A.rows_off = h->rows_off.p; A.frow = h->frow.p; A.fpos = h->fpos.p; A.piv = h->piv.p;
    A.child_off = h->child_off.p; A.child = h->child.p; A.relmap_off = h->relmap_off.p; A.relmap = h->relmap.p;
    A.L_off = h->L_off.p; A.L = h->L.p; A.w = h->w.p; A.cvec = h->cvec.p;
    auto run = [&](const SolveLaunch& L, bool forward) -> hipError_t {
        const int32_t* fr = h->solve_fronts.p + L.begin;
        return L.wave ? launch_solve_wave(A, fr, L.count, L.lds, forward, s)
                      : launch_solve(A, fr, L.count, L.mmax, L.pmax, forward, s);
    };
    for (size_t q = 0; q < h->sol_launches.size(); ++q) {
        TimerScope t(h, KC_SOLVE_FWD);
        HIPCHK(h, run(h->sol_launches[q], true));
    }
    for (size_t q = h->sol_launches.size(); q-- > 0;) {
        TimerScope t(h, KC_SOLVE_BWD);
        HIPCHK(h, run(h->sol_launches[q], false));
    }
    double* xd = on_device ? x : h->bvec.p;
    {
        TimerScope t(h, KC_RHS);
        HIPCHK(h, launch_unscale(h->w.p, h->scale.p, xd, S.n, s));
    }
    h->st.solves++;
    if (!on_device) {
        if (S.n > 0) HIPCHK(h, hipMemcpyAsync(x, xd, S.n * sizeof(double), hipMemcpyDeviceToHost, s));
        HIPCHK(h, hipStreamSynchronize(s));
    }
    if (h->factor_enqueued) {
        int rc = finish_factorization(h);
        if (rc != UNO_KKT_OK) return rc;
    }
    return UNO_KKT_OK;
}

int uno_kkt_stats(uno_kkt_t h, uno_kkt_stats_t* out) {
    if (!h || !out) return UNO_KKT_ERR_ARG;
    if (h->factor_enqueued) finish_factorization(h);
    *out = h->st;
    out->fronts_merged = h->merges_total;
    return UNO_KKT_OK;
}

int uno_kkt_kernel_times(uno_kkt_t h, char* names, int cap, double* ms, int64_t* launches, int max_classes) {
    if (!h) return UNO_KKT_ERR_ARG;
    flush_timing(h);
    std::string all;
    for (int c = 0; c < KC_COUNT; ++c) {
        if (c) all += ",";
        all += kClassNames[c];
        if (c < max_classes) {
            if (ms) ms[c] = h->t_ms[c];
            if (launches) launches[c] = h->t_n[c];
        }
    }
    if (names && cap > 0) {
        strncpy(names, all.c_str(), (size_t)cap - 1);
        names[cap - 1] = 0;
    }
    return KC_COUNT;
}

int uno_kkt_reset_kernel_times(uno_kkt_t h) {
    if (!h) return UNO_KKT_ERR_ARG;
    flush_timing(h);
    for (int c = 0; c < KC_COUNT; ++c) { h->t_ms[c] = 0; h->t_n[c] = 0; }
    return UNO_KKT_OK;
}

void* uno_kkt_stream(uno_kkt_t h) { return h ? (void*)h->stream : nullptr; }

// diagnostics (include/uno_kkt_debug.h): per-front phase stamps of the last factorization
int64_t uno_kkt_debug_stamps(uno_kkt_t h, uint64_t* out, int64_t cap, int32_t* fm, int32_t* fp, int32_t* flevel) {
    if (!h || !h->stamps.p) return -1;
    if (h->factor_enqueued) finish_factorization(h);
    int64_t nf = h->S.nf;
    if (cap < 8 * nf) return -(8 * nf);
    hipMemcpy(out, h->stamps.p, sizeof(uint64_t) * 8 * nf, hipMemcpyDeviceToHost);
    for (int64_t f = 0; f < nf; ++f) { fm[f] = h->S.f_m[f]; fp[f] = h->S.f_p[f]; flevel[f] = h->S.f_level[f]; }
    return nf;
}

const char* uno_kkt_last_error(uno_kkt_t h) { return h ? h->err.c_str() : "null handle"; }

}  // extern "C"
