// kkt_api.cpp -- implementation of the uno_kkt C ABI (include/uno_kkt.h).
//
// Host orchestration of one factor/solve handle: symbolic analysis on the host (analysis.cpp),
// device-resident layout, level-scheduled launches of the kernels in kkt_kernels.hip on one HIP
// stream.  Mirrors the call sequence of Uno's MUMPS adapter
// (uno/ingredients/subproblem_solvers/MUMPS/MUMPSSolver.cpp:72-147) but keeps the factor on the GPU.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cfloat>
#include <cmath>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/uno_kkt.h"
#include "../../include/uno_kkt_debug.h"
#include "analysis.hpp"
#include "comm.hpp"
#include "ipm_kernels.hpp"
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

enum KernelClass { KC_PACK = 0, KC_SCALE, KC_FACTOR_LDS, KC_FACTOR_GLOBAL, KC_SOLVE_FWD, KC_SOLVE_BWD, KC_RHS, KC_SYMV, KC_ROWSUM, KC_COUNT };
const char* kClassNames[KC_COUNT] = {"pack", "scale", "factor_lds", "factor_global", "solve_fwd", "solve_bwd", "rhs", "symv",
                                     "rowsum"};

struct Launch {
    int begin, count, mmax;
    bool global;
    int level;
    int pmax = 0, maxch = 0;  // large fronts: widest panel sequence, most children (assembly passes)
};

// one solve launch: fronts solve_fronts[begin, begin+count) of one level; wave kernels (p <= 64,
// m <= kMaxLdsFront) are grouped by the LDS their packed panel needs so small fronts keep occupancy
struct SolveLaunch {
    int level, begin, count, lds, mmax, pmax;
    bool wave;
};

// launch plan of a set of fronts: factor launches index fac_fronts, solve launches sol_fronts
struct Plan {
    DBuf<int32_t> fac_fronts, sol_fronts;
    std::vector<int32_t> fac_host;  // host copy of fac_fronts (reordered by reorder_slow_first)
    std::vector<Launch> fac;
    std::vector<SolveLaunch> sol;  // ordered by level
};

// per-rank data of a distributed (subtree-partitioned) factorization, SURVEY.md 8(e)
struct DistState {
    Partition part;
    std::vector<std::pair<int64_t, int64_t>> pack_ranges;  // packed slot ranges of the rank's fronts
    DBuf<int32_t> own_new, own_orig, own_long;             // rows eliminated in the rank's subtrees
    int64_t n_own = 0;
    int32_t n_own_long = 0;
    int64_t max_own_long = 0;
    DBuf<int32_t> top_orig;                                // rows eliminated in top fronts
    int64_t n_top_rows = 0;
    DBuf<int32_t> chunk_row, pslot, ppartner;              // partial scans of the top rows
    DBuf<int64_t> chunk_begin, row_chunk;
    DBuf<double> chunk_part, own_long_part;               // chunk results (combined in chunk order)
    int64_t own_long_chunks = 0;
    int64_t nchunks = 0;
    DBuf<double> outT, tbuf, xbuf;
    DBuf<unsigned long long> tmp;
    std::vector<int64_t> own_count;                        // per rank (rank 0: gather of the solution)
    DBuf<int32_t> all_own_orig;                            // rank 0: every rank's own rows, by rank
    std::vector<int64_t> all_own_off;
    double my_flops = 0.0, top_flops = 0.0;
    int64_t my_fronts = 0;
};

}  // namespace

struct uno_kkt {
    int device = 0;
    hipStream_t stream = nullptr;
    // ||A_pre||_inf (row sums of the scaled matrix) runs on stream2 beside the factorization, which uses
    // threshold 0 and records its smallest accepted pivot; finish_factorization checks it against the
    // exact threshold and refactors with the exact one in the (rare) case it would have mattered
    hipStream_t stream2 = nullptr;
    // the size-class launches of one factorization level are independent: the second and later run on
    // stream3 beside the first (fork / join events), so one launch's tail overlaps the other's body
    hipStream_t stream3 = nullptr;
    hipStream_t stream4 = nullptr;   // third class stream (option concurrent_classes = 3)
    // uno_kkt_stage_values: host -> device value chunks while the caller is still assembling (created on
    // first use); the next uno_kkt_factorize(NULL) makes the solver's stream wait for them
    hipStream_t upload = nullptr;
    hipEvent_t ev_upload = nullptr, ev_upload_dep = nullptr;
    bool staged_pending = false;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr, ev_join4 = nullptr;
    hipEvent_t ev_scale = nullptr, ev_norm = nullptr;
    int overlap_norm = 1;
    bool exact_next = false, last_optimistic = false;
    // ||A_pre||_inf is needed only when some accepted pivot could lie at or below the null threshold.  After
    // the last equilibration sweep every scaled entry is at most 1 (|s a_ij s| <= min(r_i, r_j) /
    // sqrt(r_i r_j) with the sweep's row maxima r), so ||A_pre||_inf <= max row length: a factorization
    // run with threshold 0 whose smallest accepted pivot exceeds eps * null_fac * max_row_len is the
    // exact one and the row-sum pass is skipped (norm_valid = false).
    bool norm_valid = false;
    int64_t max_row_len = 0, norm_skips = 0;
    ScanArgs scan{};  // the last factorization's scan arguments (row sums on demand)
    int64_t exact_redos = 0;
    AnalysisOptions aopt;
    double u = 0.01, null_fac = 1e-5;
    // ICNTL(8)=8 restated as 3 symmetric infinity-norm sweeps, the oracle's value (oracle/kkt_oracle.c)
    int scale_iters = 3;
    int timing = 0;
    Pattern P;
    Symbolic S;
    int delay_relaxed = 1;      // also amalgamate fronts whose pivots needed a relaxed threshold (MUMPS: delay)
    int max_merge_rounds = 64;
    int verbose = 0;
    std::chrono::steady_clock::time_point t_factor;  // verbose >= 2: per-factorization wall time
    int64_t merges_total = 0;
    bool analyzed = false, factor_enqueued = false, factored = false;
    const double* values_ptr = nullptr;  // device values used by the last factorization
    // device arrays
    DBuf<double> values, uval, scale, L, cb, gscratch, w, cvec, rowsum, rmax, bvec;
    DBuf<int32_t> slot_src;               // k_pack: per slot its single COO position, or -1 - (multi_slots record)
    DBuf<int32_t> multi_slots;            // slots with several COO positions (k_pack_multi)
    int64_t n_multi = 0;
    DBuf<int32_t> dup_ptr, dup_pos, ent_r, ent_c, fm, fp, rows, frow, fpos, child_off, child, relmap, fstat;
    DBuf<uint32_t> ent_lpos;
    DBuf<int64_t> rows_off, ent_off, relmap_off, L_off, cb_off, gscratch_off, ch_relmap_off, ch_cb_off;
    DBuf<uint16_t> cbpos;                 // FactorArgs::cbpos
    bool use_cbpos = false;
    int cbpos_opt = 1;                    // option "cbpos"
    DBuf<int32_t> ch_cm;
    DBuf<int8_t> piv;
    DBuf<BigFrontState> big;              // large-front factorization state (fronts with m > kMaxLdsFront)
    DBuf<int32_t> big_pending;
    int32_t* h_big = nullptr;             // pinned: fronts still factoring (run_big_fronts)
    DBuf<unsigned long long> counters, stamps, fcnt;  // counters: kCounterSlots (minbits, anorm inside)
    unsigned long long* minbits_p = nullptr;  // counters.p + 8
    unsigned long long* anorm_p = nullptr;    // counters.p + 9
    DBuf<double> fmin;
    int want_stamps = 0;
    DBuf<int32_t> perm_d, cptr, rptr, rslot, long_rows, fparent, delayed, rowpartner;
    DBuf<double> uvalR;  // row-major copy of |A| (single-GPU equilibration, option front_sweeps=0)
    int front_sweeps = 1;                 // option front_sweeps: equilibration over the fronts' slots (k_sweep_front)
    bool use_front_sweeps = false;        // front_sweeps, one GPU and every front within kMaxSweepFront rows
    DBuf<int8_t> longpos;                 // by original id: index among the long rows, -1 otherwise
    DBuf<double> symv_long_part;          // symv: chunk partials of the long rows
    DBuf<int32_t> sweep_big;              // fronts of more than kSweepBigSlots slots (sliced sweeps)
    int32_t n_sweep_big = 0, sweep_slices = 1;
    DBuf<int32_t> long_orig;              // long rows, original ids
    DBuf<double> part_long;               // fronts x long rows: sweep partials
    int32_t n_long = 0;
    int64_t max_long = 0, long_chunks = 0;
    DBuf<double> long_part;  // chunk results of the long-row scans
    DBuf<uint32_t> long_cnt; // per long row: chunk arrival counter (single-GPU scans)
    unsigned long long* h_counters = nullptr;
    Plan plan[2];  // 0: the rank's own fronts (all fronts on one GPU), 1: top fronts (rank 0 of a group)
    Plan dff_plan; // factor launches of the own fronts outside the dataflow launch (dff active)
    // dataflow solve (one launch per direction, kkt_kernels.hip k_solve_*_df); every front of the walk
    // one-wave eligible; option "dataflow_solve" (default 1).  The walk is every front on one GPU and the
    // rank's own subtree fronts in distributed runs (option "dist_dataflow_solve"), whose top fronts stay
    // level-scheduled on rank 0.  The walk assumes its grid is resident (sized by the occupancy query):
    // default on with one GPU per rank (RCCL), off when ranks may share a GPU (in-process / host
    // transports: waits would run into their bound and redo the solve level by level)
    int df_enabled = 1;
    int dist_df = -1;              // -1: auto (RCCL transport)
    bool own_device = false;       // the transport guarantees one GPU per rank
    int32_t df_nwalk = 0;          // fronts of the walk
    int64_t df_top_base = 0;       // distributed: xs slots of the top rows (top_orig order)
    DBuf<int32_t> df_roots, df_topf;  // distributed: own subtree roots with a top parent; top fronts
    int32_t n_df_roots = 0, n_df_topf = 0;
    DBuf<unsigned long long> df_abort64;
    int df_grid = 0, df_lds = 0;   // 0 grid: not eligible -> level schedule
    int solve_rg = 1;              // option "solve_rg": register-resident forward walk kernel (k_solve_fwd_rg)
    int solve_flat = 0;            // option "solve_flat_levels": the walks' bottom levels as flat launches (measured
                                   // slower than the walks at C3, DESIGN.md section 4 round 6: off by default)
    int solve_rg_bwd = 0;          // option "solve_rg_bwd": register-resident backward walk (k_solve_bwd_rg; its
                                   // transpose-reduced rectangle sums in another order, so the level schedule follows)
    int rg_grid_f = 0, rg_grid_b = 0;
    int rg_wpe = 3;                // option "solve_rg_wpe": waves per SIMD of the walk kernels' register budget (3 or 4)
    bool new_bwd = false;          // option solve_rg: the backward of one-wave fronts runs the register kernels' arithmetic
                                   // in both schedules (k_solve_bwd_rg / k_solve_bwd_w2)
    int df_win = 0, df_win_opt = 0; // LDS panel window of the dataflow solve (option solve_window, 0 = auto)
    int df_piv_off = 0;
    uint32_t df_epoch = 0;
    bool df_rx_valid = false;      // rxpos matches the last factorization's pivoting
    int64_t df_aborts = 0;
    int df_consec_aborts = 0;      // consecutive aborted dataflow solves (kMaxDfAborts turns the walk off)
    int debug_abort_solves = 0;    // option debug_abort_solves: the next k dataflow solves start with the abort flag set (tests)
    DBuf<int32_t> df_order, df_desc, df_xpos, df_rxpos;
    DBuf<int32_t> df_rowx;                // per front row: xs slot of a walk front's pivot position, -2: its
                                          // contribution row, -1: not in the walk (k_xpos)
    DBuf<int32_t> rg_desc, ov_desc;  // register kernels: the walk split into p <= 32, m <= 72 fronts and the others
    int32_t rg_nf = 0, ov_nf = 0, ov_grid = 0;
    DBuf<int32_t> rgf_desc, flat_desc;  // forward: rg_desc without its flat levels, and those (k_solve_fwd_flat)
    DBuf<int32_t> bwd_desc;             // backward LDS-panel walk: df_desc without the flat levels (k_solve_bwd_flat)
    int32_t bwd_nf = 0;
    int32_t rgf_nf = 0;
    std::vector<int32_t> flat_off;      // flat_desc positions of each flat level (flat_off.size() - 1 launches)
    DBuf<int64_t> df_cvx_off, df_ch_cvx_off, df_xs_off;
    DBuf<uint32_t> df_cnt, df_done, df_abort;
    DBuf<double> df_cvx, df_xs;
    int want_solve_stamps = 0;
    DBuf<unsigned long long> df_stamps;
    // dataflow factorization of the upper tree (levels >= dff_level, every front one-wave); option
    // "dataflow_factor" (default 1)
    int concurrent_classes = 1;  // option "concurrent_classes"
    int early_xpos = 1;          // option "early_xpos": the dataflow solve's row maps queued with the factorization
    bool xpos_by_factor = false; // the last factorization wrote xpos itself (FactorArgs::xpos)
    hipEvent_t ev_counters = nullptr;  // after the counters' read-back of the last enqueued factorization
    hipEvent_t ev_wait = nullptr;      // host_wait_stream
    int spin_wait = 1;                 // option "spin_wait": host waits poll (host_wait)
    // option "host_flag" (default 0): one GPU, the host polls k_count's sequence number instead of an event.  Off
    // by default: the counters and the flag are relaxed system-scope stores ordered only by the storing wave's
    // vmcnt drain, which does not order their arrival in host memory across fabric paths; a full GPU suite with
    // it on ended with one failure in the 1465-factorization drop-in trace (unconfirmed: the box was lost)
    int host_flag = 0;
    unsigned long long count_seq = 0;  // k_count flags issued
    unsigned long long wait_seq = 0;   // the flag the last enqueued factorization writes (0: wait on ev_counters)
    DBuf<unsigned long long> rmaxk;    // front sweeps: n row maxima per sweep (elimination order)
    DBuf<int32_t> rows_sw;             // front sweeps: the fronts' rows in the elimination order
    DBuf<int8_t> longpos_sw;           // front sweeps: longpos by new index
    DBuf<int32_t> long_sw;             // front sweeps: the long rows' new indices
    bool rmaxk_clean = false;          // rmaxk all zero (left so by k_sweep_final)
    int front_scale = 0;         // option "front_scale": the scaling gathered per front row (k_front_scale) for the
                                 // factorization (1; 2 is accepted as 1)
    DBuf<double> fscale;
    DBuf<int8_t> flong;          // per front row: index of its row among the long rows, -1 otherwise
    int dff_enabled = 1;  // 0 off, 1 (default) levels >= L*, 2 also the small fronts below them (measured no faster at C3)
    int dff_level = INT32_MAX;     // first level of the dataflow launch (INT32_MAX: none)
    int dff_mmax = 0;
    uint32_t dff_epoch = 0;
    int64_t dff_aborts = 0;
    DBuf<int32_t> dff_order, dff_nch;
    std::vector<int32_t> dff_order_host;  // host copy of dff_order (reorder_slow_first)
    DBuf<int32_t> fslow;                  // per front: steps off the register path in the last factorization
    int slow_first = 1;                   // option slow_first: reorder the launches after a structure's first factorization
    bool reorder_due = false;
    DBuf<uint32_t> dff_cnt, dff_ticket;
    // distributed factorization (null comm: one GPU)
    // device-side vector work around the solve
    int64_t rhs_n = -1, rhs_m = -1;
    DBuf<int64_t> jv_ptr;                 // per variable: range into jv_ent (Jacobian entries, constraint-ascending)
    DBuf<int32_t> bar_var;                // barrier diagonal: bounded variables (ascending)
    DBuf<int8_t> bar_which;               // 1: finite lower, 2: finite upper bound
    DBuf<double> bar_lb, bar_ub;
    int64_t bar_n = -1;
    int64_t aug_reg = -1, aug_nh = 0, aug_nj = 0;  // uno_kkt_augmented_setup
    DBuf<int32_t> jv_ent, j_con;
    DBuf<int32_t> rhs_long;               // variables in more than kRhsLong constraints
    int32_t rhs_n_long = 0;
    DBuf<unsigned long long> alpha;
    DBuf<double> symv_tmp, symv_part, dot_d;
    DBuf<double> xtmp, rtmp;              // host-pointer solves / refinement residuals
    int refine = 1;                       // refinement steps after a factorization with relaxed pivots
    double refine_tol = 0.0;              // option "refine_tol": skip a step when the componentwise backward error
                                          // is already <= refine_tol (0: always refine; measured at C3 in the
                                          // plugin mode: 3.0e-9 before the step, 4.1e-16 after it)
    DBuf<double> atmp;                    // |A| |x| of the backward-error check
    DBuf<unsigned long long> omega_d;
    int resid_fronts = 1;                 // option: refinement residual over the fronts' slots (launch_resid)
    int sweep_reset = 1;                  // option: the first sweep resets the counters (no k_reset_counters)
    int sweep_pack = 1;                   // option: the COO -> slot pack fused into the first sweep (0: flat k_pack first)
    int64_t resid_long = kResidShort;     // option (tests): rows with more partials are summed by chunks
    int rz_state = 0;                     // 0: index not built, 1: built, -1: not applicable (old symv)
    DBuf<int32_t> rz_ptr, rz_pos, rz_long, rz_chunk_off, rz_chunk_row;
    DBuf<double> rz_part, rz_chunk_part;
    int32_t rz_n_long = 0;
    int64_t rz_n_chunks = 0;
    int pin_host = 0;                     // option pin_host_values
    const double* pinned_ptr = nullptr;   // caller buffer registered with hipHostRegister
    size_t pinned_bytes = 0;
    DBuf<int64_t> edit_pos;               // uno_kkt_set_values staging
    DBuf<double> edit_val;
    bool packed_valid = false;            // uval holds the current values (symv reuses the factor's pack)
    ukkt::Transport* comm = nullptr;
    int rank = 0, world = 1;      // effective: world 1 when the partition was declined (every rank a replica)
    int comm_rank = 0, comm_world = 1;  // the attached transport's
    bool dist_declined = false;   // analysis found too little top-level parallelism (SURVEY.md 8(e) gate)
    double dist_efficiency = 0.0; // estimated parallel efficiency of the partition (analysis cost model)
    double dist_min_eff = 0.5;    // option dist_min_efficiency
    int dist_force = 0;           // option dist_force: partition whatever the estimate (tests, experiments)
    int comm_trace = 0;           // option comm_trace: the transport records its calls (uno_kkt_debug_comm_trace)
    int side_pending = 0;         // side streams (bit 0: stream3, bit 1: stream4) with factor launches not yet joined
                                  // into `stream` (the comm trace's order records check it is 0 at every exchange)
    int gather_solution = 1;
    DistState dist;
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

// comm trace (tests): every exchange records whether it is enqueued on the main stream after every producing
// launch -- the RCCL call is stream-ordered, so that is what makes its buffer the finished one
void install_order_probe(uno_kkt_t h) {
    ukkt::comm_trace_set_probe(h->comm, [h](hipStream_t s) { return std::make_pair(s == h->stream ? 1 : 0, h->side_pending); });
}

// hipHostUnregister of the caller's page-locked buffer (option pin_host_values) waits for every copy that
// may still read it: the staged chunks on the upload stream and the factorize / factorize_update copies on
// the solver's stream (a copy from page-locked memory is a DMA that reads the buffer until it completes)
void unpin_host_buffer(uno_kkt_t h) {
    if (!h->pinned_ptr) return;
    if (h->upload) (void)hipStreamSynchronize(h->upload);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    (void)hipHostUnregister(const_cast<double*>(h->pinned_ptr));
    (void)hipGetLastError();
    h->pinned_ptr = nullptr;
    h->pinned_bytes = 0;
}

// value edits on the solver's stream (set_values, fill_values, factorize_update) come after the chunks staged
// so far (uno_kkt_stage_values): the stream waits for the upload stream's last chunk, so a staged chunk of the
// same positions can never land after the edit (calls take effect in call order)
hipError_t order_after_staged(uno_kkt_t h) {
    if (!h->staged_pending) return hipSuccess;
    hipError_t e = hipEventRecord(h->ev_upload, h->upload);
    if (e != hipSuccess) return e;
    return hipStreamWaitEvent(h->stream, h->ev_upload, 0);
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
    hipStream_t s;
    hipEvent_t a = nullptr;
    TimerScope(uno_kkt_t h_, int c, hipStream_t st = nullptr) : h(h_), cls(c), s(st ? st : h_->stream) {
        if (h->timing) {
            a = get_event(h);
            hipEventRecord(a, s);
        }
    }
    ~TimerScope() {
        if (a) {
            hipEvent_t b = get_event(h);
            hipEventRecord(b, s);
            h->pending.push_back({cls, a, b});
        }
    }
};

void flush_timing(uno_kkt_t h) {
    if (h->pending.empty()) return;
    hipStreamSynchronize(h->stream);
    if (h->stream2) hipStreamSynchronize(h->stream2);
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
int reorder_slow_first(uno_kkt_t h);
int symv_impl(uno_kkt_t h, const double* x, double* y, const double* w, double* dot, bool absval = false);

// Fronts beyond LDS (m > kMaxLdsFront): blocked factorization in HBM scratch (kkt_kernels.hip k_big_*).
// Every panel + update step advances each unfinished front by at least one pivot; the host queues
// batches of steps and checks (one small copy + stream sync per batch) until no front is left.
int run_big_fronts(uno_kkt_t h, const FactorArgs& A, const int32_t* fronts, const Launch& L, hipStream_t s);

int run_big_fronts(uno_kkt_t h, const FactorArgs& A, const int32_t* fronts, const Launch& L, hipStream_t s) {
    const int count = L.count, mmax = L.mmax;
    if (count <= 0) return UNO_KKT_OK;
    HIPCHK(h, launch_big_assemble(A, fronts, count, mmax, L.maxch, s));
    const int nb = big_panel_width();
    // one panel step per nb pivots of the widest front (+2 for early panel stops before the first check)
    int batch = (L.pmax + nb - 1) / nb + 2;
    int64_t steps = 0;
    for (;;) {
        for (int r = 0; r < batch; ++r) HIPCHK(h, launch_big_step(A, fronts, count, mmax, s));
        steps += batch;
        HIPCHK(h, launch_big_pending(A, fronts, count, h->big_pending.p, s));
        HIPCHK(h, hipMemcpyAsync(h->h_big, h->big_pending.p, sizeof(int32_t), hipMemcpyDeviceToHost, s));
        HIPCHK(h, hipStreamSynchronize(s));
        if (*h->h_big == 0) break;
        if (steps > 2 * (int64_t)mmax + 64)
            return set_err(h, UNO_KKT_ERR_HIP, "internal: large-front factorization made no progress");
        batch = 8;  // early panel stops (interchanges, 2x2 / null pivots): a few more steps
    }
    HIPCHK(h, launch_big_finish(A, fronts, count, mmax, s));
    if (h->verbose >= 2) fprintf(stderr, "[uno_kkt] large fronts: %d of order <= %d, %lld panel steps\n", count, mmax, (long long)steps);
    return UNO_KKT_OK;
}

DfArgs dataflow_args(uno_kkt_t h) {
    DfArgs D;
    D.order = h->df_order.p; D.desc = h->df_desc.p; D.nf = h->df_nwalk; D.parent = h->fparent.p; D.cnt = h->df_cnt.p;
    D.done = h->df_done.p; D.epoch = h->df_epoch; D.cvx = h->df_cvx.p; D.cvx_off = h->df_cvx_off.p;
    D.ch_cvx_off = h->df_ch_cvx_off.p; D.xs = h->df_xs.p; D.xs_off = h->df_xs_off.p; D.rxpos = h->df_rxpos.p;
    D.rowx = h->df_rowx.p; D.rows_total = (int64_t)h->S.rows.size();
    D.abort_flag = h->df_abort.p;
    D.win = h->df_win;
    D.piv_off = h->df_piv_off;
    D.stamps = h->want_solve_stamps ? h->df_stamps.p : nullptr;
    D.rg_desc = h->rg_desc.p; D.rg_nf = h->rg_nf;
    D.ov_desc = h->ov_desc.p; D.ov_nf = h->ov_nf; D.ov_grid = h->ov_grid;
    D.rgf_desc = h->rgf_desc.p; D.rgf_nf = h->rgf_nf;
    D.flat_desc = h->flat_desc.p;
    D.bdesc = h->bwd_desc.p; D.bnf = h->bwd_nf;
    return D;
}

// After the stream has drained: a dataflow solve whose waits hit their limit produced no valid
// solution (k_xs_out then leaves x untouched); the flag is cleared, the caller redoes that one solve with
// the level schedule and the dataflow solve stays armed for the next one.  Only a run of kMaxDfAborts
// consecutive aborts (a grid that cannot be resident, e.g. ranks sharing one GPU) turns it off for the
// handle.  Returns true if the solve aborted.
constexpr int kMaxDfAborts = 3;
bool dataflow_aborted(uno_kkt_t h) {
    uint32_t ab = 0;
    memcpy(&ab, h->h_counters + 10, sizeof(ab));
    if (ab == 0) {
        h->df_consec_aborts = 0;
        return false;
    }
    h->df_aborts++;
    if (++h->df_consec_aborts >= kMaxDfAborts) {
        h->df_enabled = 0;
        h->df_grid = 0;
    }
    memset(h->h_counters + 10, 0, 8);
    return true;
}

// Launch plan of the fronts selected by `take`: per level, fronts sorted by order (descending) cut
// into size classes -- factor: one kernel instance per LDS class; solve: one-wave kernels grouped by
// the LDS their packed panel needs, larger fronts in the 256-thread kernels.
template <class Pred>
hipError_t build_plan(uno_kkt_t h, Pred take, Plan& P) {
    const Symbolic& S = h->S;
    P.fac.clear();
    P.sol.clear();
    std::vector<int32_t> ffr, sfr;
    ffr.reserve(S.nf);
    sfr.reserve(S.nf);
    for (int l = 0; l < S.nlevels; ++l) {
        std::vector<int32_t> lv;
        for (int q = S.level_off[l]; q < S.level_off[l + 1]; ++q)
            if (take(S.level_fronts[q])) lv.push_back(S.level_fronts[q]);  // keeps the m-descending order
        if (lv.empty()) continue;
        {
            std::vector<std::pair<int, int32_t>> wv;  // (LDS doubles, front)
            std::vector<int32_t> big;
            for (int32_t f : lv) {
                const int m = S.f_m[f], p = S.f_p[f];
                if (p <= 64 && m <= kMaxLdsFront) {
                    const int sz = p * m - p * (p - 1) / 2;
                    wv.push_back({((sz + 1) & ~1) + ((m + 1) & ~1) + (m + 1) / 2, f});
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
                P.sol.push_back(sl);
                q = r;
            }
            if (!big.empty()) {
                SolveLaunch sl{l, (int)sfr.size(), (int)big.size(), 0, 0, 0, false};
                for (int32_t f : big) {
                    sfr.push_back(f);
                    sl.mmax = std::max(sl.mmax, S.f_m[f]);
                    sl.pmax = std::max(sl.pmax, S.f_p[f]);
                }
                P.sol.push_back(sl);
            }
        }
        const int base = (int)ffr.size();
        ffr.insert(ffr.end(), lv.begin(), lv.end());
        // factor launches: one per kernel instance and level (the launch reserves LDS for its largest
        // front).  Finer LDS classes ({16, 24, .., 128}) were measured slower on C3 (2.36 vs 1.99 ms):
        // the one-wave kernel is VALU-issue bound at levels 0-1 and more co-resident fronts per CU
        // only lengthen every front; a class smaller than kMinClass absorbs the next smaller one.
        static const std::vector<int> caps = [] {  // LDS size classes; UNO_KKT_CAPS: experiments
            std::vector<int> c{32, 64, kMaxWaveFront, 128};
            if (const char* e = getenv("UNO_KKT_CAPS")) {
                std::vector<int> v;
                for (const char* q = e; *q;) {
                    char* end = nullptr;
                    const long x = strtol(q, &end, 10);
                    if (end == q) break;
                    v.push_back((int)x);
                    q = *end ? end + 1 : end;
                }
                if (!v.empty()) c = v;
            }
            return c;
        }();
        constexpr int kMinClass = 2048;
        auto prev_cap = [](int c) {
            int pc = 0;
            for (int x : caps) if (x < c) pc = x;
            return pc;
        };
        auto kernel_of = [](int mm) {
            return mm > kMaxLdsFront ? 4 : (mm > kMaxWaveFront ? 3 : (mm > 64 ? 2 : (mm > 32 ? 1 : 0)));
        };
        const int e = (int)lv.size();
        int q = 0;
        while (q < e) {
            const int m0 = S.f_m[lv[q]];
            const bool global = m0 > kMaxLdsFront;
            int r = q;
            if (global) {
                while (r < e && S.f_m[lv[r]] > kMaxLdsFront) ++r;
            } else {
                int floor_ = 0;  // largest cap below m0 is the class floor
                for (int x : caps) if (x < m0) floor_ = x;
                while (true) {
                    while (r < e && S.f_m[lv[r]] > floor_) ++r;
                    if (r >= e || r - q >= kMinClass || floor_ == 0 || kernel_of(S.f_m[lv[r]]) != kernel_of(m0)) break;
                    floor_ = prev_cap(floor_);
                }
            }
            Launch L{base + q, r - q, m0, global, l};
            for (int t = q; t < r; ++t) {
                L.pmax = std::max(L.pmax, S.f_p[lv[t]]);
                L.maxch = std::max(L.maxch, S.f_child_off[lv[t] + 1] - S.f_child_off[lv[t]]);
            }
            P.fac.push_back(L);
            q = r;
        }
    }
    hipError_t e = P.fac_fronts.upload(ffr, h->stream);
    if (e == hipSuccess) e = P.sol_fronts.upload(sfr, h->stream);
    P.fac_host.swap(ffr);
    return e;
}

// Slow fronts first (option slow_first, default 1).  The level launches and the dataflow launch dispatch a
// level's fronts in their list order, and a level ends with its slowest front: a one-wave front whose pivots
// leave the register path (2x2 pivots, interchanges, null pivots: each such step spills the front to LDS) takes
// 5-10x the level's mean (C3: 160 us against 33 us at level 1), so a late start of one such front is the
// level's tail.  After the first factorization of a structure, the per-front count of those steps (fslow)
// reorders every launch's fronts and the dataflow order within each level, slowest first (ties keep the
// order by size); the values of later factorizations may move a few pivots, the order stays valid.
int reorder_slow_first(uno_kkt_t h) {
    const Symbolic& S = h->S;
    h->reorder_due = false;
    if (!h->slow_first || S.nf == 0 || !h->fslow.p) return UNO_KKT_OK;
    std::vector<int32_t> slow(S.nf);
    HIPCHK(h, hipMemcpy(slow.data(), h->fslow.p, sizeof(int32_t) * S.nf, hipMemcpyDeviceToHost));
    int64_t moved = 0;
    auto by_slow = [&](int32_t a, int32_t b) { return slow[a] > slow[b]; };
    for (Plan* P : {&h->plan[0], &h->plan[1], &h->dff_plan}) {
        if (P->fac_host.empty()) continue;
        if (P == &h->dff_plan && h->dff_level == INT32_MAX) continue;  // no dataflow factor: its plan is unused
        bool valid = true;
        for (int32_t f : P->fac_host) valid = valid && f >= 0 && f < S.nf;
        if (!valid) return set_err(h, UNO_KKT_ERR_HIP, "internal: launch list holds front ids of another structure");
        bool any = false;
        for (const Launch& L : P->fac) {
            if (L.global || L.count < 2) continue;  // large fronts keep their host-driven order
            auto b = P->fac_host.begin() + L.begin, e = b + L.count;
            bool has = false;
            for (auto it = b; it != e && !has; ++it) has = slow[*it] > 0;
            if (!has) continue;
            std::stable_sort(b, e, by_slow);
            any = true;
            moved++;
        }
        if (any) HIPCHK(h, P->fac_fronts.upload(P->fac_host, h->stream));
    }
    if (h->dff_level != INT32_MAX && !h->dff_order_host.empty()) {
        for (int32_t f : h->dff_order_host)
            if (f < 0 || f >= S.nf) return set_err(h, UNO_KKT_ERR_HIP, "internal: dataflow order of another structure");
        std::stable_sort(h->dff_order_host.begin(), h->dff_order_host.end(), [&](int32_t a, int32_t b) {
            if (S.f_level[a] != S.f_level[b]) return S.f_level[a] < S.f_level[b];  // children before parents
            return slow[a] > slow[b];
        });
        HIPCHK(h, h->dff_order.upload(h->dff_order_host, h->stream));
        moved++;
    }
    if (h->verbose) fprintf(stderr, "[uno_kkt] slow fronts first: %lld launch lists reordered\n", (long long)moved);
    return UNO_KKT_OK;
}

// Rank-local layout of a distributed factorization: subtree partition (identical on every rank),
// the rank's packed slot ranges, its own rows (complete row scans) and the partial scans of the top
// rows, whose per-rank partials are all-reduced.  See DESIGN.md section 6.
int setup_distribution(uno_kkt_t h) {
    const Symbolic& S = h->S;
    DistState& D = h->dist;
    hipStream_t s = h->stream;
    partition_tree(S, h->world, D.part);
    const Partition& Pt = D.part;
    auto mine = [&](int32_t f) { return Pt.owner[f] == h->rank || (h->rank == 0 && Pt.owner[f] < 0); };
    // packed slot ranges of every front this rank factors (consecutive fronts merged)
    D.pack_ranges.clear();
    D.my_flops = D.top_flops = 0.0;
    D.my_fronts = 0;
    for (int32_t f = 0; f < S.nf; ++f) {
        double fl = 0.0;
        for (int k = 0; k < S.f_p[f]; ++k) {
            const double r = S.f_m[f] - k - 1;
            fl += r + r * (r + 1.0);
        }
        if (Pt.owner[f] < 0) D.top_flops += fl;
        else if (Pt.owner[f] == h->rank) { D.my_flops += fl; D.my_fronts++; }
        if (!mine(f)) continue;
        const int64_t b = S.f_ent_off[f], e = S.f_ent_off[f + 1];
        if (b == e) continue;
        if (!D.pack_ranges.empty() && D.pack_ranges.back().second == b) D.pack_ranges.back().second = e;
        else D.pack_ranges.push_back({b, e});
    }
    // own rows (fully-summed columns of the rank's subtree fronts) and top rows
    std::vector<int32_t> own_new, own_orig, own_long, top_orig, top_new;
    std::vector<std::vector<int32_t>> per_rank(h->world);
    for (int32_t f = 0; f < S.nf; ++f) {
        const int64_t o = S.f_rows_off[f];
        for (int k = 0; k < S.f_p[f]; ++k) {
            const int32_t v = S.rows[o + k];
            if (Pt.owner[f] < 0) { top_orig.push_back(v); top_new.push_back(S.iperm[v]); }
            else per_rank[Pt.owner[f]].push_back(v);
        }
    }
    own_orig = per_rank[h->rank];
    for (int32_t v : own_orig) own_new.push_back(S.iperm[v]);
    D.max_own_long = 0;
    for (int32_t i : own_new) {
        const int64_t len = (S.cptr[i + 1] - S.cptr[i]) + (S.rptr[i + 1] - S.rptr[i]);
        if (len > kLongRow) { own_long.push_back(i); D.max_own_long = std::max(D.max_own_long, len); }
    }
    D.n_own = (int64_t)own_new.size();
    D.n_own_long = (int32_t)own_long.size();
    D.n_top_rows = (int64_t)top_orig.size();
    HIPCHK(h, D.own_new.upload(own_new, s));
    HIPCHK(h, D.own_orig.upload(own_orig, s));
    HIPCHK(h, D.own_long.upload(own_long, s));
    HIPCHK(h, D.top_orig.upload(top_orig, s));
    // partial scans of the top rows: this rank's slots of each top row, in chunks
    std::vector<int32_t> crow, pslot, ppart;
    std::vector<int64_t> cbeg, rchunk;
    auto slot_front = [&](int64_t q) {
        return (int32_t)(std::upper_bound(S.f_ent_off.begin(), S.f_ent_off.end(), q) - S.f_ent_off.begin() - 1);
    };
    for (int64_t t = 0; t < D.n_top_rows; ++t) {
        const int32_t i = top_new[t], o = top_orig[t];
        const size_t start = pslot.size();
        if (h->rank == 0)  // column part: slots of the top front eliminating i
            for (int32_t q = S.cptr[i]; q < S.cptr[i + 1]; ++q) { pslot.push_back(q); ppart.push_back(S.ent_r[q]); }
        for (int32_t t2 = S.rptr[i]; t2 < S.rptr[i + 1]; ++t2) {
            const int32_t q = S.rslot[t2];
            if (mine(slot_front(q))) { pslot.push_back(q); ppart.push_back(S.ent_c[q] == o ? S.ent_r[q] : S.ent_c[q]); }
        }
        rchunk.push_back((int64_t)crow.size());
        for (size_t b = start; b < pslot.size(); b += kLongChunk) { crow.push_back((int32_t)t); cbeg.push_back((int64_t)b); }
    }
    cbeg.push_back((int64_t)pslot.size());
    rchunk.push_back((int64_t)crow.size());
    D.nchunks = (int64_t)crow.size();
    HIPCHK(h, D.row_chunk.upload(rchunk, s));
    HIPCHK(h, D.chunk_part.alloc(std::max<int64_t>(D.nchunks, 1)));
    D.own_long_chunks = (D.max_own_long + kLongChunk - 1) / kLongChunk;
    HIPCHK(h, D.own_long_part.alloc(std::max<int64_t>((int64_t)D.n_own_long * D.own_long_chunks, 1)));
    HIPCHK(h, D.chunk_row.upload(crow, s));
    HIPCHK(h, D.chunk_begin.upload(cbeg, s));
    HIPCHK(h, D.pslot.upload(pslot, s));
    HIPCHK(h, D.ppartner.upload(ppart, s));
    HIPCHK(h, D.outT.alloc(std::max<int64_t>(D.n_top_rows, 1)));
    HIPCHK(h, D.tbuf.alloc(std::max<int64_t>(D.n_top_rows, 1)));
    // gather of the solution on rank 0
    D.own_count.assign(h->world, 0);
    for (int q = 0; q < h->world; ++q) D.own_count[q] = (int64_t)per_rank[q].size();
    if (h->rank == 0) {
        std::vector<int32_t> all;
        D.all_own_off.assign(h->world + 1, 0);
        for (int q = 0; q < h->world; ++q) {
            D.all_own_off[q + 1] = D.all_own_off[q] + (q == 0 ? 0 : D.own_count[q]);
            if (q > 0) all.insert(all.end(), per_rank[q].begin(), per_rank[q].end());
        }
        HIPCHK(h, D.all_own_orig.upload(all, s));
        HIPCHK(h, D.xbuf.alloc(std::max<int64_t>((int64_t)all.size(), 1)));
    } else {
        HIPCHK(h, D.xbuf.alloc(std::max<int64_t>(D.n_own, 1)));
    }
    return UNO_KKT_OK;
}

// Subtree roots whose parent is a top front: their blocks (contribution blocks after the factor,
// update vectors after the forward solve) go to rank 0 at the same offsets (same layout everywhere).
template <class Off, class Size>
int exchange_roots(uno_kkt_t h, double* base, Off off, Size size) {
    const Partition& Pt = h->dist.part;
    hipStream_t s = h->stream;
    HIPCHK(h, h->comm->group_begin());
    for (size_t k = 0; k < Pt.send_roots.size(); ++k) {
        const int32_t f = Pt.send_roots[k];
        const int src = Pt.root_rank[k];
        const int64_t n = size(f);
        if (src == 0 || n <= 0) continue;
        if (h->rank == src) HIPCHK(h, h->comm->send(base + off(f), (size_t)n * sizeof(double), 0, s));
        else if (h->rank == 0) HIPCHK(h, h->comm->recv(base + off(f), (size_t)n * sizeof(double), src, s));
    }
    HIPCHK(h, h->comm->group_end());
    return UNO_KKT_OK;
}

// Distributed equilibration: rows of the rank's subtrees are complete on the rank (every entry of such
// a row lies in one of its fronts) and are scanned as on one GPU; the top rows' partials from every
// rank are combined with all-reduces (max for the scaling sweeps, sum for the row sums), and
// ||A_pre||_inf is the all-reduced max.  Same values as the single-GPU scan (max is exact; the
// row-sum additions of a top row are regrouped by rank).
int dist_scale(uno_kkt_t h, ScanArgs SA) {
    DistState& D = h->dist;
    hipStream_t s = h->stream;
    SA.list = D.own_new.p;
    SA.n = D.n_own;
    SA.long_rows = D.own_long.p;
    SA.n_long = D.n_own_long;
    SA.max_long = D.max_own_long;
    SA.long_chunks = D.own_long_chunks;
    SA.part = D.own_long_part.p;
    PartArgs PA;
    PA.nchunks = D.nchunks; PA.chunk_row = D.chunk_row.p; PA.chunk_begin = D.chunk_begin.p; PA.pslot = D.pslot.p;
    PA.ppartner = D.ppartner.p; PA.trow_orig = D.top_orig.p; PA.uval = h->uval.p; PA.scale = h->scale.p;
    PA.outT = D.outT.p;
    PA.nrows = D.n_top_rows; PA.row_chunk = D.row_chunk.p; PA.part = D.chunk_part.p;
    const int64_t nt = D.n_top_rows;
    auto top_pass = [&](int mode, double* out, RedOp op) -> int {
        if (nt == 0) return UNO_KKT_OK;
        HIPCHK(h, launch_rowscan_part(PA, mode, s));
        HIPCHK(h, h->comm->allreduce(D.outT.p, (size_t)nt, op, s));
        HIPCHK(h, launch_scatter(D.outT.p, D.top_orig.p, out, nt, s));
        return UNO_KKT_OK;
    };
    int rc;
    for (int it = 0; it < h->scale_iters; ++it) {
        SA.out = h->rmax.p;
        HIPCHK(h, launch_rowscan(SA, it == 0 ? 0 : 1, s));
        if ((rc = top_pass(it == 0 ? 0 : 1, h->rmax.p, RedOp::MaxF64)) != UNO_KKT_OK) return rc;
        HIPCHK(h, launch_scale_update(h->rmax.p, h->scale.p, D.own_orig.p, D.n_own, it == 0, s));
        HIPCHK(h, launch_scale_update(h->rmax.p, h->scale.p, D.top_orig.p, nt, it == 0, s));
    }
    if (h->scale_iters == 0) {
        HIPCHK(h, hipMemsetAsync(h->rmax.p, 0, sizeof(double) * h->S.n, s));
        HIPCHK(h, launch_scale_update(h->rmax.p, h->scale.p, nullptr, h->S.n, 1, s));
    }
    SA.out = h->rowsum.p;
    HIPCHK(h, launch_rowscan(SA, 2, s));
    if ((rc = top_pass(2, h->rowsum.p, RedOp::SumF64)) != UNO_KKT_OK) return rc;
    HIPCHK(h, launch_normmax(h->rowsum.p, D.own_orig.p, D.n_own, h->anorm_p, s));
    HIPCHK(h, launch_normmax(h->rowsum.p, D.top_orig.p, nt, h->anorm_p, s));
    HIPCHK(h, h->comm->allreduce(h->anorm_p, 1, RedOp::MaxU64, s));
    return UNO_KKT_OK;
}

// host-side all-reduce of a small vector (delayed-pivot rounds only)
int allreduce_host(uno_kkt_t h, std::vector<unsigned long long>& v, RedOp op) {
    if (h->world <= 1 || v.empty()) return UNO_KKT_OK;
    HIPCHK(h, h->dist.tmp.alloc(v.size()));
    HIPCHK(h, hipMemcpyAsync(h->dist.tmp.p, v.data(), v.size() * 8, hipMemcpyHostToDevice, h->stream));
    HIPCHK(h, h->comm->allreduce(h->dist.tmp.p, v.size(), op, h->stream));
    HIPCHK(h, hipMemcpyAsync(v.data(), h->dist.tmp.p, v.size() * 8, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return UNO_KKT_OK;
}


// wait for the factorization; if it ran with the overlapped norm (threshold 0), check that no
// accepted pivot is at or below the exact null-pivot threshold, else refactor with the exact one
// Host wait for an event.  Option "spin_wait" (default 1) polls it: hipEventSynchronize falls back to an
// interrupt wait once the GPU has run for a while, and its wake-up adds tens of microseconds to every
// factorization and solve (measured r03, tools/timeline.py)
hipError_t host_wait(uno_kkt_t h, hipEvent_t ev) {
    if (!h->spin_wait) return hipEventSynchronize(ev);
    for (;;) {
        const hipError_t e = hipEventQuery(ev);
        if (e != hipErrorNotReady) return e;
        __builtin_ia32_pause();
    }
}

hipError_t host_wait_stream(uno_kkt_t h, hipStream_t s) {
    if (!h->spin_wait) return hipStreamSynchronize(s);
    const hipError_t e = hipEventRecord(h->ev_wait, s);
    return e != hipSuccess ? e : host_wait(h, h->ev_wait);
}

// Host wait for k_count's sequence number in the page-locked block (slot 10, written after the counters with
// system-scope stores): a device error or a stream that finished without it ends the wait
hipError_t host_wait_flag(uno_kkt_t h, unsigned long long seq) {
    volatile unsigned long long* flag = h->h_counters + 10;
    for (unsigned it = 1;; ++it) {
        if (*flag == seq) break;
        if ((it & 255) == 0) {
            const hipError_t e = hipStreamQuery(h->stream);
            if (e == hipSuccess) {
                if (*flag == seq) break;
                return hipErrorUnknown;  // the stream is done and the flag never came
            }
            if (e != hipErrorNotReady) return e;
        }
        __builtin_ia32_pause();
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    return hipSuccess;
}

int sync_and_verify(uno_kkt_t h) {
    // the counters (and the dataflow abort word) are on the host
    if (h->wait_seq) HIPCHK(h, host_wait_flag(h, h->wait_seq));
    else HIPCHK(h, host_wait(h, h->ev_counters));
    uint32_t ab = 0;
    memcpy(&ab, h->h_counters + 11, sizeof(ab));
    if (ab != 0) {
        // a dependency wait of the dataflow factorization hit its limit: the factorization is invalid;
        // level-scheduled launches from now on, and this one is redone
        h->dff_aborts++;
        h->dff_enabled = 0;
        h->dff_level = INT32_MAX;
        memset(h->h_counters + 11, 0, 8);
        HIPCHK(h, hipMemsetAsync(h->df_abort.p, 0, sizeof(uint32_t), h->stream));
        if (h->verbose) fprintf(stderr, "[uno_kkt] dataflow factorization aborted: refactoring level by level\n");
        int rc = enqueue_factorization(h);
        if (rc != UNO_KKT_OK) return rc;
        HIPCHK(h, hipStreamSynchronize(h->stream));
    }
    if (h->last_optimistic) {
        double anorm, mp;
        memcpy(&mp, h->h_counters + 8, 8);
        const double bound = DBL_EPSILON * h->null_fac * (double)h->max_row_len * (1.0 + 1e-9);
        if (mp > bound && h->scale_iters > 0) {  // no pivot near any possible threshold: exact as it stands
            h->norm_skips++;
            flush_timing(h);
            return UNO_KKT_OK;
        }
        {
            TimerScope t2(h, KC_ROWSUM);
            if (h->use_front_sweeps) HIPCHK(h, launch_rowsum_norm_orig(h->scan, h->rowsum.p, h->stream));
            else HIPCHK(h, launch_rowsum_norm(h->scan, h->rowsum.p, h->stream));
        }
        HIPCHK(h, hipMemcpyAsync(h->h_counters + 9, h->anorm_p, 8, hipMemcpyDeviceToHost, h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
        h->norm_valid = true;
        memcpy(&anorm, h->h_counters + 9, 8);
        const double thres = DBL_EPSILON * h->null_fac * anorm;
        if (!(mp > thres)) {
            h->exact_next = true;
            int rc = enqueue_factorization(h);
            h->exact_next = false;
            if (rc != UNO_KKT_OK) return rc;
            HIPCHK(h, hipStreamSynchronize(h->stream));
            h->exact_redos++;
            if (h->verbose) fprintf(stderr, "[uno_kkt] pivot %.3e <= null threshold %.3e: refactored exactly\n", mp, thres);
        }
    }
    flush_timing(h);
    return UNO_KKT_OK;
}

int finish_factorization(uno_kkt_t h) {
    if (!h->factor_enqueued) return h->factored ? UNO_KKT_OK : set_err(h, UNO_KKT_ERR_STATE, "no factorization");
    {
        int rc = sync_and_verify(h);
        if (rc != UNO_KKT_OK) return rc;
    }
    h->factor_enqueued = false;
    // delayed pivots: a front that could not pivot a fully-summed column (or, optionally, needed a
    // relaxed threshold) is amalgamated into its parent and the factorization is redone.  The merge
    // is sticky for later factorizations of the same pattern.
    for (int round = 0; round < h->max_merge_rounds; ++round) {
        const unsigned long long* c = h->h_counters;
        int64_t nd = (int64_t)std::min<unsigned long long>(c[6], (unsigned long long)h->S.n);
        bool need = c[5] != 0 || (h->delay_relaxed && nd > 0);
        if (!need) break;
        std::vector<int32_t> dv;
        if (h->world == 1) {
            dv.resize(nd);
            if (nd > 0) HIPCHK(h, hipMemcpy(dv.data(), h->delayed.p, sizeof(int32_t) * nd, hipMemcpyDeviceToHost));
        } else {
            // every rank applies the union of all ranks' delayed columns (same structure everywhere)
            std::vector<unsigned long long> cnt(h->world, 0);
            cnt[h->rank] = std::min<unsigned long long>(c[7], (unsigned long long)h->S.n);
            int rc = allreduce_host(h, cnt, RedOp::SumU64);
            if (rc != UNO_KKT_OK) return rc;
            int64_t total = 0, mine_off = 0;
            for (int q = 0; q < h->world; ++q) { if (q == h->rank) mine_off = total; total += (int64_t)cnt[q]; }
            std::vector<int32_t> my((size_t)cnt[h->rank]);
            if (!my.empty()) HIPCHK(h, hipMemcpy(my.data(), h->delayed.p, sizeof(int32_t) * my.size(), hipMemcpyDeviceToHost));
            std::vector<unsigned long long> all((size_t)total, 0);
            for (size_t q = 0; q < my.size(); ++q) all[mine_off + q] = (unsigned long long)my[q];
            if ((rc = allreduce_host(h, all, RedOp::SumU64)) != UNO_KKT_OK) return rc;
            for (unsigned long long v : all) dv.push_back((int32_t)v);
        }
        std::sort(dv.begin(), dv.end());  // deterministic merge order
        int64_t moved = delay_columns(h->P, h->S, dv);
        if (moved == 0) {
            // fall back to whole-front amalgamation for stuck fronts (cannot happen at roots)
            std::vector<int32_t> fs(h->S.nf);
            if (h->S.nf > 0) HIPCHK(h, hipMemcpy(fs.data(), h->fstat.p, sizeof(int32_t) * fs.size(), hipMemcpyDeviceToHost));
            std::vector<unsigned long long> stuck(h->S.nf);
            for (int64_t f = 0; f < h->S.nf; ++f) stuck[f] = (fs[f] & 0xffff) != 0;
            int rc = allreduce_host(h, stuck, RedOp::MaxU64);
            if (rc != UNO_KKT_OK) return rc;
            std::vector<char> merge(h->S.nf, 0);
            for (int64_t f = 0; f < h->S.nf; ++f) merge[f] = stuck[f] != 0;
            moved = amalgamate(h->P, h->S, merge);
        }
        if (moved == 0) break;
        h->merges_total += moved;
        auto tb = std::chrono::steady_clock::now();
        std::string msg = build_structure(h->P, h->S);
        if (!msg.empty()) return set_err(h, UNO_KKT_ERR_ARG, msg);
        int rc = upload_structure(h);
        if (rc != UNO_KKT_OK) return rc;
        auto tu = std::chrono::steady_clock::now();
        rc = enqueue_factorization(h);
        if (rc != UNO_KKT_OK) return rc;
        if ((rc = sync_and_verify(h)) != UNO_KKT_OK) return rc;
        h->factor_enqueued = false;
        if (h->verbose)
            fprintf(stderr, "[uno_kkt] merge round %d: %lld delayed columns listed, %lld moved, stuck %llu; "
                            "rebuild %.3f s, upload %.3f s, refactor %.3f s, fronts %lld, max front %lld\n", round, (long long)dv.size(),
                    (long long)moved, (unsigned long long)c[5],
                    std::chrono::duration<double>(tu - tb).count() - 0.0,
                    0.0, std::chrono::duration<double>(std::chrono::steady_clock::now() - tu).count(), (long long)h->S.nf,
                    (long long)h->S.max_m);
    }
    const unsigned long long* c = h->h_counters;
    if (h->verbose >= 2)
        fprintf(stderr, "[uno_kkt] factorization %lld: %.3f ms (enqueue to checked), inertia (%llu, %llu, %llu), merges %lld\n",
                (long long)h->st.factorizations,
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - h->t_factor).count(), c[0], c[1],
                c[2], (long long)h->merges_total);
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
    if (h->reorder_due) return reorder_slow_first(h);
    return UNO_KKT_OK;
}

// Dataflow solve layout: topological front order (the level order), 128-byte-aligned per-front slots
// for the forward update vectors and the backward solution values, arrival counters.
hipError_t setup_factor_dataflow(uno_kkt_t h) {
    const Symbolic& S = h->S;
    h->dff_level = INT32_MAX;
    h->dff_epoch = 0;
    // a plan or order of an earlier structure must not survive an early return (reorder_slow_first walks them)
    h->dff_plan.fac.clear();
    h->dff_plan.fac_host.clear();
    h->dff_plan.sol.clear();
    h->dff_order_host.clear();
    if (!h->dff_enabled || S.nf == 0) return hipSuccess;
    // the fronts of plan[0]: all fronts on one GPU, the rank's own subtrees in a distributed run (the
    // top fronts are factored after the root exchange by the level launches of plan[1])
    auto mine = [&](int32_t f) { return h->world == 1 || h->dist.part.owner[f] == h->rank; };
    // lowest level from which every own front fits the one-wave register kernel (m <= 64)
    int L = S.nlevels;
    while (L > 0) {
        bool ok = true;
        for (int q = S.level_off[L - 1]; q < S.level_off[L] && ok; ++q)
            ok = !mine(S.level_fronts[q]) || S.f_m[S.level_fronts[q]] <= 64;
        if (!ok) break;
        --L;
    }
    if (L >= S.nlevels) return hipSuccess;
    // the set grows downwards (option 2, default): every own front of order <= M (M = largest order at
    // levels >= L, so the launch keeps that LDS size) whose ancestors are all <= M; the rest (downward
    // closed: a front above M makes its whole subtree "low") runs in level launches before
    int M = 1;
    for (int q = S.level_off[L]; q < S.level_off[S.nlevels]; ++q)
        if (mine(S.level_fronts[q])) M = std::max(M, S.f_m[S.level_fronts[q]]);
    std::vector<char> in(S.nf, 0);
    for (int l = S.nlevels - 1; l >= 0; --l) {
        for (int q = S.level_off[l]; q < S.level_off[l + 1]; ++q) {
            const int32_t f = S.level_fronts[q];
            if (!mine(f)) continue;
            const int32_t par = S.f_parent[f];
            const bool parent_ok = par < 0 || !mine(par) || in[par];
            in[f] = l >= L || (h->dff_enabled >= 2 && parent_ok && S.f_m[f] <= M);
        }
    }
    std::vector<int32_t> order;
    for (int q = 0; q < S.level_off[S.nlevels]; ++q)
        if (in[S.level_fronts[q]]) order.push_back(S.level_fronts[q]);
    if (order.empty()) return hipSuccess;
    std::vector<int32_t> nch(S.nf, 0);
    int mmax = 1;
    for (int32_t f : order) {
        mmax = std::max(mmax, S.f_m[f]);
        for (int q = S.f_child_off[f]; q < S.f_child_off[f + 1]; ++q) nch[f] += in[S.child[q]];
    }
    // level launches of the other own fronts (downward closed: all their descendants are among them)
    if (hipError_t e = build_plan(h, [&](int32_t f) { return mine(f) && !in[f]; }, h->dff_plan); e != hipSuccess)
        return e;
    hipStream_t s = h->stream;
    hipError_t e;
    if ((e = h->dff_order.upload(order, s)) != hipSuccess) return e;
    h->dff_order_host = order;
    if ((e = h->dff_nch.upload(nch, s)) != hipSuccess) return e;
    if ((e = h->dff_cnt.alloc(S.nf)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(h->dff_cnt.p, 0, sizeof(uint32_t) * S.nf, s)) != hipSuccess) return e;
    if (!h->dff_ticket.p && (e = h->dff_ticket.alloc(1)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(h->dff_ticket.p, 0, sizeof(uint32_t), s)) != hipSuccess) return e;
    if (!h->df_abort.p && (e = h->df_abort.alloc(1)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(h->df_abort.p, 0, sizeof(uint32_t), s)) != hipSuccess) return e;
    h->dff_mmax = mmax;
    h->dff_level = L;
    if (h->verbose)
        fprintf(stderr, "[uno_kkt] dataflow factorization: %zu fronts (levels >= %d and fronts <= %d rows below them), "
                        "%d level launches before\n", order.size(), L, M, (int)h->dff_plan.fac.size());
    return hipSuccess;
}

// the register kernels' launch: resident blocks (occupancy), the last ov_grid of them walk the oversized fronts
void set_rg_grids(uno_kkt_t h) {
    h->ov_grid = std::min(h->ov_nf, 32);
    for (int d = 0; d < 2; ++d) {
        const int resident = solve_rg_grid(d == 0, 1 << 30, h->rg_wpe);
        const int nwalk = d == 0 ? h->rgf_nf : h->rg_nf;  // the forward walk leaves its leaves to k_solve_fwd_leaf
        int g = std::min(resident, nwalk + h->ov_grid);
        if (resident <= h->ov_grid || (nwalk > 0 && g - h->ov_grid < 1)) g = 0;  // no room: df kernels
        (d == 0 ? h->rg_grid_f : h->rg_grid_b) = g;
    }
}

hipError_t setup_dataflow(uno_kkt_t h) {
    const Symbolic& S = h->S;
    h->new_bwd = h->solve_rg_bwd != 0;
    h->df_grid = 0;
    h->df_rx_valid = false;
    h->df_epoch = 0;
    h->df_nwalk = 0;
    const bool dist = h->world > 1;
    const bool dist_want = h->dist_df >= 0 ? h->dist_df != 0 : h->own_device;
    if (!h->df_enabled || S.nf == 0 || (dist && !dist_want)) return hipSuccess;
    std::vector<int32_t> walk;  // children before parents (level order)
    walk.reserve(S.nf);
    for (int32_t f : S.level_fronts)
        if (!dist || h->dist.part.owner[f] == h->rank) walk.push_back(f);
    if (walk.empty()) return hipSuccess;
    // every front of the walk is one-wave eligible; inside it, fronts beyond the register class (p <= 32,
    // m <= 72) go to the register kernels' second walk (ov_desc, LDS-panel path) -- the split below
    int max_sz = 0, mmax = 0;
    for (int32_t f : walk) {
        const int m = S.f_m[f], p = S.f_p[f];
        if (p > 64 || m > kMaxLdsFront) {  // a front needs the 256-thread kernels
            if (h->verbose) fprintf(stderr, "[uno_kkt] dataflow solve off: front %lld m %d p %d\n", (long long)f, m, p);
            return hipSuccess;
        }
        max_sz = std::max(max_sz, p * m - p * (p - 1) / 2);
        mmax = std::max(mmax, m);
    }
    // panel window: sized so that 16 one-wave blocks (4 per SIMD, the register limit of the dataflow
    // kernels) fit the 160 KB LDS of a CU; larger panels are processed in column windows
    const int rows_lds = ((mmax + 1) & ~1) + (mmax + 1) / 2;
    int win = h->df_win_opt > 0 ? h->df_win_opt : (160 * 1024 / 16 - 16) / 8 - solve_slack_doubles() - rows_lds - 32;
    win = std::max(win, mmax + 1) & ~1;
    win = std::min(win, (max_sz + 1) & ~1);
    win = std::max(win, 2);
    h->df_win = win;
    h->df_piv_off = win + rows_lds;
    const int lds = win + rows_lds + 32;  // + 64 pivot-kind words
    std::vector<int64_t> cvx(S.nf), xs(S.nf), chx(S.child.size());
    int64_t tc = 0, tx = 0;
    for (int64_t f = 0; f < S.nf; ++f) {
        cvx[f] = tc;
        tc += (S.f_m[f] - S.f_p[f] + 15) & ~15;
        xs[f] = tx;
        tx += (S.f_p[f] + 15) & ~15;
    }
    h->df_top_base = tx;
    if (dist) tx += (h->dist.n_top_rows + 15) & ~15;
    if (tx >= INT32_MAX) return hipSuccess;
    for (size_t q = 0; q < S.child.size(); ++q) chx[q] = cvx[S.child[q]];
    hipStream_t s = h->stream;
    hipError_t e;
    if ((e = h->df_order.upload(walk, s)) != hipSuccess) return e;
    if (dist) {
        const Partition& Pt = h->dist.part;
        std::vector<int32_t> roots, topf;
        for (int32_t f = 0; f < (int32_t)S.nf; ++f) {
            if (Pt.owner[f] < 0) topf.push_back(f);
            else if (Pt.owner[f] == h->rank && S.f_parent[f] >= 0 && Pt.owner[S.f_parent[f]] < 0) roots.push_back(f);
        }
        h->n_df_roots = (int32_t)roots.size();
        h->n_df_topf = (int32_t)topf.size();
        if (!roots.empty() && (e = h->df_roots.upload(roots, s)) != hipSuccess) return e;
        if (!topf.empty() && (e = h->df_topf.upload(topf, s)) != hipSuccess) return e;
    }
    {
        std::vector<int32_t> desc(walk.size() * 16, 0);
        auto put64 = [&](int32_t* d, int64_t v) { d[0] = (int32_t)(uint32_t)v; d[1] = (int32_t)(uint32_t)((uint64_t)v >> 32); };
        // the bottom solve_flat levels of the register class go to k_solve_fwd_flat (one flat launch per level
        // before the forward walk): a front is flat when its level is < solve_flat, it fits the register kernels
        // and all its children are flat -- unless the walk would then be empty (tiny systems); kDescNW counts the
        // children a walk front waits for
        std::vector<char> leaf(S.nf, 0);  // flat
        int64_t nleaf = 0, nrg = 0;
        for (int32_t f : walk) {  // children before parents
            const bool rg = S.f_p[f] <= 32 && S.f_m[f] <= 72;
            nrg += rg;
            bool ok = rg && S.f_level[f] < h->solve_flat;
            for (int q = S.f_child_off[f]; q < S.f_child_off[f + 1] && ok; ++q) ok = leaf[S.child[q]] != 0;
            if (ok) { leaf[f] = 1; ++nleaf; }
        }
        if (nleaf == nrg) std::fill(leaf.begin(), leaf.end(), 0);
        for (size_t t = 0; t < walk.size(); ++t) {
            const int32_t f = walk[t];
            int32_t* d = desc.data() + 16 * t;
            d[kDescF] = f; d[kDescM] = S.f_m[f]; d[kDescP] = S.f_p[f]; d[kDescPar] = S.f_parent[f];
            d[kDescC0] = S.f_child_off[f]; d[kDescC1] = S.f_child_off[f + 1];
            int nw = 0;
            for (int q = S.f_child_off[f]; q < S.f_child_off[f + 1]; ++q) nw += !leaf[S.child[q]];
            d[kDescNW] = nw;
            put64(d + kDescRo, S.f_rows_off[f]); put64(d + kDescLo, S.f_L_off[f]);
            put64(d + kDescCvx, cvx[f]); put64(d + kDescXs, xs[f]);
        }
        if ((e = h->df_desc.upload(desc, s)) != hipSuccess) return e;
        std::vector<int32_t> bwd;  // filled below with the flat set (the backward walk without the flat levels)
        // the register kernels' two walks (same order): p <= 32, m <= 72 fronts, and the rest
        std::vector<int32_t> rgd, ovd;
        for (size_t t = 0; t < walk.size(); ++t) {
            const int32_t f = walk[t];
            auto& dst = (S.f_p[f] <= 32 && S.f_m[f] <= 72) ? rgd : ovd;
            dst.insert(dst.end(), desc.begin() + 16 * t, desc.begin() + 16 * (t + 1));
        }
        std::vector<int32_t> rgf, lfd;  // the forward register walk without the flat levels, and those by level
        h->flat_off.assign(1, 0);
        for (int lev = 0; lev < h->solve_flat; ++lev) {
            for (size_t t = 0; t < rgd.size() / 16; ++t) {
                const int32_t f = rgd[16 * t + kDescF];
                if (leaf[f] && S.f_level[f] == lev) lfd.insert(lfd.end(), rgd.begin() + 16 * t, rgd.begin() + 16 * (t + 1));
            }
            h->flat_off.push_back((int32_t)(lfd.size() / 16));
        }
        for (size_t t = 0; t < rgd.size() / 16; ++t)
            if (!leaf[rgd[16 * t + kDescF]]) rgf.insert(rgf.end(), rgd.begin() + 16 * t, rgd.begin() + 16 * (t + 1));
        h->rg_nf = (int32_t)(rgd.size() / 16);
        h->ov_nf = (int32_t)(ovd.size() / 16);
        h->rgf_nf = (int32_t)(rgf.size() / 16);
        if (rgd.empty()) rgd.assign(16, 0);
        if (ovd.empty()) ovd.assign(16, 0);
        if (rgf.empty()) rgf.assign(16, 0);
        if (lfd.empty()) lfd.assign(16, 0);
        if ((e = h->rg_desc.upload(rgd, s)) != hipSuccess) return e;
        if ((e = h->ov_desc.upload(ovd, s)) != hipSuccess) return e;
        if ((e = h->rgf_desc.upload(rgf, s)) != hipSuccess) return e;
        if ((e = h->flat_desc.upload(lfd, s)) != hipSuccess) return e;
        for (size_t t = 0; t < desc.size() / 16; ++t)
            if (!leaf[desc[16 * t + kDescF]]) bwd.insert(bwd.end(), desc.begin() + 16 * t, desc.begin() + 16 * (t + 1));
        h->bwd_nf = (int32_t)(bwd.size() / 16);
        if (bwd.empty()) bwd.assign(16, 0);
        if ((e = h->bwd_desc.upload(bwd, s)) != hipSuccess) return e;
    }
    if ((e = h->df_cvx_off.upload(cvx, s)) != hipSuccess) return e;
    if ((e = h->df_ch_cvx_off.upload(chx, s)) != hipSuccess) return e;
    if ((e = h->df_xs_off.upload(xs, s)) != hipSuccess) return e;
    if ((e = h->df_cvx.alloc(std::max<int64_t>(tc, 16))) != hipSuccess) return e;
    if ((e = h->df_xs.alloc(std::max<int64_t>(tx, 16))) != hipSuccess) return e;
    if ((e = h->df_xpos.alloc(std::max<int64_t>(S.n, 1))) != hipSuccess) return e;
    if ((e = h->df_rxpos.alloc(std::max<size_t>(S.rows.size(), 1))) != hipSuccess) return e;
    {
        std::vector<int32_t> rowx(std::max<size_t>(S.rows.size(), 1), -1);
        for (int32_t f : walk) {
            const int64_t ro = S.f_rows_off[f];
            for (int i = 0; i < S.f_m[f]; ++i) rowx[ro + i] = i < S.f_p[f] ? (int32_t)(xs[f] + i) : -2;
        }
        if ((e = h->df_rowx.upload(rowx, s)) != hipSuccess) return e;
    }
    if ((e = h->df_cnt.alloc(S.nf)) != hipSuccess) return e;
    if ((e = h->df_done.alloc(S.nf)) != hipSuccess) return e;
    if (!h->df_abort.p && (e = h->df_abort.alloc(1)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(h->df_cnt.p, 0, sizeof(uint32_t) * S.nf, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(h->df_done.p, 0, sizeof(uint32_t) * S.nf, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(h->df_abort.p, 0, sizeof(uint32_t), s)) != hipSuccess) return e;
    h->df_lds = lds;
    h->df_nwalk = (int32_t)walk.size();
    h->df_grid = solve_df_grid(lds, h->df_nwalk);
    set_rg_grids(h);
    if (h->verbose)
        fprintf(stderr, "[uno_kkt] dataflow solve: %d of %lld fronts, panel window %d of %d doubles, lds %d doubles, grid %d\n",
                h->df_nwalk, (long long)S.nf, win, max_sz, lds, h->df_grid);
    return hipSuccess;
}

int upload_structure(uno_kkt_t h) {
    Symbolic& S = h->S;
    if (S.max_m > kMaxGlobalFront)
        return set_err(h, UNO_KKT_ERR_ARG, "front of order " + std::to_string(S.max_m) + " exceeds " +
                                               std::to_string(kMaxGlobalFront));
    const int64_t n = S.n;
    // global scratch for fronts too large for LDS
    std::vector<int64_t> goff(S.nf + 1, 0);
    int64_t gtot = 0;
    for (int64_t f = 0; f < S.nf; ++f) {
        // element -1 of every global front is its own trash slot (masked-off lanes of the assembly
        // read-add-write it; a slot shared with the previous front would race with that front)
        if (S.f_m[f] > kMaxLdsFront) {
            gtot += 8;
            goff[f] = gtot;
            // the front, then the a-posteriori step's panel (m x kAppNB) and its AppSlot
            gtot += (int64_t)S.f_m[f] * S.f_m[f] + (int64_t)S.f_m[f] * kAppNB + kAppSlotDoubles;
        } else {
            goff[f] = gtot;
        }
    }
    gtot += 8;
    hipStream_t s = h->stream;
    HIPCHK(h, S.identity_dups ? (h->dup_ptr.release(), hipSuccess) : h->dup_ptr.upload(S.dup_ptr, s));
    HIPCHK(h, h->dup_pos.upload(S.dup_pos, s));
    if (S.identity_dups) {
        h->slot_src.release();
    } else {
        // multi_slots: per slot with several COO positions {slot, p0, p1, p2} (-1 padded), or {slot, -2 - q0,
        // count, 0} (dup_pos[q0 ..]) for more than three
        std::vector<int32_t> src((size_t)S.nu), multi;
        for (int64_t e = 0; e < S.nu; ++e) {
            const int32_t q0 = S.dup_ptr[e], cnt = S.dup_ptr[e + 1] - q0;
            src[e] = cnt == 1 ? S.dup_pos[q0] : -1 - (int32_t)(multi.size() / 4);  // < 0: its multi record
            if (cnt == 1) continue;
            multi.push_back((int32_t)e);
            if (cnt <= 3) {
                for (int t = 0; t < 3; ++t) multi.push_back(t < cnt ? S.dup_pos[q0 + t] : -1);
            } else {
                multi.push_back(-2 - q0);
                multi.push_back(cnt);
                multi.push_back(0);
            }
        }
        HIPCHK(h, h->slot_src.upload(src, s));
        HIPCHK(h, h->multi_slots.upload(multi, s));
        h->n_multi = (int64_t)multi.size() / 4;
    }
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
    {  // cbpos: each contribution-block entry's packed position i (i + 1) / 2 + j in its parent's LDS front
        h->use_cbpos = false;
        if (h->cbpos_opt && S.cb_size > 0 && S.cb_size < INT32_MAX) {
            std::vector<uint16_t> cp((size_t)S.cb_size, 0);
            bool ok = true;
            for (int64_t c = 0; c < S.nf && ok; ++c) {
                const int32_t par = S.f_parent[c];
                if (par < 0 || S.f_m[par] > kMaxLdsFront) continue;  // roots; large parents use k_big_child
                const int cm = S.f_m[c] - S.f_p[c];
                const int32_t* rm = S.relmap.data() + S.f_relmap_off[c];
                int64_t t = S.f_cb_off[c];
                for (int r = 0; r < cm; ++r) {
                    const int64_t i = rm[r], base = i * (i + 1) / 2;
                    if (base + i >= 65536) { ok = false; break; }
                    for (int q = 0; q <= r; ++q) cp[t++] = (uint16_t)(base + rm[q]);
                }
            }
            if (ok) {
                HIPCHK(h, h->cbpos.upload(cp, s));
                HIPCHK(h, hipStreamSynchronize(s));
                h->use_cbpos = true;
            }
        }
    }
    HIPCHK(h, h->gscratch_off.upload(goff, s));
    HIPCHK(h, h->fstat.alloc(S.nf));
    HIPCHK(h, h->fcnt.alloc(S.nf));
    HIPCHK(h, h->fslow.alloc(S.nf));
    h->reorder_due = true;
    h->rz_state = 0;
    HIPCHK(h, h->fmin.alloc(S.nf));
    if (S.nf > 0) HIPCHK(h, hipMemsetAsync(h->fmin.p, 0x7f, sizeof(double) * S.nf, s));  // 1.4e306: above any threshold
    HIPCHK(h, h->perm_d.upload(S.perm, s));
    HIPCHK(h, h->cptr.upload(S.cptr, s));
    HIPCHK(h, h->rptr.upload(S.rptr, s));
    HIPCHK(h, h->rslot.upload(S.rslot, s));
    h->use_front_sweeps = h->world == 1 && h->front_sweeps && S.max_m <= kMaxSweepFront;
    {
        std::vector<int32_t> big;
        int64_t most = 0;
        for (int32_t f = 0; f < (int32_t)S.nf; ++f) {
            const int64_t ns = S.f_ent_off[f + 1] - S.f_ent_off[f];
            if (ns > kSweepBigSlots) { big.push_back(f); most = std::max(most, ns); }
        }
        h->n_sweep_big = (int32_t)big.size();
        h->sweep_slices = (int32_t)std::min<int64_t>(256, (most + kSweepBigSlots - 1) / kSweepBigSlots);
        if (!big.empty()) HIPCHK(h, h->sweep_big.upload(big, s));
    }
    if (h->world == 1 && !h->use_front_sweeps) {
        HIPCHK(h, h->rowpartner.upload(S.rowpartner, s));
        HIPCHK(h, h->uvalR.alloc(S.rowpartner.size()));
    }
    HIPCHK(h, h->fparent.upload(S.f_parent, s));
    {
        std::vector<int32_t> lr;
        h->max_long = 0;
        h->max_row_len = 0;
        for (int64_t i = 0; i < n; ++i) {
            int64_t len = (S.cptr[i + 1] - S.cptr[i]) + (S.rptr[i + 1] - S.rptr[i]);
            h->max_row_len = std::max(h->max_row_len, len);
            if (len > kLongRow) { lr.push_back((int32_t)i); h->max_long = std::max(h->max_long, len); }
        }
        h->n_long = (int32_t)lr.size();
        HIPCHK(h, h->long_rows.upload(lr, s));
        if (h->use_front_sweeps) {
            std::vector<int8_t> lp((size_t)std::max<int64_t>(n, 1), (int8_t)-1);
            std::vector<int32_t> lo(lr.size());
            for (size_t k = 0; k < lr.size(); ++k) {
                lo[k] = S.perm[lr[k]];
                lp[lo[k]] = (int8_t)k;
            }
            if (lr.size() > 127) h->use_front_sweeps = false;  // int8 index
            HIPCHK(h, h->longpos.upload(lp, s));
            HIPCHK(h, h->long_orig.upload(lo, s));
            {  // the sweeps index rows in the elimination order (a front's rows are then clustered: the
               // scaling gathers and row-maximum atomics touch fewer cache lines than by original id)
                std::vector<int8_t> lpn((size_t)std::max<int64_t>(n, 1), (int8_t)-1);
                for (size_t k = 0; k < lr.size(); ++k) lpn[lr[k]] = (int8_t)k;
                std::vector<int32_t> rn(std::max<size_t>(S.rows.size(), 1), 0);
                for (size_t t = 0; t < S.rows.size(); ++t) rn[t] = S.iperm[S.rows[t]];
                HIPCHK(h, h->longpos_sw.upload(lpn, s));
                HIPCHK(h, h->long_sw.upload(lr, s));
                HIPCHK(h, h->rows_sw.upload(rn, s));
            }
            {  // the same per front row (the sweeps read it with the row ids, no dependent gather)
                std::vector<int8_t> fl(std::max<size_t>(S.rows.size(), 1), (int8_t)-1);
                for (size_t t = 0; t < S.rows.size(); ++t) fl[t] = lp[S.rows[t]];
                HIPCHK(h, h->flong.upload(fl, s));
            }
            const int64_t npl = std::max<int64_t>((int64_t)S.nf * (int64_t)lr.size(), 1);
            HIPCHK(h, h->part_long.alloc(npl));
            // fronts without a given long row never write its partial: those slots stay 0
            HIPCHK(h, hipMemsetAsync(h->part_long.p, 0, sizeof(double) * npl, s));
            if (!h->use_front_sweeps) {  // more than 127 dense rows: the row-major sweeps
                HIPCHK(h, h->rowpartner.upload(S.rowpartner, s));
                HIPCHK(h, h->uvalR.alloc(S.rowpartner.size()));
            }
        }
        h->long_chunks = (h->max_long + kLongChunk - 1) / kLongChunk;
        HIPCHK(h, h->long_part.alloc(std::max<int64_t>((int64_t)h->n_long * h->long_chunks, 1)));
        HIPCHK(h, h->long_cnt.alloc(std::max<int64_t>(h->n_long, 1)));
        HIPCHK(h, hipMemsetAsync(h->long_cnt.p, 0, sizeof(uint32_t) * std::max<int64_t>(h->n_long, 1), s));
    }
    if (h->delayed.n != (size_t)std::max<int64_t>(n, 1)) HIPCHK(h, h->delayed.alloc(std::max<int64_t>(n, 1)));
    if (h->uval.n != (size_t)S.nu) HIPCHK(h, h->uval.alloc(S.nu));
    if (h->scale.n != (size_t)n) {
        HIPCHK(h, h->scale.alloc(n));
        if (n > 0) HIPCHK(h, hipMemsetAsync(h->scale.p, 0, sizeof(double) * n, s));  // rows of other ranks: x = 0
        HIPCHK(h, h->rowsum.alloc(n));
        HIPCHK(h, h->rmax.alloc(n));
        HIPCHK(h, h->w.alloc(n));
        HIPCHK(h, h->bvec.alloc(n));
        HIPCHK(h, h->xtmp.alloc(n));
        HIPCHK(h, h->rtmp.alloc(n));
    }
    HIPCHK(h, h->L.alloc(S.L_size));
    HIPCHK(h, h->cb.alloc(S.cb_size));
    HIPCHK(h, h->cvec.alloc(S.f_relmap_off.empty() ? 0 : S.f_relmap_off.back()));
    HIPCHK(h, h->gscratch.alloc(gtot));
    HIPCHK(h, h->big.alloc(S.max_m > kMaxLdsFront ? S.nf : 0));
    if (!h->big_pending.p) HIPCHK(h, h->big_pending.alloc(1));
    HIPCHK(h, h->frow.alloc(S.rows.size()));
    HIPCHK(h, h->fscale.alloc(S.rows.size()));
    HIPCHK(h, h->fpos.alloc(S.rows.size()));
    HIPCHK(h, h->piv.alloc(S.rows.size()));
    if (!h->counters.p) {
        HIPCHK(h, h->counters.alloc(kCounterSlots));
        h->minbits_p = h->counters.p + 8;
        h->anorm_p = h->counters.p + 9;
    }
    if (S.nf > 0) {  // fronts another rank factors keep zero records
        HIPCHK(h, hipMemsetAsync(h->fstat.p, 0, sizeof(int32_t) * S.nf, s));
        HIPCHK(h, hipMemsetAsync(h->fcnt.p, 0, sizeof(unsigned long long) * S.nf, s));
    }
    if (h->world > 1) {
        int rc = setup_distribution(h);
        if (rc != UNO_KKT_OK) return rc;
        const Partition& Pt = h->dist.part;
        HIPCHK(h, build_plan(h, [&](int32_t f) { return Pt.owner[f] == h->rank; }, h->plan[0]));
        HIPCHK(h, build_plan(h, [&](int32_t f) { return h->rank == 0 && Pt.owner[f] < 0; }, h->plan[1]));
    } else {
        HIPCHK(h, build_plan(h, [](int32_t) { return true; }, h->plan[0]));
        HIPCHK(h, build_plan(h, [](int32_t) { return false; }, h->plan[1]));
    }
    HIPCHK(h, setup_dataflow(h));  // after the partition (distributed: the walk is the rank's own fronts)
    HIPCHK(h, setup_factor_dataflow(h));  // after the partition: a rank's own subtrees
    HIPCHK(h, hipStreamSynchronize(s));
    double an = h->st.analysis_seconds;
    int64_t nfac = h->st.factorizations, nsol = h->st.solves;
    memset(&h->st, 0, sizeof(h->st));
    h->st.last_backward_error = -1.0;
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

// rxpos / xpos of the dataflow solve for the factorization just enqueued (they depend on its pivoting, not on
// the right-hand side): queued right behind the counters' read-back, so they run while the host checks the
// inertia instead of at the start of the next solve (one GPU)
hipError_t enqueue_xpos(uno_kkt_t h) {
    if (h->world != 1 || !h->df_enabled || h->df_grid <= 0 || !h->early_xpos) return hipSuccess;
    SolveArgs A;
    A.fm = h->fm.p; A.fp = h->fp.p; A.rows_off = h->rows_off.p; A.frow = h->frow.p; A.fpos = h->fpos.p; A.piv = h->piv.p;
    A.child_off = h->child_off.p; A.child = h->child.p; A.relmap_off = h->relmap_off.p; A.relmap = h->relmap.p;
    A.L_off = h->L_off.p; A.L = h->L.p; A.w = h->w.p; A.cvec = h->cvec.p; A.ch_cm = h->ch_cm.p;
    A.ch_relmap_off = h->ch_relmap_off.p;
    const DfArgs Df = dataflow_args(h);
    hipError_t e = launch_xpos(A, Df, h->df_xpos.p, h->df_rxpos.p, nullptr, 0, h->df_top_base, h->stream, !h->xpos_by_factor);
    if (e == hipSuccess) h->df_rx_valid = true;
    return e;
}

int enqueue_factorization(uno_kkt_t h) {
    Symbolic& S = h->S;
    hipStream_t s = h->stream;
    // counters, minbits, anorm: reset by the first equilibration sweep when it runs (no launch of its own)
    // the pack fused into the first sweep (option sweep_pack, one GPU, scaling on), else the flat k_pack grid
    const bool fused_pack = h->use_front_sweeps && (h->sweep_pack || h->world != 1 || h->scale_iters <= 0);
    const bool reset_in_sweep = fused_pack && S.nf > 0 && h->sweep_reset;
    if (!reset_in_sweep) HIPCHK(h, launch_reset_counters(h->counters.p, s));
    if (fused_pack) {
        // k_pack runs inside launch_front_sweeps (timed with the scaling)
    } else {
        TimerScope t(h, KC_PACK);
        if (h->world == 1) {
            HIPCHK(h, launch_pack(h->values_ptr, h->dup_ptr.p, h->dup_pos.p, h->slot_src.p, 0, S.nu, h->uval.p, s));
            if (h->slot_src.p) HIPCHK(h, launch_pack_multi(h->values_ptr, h->dup_ptr.p, h->dup_pos.p, h->multi_slots.p, h->n_multi, h->uval.p, s));
        } else {
            for (const auto& r : h->dist.pack_ranges)
                HIPCHK(h, launch_pack(h->values_ptr, h->dup_ptr.p, h->dup_pos.p, nullptr, r.first, r.second, h->uval.p, s));
        }
    }
    {
        TimerScope t(h, KC_SCALE);
        ScanArgs SA;
        SA.n = S.n; SA.list = nullptr; SA.perm = h->perm_d.p; SA.cptr = h->cptr.p; SA.rptr = h->rptr.p;
        SA.rslot = h->rslot.p; SA.ent_r = h->ent_r.p; SA.ent_c = h->ent_c.p; SA.uval = h->uval.p;
        SA.scale = h->scale.p; SA.out = nullptr; SA.anorm = h->anorm_p; SA.long_rows = h->long_rows.p;
        SA.n_long = h->n_long; SA.max_long = h->max_long; SA.long_chunks = h->long_chunks; SA.part = h->long_part.p;
        SA.uvalR = h->uvalR.p; SA.rowpartner = h->rowpartner.p; SA.long_cnt = h->long_cnt.p;
        SA.scale_out = h->rmax.p;  // scratch of the double-buffered sweeps (new numbering); final scaling after them
        SA.scale_in = h->w.p;      // (free until the solve)
        h->scan = SA;
        h->norm_valid = false;
        if (h->use_front_sweeps) {
            SweepArgs W;
            W.nf = S.nf; W.n = S.n; W.fm = h->fm.p; W.rows_off = h->rows_off.p; W.rows = h->rows_sw.p;
            W.perm = h->perm_d.p;
            W.ent_off = h->ent_off.p; W.ent_lpos = h->ent_lpos.p; W.values = h->values_ptr; W.dup_ptr = h->dup_ptr.p;
            W.dup_pos = h->dup_pos.p; W.slot_src = h->slot_src.p; W.uval = h->uval.p;
            W.multi = h->multi_slots.p; W.n_multi = h->n_multi; W.scale = h->scale.p; W.ent_total = S.nu;
            const size_t need = (size_t)S.n * std::max(h->scale_iters, 1);
            if (h->rmaxk.n != need) {
                HIPCHK(h, h->rmaxk.alloc(need));
                h->rmaxk_clean = false;
            }
            W.rmax_all = h->rmaxk.p; W.rmax = h->rmaxk.p; W.longpos = h->longpos_sw.p;
            W.long_orig = h->long_sw.p; W.n_long = h->n_long; W.part_long = h->part_long.p; W.max_m = (int)S.max_m;
            W.big_list = h->sweep_big.p; W.n_big = h->n_sweep_big; W.big_slices = h->sweep_slices;
            W.rows_total = (int64_t)S.rows.size();
            W.flong = h->n_long > 0 ? h->flong.p : nullptr;
            W.rmax_zero = h->rmaxk_clean;
            W.counters = reset_in_sweep ? h->counters.p : nullptr;
            HIPCHK(h, launch_front_sweeps(W, h->scale_iters, s, fused_pack));
            h->rmaxk_clean = true;  // k_sweep_final cleared it
            if (h->overlap_norm && !h->exact_next) {
                h->last_optimistic = true;  // row sums only if a pivot is small (sync_and_verify)
            } else {
                HIPCHK(h, launch_rowsum_norm_orig(SA, h->rowsum.p, s));
                h->last_optimistic = false;
                h->norm_valid = true;
            }
        } else if (h->world == 1 && h->overlap_norm && !h->exact_next) {
            // threshold 0 and a record of the smallest accepted pivot; the row sums only if it is small
            // (sync_and_verify)
            HIPCHK(h, launch_scale_sweeps(SA, h->scale_iters, h->rmax.p, s));
            h->last_optimistic = true;
        } else if (h->world == 1) {
            HIPCHK(h, launch_scale(SA, h->scale_iters, h->rmax.p, h->rowsum.p, s));
            h->last_optimistic = false;
            h->norm_valid = true;
        } else {
            h->last_optimistic = false;
            int rc = dist_scale(h, SA);
            if (rc != UNO_KKT_OK) return rc;
        }
    }
    // the scaling per front row
    if (h->front_scale)
        HIPCHK(h, launch_front_scale(h->rows.p, h->scale.p, h->fscale.p, (int64_t)S.rows.size(), s));
    FactorArgs A;
    A.fscale = h->front_scale ? h->fscale.p : nullptr;
    // one GPU with the dataflow solve: the factor write-outs also fill xpos (k_xpos pass 0)
    h->xpos_by_factor = h->world == 1 && h->df_enabled && h->df_grid > 0 && h->early_xpos && h->df_xpos.p && h->df_xs_off.p;
    A.xpos = h->xpos_by_factor ? h->df_xpos.p : nullptr;
    A.xs_off = h->xpos_by_factor ? h->df_xs_off.p : nullptr;
    A.fm = h->fm.p; A.fp = h->fp.p; A.rows_off = h->rows_off.p; A.rows = h->rows.p;
    A.ent_off = h->ent_off.p; A.ent_lpos = h->ent_lpos.p; A.uval = h->uval.p; A.scale = h->scale.p;
    A.child_off = h->child_off.p; A.child = h->child.p; A.relmap_off = h->relmap_off.p; A.relmap = h->relmap.p;
    A.ch_cm = h->ch_cm.p; A.ch_relmap_off = h->ch_relmap_off.p; A.ch_cb_off = h->ch_cb_off.p;
    A.L_off = h->L_off.p; A.cb_off = h->cb_off.p; A.gscratch_off = h->gscratch_off.p; A.anorm_bits = h->anorm_p;
    A.cbpos = h->use_cbpos ? h->cbpos.p : nullptr;
    A.L = h->L.p; A.cb = h->cb.p; A.gscratch = h->gscratch.p; A.frow = h->frow.p; A.fpos = h->fpos.p; A.piv = h->piv.p;
    A.counters = h->counters.p; A.fstat = h->fstat.p; A.fslow = h->fslow.p; A.fcnt = h->fcnt.p; A.u = h->u; A.null_fac = h->null_fac;
    A.fmin = h->fmin.p;
    A.big = h->big.p;
    if (h->last_optimistic) A.anorm_bits = nullptr;
    A.fparent = h->fparent.p; A.delayed = h->delayed.p; A.record_delays = h->delay_relaxed;
    A.stamps = nullptr;
    A.stamp_mode = h->want_stamps;
    if (h->want_stamps) {
        if (h->stamps.n != (size_t)(8 * S.nf)) HIPCHK(h, h->stamps.alloc(8 * S.nf));
        HIPCHK(h, hipMemsetAsync(h->stamps.p, 0, sizeof(unsigned long long) * 8 * S.nf, s));
        A.stamps = h->stamps.p;
    }
    A.df_order = nullptr; A.df_nf = 0; A.df_nch = nullptr; A.df_cnt = nullptr; A.df_epoch = 0; A.df_abort = nullptr;
    A.df_ticket = nullptr;
    const bool dff = h->dff_level != INT32_MAX;
    const Plan& lp = dff ? h->dff_plan : h->plan[0];
    // two-stream levels back to back: each stream waits for the other's previous level directly (one event
    // hop) instead of a join into the main stream followed by a fork out of it (two hops, ~18 us of idle
    // between levels 0 and 1 at C3)
    bool split = false;  // stream3 holds launches of the previous level not yet joined into s
    auto join3 = [&]() -> hipError_t {
        hipError_t e = hipEventRecord(h->ev_join, h->stream3);
        if (e == hipSuccess) h->side_pending &= ~1;
        return e == hipSuccess ? hipStreamWaitEvent(s, h->ev_join, 0) : e;
    };
    for (size_t q = 0; q < lp.fac.size();) {
        size_t r = q + 1;  // launches [q, r) of one level
        while (r < lp.fac.size() && lp.fac[r].level == lp.fac[q].level) ++r;
        TimerScope t(h, lp.fac[q].global ? KC_FACTOR_GLOBAL : KC_FACTOR_LDS);
        const bool three = h->concurrent_classes == 3 && r - q > 2;
        const bool multi = r - q > 1 && h->concurrent_classes;
        if (multi && split && !three) {  // cross waits (the previous level was split over s / stream3)
            HIPCHK(h, hipEventRecord(h->ev_fork, s));
            HIPCHK(h, hipEventRecord(h->ev_join, h->stream3));
            HIPCHK(h, hipStreamWaitEvent(s, h->ev_join, 0));
            HIPCHK(h, hipStreamWaitEvent(h->stream3, h->ev_fork, 0));
            h->side_pending &= ~1;
        } else {
            if (split) HIPCHK(h, join3());
            if (multi) {
                HIPCHK(h, hipEventRecord(h->ev_fork, s));
                HIPCHK(h, hipStreamWaitEvent(h->stream3, h->ev_fork, 0));
                if (three) HIPCHK(h, hipStreamWaitEvent(h->stream4, h->ev_fork, 0));
            }
        }
        split = false;
        for (size_t u = q; u < r; ++u) {
            const Launch& L = lp.fac[u];
            // classes alternate between the streams (a level's two large one-wave classes overlap instead
            // of queueing behind each other on the second stream: factor 1.32 -> 1.18 ms at C3); option
            // concurrent_classes = 2 keeps the earlier rule (first class on the main stream, every other
            // one on the second), 3 deals the classes over three streams
            hipStream_t ls = s;
            if (h->concurrent_classes == 2) ls = u > q ? h->stream3 : s;
            else if (three) ls = (u - q) % 3 == 0 ? s : ((u - q) % 3 == 1 ? h->stream3 : h->stream4);
            else if (h->concurrent_classes) ls = ((u - q) & 1) ? h->stream3 : s;
            if (ls == h->stream3) h->side_pending |= 1;
            if (ls == h->stream4) h->side_pending |= 2;
            if (L.global) {
                const int rc = run_big_fronts(h, A, lp.fac_fronts.p + L.begin, L, ls);
                if (rc != UNO_KKT_OK) return rc;
            } else {
                HIPCHK(h, launch_factor(A, lp.fac_fronts.p + L.begin, L.count, L.mmax, false, ls));
            }
        }
        if (multi && !three) {
            split = true;  // joined by the next level's waits or after the loop
        } else if (multi) {
            HIPCHK(h, join3());
            HIPCHK(h, hipEventRecord(h->ev_join4, h->stream4));
            HIPCHK(h, hipStreamWaitEvent(s, h->ev_join4, 0));
            h->side_pending &= ~2;
        }
        q = r;
    }
    if (split) {  // inside a timer scope: the per-class device times keep the last level's stream3 tail
        TimerScope t(h, KC_FACTOR_LDS);
        HIPCHK(h, join3());
    }
    if (dff) {
        TimerScope t(h, KC_FACTOR_LDS);
        A.df_order = h->dff_order.p;
        A.df_nf = (int32_t)h->dff_order.n;
        A.df_nch = h->dff_nch.p;
        A.df_cnt = h->dff_cnt.p;
        A.df_epoch = ++h->dff_epoch;
        A.df_abort = h->df_abort.p;
        A.df_ticket = h->dff_ticket.p;
        HIPCHK(h, launch_factor_df(A, h->dff_mmax, s));
        // one GPU: k_count writes the abort word to the host block itself
        if (h->world > 1) HIPCHK(h, hipMemcpyAsync(h->h_counters + 11, h->df_abort.p, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    }
    if (h->world > 1) {
        // subtree roots' contribution blocks -> rank 0 (same arena offsets on every rank)
        int rc = exchange_roots(h, h->cb.p, [&](int32_t f) { return S.f_cb_off[f]; },
                                [&](int32_t f) { return S.f_cb_off[f + 1] - S.f_cb_off[f]; });
        if (rc != UNO_KKT_OK) return rc;
        for (const Launch& L : h->plan[1].fac) {
            TimerScope t(h, L.global ? KC_FACTOR_GLOBAL : KC_FACTOR_LDS);
            if (L.global) {
                rc = run_big_fronts(h, A, h->plan[1].fac_fronts.p + L.begin, L, s);
                if (rc != UNO_KKT_OK) return rc;
            } else {
                HIPCHK(h, launch_factor(A, h->plan[1].fac_fronts.p + L.begin, L.count, L.mmax, false, s));
            }
        }
    }
    h->wait_seq = 0;
    if (h->world == 1) {  // counters and the dataflow abort word straight into the page-locked host block
        // option host_flag (with spin_wait): the host polls the sequence number k_count writes last
        if (h->host_flag && h->spin_wait) h->wait_seq = ++h->count_seq;
        HIPCHK(h, launch_count(h->fcnt.p, h->fstat.p, h->fmin.p, S.nf, h->counters.p, h->minbits_p, s,
                               dff ? h->df_abort.p : nullptr, h->h_counters, h->wait_seq));
    } else {
        HIPCHK(h, launch_count(h->fcnt.p, h->fstat.p, h->fmin.p, S.nf, h->counters.p, h->minbits_p, s));
    }
    if (h->world > 1) {
        // counters[7] keeps this rank's delayed-column count; 0..6 are summed over the ranks
        HIPCHK(h, hipMemcpyAsync(h->counters.p + 7, h->counters.p + 6, sizeof(unsigned long long), hipMemcpyDeviceToDevice, s));
        HIPCHK(h, h->comm->allreduce(h->counters.p, 7, RedOp::SumU64, s));
    }
    // counters and minbits in one copy (h_counters[8] is the min pivot bits)
    if (h->world > 1) HIPCHK(h, hipMemcpyAsync(h->h_counters, h->counters.p, 9 * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    // sync_and_verify waits for this, not for the xpos below (or for k_count's flag: no event marker between
    // k_count and the xpos launch)
    if (!h->wait_seq) HIPCHK(h, hipEventRecord(h->ev_counters, s));
    h->factor_enqueued = true;
    h->df_rx_valid = false;  // pivoting may have permuted rows
    HIPCHK(h, enqueue_xpos(h));
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
        hipStreamCreateWithFlags(&h->stream2, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&h->stream3, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&h->stream4, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&h->ev_fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&h->ev_join, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&h->ev_join4, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&h->ev_scale, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&h->ev_norm, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&h->ev_counters, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&h->ev_wait, hipEventDisableTiming) != hipSuccess ||
        hipHostMalloc((void**)&h->h_counters, 12 * sizeof(unsigned long long)) != hipSuccess ||
        hipHostMalloc((void**)&h->h_big, sizeof(int32_t)) != hipSuccess) {
        delete h;
        return UNO_KKT_ERR_HIP;
    }
    memset(h->h_counters, 0, 12 * sizeof(unsigned long long));
    if (const char* v = getenv("UNO_KKT_VERBOSE")) h->verbose = atoi(v);  // diagnostics of embedded uses
    *handle = h;
    // UNO_KKT_OPTIONS="name=value,name=value": options for embedded uses (the Uno plugin has no option path)
    if (const char* o = getenv("UNO_KKT_OPTIONS")) {
        std::string all(o);
        size_t b = 0;
        while (b < all.size()) {
            size_t e = all.find(',', b);
            if (e == std::string::npos) e = all.size();
            const std::string kv = all.substr(b, e - b);
            const size_t eq = kv.find('=');
            if (eq != std::string::npos) uno_kkt_set_option(h, kv.substr(0, eq).c_str(), atof(kv.c_str() + eq + 1));
            b = e + 1;
        }
    }
    return UNO_KKT_OK;
}

void uno_kkt_destroy(uno_kkt_t h) {
    if (!h) return;
    hipSetDevice(h->device);
    if (h->stream) hipStreamSynchronize(h->stream);
    for (auto& t : h->pending) { hipEventDestroy(t.a); hipEventDestroy(t.b); }
    for (auto e : h->ev_pool) hipEventDestroy(e);
    if (h->h_counters) hipHostFree(h->h_counters);
    if (h->h_big) hipHostFree(h->h_big);
    unpin_host_buffer(h);
    if (h->stream2) hipStreamSynchronize(h->stream2);
    if (h->ev_scale) hipEventDestroy(h->ev_scale);
    if (h->ev_norm) hipEventDestroy(h->ev_norm);
    if (h->ev_counters) hipEventDestroy(h->ev_counters);
    if (h->ev_wait) hipEventDestroy(h->ev_wait);
    if (h->stream2) hipStreamDestroy(h->stream2);
    if (h->stream3) { hipStreamSynchronize(h->stream3); hipStreamDestroy(h->stream3); }
    if (h->ev_fork) hipEventDestroy(h->ev_fork);
    if (h->ev_join) hipEventDestroy(h->ev_join);
    if (h->ev_join4) hipEventDestroy(h->ev_join4);
    if (h->stream4) { hipStreamSynchronize(h->stream4); hipStreamDestroy(h->stream4); }
    if (h->upload) { hipStreamSynchronize(h->upload); hipStreamDestroy(h->upload); }
    if (h->ev_upload) hipEventDestroy(h->ev_upload);
    if (h->ev_upload_dep) hipEventDestroy(h->ev_upload_dep);
    delete h->comm;
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
    else if (n == "wide_group") h->aopt.wide_group = std::max(1, (int)value);
    else if (n == "wide_block") h->aopt.wide_block = std::max(1, std::min((int)value, 32767));
    else if (n == "dense_factor") h->aopt.dense_factor = value;
    else if (n == "timing") h->timing = value != 0.0;
    else if (n == "delay_relaxed") h->delay_relaxed = value != 0.0;
    else if (n == "refine") h->refine = std::max(0, (int)value);
    else if (n == "refine_tol") h->refine_tol = std::max(0.0, value);
    else if (n == "sweep_reset") h->sweep_reset = value != 0.0;
    else if (n == "sweep_pack") h->sweep_pack = value != 0.0;
    else if (n == "cbpos") h->cbpos_opt = value != 0.0;  // takes effect at the next analysis
    else if (n == "resid_fronts") { h->resid_fronts = value != 0.0; h->rz_state = 0; }
    else if (n == "resid_long") { h->resid_long = std::max<int64_t>(1, (int64_t)value); h->rz_state = 0; }
    else if (n == "pin_host_values") h->pin_host = value != 0.0;
    else if (n == "front_sweeps") h->front_sweeps = value != 0.0;
    else if (n == "stamps") h->want_stamps = (int)value;
    else if (n == "max_merge_rounds") h->max_merge_rounds = std::max(0, (int)value);
    else if (n == "gather_solution") h->gather_solution = value != 0.0;
    else if (n == "verbose") h->verbose = (int)value;
    else if (n == "overlap_norm") h->overlap_norm = value != 0.0;
    else if (n == "solve_stamps") h->want_solve_stamps = (int)value;
    else if (n == "concurrent_classes") h->concurrent_classes = (int)value;
    else if (n == "early_xpos") h->early_xpos = value != 0.0;
    else if (n == "spin_wait") h->spin_wait = value != 0.0;
    else if (n == "host_flag") h->host_flag = value != 0.0;
    else if (n == "front_scale") h->front_scale = std::max(0, std::min(2, (int)value));
    else if (n == "debug_abort_solves") h->debug_abort_solves = std::max(0, (int)value);
    else if (n == "dist_min_efficiency") h->dist_min_eff = value;
    else if (n == "dist_force") h->dist_force = value != 0.0;
    else if (n == "slow_first") h->slow_first = value != 0.0;
    else if (n == "comm_trace") {  // record the transport calls (tests): wraps the attached transport, if any
        h->comm_trace = value != 0.0;
        std::vector<int64_t> dummy;
        if (h->comm_trace && h->comm && !ukkt::comm_trace_records(h->comm, dummy, false)) {
            h->comm = ukkt::make_tracing_transport(h->comm);
            install_order_probe(h);
        }
    }
    else if (n == "dataflow_factor") {
        h->dff_enabled = std::max(0, std::min(2, (int)value));
        if (h->analyzed) {
            HIPCHK(h, setup_factor_dataflow(h));
            HIPCHK(h, hipStreamSynchronize(h->stream));
        }
    }
    else if (n == "solve_window") {
        h->df_win_opt = std::max(0, (int)value);
        if (h->analyzed) {
            HIPCHK(h, setup_dataflow(h));
            HIPCHK(h, hipStreamSynchronize(h->stream));
        }
    }
    else if (n == "dist_dataflow_solve") {
        h->dist_df = value < 0.0 ? -1 : value != 0.0;
        if (h->analyzed) {
            HIPCHK(h, setup_dataflow(h));
            HIPCHK(h, hipStreamSynchronize(h->stream));
        }
    }
    else if (n == "solve_rg" || n == "solve_rg_bwd" || n == "solve_flat_levels") {
        if (n == "solve_flat_levels") h->solve_flat = std::max(0, (int)value);
        else (n == "solve_rg" ? h->solve_rg : h->solve_rg_bwd) = value != 0.0;
        if (h->analyzed) {
            HIPCHK(h, setup_dataflow(h));
            HIPCHK(h, hipStreamSynchronize(h->stream));
        }
    }
    else if (n == "solve_rg_wpe") {
        h->rg_wpe = (int)value == 4 ? 4 : 3;
        if (h->analyzed) set_rg_grids(h);
    }
    else if (n == "dataflow_solve") {
        h->df_enabled = value != 0.0;
        if (h->analyzed) {
            HIPCHK(h, setup_dataflow(h));
            HIPCHK(h, hipStreamSynchronize(h->stream));
        }
    }
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
    unpin_host_buffer(h);
    auto t0 = std::chrono::steady_clock::now();
    std::string msg = ukkt::analyze(n, nnz, row, col, h->aopt, h->P, h->S);
    if (!msg.empty()) return set_err(h, UNO_KKT_ERR_ARG, msg);
    // multi-GPU gate (north_star: partition "only when the ordering exposes enough top-level
    // parallelism"): the subtree partition is used only if it has at least `world` subtrees and its estimated
    // parallel efficiency total / (world * (max rank work + top work)) reaches dist_min_efficiency; otherwise
    // every rank factors and solves the whole matrix on its own GPU (replicas, no collective).  The decision
    // is a pure function of the pattern and the options, all-reduced so every rank takes the same one;
    // delayed-pivot rebuilds keep it.
    h->world = h->comm_world;
    h->rank = h->comm_rank;
    h->dist_declined = false;
    h->dist_efficiency = 0.0;
    if (h->world > 1) {
        Partition Pt;
        partition_tree(h->S, h->world, Pt);
        const double denom = (double)h->world * (Pt.max_rank_work + Pt.top_work);
        h->dist_efficiency = denom > 0.0 ? Pt.total_work / denom : 0.0;
        bool decline = !h->dist_force && (Pt.n_subtrees < h->world || h->dist_efficiency < h->dist_min_eff);
        {
            // the ranks agree on the gate even if their options differ: any rank declining makes all decline
            // (otherwise a partitioned rank would wait in collectives a replica never joins)
            if (!h->df_abort64.p) HIPCHK(h, h->df_abort64.alloc(1));
            unsigned long long flag = decline ? 1ull : 0ull;
            HIPCHK(h, hipMemcpyAsync(h->df_abort64.p, &flag, sizeof(flag), hipMemcpyHostToDevice, h->stream));
            HIPCHK(h, h->comm->allreduce(h->df_abort64.p, 1, RedOp::MaxU64, h->stream));
            HIPCHK(h, hipMemcpyAsync(&flag, h->df_abort64.p, sizeof(flag), hipMemcpyDeviceToHost, h->stream));
            HIPCHK(h, hipStreamSynchronize(h->stream));
            decline = flag != 0;
        }
        if (decline) {
            h->dist_declined = true;
            h->world = 1;
            h->rank = 0;
            if (h->verbose)
                fprintf(stderr, "[uno_kkt] partition declined: %lld subtrees for %d ranks, efficiency %.3f < %.3f: replicas\n",
                        (long long)Pt.n_subtrees, h->comm_world, h->dist_efficiency, h->dist_min_eff);
        }
    }
    if (h->upload) HIPCHK(h, hipStreamSynchronize(h->upload));  // staged chunks of the previous pattern
    h->staged_pending = false;
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
    for (int64_t i = 0; i < count; ++i)
        if (positions[i] < 0 || positions[i] >= h->S.nnz) return set_err(h, UNO_KKT_ERR_ARG, "position out of range");
    // the values of a queued factorization are final only once it has been checked (its redos re-pack
    // from the same buffer): finish it before editing
    if (h->factor_enqueued) {
        const int rc = finish_factorization(h);
        if (rc != UNO_KKT_OK && rc != UNO_KKT_ERR_PIVOT) return rc;
    }
    h->packed_valid = false;
    if (count == 0) return UNO_KKT_OK;
    HIPCHK(h, order_after_staged(h));
    // a position listed twice keeps its LAST value (the sequential-copy semantics): duplicates are resolved
    // here, so the parallel scatter below writes every position once
    std::vector<int64_t> order((size_t)count);
    for (int64_t i = 0; i < count; ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](int64_t a, int64_t b) { return positions[a] < positions[b]; });
    std::vector<int64_t> upos;
    std::vector<double> uv;
    for (int64_t q = 0; q < count; ++q) {
        const int64_t i = order[q];
        if (q + 1 < count && positions[order[q + 1]] == positions[i]) continue;  // a later edit of the same position wins
        upos.push_back(positions[i]);
        uv.push_back(v[i]);
    }
    count = (int64_t)upos.size();
    // one H2D copy of (positions, values), one scatter kernel
    HIPCHK(h, h->edit_pos.alloc(count));
    HIPCHK(h, h->edit_val.alloc(count));
    HIPCHK(h, hipMemcpyAsync(h->edit_pos.p, upos.data(), sizeof(int64_t) * count, hipMemcpyHostToDevice, h->stream));
    HIPCHK(h, hipMemcpyAsync(h->edit_val.p, uv.data(), sizeof(double) * count, hipMemcpyHostToDevice, h->stream));
    HIPCHK(h, launch_scatter64(h->edit_val.p, h->edit_pos.p, const_cast<double*>(h->values_ptr), count, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));  // the host arrays may be reused on return
    return UNO_KKT_OK;
}

}  // extern "C"

__global__ void k_fill(double* p, int64_t n, double v) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = v;
}

// option pin_host_values: the caller's buffer is page-locked once (hipHostRegister) so every later upload
// is a direct DMA; it is unregistered when the pointer changes or the handle is destroyed (a registration is
// keyed by pointer AND length: the same address with another pattern size is a new buffer).  The caller keeps
// a registered buffer allocated until it passes another pointer, calls uno_kkt_analyze again or destroys the
// handle (include/uno_kkt.h).
static void pin_host_buffer(uno_kkt_t h, const double* values) {
    const int64_t nnz = h->S.nnz;
    if (!h->pin_host || nnz <= 0) return;
    if (values == h->pinned_ptr && h->pinned_bytes == (size_t)nnz * sizeof(double)) return;
    unpin_host_buffer(h);
    h->pinned_bytes = (size_t)nnz * sizeof(double);
    h->pinned_ptr = hipHostRegister(const_cast<double*>(values), h->pinned_bytes, hipHostRegisterDefault) == hipSuccess
                        ? values : nullptr;
    (void)hipGetLastError();
}

extern "C" {

int uno_kkt_fill_values(uno_kkt_t h, int64_t first, int64_t count, double value) {
    if (!h) return UNO_KKT_ERR_ARG;
    if (!h->analyzed || !h->values_ptr) return set_err(h, UNO_KKT_ERR_STATE, "fill_values before a factorization");
    if (first < 0 || count < 0 || first + count > h->S.nnz) return set_err(h, UNO_KKT_ERR_ARG, "range out of bounds");
    if (count == 0) return UNO_KKT_OK;
    HIPCHK(h, hipSetDevice(h->device));
    if (h->factor_enqueued) {  // see uno_kkt_set_values
        const int rc = finish_factorization(h);
        if (rc != UNO_KKT_OK && rc != UNO_KKT_ERR_PIVOT) return rc;
    }
    h->packed_valid = false;
    HIPCHK(h, order_after_staged(h));
    int grid = (int)std::min<int64_t>((count + 255) / 256, 4096);
    hipLaunchKernelGGL(k_fill, dim3(grid), dim3(256), 0, h->stream, const_cast<double*>(h->values_ptr) + first, count, value);
    HIPCHK(h, hipGetLastError());
    return UNO_KKT_OK;
}

int uno_kkt_factorize_update(uno_kkt_t h, const double* values, int64_t first, int64_t count) {
    if (!h || !values) return UNO_KKT_ERR_ARG;
    if (!h->analyzed) return set_err(h, UNO_KKT_ERR_STATE, "factorize before analyze");
    if (h->values_ptr != h->values.p) return set_err(h, UNO_KKT_ERR_STATE, "factorize_update needs a previous host-pointer factorization");
    if (first < 0 || count < 0 || first + count > h->S.nnz) return set_err(h, UNO_KKT_ERR_ARG, "range out of bounds");
    HIPCHK(h, hipSetDevice(h->device));
    if (h->factor_enqueued) {  // its redos re-pack from the device copy: finish it before the copy changes
        const int rc = finish_factorization(h);
        if (rc != UNO_KKT_OK && rc != UNO_KKT_ERR_PIVOT) return rc;
    }
    HIPCHK(h, order_after_staged(h));
    if (count > 0)
        HIPCHK(h, hipMemcpyAsync(h->values.p + first, values + first, count * sizeof(double), hipMemcpyHostToDevice, h->stream));
    return uno_kkt_factorize(h, nullptr, 0);
}

int uno_kkt_stage_values(uno_kkt_t h, const double* values, int64_t first, int64_t count) {
    if (!h || !values) return UNO_KKT_ERR_ARG;
    if (!h->analyzed) return set_err(h, UNO_KKT_ERR_STATE, "stage_values before analyze");
    if (h->world != 1) return set_err(h, UNO_KKT_ERR_STATE, "stage_values: one-GPU handles only");
    if (first < 0 || count < 0 || first + count > h->S.nnz) return set_err(h, UNO_KKT_ERR_ARG, "range out of bounds");
    if (count == 0) return UNO_KKT_OK;
    HIPCHK(h, hipSetDevice(h->device));
    if (!h->upload) {
        HIPCHK(h, hipStreamCreateWithFlags(&h->upload, hipStreamNonBlocking));
        HIPCHK(h, hipEventCreateWithFlags(&h->ev_upload, hipEventDisableTiming));
        HIPCHK(h, hipEventCreateWithFlags(&h->ev_upload_dep, hipEventDisableTiming));
    }
    if (!h->staged_pending) {
        // first chunk of a new set of values: the work queued so far (a factorization whose redos re-pack
        // from the device copy, a refined solve whose residual reads it) must be done with the old copy
        if (h->factor_enqueued) {
            const int rc = finish_factorization(h);
            if (rc != UNO_KKT_OK && rc != UNO_KKT_ERR_PIVOT) return rc;
        }
        HIPCHK(h, hipEventRecord(h->ev_upload_dep, h->stream));
        HIPCHK(h, hipStreamWaitEvent(h->upload, h->ev_upload_dep, 0));
        h->staged_pending = true;
        h->packed_valid = false;
    }
    pin_host_buffer(h, values);
    HIPCHK(h, hipMemcpyAsync(h->values.p + first, values + first, count * sizeof(double), hipMemcpyHostToDevice, h->upload));
    return UNO_KKT_OK;
}

int uno_kkt_factorize(uno_kkt_t h, const double* values, int values_on_device) {
    if (!h) return UNO_KKT_ERR_ARG;
    if (!h->analyzed) return set_err(h, UNO_KKT_ERR_STATE, "factorize before analyze");
    HIPCHK(h, hipSetDevice(h->device));
    Symbolic& S = h->S;
    if (h->factor_enqueued) {  // previous factorization never queried: drain it first
        // a device / runtime failure is reported; a pivoting failure (ERR_PIVOT) only concerned the
        // drained values, which this factorization replaces
        int rc = finish_factorization(h);
        if (rc != UNO_KKT_OK && rc != UNO_KKT_ERR_PIVOT) return rc;
    }
    h->factored = false;
    if (h->staged_pending) {  // chunks of uno_kkt_stage_values: the solver's stream waits for the last one
        HIPCHK(h, hipEventRecord(h->ev_upload, h->upload));
        HIPCHK(h, hipStreamWaitEvent(h->stream, h->ev_upload, 0));
        h->staged_pending = false;
        if (values == nullptr) h->values_ptr = h->values.p;
    }
    if (values == nullptr) {
        if (!h->values_ptr && S.nnz > 0) return set_err(h, UNO_KKT_ERR_STATE, "no device values to reuse");
    } else if (values_on_device) {
        h->values_ptr = values;
    } else {
        pin_host_buffer(h, values);
        if (S.nnz > 0)
            HIPCHK(h, hipMemcpyAsync(h->values.p, values, S.nnz * sizeof(double), hipMemcpyHostToDevice, h->stream));
        h->values_ptr = h->values.p;
    }
    h->t_factor = std::chrono::steady_clock::now();
    int rc = enqueue_factorization(h);
    if (rc != UNO_KKT_OK) return rc;
    h->packed_valid = h->world == 1;  // one GPU packs every slot
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

}  // extern "C"

namespace {
// One solve with the last factorization, device pointers (b may alias xd: b is read by the first kernel,
// xd written by the last).  Returns after the stream has drained when the dataflow solve ran (its abort
// flag is checked in the same call; an aborted solve is redone with the level schedule, allow_df = false).
// check = false (refined solves): the dataflow abort flag is not read here; the caller reads it once after
// the refinement (the flag stays set through the later walks) and redoes the whole solve level by level
// sub_into (a refinement correction): x = A^-1 b is subtracted from sub_into (xd is scratch then)
int solve_core(uno_kkt_t h, const double* b, double* xd, bool allow_df = true, bool check = true, double* sub_into = nullptr) {
    Symbolic& S = h->S;
    hipStream_t s = h->stream;
    const bool df = allow_df && h->df_enabled && h->df_grid > 0;
    const bool dist = h->world > 1;
    SolveArgs A;
    A.fm = h->fm.p; A.fp = h->fp.p; A.rows_off = h->rows_off.p; A.frow = h->frow.p; A.fpos = h->fpos.p; A.piv = h->piv.p;
    A.child_off = h->child_off.p; A.child = h->child.p; A.relmap_off = h->relmap_off.p; A.relmap = h->relmap.p;
    A.L_off = h->L_off.p; A.L = h->L.p; A.w = h->w.p; A.cvec = h->cvec.p; A.ch_cm = h->ch_cm.p;
    A.ch_relmap_off = h->ch_relmap_off.p;
    auto run = [&](const Plan& P, const SolveLaunch& L, bool forward) -> hipError_t {
        const int32_t* fr = P.sol_fronts.p + L.begin;
        if (L.wave && !forward && h->new_bwd) return launch_solve_bwd_w2(A, fr, L.count, s);
        return L.wave ? launch_solve_wave(A, fr, L.count, L.lds, forward, s)
                      : launch_solve(A, fr, L.count, L.mmax, L.pmax, forward, s);
    };
    const Plan& P0 = h->plan[0];
    const Plan& P1 = h->plan[1];
    if (!df || dist) {  // level schedule (distributed: rank 0's top fronts read the scaled rhs from w)
        TimerScope t(h, KC_RHS);
        HIPCHK(h, launch_rhs_scale(b, h->scale.p, h->w.p, S.n, s));
    }
    DfArgs Df;
    auto walk = [&](bool forward) -> hipError_t {
        const int g = forward ? h->rg_grid_f : h->rg_grid_b;
        if ((forward ? h->solve_rg != 0 : h->new_bwd) && g > 0) {
            if (forward) {  // the flat levels first, level by level (no counters), then the walk of the rest
                for (size_t l = 0; l + 1 < h->flat_off.size(); ++l) {
                    const hipError_t e = launch_solve_fwd_flat(A, Df, h->flat_off[l], h->flat_off[l + 1] - h->flat_off[l], s);
                    if (e != hipSuccess) return e;
                }
            }
            return launch_solve_rg(A, Df, g, forward, h->rg_wpe, s);
        }
        if (forward) return launch_solve_df(A, Df, h->df_grid, h->df_lds, true, s);  // every front (no flat launches)
        // backward: the walk without the flat levels, then those level by level, top level first
        hipError_t e = launch_solve_df(A, Df, h->df_grid, h->df_lds, false, s);
        for (size_t l = h->flat_off.size(); e == hipSuccess && l-- > 1;)
            e = launch_solve_bwd_flat(A, Df, h->flat_off[l - 1], h->flat_off[l] - h->flat_off[l - 1], h->df_lds, s);
        return e;
    };
    if (df) {
        Df = dataflow_args(h);
        if (!h->df_rx_valid) {
            HIPCHK(h, launch_xpos(A, Df, h->df_xpos.p, h->df_rxpos.p, dist ? h->dist.top_orig.p : nullptr,
                                  dist ? h->dist.n_top_rows : 0, h->df_top_base, s));
            h->df_rx_valid = true;
        }
        {
            TimerScope t(h, KC_RHS);
            HIPCHK(h, launch_xs_in(b, h->scale.p, h->df_xpos.p, h->df_xs.p, dist ? h->dist.n_own : S.n, s,
                                   dist ? h->dist.own_orig.p : nullptr));
        }
        Df.epoch = ++h->df_epoch;
        if (h->debug_abort_solves > 0) {  // tests: an abort of this rank's walk (its waits give up at once)
            h->debug_abort_solves--;
            HIPCHK(h, hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(h->df_abort.p), 1, 1, s));
        }
        if (h->want_solve_stamps) {
            if (h->df_stamps.n != (size_t)(8 * S.nf)) HIPCHK(h, h->df_stamps.alloc(8 * S.nf));
            Df.stamps = h->df_stamps.p;
        }
        {
            TimerScope t(h, KC_SOLVE_FWD);
            HIPCHK(h, walk(true));
        }
        if (!dist) {
            TimerScope t(h, KC_SOLVE_BWD);
            HIPCHK(h, walk(false));
        }
    }
    for (size_t q = 0; q < P0.sol.size() && !df; ++q) {
        TimerScope t(h, KC_SOLVE_FWD);
        HIPCHK(h, run(P0, P0.sol[q], true));
    }
    if (dist) {
        DistState& D = h->dist;
        // forward: subtree roots' update vectors -> rank 0, which solves the top of the tree
        if (df) HIPCHK(h, launch_cvx_to_cvec(Df, A, h->df_roots.p, h->n_df_roots, h->cvec.p, s));
        int rc = exchange_roots(h, h->cvec.p, [&](int32_t f) { return S.f_relmap_off[f]; },
                                [&](int32_t f) { return (int64_t)(S.f_m[f] - S.f_p[f]); });
        if (rc != UNO_KKT_OK) return rc;
        for (size_t q = 0; q < P1.sol.size(); ++q) {
            TimerScope t(h, KC_SOLVE_FWD);
            HIPCHK(h, run(P1, P1.sol[q], true));
        }
        for (size_t q = P1.sol.size(); q-- > 0;) {
            TimerScope t(h, KC_SOLVE_BWD);
            HIPCHK(h, run(P1, P1.sol[q], false));
        }
        // backward: the top rows' solution is broadcast, then every rank finishes its subtrees
        if (D.n_top_rows > 0) {
            if (h->rank == 0) HIPCHK(h, launch_gather(h->w.p, D.top_orig.p, D.tbuf.p, D.n_top_rows, s));
            HIPCHK(h, h->comm->broadcast(D.tbuf.p, sizeof(double) * D.n_top_rows, 0, s));
            if (df) {
                HIPCHK(h, hipMemcpyAsync(h->df_xs.p + h->df_top_base, D.tbuf.p, sizeof(double) * D.n_top_rows,
                                         hipMemcpyDeviceToDevice, s));
            } else if (h->rank != 0) {
                HIPCHK(h, launch_scatter(D.tbuf.p, D.top_orig.p, h->w.p, D.n_top_rows, s));
            }
        }
        if (df) {  // the subtree roots' parents (top fronts) have published
            HIPCHK(h, launch_set_done(h->df_done.p, h->df_topf.p, h->n_df_topf, Df.epoch, s));
            TimerScope t(h, KC_SOLVE_BWD);
            HIPCHK(h, walk(false));
        }
    }
    for (size_t q = P0.sol.size(); q-- > 0 && !df;) {
        TimerScope t(h, KC_SOLVE_BWD);
        HIPCHK(h, run(P0, P0.sol[q], false));
    }
    if (dist && allow_df) {
        // distributed: the abort flag is all-reduced BEFORE anything writes x (a rank whose walk is empty or
        // ineligible ran the level schedule and contributes 0), so every rank sees the same verdict, none
        // writes x from a peer's invalid root / top values (x may alias the rhs), and every rank redoes the
        // solve if any aborted, keeping the same path through the collectives
        if (!h->df_abort64.p) HIPCHK(h, h->df_abort64.alloc(1));
        HIPCHK(h, hipMemsetAsync(h->df_abort64.p, 0, sizeof(unsigned long long), s));
        if (df) HIPCHK(h, hipMemcpyAsync(h->df_abort64.p, h->df_abort.p, sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
        HIPCHK(h, h->comm->allreduce(h->df_abort64.p, 1, RedOp::MaxU64, s));
        HIPCHK(h, hipMemcpyAsync(h->h_counters + 10, h->df_abort64.p, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
        HIPCHK(h, hipStreamSynchronize(s));
        if (dataflow_aborted(h)) {
            if (h->df_abort.p) HIPCHK(h, hipMemsetAsync(h->df_abort.p, 0, sizeof(uint32_t), s));
            if (h->verbose) fprintf(stderr, "[uno_kkt] dataflow solve aborted on some rank: this solve redone level by level\n");
            return solve_core(h, b, xd, false);
        }
    }
    {
        TimerScope t(h, KC_RHS);
        if (df && dist) {  // own rows and top rows (the rows a rank's solution holds)
            HIPCHK(h, launch_xs_out(h->df_xs.p, h->scale.p, h->df_xpos.p, h->df_abort.p, xd, h->dist.n_own, s, h->dist.own_orig.p));
            HIPCHK(h, launch_xs_out(h->df_xs.p, h->scale.p, h->df_xpos.p, h->df_abort.p, xd, h->dist.n_top_rows, s, h->dist.top_orig.p));
        } else if (df) {
            if (sub_into) HIPCHK(h, launch_xs_out(h->df_xs.p, h->scale.p, h->df_xpos.p, h->df_abort.p, sub_into, S.n, s, nullptr, true));
            else HIPCHK(h, launch_xs_out(h->df_xs.p, h->scale.p, h->df_xpos.p, h->df_abort.p, xd, S.n, s));
        } else {
            HIPCHK(h, launch_unscale(h->w.p, h->scale.p, xd, S.n, s));
            if (sub_into) HIPCHK(h, launch_sub(sub_into, xd, S.n, s));
        }
    }
    if (dist && h->gather_solution) {
        // MUMPS-style centralized solution on rank 0 (ICNTL(21) = 0): own rows of every other rank
        DistState& D = h->dist;
        if (h->rank != 0 && D.n_own > 0) HIPCHK(h, launch_gather(xd, D.own_orig.p, D.xbuf.p, D.n_own, s));
        HIPCHK(h, h->comm->group_begin());
        for (int q = 1; q < h->world; ++q) {
            const int64_t k = D.own_count[q];
            if (k == 0) continue;
            if (h->rank == q) HIPCHK(h, h->comm->send(D.xbuf.p, sizeof(double) * k, 0, s));
            else if (h->rank == 0) HIPCHK(h, h->comm->recv(D.xbuf.p + D.all_own_off[q], sizeof(double) * k, q, s));
        }
        HIPCHK(h, h->comm->group_end());
        if (h->rank == 0)
            HIPCHK(h, launch_scatter(D.xbuf.p, D.all_own_orig.p, xd, D.all_own_off[h->world], s));
    }
    if (df && !dist && check) {
        // one GPU: k_xs_out itself skips the write of x on an abort (x may alias the rhs); the flag is read
        // in the same call and the solve redone with the level schedule
        HIPCHK(h, hipMemcpyAsync(h->h_counters + 10, h->df_abort.p, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
        HIPCHK(h, host_wait_stream(h, s));
        if (dataflow_aborted(h)) {
            if (h->df_abort.p) HIPCHK(h, hipMemsetAsync(h->df_abort.p, 0, sizeof(uint32_t), s));
            if (h->verbose) fprintf(stderr, "[uno_kkt] dataflow solve aborted: this solve redone level by level\n");
            return solve_core(h, b, xd, false, true, sub_into);
        }
    }
    return UNO_KKT_OK;
}

// The row -> front-row index of launch_resid, built on the first refinement of a structure: the front rows
// (f, q) that hold a slot of their row (q is one of the slot's two local indices), per row in front order.
// Not applicable (the COO symv then): fronts with more than kSweepBigSlots slots (one wave would take them
// alone), fronts beyond the sweeps' LDS, or more front rows than int32 positions.
int build_resid_index(uno_kkt_t h) {
    Symbolic& S = h->S;
    hipStream_t s = h->stream;
    const int64_t nr = (int64_t)S.rows.size();
    bool ok = h->resid_fronts != 0 && S.max_m <= kMaxSweepFront && nr < INT32_MAX && S.n < INT32_MAX;
    for (int64_t f = 0; ok && f < S.nf; ++f) ok = S.f_ent_off[f + 1] - S.f_ent_off[f] <= kSweepBigSlots;
    if (!ok) {
        h->rz_state = -1;
        return UNO_KKT_OK;
    }
    std::vector<uint8_t> act((size_t)std::max<int64_t>(nr, 1), 0);
    for (int64_t f = 0; f < S.nf; ++f) {
        const int64_t ro = S.f_rows_off[f];
        for (int64_t e = S.f_ent_off[f]; e < S.f_ent_off[f + 1]; ++e) {
            act[ro + (S.ent_lpos[e] >> 16)] = 1;
            act[ro + (S.ent_lpos[e] & 0x7fffu)] = 1;
        }
    }
    std::vector<int32_t> ptr((size_t)S.n + 1, 0);
    for (int64_t t = 0; t < nr; ++t)
        if (act[t]) ptr[S.rows[t] + 1]++;
    for (int64_t i = 0; i < S.n; ++i) ptr[i + 1] += ptr[i];
    std::vector<int32_t> pos((size_t)std::max<int32_t>(ptr[S.n], 1)), fill(ptr.begin(), ptr.end() - 1);
    for (int64_t t = 0; t < nr; ++t)  // t ascending = front ascending
        if (act[t]) pos[fill[S.rows[t]]++] = (int32_t)t;
    std::vector<int32_t> lr, coff(1, 0), crow;
    for (int64_t i = 0; i < S.n; ++i) {
        const int64_t len = ptr[i + 1] - ptr[i];
        if (len <= std::min<int64_t>(h->resid_long, kResidShort)) continue;
        const int32_t nc = (int32_t)((len + kResidChunk - 1) / kResidChunk);
        crow.insert(crow.end(), nc, (int32_t)lr.size());
        lr.push_back((int32_t)i);
        coff.push_back(coff.back() + nc);
    }
    HIPCHK(h, h->rz_ptr.upload(ptr, s));
    HIPCHK(h, h->rz_pos.upload(pos, s));
    HIPCHK(h, h->rz_part.alloc(std::max<int64_t>(nr, 1)));
    h->rz_n_long = (int32_t)lr.size();
    h->rz_n_chunks = (int64_t)crow.size();
    if (!lr.empty()) {
        HIPCHK(h, h->rz_long.upload(lr, s));
        HIPCHK(h, h->rz_chunk_off.upload(coff, s));
        HIPCHK(h, h->rz_chunk_row.upload(crow, s));
        HIPCHK(h, h->rz_chunk_part.alloc(h->rz_n_chunks));
    }
    HIPCHK(h, hipStreamSynchronize(s));  // the host vectors go out of scope
    h->rz_state = 1;
    return UNO_KKT_OK;
}

// r = A x - b (refinement residual): launch_resid over the fronts' slots, or the COO symv (r = -b, r += A x)
int resid_impl(uno_kkt_t h, const double* x, const double* b, double* r) {
    Symbolic& S = h->S;
    hipStream_t s = h->stream;
    if (h->rz_state == 0) {
        int rc = build_resid_index(h);
        if (rc != UNO_KKT_OK) return rc;
    }
    if (h->rz_state < 0 || h->resid_fronts == 0) {
        HIPCHK(h, launch_neg(b, r, S.n, s));
        return symv_impl(h, x, r, nullptr, nullptr);
    }
    if (!h->packed_valid) {
        HIPCHK(h, launch_pack(h->values_ptr, h->dup_ptr.p, h->dup_pos.p, h->slot_src.p, 0, S.nu, h->uval.p, s));
        if (h->slot_src.p) HIPCHK(h, launch_pack_multi(h->values_ptr, h->dup_ptr.p, h->dup_pos.p, h->multi_slots.p, h->n_multi, h->uval.p, s));
        h->packed_valid = true;
    }
    ResidArgs A;
    A.nf = S.nf; A.n = S.n; A.fm = h->fm.p; A.rows_off = h->rows_off.p; A.rows = h->rows.p; A.ent_off = h->ent_off.p;
    A.ent_lpos = h->ent_lpos.p; A.uval = h->uval.p; A.x = x; A.b = b; A.part = h->rz_part.p; A.rz_ptr = h->rz_ptr.p;
    A.rz_pos = h->rz_pos.p; A.r = r; A.max_m = (int)S.max_m;
    A.short_len = (int32_t)std::min<int64_t>(h->resid_long, kResidShort);
    if (h->rz_n_long > 0) {
        A.long_rows = h->rz_long.p; A.n_long = h->rz_n_long; A.chunk_off = h->rz_chunk_off.p;
        A.n_chunks = h->rz_n_chunks; A.chunk_row = h->rz_chunk_row.p; A.chunk_part = h->rz_chunk_part.p;
    }
    TimerScope t(h, KC_SYMV);
    HIPCHK(h, launch_resid(A, s));
    return UNO_KKT_OK;
}
}  // namespace

extern "C" {

int uno_kkt_solve(uno_kkt_t h, const double* rhs, double* x, int on_device) {
    if (!h || !rhs || !x) return UNO_KKT_ERR_ARG;
    if (!h->analyzed || (!h->factored && !h->factor_enqueued))
        return set_err(h, UNO_KKT_ERR_STATE, "solve before factorize");
    HIPCHK(h, hipSetDevice(h->device));
    Symbolic& S = h->S;
    hipStream_t s = h->stream;
    if (h->factor_enqueued) {  // the factorization is final only once checked (delays, null threshold)
        int rc = finish_factorization(h);
        if (rc != UNO_KKT_OK) return rc;
    }
    // iterative refinement when the last factorization accepted pivots below the threshold u (threshold
    // relaxation instead of delayed pivots, option delay_relaxed = 0): r = A x - b with the analysed COO
    // values (uno_kkt_symv), x -= A^-1 r
    const int refine = (h->world == 1 && h->st.pivots_relaxed > 0 && h->values_ptr) ? h->refine : 0;
    const double* b = rhs;
    double* xd = x;
    if (!on_device) {
        if (S.n > 0) HIPCHK(h, hipMemcpyAsync(h->bvec.p, rhs, S.n * sizeof(double), hipMemcpyHostToDevice, s));
        b = h->bvec.p;
        xd = h->xtmp.p;
    } else if (refine > 0 && rhs == x) {  // keep the right-hand side for the residuals
        if (S.n > 0) HIPCHK(h, hipMemcpyAsync(h->bvec.p, rhs, S.n * sizeof(double), hipMemcpyDeviceToDevice, s));
        b = h->bvec.p;
    }
    // with refinement the dataflow abort flag is read once, after the last correction (one host wait per
    // solve instead of one per solve_core); an abort redoes the solve and its refinement level by level
    auto refined_solve = [&](bool allow_df) -> int {
        int rc = solve_core(h, b, xd, allow_df, refine == 0);
        if (rc != UNO_KKT_OK) return rc;
        for (int it = 0; it < refine; ++it) {
            if ((rc = resid_impl(h, xd, b, h->rtmp.p)) != UNO_KKT_OK) return rc;  // r = A x - b
            if (h->refine_tol > 0.0) {
                // componentwise backward error omega = max_i |r_i| / (|A| |x| + |b|)_i; the step is skipped when
                // x already satisfies omega <= refine_tol (one extra |A| |x| product and a scalar read-back)
                if (h->atmp.n != (size_t)S.n) HIPCHK(h, h->atmp.alloc(std::max<int64_t>(S.n, 1)));
                if (!h->omega_d.p) HIPCHK(h, h->omega_d.alloc(1));
                if (S.n > 0) HIPCHK(h, hipMemsetAsync(h->atmp.p, 0, sizeof(double) * S.n, s));
                if ((rc = symv_impl(h, xd, h->atmp.p, nullptr, nullptr, true)) != UNO_KKT_OK) return rc;
                HIPCHK(h, launch_backward_error(h->rtmp.p, h->atmp.p, b, S.n, h->omega_d.p, s));
                unsigned long long bits = 0;
                HIPCHK(h, hipMemcpyAsync(&bits, h->omega_d.p, sizeof(bits), hipMemcpyDeviceToHost, s));
                HIPCHK(h, hipStreamSynchronize(s));
                double omega;
                memcpy(&omega, &bits, sizeof(omega));
                h->st.last_backward_error = omega;
                if (omega <= h->refine_tol) { h->st.refinements_skipped++; break; }
            }
            // x -= A^-1 r (the subtraction fused into the solve's write-out)
            if ((rc = solve_core(h, h->rtmp.p, h->rtmp.p, allow_df, false, xd)) != UNO_KKT_OK) return rc;
            h->st.refinements++;
        }
        return UNO_KKT_OK;
    };
    // the statistics of a refined solve whose dataflow walk aborted are rolled back before the redo (its x, residual
    // and omega were computed from an x the aborted walk never wrote)
    const int64_t ref0 = h->st.refinements, refskip0 = h->st.refinements_skipped;
    const double omega0 = h->st.last_backward_error;
    int rc = refined_solve(true);
    if (rc != UNO_KKT_OK) return rc;
    if (refine > 0 && h->df_enabled && h->df_grid > 0) {
        HIPCHK(h, hipMemcpyAsync(h->h_counters + 10, h->df_abort.p, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
        HIPCHK(h, host_wait_stream(h, s));
        if (dataflow_aborted(h)) {
            if (h->df_abort.p) HIPCHK(h, hipMemsetAsync(h->df_abort.p, 0, sizeof(uint32_t), s));
            if (h->verbose) fprintf(stderr, "[uno_kkt] dataflow solve aborted: the refined solve redone level by level\n");
            h->st.refinements = ref0;
            h->st.refinements_skipped = refskip0;
            h->st.last_backward_error = omega0;
            if ((rc = refined_solve(false)) != UNO_KKT_OK) return rc;
        }
    }
    h->st.solves++;
    if (!on_device) {
        if (S.n > 0) HIPCHK(h, hipMemcpyAsync(x, xd, S.n * sizeof(double), hipMemcpyDeviceToHost, s));
        HIPCHK(h, hipStreamSynchronize(s));
    }
    return UNO_KKT_OK;
}

int uno_kkt_stats(uno_kkt_t h, uno_kkt_stats_t* out) {
    if (!h || !out) return UNO_KKT_ERR_ARG;
    if (h->factor_enqueued) {
        const int rc = finish_factorization(h);
        if (rc != UNO_KKT_OK && rc != UNO_KKT_ERR_PIVOT) return rc;
    }
    *out = h->st;
    out->fronts_merged = h->merges_total;
    out->solve_grid = h->df_enabled ? h->df_grid : 0;
    out->solve_aborts = h->df_aborts;
    out->factor_df_fronts = h->dff_level != INT32_MAX ? (int64_t)h->dff_order.n : 0;
    out->factor_df_aborts = h->dff_aborts;
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

// diagnostics (include/uno_kkt_debug.h): host-only analysis + subtree partition (no device needed)
int64_t uno_kkt_debug_partition(int64_t n, int64_t nnz, const int64_t* row, const int64_t* col, int world,
                                int32_t* owner, int32_t* parent, int64_t cap, int64_t* n_subtrees) {
    Pattern P;
    Symbolic S;
    if (!ukkt::analyze(n, nnz, row, col, AnalysisOptions(), P, S).empty()) return -1;
    Partition Pt;
    partition_tree(S, world, Pt);
    if (cap < S.nf) return -S.nf;
    for (int64_t f = 0; f < S.nf; ++f) { owner[f] = Pt.owner[f]; parent[f] = S.f_parent[f]; }
    if (n_subtrees) *n_subtrees = Pt.n_subtrees;
    return S.nf;
}

// diagnostics (include/uno_kkt_debug.h): the multi-GPU gate of uno_kkt_analyze on a pattern (no device)
int uno_kkt_debug_partition_gate(int64_t n, int64_t nnz, const int64_t* row, const int64_t* col, int world,
                                 double min_efficiency, double* efficiency, int64_t* n_subtrees) {
    Pattern P;
    Symbolic S;
    if (!ukkt::analyze(n, nnz, row, col, AnalysisOptions(), P, S).empty()) return -1;
    Partition Pt;
    partition_tree(S, world, Pt);
    const double denom = (double)world * (Pt.max_rank_work + Pt.top_work);
    const double eff = denom > 0.0 ? Pt.total_work / denom : 0.0;
    if (efficiency) *efficiency = eff;
    if (n_subtrees) *n_subtrees = Pt.n_subtrees;
    return (world > 1 && Pt.n_subtrees >= world && eff >= min_efficiency) ? 1 : 0;
}

// diagnostics (include/uno_kkt_debug.h): host-only analysis, per front order / pivots / level
int64_t uno_kkt_debug_fronts(int64_t n, int64_t nnz, const int64_t* row, const int64_t* col, int32_t* fm, int32_t* fp,
                             int32_t* flevel, int64_t cap) {
    Pattern P;
    Symbolic S;
    AnalysisOptions opt;  // defaults; UNO_KKT_LEAF / UNO_KKT_BLOCK override them for layout studies
    if (const char* e = getenv("UNO_KKT_LEAF")) opt.leaf_size = std::max(1, atoi(e));
    if (const char* e = getenv("UNO_KKT_BLOCK")) opt.max_block = std::max(1, atoi(e));
    if (!ukkt::analyze(n, nnz, row, col, opt, P, S).empty()) return -1;
    if (cap < S.nf) return -S.nf;
    for (int64_t f = 0; f < S.nf; ++f) { fm[f] = S.f_m[f]; fp[f] = S.f_p[f]; flevel[f] = S.f_level[f]; }
    return S.nf;
}

// diagnostics (include/uno_kkt_debug.h): per-front phase stamps of the last factorization
int64_t uno_kkt_debug_stamps(uno_kkt_t h, uint64_t* out, int64_t cap, int32_t* fm, int32_t* fp, int32_t* flevel) {
    if (!h || !h->stamps.p) return -1;
    if (h->factor_enqueued) {
        const int rc = finish_factorization(h);
        if (rc != UNO_KKT_OK && rc != UNO_KKT_ERR_PIVOT) return rc;  // a device / runtime failure is reported
    }
    int64_t nf = h->S.nf;
    if (cap < 8 * nf) return -(8 * nf);
    if (hipMemcpy(out, h->stamps.p, sizeof(uint64_t) * 8 * nf, hipMemcpyDeviceToHost) != hipSuccess)
        return set_err(h, UNO_KKT_ERR_HIP, "stamps copy failed");
    for (int64_t f = 0; f < nf; ++f) { fm[f] = h->S.f_m[f]; fp[f] = h->S.f_p[f]; flevel[f] = h->S.f_level[f]; }
    return nf;
}

// diagnostics: per front {fwd start, dependency met, staged, published, bwd ...} of the last dataflow solve
int64_t uno_kkt_debug_solve_stamps(uno_kkt_t h, uint64_t* out, int64_t cap) {
    if (!h || !h->df_stamps.p) return -1;
    const int64_t nf = h->S.nf;
    if (cap < 8 * nf) return -(8 * nf);
    HIPCHK(h, hipStreamSynchronize(h->stream));
    HIPCHK(h, hipMemcpy(out, h->df_stamps.p, sizeof(uint64_t) * 8 * nf, hipMemcpyDeviceToHost));
    return nf;
}

int64_t uno_kkt_debug_front_info(uno_kkt_t h, int32_t* fm, int32_t* fp, int32_t* flevel, int64_t cap) {
    if (!h) return -1;
    const int64_t nf = h->S.nf;
    if (cap < nf) return -nf;
    for (int64_t f = 0; f < nf; ++f) { fm[f] = h->S.f_m[f]; fp[f] = h->S.f_p[f]; flevel[f] = h->S.f_level[f]; }
    return nf;
}

int uno_kkt_debug_scaling(uno_kkt_t h, double* scale, double* anorm) {
    if (!h || !scale || !anorm) return UNO_KKT_ERR_ARG;
    if (h->factor_enqueued) {
        const int rc = finish_factorization(h);
        if (rc != UNO_KKT_OK && rc != UNO_KKT_ERR_PIVOT) return rc;
    }
    if (!h->factored && h->st.factorizations == 0) return set_err(h, UNO_KKT_ERR_STATE, "no factorization");
    HIPCHK(h, hipSetDevice(h->device));
    if (h->world == 1 && !h->norm_valid && h->scan.n > 0) {  // skipped by the bound: compute it now
        if (h->use_front_sweeps) HIPCHK(h, launch_rowsum_norm_orig(h->scan, h->rowsum.p, h->stream));
        else HIPCHK(h, launch_rowsum_norm(h->scan, h->rowsum.p, h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
        h->norm_valid = true;
    }
    if (h->S.n > 0) HIPCHK(h, hipMemcpy(scale, h->scale.p, sizeof(double) * h->S.n, hipMemcpyDeviceToHost));
    unsigned long long b = 0;
    HIPCHK(h, hipMemcpy(&b, h->anorm_p, sizeof(b), hipMemcpyDeviceToHost));
    memcpy(anorm, &b, sizeof(b));
    return UNO_KKT_OK;
}

const char* uno_kkt_last_error(uno_kkt_t h) { return h ? h->err.c_str() : "null handle"; }

// ---- device-side vector work around the solve ----
int uno_kkt_rhs_setup(uno_kkt_t h, int64_t n_vars, int64_t n_cons, int64_t nnz_jac, const int64_t* jac_con,
                      const int64_t* jac_var) {
    if (!h || n_vars < 0 || n_cons < 0 || nnz_jac < 0 || (nnz_jac > 0 && (!jac_con || !jac_var))) return UNO_KKT_ERR_ARG;
    HIPCHK(h, hipSetDevice(h->device));
    std::vector<int64_t> ptr(n_vars + 1, 0);
    std::vector<int32_t> con(nnz_jac);
    for (int64_t e = 0; e < nnz_jac; ++e) {
        if (jac_con[e] < 0 || jac_con[e] >= n_cons || jac_var[e] < 0 || jac_var[e] >= n_vars)
            return set_err(h, UNO_KKT_ERR_ARG, "Jacobian index out of range");
        ptr[jac_var[e] + 1]++;
        con[e] = (int32_t)jac_con[e];
    }
    for (int64_t i = 0; i < n_vars; ++i) ptr[i + 1] += ptr[i];
    // per variable, entries in ascending (constraint, position): the reference's accumulation order
    std::vector<int32_t> ent(nnz_jac);
    {
        std::vector<int64_t> fill(ptr.begin(), ptr.end() - 1);
        std::vector<int32_t> order(nnz_jac);
        for (int64_t e = 0; e < nnz_jac; ++e) order[e] = (int32_t)e;
        std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) { return jac_con[a] < jac_con[b]; });
        for (int32_t e : order) ent[fill[jac_var[e]]++] = e;
    }
    hipStream_t s = h->stream;
    HIPCHK(h, h->jv_ptr.upload(ptr, s));
    HIPCHK(h, h->jv_ent.upload(ent, s));
    HIPCHK(h, h->j_con.upload(con, s));
    std::vector<int32_t> lv;  // variables in more than kRhsLong constraints (k_rhs_long)
    for (int64_t i = 0; i < n_vars; ++i)
        if (ptr[i + 1] - ptr[i] > kRhsLong) lv.push_back((int32_t)i);
    h->rhs_n_long = (int32_t)lv.size();
    if (!lv.empty()) HIPCHK(h, h->rhs_long.upload(lv, s));
    HIPCHK(h, hipStreamSynchronize(s));
    h->rhs_n = n_vars;
    h->rhs_m = n_cons;
    return UNO_KKT_OK;
}

int uno_kkt_barrier_setup(uno_kkt_t h, int64_t n_vars, const double* lb, const double* ub) {
    if (!h || n_vars < 0 || (n_vars > 0 && (!lb || !ub))) return UNO_KKT_ERR_ARG;
    HIPCHK(h, hipSetDevice(h->device));
    std::vector<int32_t> var;
    std::vector<int8_t> which;
    for (int64_t i = 0; i < n_vars; ++i) {  // is_finite (uno/tools/Infinity.hpp): |b| < INF
        const int8_t w = (int8_t)((std::fabs(lb[i]) < INFINITY ? 1 : 0) | (std::fabs(ub[i]) < INFINITY ? 2 : 0));
        if (w) { var.push_back((int32_t)i); which.push_back(w); }
    }
    hipStream_t s = h->stream;
    HIPCHK(h, h->bar_var.upload(var, s));
    HIPCHK(h, h->bar_which.upload(which, s));
    HIPCHK(h, h->bar_lb.alloc(std::max<int64_t>(n_vars, 1)));
    HIPCHK(h, h->bar_ub.alloc(std::max<int64_t>(n_vars, 1)));
    if (n_vars > 0) {
        HIPCHK(h, hipMemcpyAsync(h->bar_lb.p, lb, sizeof(double) * n_vars, hipMemcpyHostToDevice, s));
        HIPCHK(h, hipMemcpyAsync(h->bar_ub.p, ub, sizeof(double) * n_vars, hipMemcpyHostToDevice, s));
    }
    HIPCHK(h, hipStreamSynchronize(s));
    h->bar_n = (int64_t)var.size();
    return UNO_KKT_OK;
}

int64_t uno_kkt_barrier_count(uno_kkt_t h) { return h ? h->bar_n : -1; }

int uno_kkt_assemble_barrier(uno_kkt_t h, const double* x, const double* zl, const double* zu, double* values) {
    if (!h || !x || !zl || !zu || !values) return UNO_KKT_ERR_ARG;
    if (h->bar_n < 0) return set_err(h, UNO_KKT_ERR_STATE, "assemble_barrier before barrier_setup");
    HIPCHK(h, hipSetDevice(h->device));
    HIPCHK(h, launch_barrier(h->bar_var.p, h->bar_which.p, h->bar_lb.p, h->bar_ub.p, x, zl, zu, h->bar_n, values, h->stream));
    return UNO_KKT_OK;
}

int uno_kkt_augmented_setup(uno_kkt_t h, int64_t reg_size, int64_t nnz_hess, int64_t nnz_jac) {
    if (!h || reg_size < 0 || nnz_hess < 0 || nnz_jac < 0) return UNO_KKT_ERR_ARG;
    if (h->bar_n < 0) return set_err(h, UNO_KKT_ERR_STATE, "augmented_setup before barrier_setup");
    if (h->analyzed && reg_size + nnz_hess + h->bar_n + nnz_jac != h->S.nnz)
        return set_err(h, UNO_KKT_ERR_ARG, "augmented layout (" + std::to_string(reg_size + nnz_hess + h->bar_n + nnz_jac) +
                                               " entries) differs from the analysed pattern (" + std::to_string(h->S.nnz) + ")");
    h->aug_reg = reg_size;
    h->aug_nh = nnz_hess;
    h->aug_nj = nnz_jac;
    return UNO_KKT_OK;
}

int uno_kkt_assemble_augmented(uno_kkt_t h, double hess_scale, const double* hess, const double* jac, const double* x,
                               const double* zl, const double* zu, double* values) {
    if (!h || !values) return UNO_KKT_ERR_ARG;
    if (h->aug_reg < 0) return set_err(h, UNO_KKT_ERR_STATE, "assemble_augmented before augmented_setup");
    if ((h->aug_nh > 0 && !hess) || (h->aug_nj > 0 && !jac) || (h->bar_n > 0 && (!x || !zl || !zu)))
        return UNO_KKT_ERR_ARG;
    HIPCHK(h, hipSetDevice(h->device));
    if (h->factor_enqueued && values == h->values_ptr) {  // the queued factorization's redos re-pack from these values
        const int rc = finish_factorization(h);
        if (rc != UNO_KKT_OK && rc != UNO_KKT_ERR_PIVOT) return rc;
    }
    // the layout is re-checked here: a barrier_setup with another bound count or a re-analysis after
    // augmented_setup would otherwise let the kernel write past the analysed value array
    if (h->analyzed && h->aug_reg + h->aug_nh + h->bar_n + h->aug_nj != h->S.nnz)
        return set_err(h, UNO_KKT_ERR_ARG, "augmented layout (" + std::to_string(h->aug_reg + h->aug_nh + h->bar_n + h->aug_nj) +
                                           " entries) does not match the analysed nnz " + std::to_string(h->S.nnz));
    AugArgs A;
    A.reg = h->aug_reg; A.nh = h->aug_nh; A.nb = h->bar_n; A.nj = h->aug_nj;
    A.hscale = hess_scale; A.hess = hess; A.jac = jac;
    A.bvar = h->bar_var.p; A.bwhich = h->bar_which.p; A.lb = h->bar_lb.p; A.ub = h->bar_ub.p;
    A.x = x; A.zl = zl; A.zu = zu; A.values = values;
    HIPCHK(h, launch_assemble_augmented(A, h->stream));
    if (values == h->values_ptr) h->packed_valid = false;
    return UNO_KKT_OK;
}

int uno_kkt_assemble_rhs(uno_kkt_t h, const double* grad, const double* cons, const double* y, const double* jac_values,
                         double* rhs) {
    if (!h || !rhs) return UNO_KKT_ERR_ARG;
    if (h->rhs_n < 0) return set_err(h, UNO_KKT_ERR_STATE, "assemble_rhs before rhs_setup");
    HIPCHK(h, hipSetDevice(h->device));
    HIPCHK(h, launch_rhs(grad, cons, y, jac_values, h->jv_ptr.p, h->jv_ent.p, h->j_con.p, h->rhs_n, h->rhs_m, rhs,
                         h->stream, h->rhs_long.p, h->rhs_n_long, kRhsLong));
    return UNO_KKT_OK;
}

int uno_kkt_assemble_direction(uno_kkt_t h, int64_t n_vars, int64_t n_cons, const double* solution, const double* x,
                               const double* lb, const double* ub, const double* zl, const double* zu,
                               double barrier_parameter, double tau_min, double* dx, double* dy, double* dzl,
                               double* dzu, double* step_lengths) {
    if (!h || n_vars < 0 || n_cons < 0 || !step_lengths) return UNO_KKT_ERR_ARG;
    HIPCHK(h, hipSetDevice(h->device));
    if (!h->alpha.p) HIPCHK(h, h->alpha.alloc(2));
    DirArgs A;
    A.n = n_vars; A.m = n_cons; A.sol = solution; A.x = x; A.lb = lb; A.ub = ub; A.zl = zl; A.zu = zu;
    A.mu = barrier_parameter;
    A.tau = std::max(tau_min, 1.0 - barrier_parameter);  // PrimalDualInteriorPointProblem.cpp:183
    A.dx = dx; A.dy = dy; A.dzl = dzl; A.dzu = dzu; A.alpha = h->alpha.p;
    HIPCHK(h, launch_direction(A, h->stream));
    unsigned long long b[2];
    HIPCHK(h, hipMemcpyAsync(b, h->alpha.p, sizeof(b), hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    memcpy(step_lengths, b, sizeof(b));
    return UNO_KKT_OK;
}

}  // extern "C"

namespace {
int symv_impl(uno_kkt_t h, const double* x, double* y, const double* w, double* dot, bool absval) {
    if (!h->analyzed || !h->values_ptr) return set_err(h, UNO_KKT_ERR_STATE, "symv needs analysed pattern and values");
    if (h->world > 1) return set_err(h, UNO_KKT_ERR_STATE, "symv on a distributed handle");
    Symbolic& S = h->S;
    hipStream_t s = h->stream;
    if (h->factor_enqueued) {
        int rc = finish_factorization(h);
        if (rc != UNO_KKT_OK) return rc;
    }
    if (!h->packed_valid) {
        HIPCHK(h, launch_pack(h->values_ptr, h->dup_ptr.p, h->dup_pos.p, h->slot_src.p, 0, S.nu, h->uval.p, s));
        if (h->slot_src.p) HIPCHK(h, launch_pack_multi(h->values_ptr, h->dup_ptr.p, h->dup_pos.p, h->multi_slots.p, h->n_multi, h->uval.p, s));
        h->packed_valid = true;
    }
    SymvArgs A;
    A.n = S.n; A.perm = h->perm_d.p; A.cptr = h->cptr.p; A.rptr = h->rptr.p; A.rslot = h->rslot.p;
    A.ent_r = h->ent_r.p; A.ent_c = h->ent_c.p; A.uval = h->uval.p; A.x = x; A.y = y; A.dot_w = w;
    A.absval = absval ? 1 : 0;
    A.dot_part = nullptr;
    if (h->n_long > 0) {
        const int32_t nch = (int32_t)((h->max_long + kSymvChunk - 1) / kSymvChunk);
        const size_t need = (size_t)h->n_long * nch;
        if (h->symv_long_part.n < need) HIPCHK(h, h->symv_long_part.alloc(need));
        A.long_len = kLongRow; A.long_rows = h->long_rows.p; A.n_long = h->n_long; A.long_chunks = nch;
        A.long_part = h->symv_long_part.p;
    }
    if (w) {
        if (h->symv_part.n != (size_t)S.n) HIPCHK(h, h->symv_part.alloc(std::max<int64_t>(S.n, 1)));
        if (!h->dot_d.p) HIPCHK(h, h->dot_d.alloc(1 + kSumParts));
        A.dot_part = h->symv_part.p;
    }
    {
        TimerScope t(h, KC_SYMV);
        HIPCHK(h, launch_symv(A, h->dot_d.p, s));
    }
    if (w) {
        HIPCHK(h, hipMemcpyAsync(dot, h->dot_d.p, sizeof(double), hipMemcpyDeviceToHost, s));
        HIPCHK(h, hipStreamSynchronize(s));
    }
    return UNO_KKT_OK;
}

}  // namespace

extern "C" {

int uno_kkt_symv(uno_kkt_t h, const double* x, double* y) {
    if (!h || !x || !y) return UNO_KKT_ERR_ARG;
    HIPCHK(h, hipSetDevice(h->device));
    return symv_impl(h, x, y, nullptr, nullptr);
}

int uno_kkt_quadratic_product(uno_kkt_t h, const double* x, const double* y, double* result) {
    if (!h || !x || !y || !result) return UNO_KKT_ERR_ARG;
    HIPCHK(h, hipSetDevice(h->device));
    if (h->symv_tmp.n != (size_t)h->S.n) HIPCHK(h, h->symv_tmp.alloc(std::max<int64_t>(h->S.n, 1)));
    if (h->S.n > 0) HIPCHK(h, hipMemsetAsync(h->symv_tmp.p, 0, sizeof(double) * h->S.n, h->stream));
    return symv_impl(h, y, h->symv_tmp.p, x, result);  // x^T (A y)
}

// ---- distributed factorization ----
int uno_kkt_comm_unique_id(unsigned char id[128]) {
    if (!id) return UNO_KKT_ERR_ARG;
    return ukkt::rccl_unique_id(id) == 0 ? UNO_KKT_OK : UNO_KKT_ERR_HIP;
}

static int attach(uno_kkt_t h, ukkt::Transport* t) {
    delete h->comm;
    h->comm = h->comm_trace ? ukkt::make_tracing_transport(t) : t;
    if (h->comm_trace) install_order_probe(h);
    h->own_device = false;
    h->rank = h->comm_rank = t->rank();
    h->world = h->comm_world = t->size();
    h->analyzed = h->factored = h->factor_enqueued = false;
    return UNO_KKT_OK;
}

int uno_kkt_attach_rccl(uno_kkt_t h, const unsigned char id[128], int rank, int world) {
    if (!h || !id || world < 1 || rank < 0 || rank >= world) return UNO_KKT_ERR_ARG;
    std::string err;
    ukkt::Transport* t = ukkt::make_rccl_transport(id, rank, world, h->device, err);
    if (!t) return set_err(h, UNO_KKT_ERR_HIP, err);
    const int rc = attach(h, t);
    h->own_device = true;  // RCCL refuses two ranks on one GPU
    return rc;
}

int uno_kkt_group_create(uno_kkt_group_t* g, int world) {
    if (!g || world < 1) return UNO_KKT_ERR_ARG;
    *g = reinterpret_cast<uno_kkt_group_t>(ukkt::local_group_create(world));
    return UNO_KKT_OK;
}

void uno_kkt_group_destroy(uno_kkt_group_t g) { ukkt::local_group_destroy(reinterpret_cast<ukkt::LocalGroup*>(g)); }

int uno_kkt_attach_local(uno_kkt_t h, uno_kkt_group_t g, int rank) {
    if (!h || !g) return UNO_KKT_ERR_ARG;
    ukkt::Transport* t = ukkt::make_local_transport(reinterpret_cast<ukkt::LocalGroup*>(g), rank);
    if (!t) return set_err(h, UNO_KKT_ERR_ARG, "bad rank for local group");
    return attach(h, t);
}

int uno_kkt_attach_host(uno_kkt_t h, const uno_kkt_host_comm_t* comm, int rank, int world) {
    if (!h || !comm) return UNO_KKT_ERR_ARG;
    ukkt::HostComm cb{comm->ctx, comm->send, comm->recv, comm->group_end, comm->allreduce, comm->broadcast};
    ukkt::Transport* t = ukkt::make_host_transport(cb, rank, world);
    if (!t) return set_err(h, UNO_KKT_ERR_ARG, "incomplete host transport or bad rank");
    return attach(h, t);
}

int64_t uno_kkt_debug_comm_trace(uno_kkt_t h, int64_t* out, int64_t cap, int clear) {
    if (!h || !h->comm) return -1;
    std::vector<int64_t> rec;
    if (!ukkt::comm_trace_records(h->comm, rec, clear != 0)) return -1;
    const int64_t n = (int64_t)rec.size() / 4;
    if (out) memcpy(out, rec.data(), sizeof(int64_t) * (size_t)std::min<int64_t>(4 * n, std::max<int64_t>(cap, 0)));
    return n;
}

int uno_kkt_dist_info(uno_kkt_t h, uno_kkt_dist_info_t* out) {
    if (!h || !out) return UNO_KKT_ERR_ARG;
    memset(out, 0, sizeof(*out));
    out->rank = h->comm_rank;
    out->world = h->comm_world;
    out->partitioned = h->analyzed && h->world > 1;
    out->est_efficiency = h->dist_efficiency;
    if (h->world > 1 && h->analyzed) {
        const DistState& D = h->dist;
        out->subtrees = D.part.n_subtrees;
        out->top_fronts = D.part.n_top;
        out->my_fronts = D.my_fronts;
        out->own_rows = D.n_own;
        out->top_rows = D.n_top_rows;
        out->my_flops = D.my_flops;
        out->top_flops = D.top_flops;
        out->est_imbalance = D.part.total_work > 0 ? D.part.max_rank_work * h->world / D.part.total_work : 1.0;
    }
    return UNO_KKT_OK;
}

}  // extern "C"
