// kkt_kernels.hpp -- device-argument structs and launch wrappers of kkt_kernels.hip.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace ukkt {

// Per-front state of the blocked large-front factorization (kkt_kernels.hip k_big_*), by front id.
struct BigFrontState {
    int32_t k;          // next pivot position
    int32_t k0, k1;     // pivots of the last panel: [k0, k1) (its trailing update is applied by k_big_update)
    int32_t done;
    int32_t npos, nneg, nzero, n2, nrel, nstuck, delays, pad;
    int32_t exact;      // a-posteriori step (FactorArgs::big_app) stopped at a failing column: the register
                        // panel's exact search runs next (k_big_panel_reg / k_big_panel), then clears it
    double minpiv;      // smallest pivot magnitude accepted as non-null
};

// a-posteriori blocked steps of the large fronts (k_app_*): kAppNB columns per step; per big front the
// global scratch holds, after its m x m front, the step's panel (m x kAppNB, row-major) and an AppSlot
constexpr int kAppNB = 64;
struct AppSlot {
    unsigned long long cmax[kAppNB];  // max |W(i, c)| over the rows below the diagonal (bits; atomic max); for a
                                      // 2x2 pair, over the rows below the pair
    double d[kAppNB];                 // the diagonal block's pivots (a 2x2 pair: its two diagonal entries)
    double offd[kAppNB];              // a 2x2 pair's off-diagonal entry (both columns)
    int8_t kind[kAppNB];              // PIV_1X1, PIV_2X2_A / PIV_2X2_B (pair with the next / previous column)
    int32_t k0, nbt, nacc, nb;        // first column, columns passing the in-block test, accepted, block width
    uint32_t arrive;                  // k_app_rows blocks done (the last one decides nacc)
    int32_t pad_[3];
};
constexpr int64_t kAppSlotDoubles = 208;
static_assert(sizeof(AppSlot) <= kAppSlotDoubles * sizeof(double), "AppSlot");

// Arguments of the front factorization kernels (device pointers, SoA per front).
struct FactorArgs {
    const int32_t* fm;          // front order
    const int32_t* fp;          // fully-summed columns
    const int64_t* rows_off;    // nf+1
    const int32_t* rows;        // original ids, analysis order
    const int64_t* ent_off;     // nf+1 packed slot ranges
    const uint32_t* ent_lpos;   // (lr << 16) | flip << 15 | lc (flip: scale the column's side first)
    const double* uval;         // packed summed values
    const double* scale;        // equilibration, by original id
    const double* fscale;       // the same gathered per front row (layout of rows; k_front_scale), or nullptr
    const int32_t* child_off;   // nf+1
    const int32_t* child;
    const int32_t* ch_cm;       // per child edge (aligned with child): contribution-block order
    const int64_t* ch_relmap_off;
    const int64_t* ch_cb_off;
    const int64_t* relmap_off;  // per front: cb rows into relmap / cvec
    const int32_t* relmap;
    const int64_t* L_off;
    const int64_t* cb_off;
    const int64_t* gscratch_off;  // per front, only used by k_factor_global
    const unsigned long long* anorm_bits;  // ||A_pre||_inf; nullptr = threshold 0 + minpiv record (norm overlapped)
    double* L;
    double* cb;
    double* gscratch;
    int32_t* frow;              // row ids after pivoting (same layout as rows)
    int32_t* fpos;              // analysis-order local row -> position after pivoting
    int8_t* piv;                // pivot kinds (same layout as rows)
    unsigned long long* counters;  // pos, neg, zero, 2x2, relaxed, stuck, delayed
    int32_t* fstat;             // per front: stuck pivots (low 16 bits) | relaxed pivots (high 16 bits)
    int32_t* fslow = nullptr;   // per front: pivot steps that left the register path (LDS search / interchange /
                                // 2x2 / null): the host launches such fronts first in their level (no level tail)
    unsigned long long* fcnt;   // per front: npos | nneg << 16 | nzero << 32 | n2x2 << 48 (summed by launch_count)
    double* fmin;               // per front: smallest pivot magnitude accepted as non-null (min by launch_count)
    const int32_t* fparent;     // assembly-tree parent (-1 = root)
    int32_t* delayed;           // original ids of columns that failed the threshold (counters[6] = count)
    int record_delays;
    unsigned long long* stamps;
    int stamp_mode;  // 1: phases + cycle counts, 2: write-out sub-phases in slots 4..7  // diagnostics (nullptr in normal runs): per front 8 words
    double u;
    double null_fac;
    // dataflow schedule of the upper tree (k_factor_df), after the level launches of the lower levels
    const int32_t* df_order;    // fronts, children before parents
    int32_t df_nf;
    const int32_t* df_nch;      // per front: children in the dataflow set
    uint32_t* df_cnt;           // per front: children arrived (cumulative: epoch * df_nch when complete)
    uint32_t df_epoch;          // 1, 2, ... per factorization since the counters were cleared
    uint32_t* df_ticket;        // block start order (cumulative: (epoch - 1) * df_nf at launch)
    uint32_t* df_abort;         // set when a wait exceeded its limit (factorization invalid, host redoes it)
    BigFrontState* big;         // per front: state of the blocked large-front factorization (m > kMaxLdsFront)
    const uint16_t* cbpos = nullptr;  // per contribution-block entry (layout of cb): its packed position in the
                                      // parent's LDS front (assemble_front without relmap gathers); nullptr: gathers
    int32_t* xpos = nullptr;        // one GPU, dataflow solve: xpos[row] = xs slot of each pivot (k_xpos pass 0)
    const int64_t* xs_off = nullptr;  // per front: its xs slot (DfArgs::xs_off)
};

struct SolveArgs {
    const int32_t* fm;
    const int32_t* fp;
    const int64_t* rows_off;
    const int32_t* frow;
    const int32_t* fpos;
    const int8_t* piv;
    const int32_t* child_off;
    const int32_t* child;
    const int64_t* relmap_off;
    const int32_t* relmap;
    const int64_t* L_off;
    const double* L;
    double* w;      // work vector by original id (scaled space)
    double* cvec;   // per-front update vectors (layout of relmap)
    const int32_t* ch_cm;          // per child edge (aligned with child): update-vector length
    const int64_t* ch_relmap_off;  // per child edge: offset into relmap / cvec
};

// Dataflow (one launch per direction) solve schedule, kkt_kernels.hip k_solve_fwd_df / k_solve_bwd_df
// walk-order front records of the dataflow solve: 16 int32 per position
// kDescNW: children whose arrival the front waits for (the forward walks' children; the flat levels solved by
// k_solve_fwd_flat before the walk are not counted)
enum : int { kDescF = 0, kDescM, kDescP, kDescPar, kDescC0, kDescC1, kDescRo = 6, kDescLo = 8, kDescCvx = 10, kDescXs = 12,
             kDescNW = 14 };
struct DfArgs {
    const int32_t* order;       // fronts, children before parents (the backward solve walks it from the end)
    const int32_t* desc;        // per walk position: 16-word record (kDesc* fields, 64-bit fields low word first)
    int32_t nf;
    const int32_t* parent;      // assembly-tree parent (-1 = root)
    uint32_t* cnt;              // forward: children arrived; epoch * children once all have (cumulative)
    uint32_t* done;             // backward: epoch of the front's last published solution
    uint32_t epoch;             // 1, 2, ... per solve since the counters were cleared
    double* cvx;                // forward update vectors, one 128-byte-aligned slot per front
    const int64_t* cvx_off;     // per front
    const int64_t* ch_cvx_off;  // per child edge (aligned with child)
    double* xs;                 // solution vector in elimination order: each front's pivots in a 128-byte-aligned slot
    const int64_t* xs_off;      // per front
    const int32_t* rxpos;       // per front row (layout of frow): xs index of the rows >= p
    const int32_t* rowx;        // per front row: xs slot of a walk front's pivot position, -2 its contribution rows, -1
    int64_t rows_total;         // length of rowx
    uint32_t* abort_flag;       // set when a wait exceeded its limit (result invalid, host falls back)
    int32_t win;                // LDS panel window (doubles, even, >= the longest column); rows follow it
    int32_t piv_off;            // LDS offset (doubles) of the 64 pivot-kind words, after the rows
    const int32_t* rg_desc;     // register kernels (k_solve_*_rg): the walk's fronts with p <= 32, m <= 72 (16 words each)
    int32_t rg_nf;
    const int32_t* ov_desc;     // ... the other fronts, same order, walked by the launch's last ov_grid blocks
    int32_t ov_nf, ov_grid;
    const int32_t* rgf_desc;    // forward register walk: rg_desc without its flat levels (option solve_flat_levels)
    int32_t rgf_nf;
    const int32_t* flat_desc;   // the flat levels' fronts, level by level: one k_solve_fwd_flat launch per level
    const int32_t* bdesc;       // the backward LDS-panel walk (k_solve_bwd_df): desc without the flat levels
    int32_t bnf;
    unsigned long long* stamps; // diagnostics (nullptr in normal runs): per front and direction 4 s_memrealtime
                                // words {start, dependency satisfied, values staged, published}
};

// row-wise scans for the equilibration and ||A_pre||_inf (kkt_kernels.hip k_rowscan)
struct ScanArgs {
    int64_t n;               // rows to scan (list entries, or rows 0..n-1 when list is null)
    const int32_t* list;     // optional row list (new numbering): a rank's own rows
    const int32_t* perm;     // new -> original
    const int32_t* cptr;     // n+1 column part of each row (contiguous slots)
    const int32_t* rptr;     // n+1 row part
    const int32_t* rslot;
    const int32_t* ent_r;    // slot -> original id of the later row
    const int32_t* ent_c;    // slot -> original id of the earlier column
    const double* uval;
    double* scale;           // by original id
    double* out;             // rmax or rowsum, by original id
    unsigned long long* anorm;
    const int32_t* long_rows;  // rows longer than kLongRow (new numbering)
    int32_t n_long;
    int64_t max_long;          // longest row length among long_rows
    int64_t long_chunks;       // chunks of the longest long row (row stride of part)
    double* part;              // n_long * long_chunks chunk results (combined in chunk order)
    // single GPU: row-major copy of |A| (k_rowscanR), double-buffered scaling sweeps in the new numbering
    double* uvalR;             // cptr[n] + rptr[n] entries, row i at [cptr[i] + rptr[i], cptr[i+1] + rptr[i+1])
    const int32_t* rowpartner; // same layout: (partner's new index << 1) | (row's original id > partner's)
    const double* scale_in;    // launch_scale_sweeps: second scratch buffer (n); in a sweep: the scaling read
    double* scale_out;         // launch_scale_sweeps: first scratch buffer (n), holds the final scaling after it
    uint32_t* long_cnt;        // per long row: chunk arrival counter (zero between launches)
};
constexpr int kLongRow = 2048;

// single-GPU equilibration sweeps over the fronts' packed slots (k_sweep_front): row maxima of a front's
// slots in LDS, merged over fronts with one atomic max per (front, row) -- rows longer than kLongRow
// (dense rows, present in every front) through per-front partials instead; scalings by original id.
struct SweepArgs {
    int64_t nf, n;
    const int32_t* fm;
    const int64_t* rows_off;
    const int32_t* rows;        // the fronts' rows, by new index (elimination order: rmax_all, longpos, long_orig too)
    const int32_t* perm;        // new index -> original id (k_sweep_final writes scale by original id)
    const int64_t* ent_off;     // nf+1 slot ranges
    const uint32_t* ent_lpos;   // (lr << 16) | flip << 15 | lc
    const double* values;       // caller's COO values (packed into uval by k_pack first)
    int64_t ent_total;          // packed slots
    const int32_t* dup_ptr;     // nullptr: one COO position per slot
    const int32_t* dup_pos;
    const int32_t* slot_src;    // single COO position per slot; < 0: record -1 - slot_src of `multi`
    const int32_t* multi;       // slots with several COO positions
    int64_t n_multi;
    double* uval;
    double* scale;              // by original id (written after the last sweep)
    unsigned long long* rmax_all;  // n per sweep (max(iters, 1) buffers), all zero on entry (left so on exit)
    unsigned long long* rmax;   // launch_front_sweeps: this sweep's buffer in rmax_all
    int iter = 0;               // launch_front_sweeps: this sweep's index
    const int8_t* longpos;      // by new index: index among the long rows, -1 otherwise
    const int32_t* long_orig;   // n_long new indices
    int32_t n_long;
    double* part_long;          // nf * n_long
    int max_m;
    int64_t rows_total = 0;     // front rows (length of rows / flong)
    const int8_t* flong = nullptr;  // per front row: longpos of its row (-1: not a long row); nullptr: no long rows
    const int32_t* big_list;    // fronts of more than kSweepBigSlots slots (swept by 2-D grids)
    int32_t n_big = 0, big_slices = 1;
    int rmax_zero = 0;  // rmax_all is known to be all zero (k_sweep_final leaves it so): no clearing memset
    unsigned long long* counters = nullptr;  // reset by the first sweep's block 0 (k_reset_counters' values:
                                             // one launch less at the head of the factorization)
};
hipError_t launch_front_sweeps(const SweepArgs& A, int iters, hipStream_t s, bool fused_pack = true);
hipError_t launch_pack_multi(const double* values, const int32_t* dup_ptr, const int32_t* dup_pos, const int32_t* multi,
                             int64_t count, double* uval, hipStream_t s);
// ||A_pre||_inf from the scaling by original id (row scans over the packed slots, no row-major copy)
hipError_t launch_rowsum_norm_orig(ScanArgs A, double* rowsum, hipStream_t s);
constexpr int kMaxSweepFront = 4096;  // largest front order of the front sweeps (LDS 16 B per row)
constexpr int64_t kSweepBigSlots = 16384;  // fronts with more slots are swept by slices (k_sweep_front<., true>)

// Residual r = A x - b of a refinement step (uno_kkt_solve after a factorization with relaxed pivots), over
// the fronts' packed slots instead of the row-wise COO symv (whose row halves gather every slot a second
// time, scattered): one wave per front accumulates its slots' products into the front's rows in LDS (one
// wave: a fixed order), writes one partial per front row, then each row sums its partials in front order
// (rz_ptr / rz_pos: the front rows that hold a slot of the row): 4 lanes per row up to kResidShort partials,
// longer rows (separator and dense rows) by chunks of kResidChunk partials, one wave each, whose sums are
// added in chunk order.  Deterministic.
struct ResidArgs {
    int64_t nf, n;
    const int32_t* fm;
    const int64_t* rows_off;
    const int32_t* rows;       // the fronts' rows by original id
    const int64_t* ent_off;    // nf+1 slot ranges
    const uint32_t* ent_lpos;  // (lr << 16) | flip << 15 | lc
    const double* uval;        // packed values (unscaled)
    const double* x;           // by original id
    const double* b;           // by original id
    double* part;              // one partial per front row
    const int32_t* rz_ptr;     // n+1, by original id
    const int32_t* rz_pos;     // front-row positions of each row's partials, ascending front
    int32_t short_len = 0;     // rows with more partials are chunked (kResidShort; smaller in tests)
    const int32_t* long_rows = nullptr;  // original ids of the chunked rows
    int32_t n_long = 0;
    const int32_t* chunk_off = nullptr;  // n_long+1: each chunked row's chunks
    int64_t n_chunks = 0;
    const int32_t* chunk_row = nullptr;  // per chunk: index among the chunked rows
    double* chunk_part = nullptr;        // per chunk: sum of its partials
    double* r;                 // out, by original id
    int max_m;
};
constexpr int kResidShort = 32;   // 4 lanes x 8 partials
constexpr int kResidChunk = 256;  // 64 lanes x 4 partials
hipError_t launch_resid(const ResidArgs& A, hipStream_t s);

// partial scans of the top (separator) rows on one rank: chunk c covers pslot[chunk_begin[c] ..
// chunk_begin[c+1]) of top row chunk_row[c]; ppartner = original id of the slot's other index
struct PartArgs {
    int64_t nchunks;
    const int32_t* chunk_row;
    const int64_t* chunk_begin;  // nchunks+1
    const int32_t* pslot;
    const int32_t* ppartner;
    const int32_t* trow_orig;    // top row t -> original id
    const double* uval;
    const double* scale;
    double* outT;                // per top row
    int64_t nrows;               // top rows
    const int64_t* row_chunk;    // nrows+1: chunks of top row t (consecutive in the chunk list)
    double* part;                // nchunks chunk results (combined in chunk order, no atomics)
};
constexpr int kLongChunk = 4096;

// pack slots [begin, end)
hipError_t launch_pack(const double* values, const int32_t* dup_ptr, const int32_t* dup_pos, const int32_t* slot_src, int64_t begin, int64_t end,
                       double* uval, hipStream_t s);
// single-GPU equilibration: `iters` max-scaling sweeps over all rows, then row sums and ||A_pre||_inf
hipError_t launch_scale(ScanArgs A, int iters, double* rmax, double* rowsum, hipStream_t s);
// the two halves of launch_scale: scaling sweeps (scale ready), then row sums + ||A_pre||_inf
hipError_t launch_scale_sweeps(ScanArgs A, int iters, double* rmax, hipStream_t s);
hipError_t launch_rowsum_norm(ScanArgs A, double* rowsum, hipStream_t s);
// building blocks of the distributed equilibration (mode 0: max |a|, 1: max |s a s|, 2: sum |s a s|)
hipError_t launch_rowscan(const ScanArgs& A, int mode, hipStream_t s);
hipError_t launch_rowscan_part(const PartArgs& A, int mode, hipStream_t s);
hipError_t launch_scale_update(const double* rmax, double* scale, const int32_t* list, int64_t n, int first, hipStream_t s);
hipError_t launch_normmax(const double* rowsum, const int32_t* list, int64_t n, unsigned long long* anorm, hipStream_t s);
hipError_t launch_scatter(const double* src, const int32_t* idx, double* dst, int64_t k, hipStream_t s);  // dst[idx[t]] = src[t]
hipError_t launch_gather(const double* src, const int32_t* idx, double* dst, int64_t k, hipStream_t s);   // dst[t] = src[idx[t]]
hipError_t launch_scatter64(const double* src, const int64_t* idx, double* dst, int64_t k, hipStream_t s);  // dst[idx[t]] = src[t]
hipError_t launch_neg(const double* b, double* r, int64_t n, hipStream_t s);  // r = -b
hipError_t launch_sub(double* x, const double* d, int64_t n, hipStream_t s);   // x -= d
size_t factor_lds_bytes(int mmax);
hipError_t launch_factor(const FactorArgs& A, const int32_t* fronts, int count, int mmax, bool global, hipStream_t s);
// one-wave solves (p <= 64, m <= kMaxLdsFront); lds_doubles >= max over the fronts of
// p*m - p*(p-1)/2 (rounded up to even) + m (rounded up to even) + m / 2 (int32 row positions)
hipError_t launch_solve_wave(const SolveArgs& A, const int32_t* fronts, int count, int lds_doubles, bool forward,
                             hipStream_t s);
// counters[0..5] = sums of the per-front pivot records (no same-address atomics inside the factor kernels)
hipError_t launch_count(const unsigned long long* fcnt, const int32_t* fstat, const double* fmin, int64_t nf,
                        unsigned long long* counters, unsigned long long* minbits, hipStream_t s,
                        const uint32_t* abort_word = nullptr, unsigned long long* host_out = nullptr,
                        unsigned long long seq = 0);  // seq != 0: written to host_out[10] after the rest (host poll)
// the factorization's device counter block: [0..7] pivot counters, [8] min pivot bits, [9] ||A_pre||_inf bits
constexpr int kCounterSlots = 11;  // [10]: k_count's block ticket (host_out)
hipError_t launch_reset_counters(unsigned long long* counters, hipStream_t s);
// fscale[t] = scale[rows[t]] for every front row t (one gather after the equilibration: the front assembly then
// loads its rows' scalings in the same round trip as the row ids instead of after them)
hipError_t launch_front_scale(const int32_t* rows, const double* scale, double* fscale, int64_t total, hipStream_t s);
hipError_t launch_rhs_scale(const double* b, const double* scale, double* w, int64_t n, hipStream_t s);
hipError_t launch_unscale(const double* w, const double* scale, double* x, int64_t n, hipStream_t s);
hipError_t launch_solve(const SolveArgs& A, const int32_t* fronts, int count, int mmax, int pmax, bool forward,
                        hipStream_t s);

// blocked large fronts (m > kMaxLdsFront): assemble, then (panel + MFMA trailing update) steps until
// launch_big_pending reports no front still factoring, then finish (L, CB, row maps, counters)
hipError_t launch_big_assemble(const FactorArgs& A, const int32_t* fronts, int count, int mmax, int maxch, hipStream_t s);
hipError_t launch_big_step(const FactorArgs& A, const int32_t* fronts, int count, int mmax, hipStream_t s);
hipError_t launch_big_pending(const FactorArgs& A, const int32_t* fronts, int count, int32_t* out, hipStream_t s);
hipError_t launch_big_finish(const FactorArgs& A, const int32_t* fronts, int count, int mmax, hipStream_t s);
int big_panel_width();  // pivots per panel step of the large-front launches

// dataflow factorization of the upper tree (one-wave fronts, m <= 64)
hipError_t launch_factor_df(const FactorArgs& A, int mmax, hipStream_t s);
// dataflow solve: one resident grid of one-wave blocks per direction (grid from the occupancy query)
int solve_df_grid(int lds_doubles, int nf);
int solve_slack_doubles();
// register-resident dataflow solve (same DfArgs walk and hand-offs as launch_solve_df; p <= 64, m <= 128)
int solve_rg_grid(bool forward, int nf, int waves_per_simd);  // waves_per_simd: 3 or 4 (the kernel variant)
hipError_t launch_solve_bwd_w2(const SolveArgs& A, const int32_t* fronts, int count, hipStream_t s);
hipError_t launch_solve_rg(const SolveArgs& A, const DfArgs& D, int grid, bool forward, int waves_per_simd, hipStream_t s);
// the forward of the flat level's fronts DfArgs::flat_desc[begin, begin + count), one wave each, before the walk
hipError_t launch_solve_fwd_flat(const SolveArgs& A, const DfArgs& D, int begin, int count, hipStream_t s);
// the backward of the flat level's fronts, one wave each, after the backward walk (LDS: the walk's lds_doubles)
hipError_t launch_solve_bwd_flat(const SolveArgs& A, const DfArgs& D, int begin, int count, int lds_doubles, hipStream_t s);
hipError_t launch_solve_df(const SolveArgs& A, const DfArgs& D, int grid, int lds_doubles, bool forward, hipStream_t s);
// rxpos for the dataflow backward solve (after every factorization); xpos: n int32 scratch.  Distributed
// runs: the walk is the rank's own fronts, and the top rows (top_orig, eliminated on rank 0) get the
// slots top_base + t of xs, where the broadcast top solution is copied before the backward launch
hipError_t launch_xpos(const SolveArgs& A, const DfArgs& D, int32_t* xpos, int32_t* rxpos, const int32_t* top_orig,
                       int64_t n_top, int64_t top_base, hipStream_t s,
                       bool pass0 = true);
// xs[xpos[i]] = scale_i b_i  /  x_i = scale_i xs[xpos[i]]; rows i = list[0 .. n) (list == nullptr: 0 .. n-1)
hipError_t launch_xs_in(const double* b, const double* scale, const int32_t* xpos, double* xs, int64_t n, hipStream_t s,
                        const int32_t* list = nullptr);
// sub: x_i -= scale_i xs[xpos[i]] (a refinement correction, rounded as the product stored and subtracted)
hipError_t launch_xs_out(const double* xs, const double* scale, const int32_t* xpos, const uint32_t* abort_flag, double* x,
                         int64_t n, hipStream_t s, const int32_t* list = nullptr, bool sub = false);
// distributed dataflow solve: subtree roots' update vectors (cvx slots) -> cvec (level-schedule layout,
// sent to rank 0); done[f] = epoch for the top fronts (the subtree roots' parents) before the backward
hipError_t launch_cvx_to_cvec(const DfArgs& D, const SolveArgs& A, const int32_t* roots, int count, double* cvec, hipStream_t s);
hipError_t launch_set_done(uint32_t* done, const int32_t* list, int count, uint32_t epoch, hipStream_t s);

constexpr int kMaxLdsFront = 128;
constexpr int kMaxWaveFront = 72;     // one-wave register-resident factorization (8 x 8 lane grid, 9 row blocks)     // fronts up to this order factor entirely in LDS
constexpr int kMaxGlobalFront = 8192; // larger fronts are rejected at analysis

}  // namespace ukkt
