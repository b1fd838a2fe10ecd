// analysis.hpp -- host-side symbolic analysis for the MI355X KKT backend.
//
// Replaces the symbolic phase Uno delegates to MUMPS JOB=1
// (uno/ingredients/subproblem_solvers/MUMPS/MUMPSSolver.cpp:72-83): canonicalises the COO pattern
// that uno/linear_algebra/COOFormat.hpp produces (duplicates, either triangle), orders it with
// nested dissection (dense "arrow" rows last), groups columns into supernodes, and lays out every
// device array the numerical phase reads: packed value slots per front, front row lists, extend-add
// maps, factor / contribution-block arenas and the level schedule.  Runs once per pattern
// (contract invariant 1 of SURVEY.md 8(b)).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace ukkt {

struct AnalysisOptions {
    int leaf_size = 32;   // nested-dissection leaf (nodes)
    int max_block = 64;   // widest supernode (fully-summed columns per front)
    // a group (separator / dense rows) longer than wide_group columns has fronts beyond the LDS kernels
    // anyway: it is cut into blocks of at most wide_block columns instead of max_block, so the large-front
    // path factors it as one front in panels instead of a chain of max_block-column fronts, each copying
    // the whole remaining group as its contribution block
    int wide_group = 128;
    int wide_block = 4096;
    double dense_factor = 10.0;  // dense node: degree > max(16, dense_factor * sqrt(n))
};

// Canonical pattern + graph + ordering, kept for the lifetime of an analysis so the supernode
// structure can be rebuilt when fronts are amalgamated after a failed pivot (delayed pivots).
struct Pattern {
    int64_t n = 0, nnz = 0, nu = 0;
    std::vector<int32_t> ur, uc;            // unique entries (ur >= uc), original numbering
    std::vector<int32_t> udp;               // nu+1: range into pos_sorted
    std::vector<int32_t> pos_sorted;        // COO positions grouped by unique entry, ascending
    std::vector<int64_t> ap;                // adjacency (no diagonal)
    std::vector<int32_t> ai;
    std::vector<int32_t> perm;              // nested-dissection order (new -> original)
    std::vector<int32_t> bfirst;            // supernode boundaries in the new order (nb+1)
    std::vector<uint8_t> delay_count;       // per original variable: times its pivot was delayed
    int64_t n_dense = 0;
};

struct Symbolic {
    int64_t n = 0, nnz = 0, nu = 0;
    // packed value slots: slot s holds unique entry (ent_r[s], ent_c[s]) in original numbering,
    // its value is the sum of COO positions dup_pos[dup_ptr[s] .. dup_ptr[s+1])
    bool identity_dups = false;        // every unique entry has exactly one COO position
    std::vector<int32_t> dup_ptr, dup_pos;
    std::vector<int32_t> ent_r, ent_c; // original ids, ent_r is the later-eliminated one
    std::vector<uint32_t> ent_lpos;    // (local row << 16) | flip << 15 | local col inside the owning front
                                       // (flip: the column has the larger original id)
    // row-wise access to the packed slots (new numbering) for atomic-free equilibration:
    // column part of row i = slots [cptr[i], cptr[i+1]) (entries (r, i), r >= i, contiguous),
    // row part = rslot[rptr[i] .. rptr[i+1]) (entries (i, c), c < i)
    std::vector<int32_t> cptr, rptr, rslot;
    std::vector<int32_t> rowpartner;   // row-major symmetric layout: (partner new index << 1) | order flag (k_rowscanR)
    // ordering (new index -> original index and inverse)
    std::vector<int32_t> perm, iperm;
    int64_t n_dense = 0;
    // fronts (supernodes), children have smaller ids than parents
    int64_t nf = 0;
    std::vector<int32_t> f_m, f_p, f_parent, f_level;
    std::vector<int64_t> f_rows_off;   // nf+1, into rows
    std::vector<int32_t> rows;         // original ids: fully-summed columns then struct rows
    std::vector<int64_t> f_ent_off;    // nf+1, packed slot ranges
    std::vector<int32_t> f_child_off;  // nf+1, into child
    std::vector<int32_t> child;
    std::vector<int64_t> f_relmap_off; // per front (as a child): cb_m entries into relmap
    std::vector<int32_t> relmap;       // contribution-block row -> parent local row
    std::vector<int64_t> f_L_off;      // packed lower trapezoid, m x p, column-major
    std::vector<int64_t> f_cb_off;     // packed lower triangle, (m-p) x (m-p), column-major
    int64_t L_size = 0, cb_size = 0, nnz_L = 0;
    double flops = 0.0;
    int64_t max_m = 0;
    int nlevels = 0;
    std::vector<int32_t> level_off;    // nlevels+1
    std::vector<int32_t> level_fronts; // fronts by level, each level sorted by m descending
};

// Canonicalise + order.  Returns "" on success, an error message otherwise.
std::string order_pattern(int64_t n, int64_t nnz, const int64_t* row, const int64_t* col,
                          const AnalysisOptions& opt, Pattern& P);
// Supernodal structure / device layout for the ordering and boundaries held in P.
std::string build_structure(const Pattern& P, Symbolic& S);
// Amalgamate every front flagged in `merge` into its parent (its columns are moved to just before
// the parent's, i.e. their pivots are delayed to the parent).  Returns the number merged.
int64_t amalgamate(Pattern& P, const Symbolic& S, const std::vector<char>& merge);
// Delayed pivots at column granularity: every listed column (original id) whose front has a parent
// is moved into its parent's block (eliminated just before the parent's own columns); a column
// delayed for the second time goes straight to the root of its tree (one rebuild instead of one per
// level of a cascade).
int64_t delay_columns(Pattern& P, const Symbolic& S, const std::vector<int32_t>& delayed_vars);

// Subtree partition of the assembly tree over `world` ranks: the top of the tree is
// cut until the remaining subtrees can be packed onto the ranks with a small makespan; every subtree
// is factored by one rank without communication, the cut-off top fronts by rank 0 after the subtree
// roots' contribution blocks arrive.  Deterministic: every rank computes the same partition.
struct Partition {
    int world = 1;
    std::vector<int32_t> owner;       // per front: rank, or -1 for a top front (rank 0, after the exchange)
    std::vector<int32_t> send_roots;  // subtree roots whose parent is a top front
    std::vector<int32_t> root_rank;   // rank owning send_roots[k]
    int64_t n_subtrees = 0, n_top = 0;
    double total_work = 0.0, top_work = 0.0, max_rank_work = 0.0;
};
void partition_tree(const Symbolic& S, int world, Partition& out);

inline std::string analyze(int64_t n, int64_t nnz, const int64_t* row, const int64_t* col,
                           const AnalysisOptions& opt, Pattern& P, Symbolic& S) {
    std::string e = order_pattern(n, nnz, row, col, opt, P);
    return e.empty() ? build_structure(P, S) : e;
}

}  // namespace ukkt
