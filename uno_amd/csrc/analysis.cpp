// analysis.cpp -- host symbolic analysis: canonical pattern, nested dissection, supernodes,
// assembly tree, device layout.  See analysis.hpp and DESIGN.md section 3.
#include "analysis.hpp"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <numeric>

namespace ukkt {
namespace {

struct Graph {
    int32_t n = 0;
    std::vector<int64_t> ap;
    std::vector<int32_t> ai;
};

// Nested dissection by BFS level-set separators (George's automatic ND) on the non-dense subgraph.
// Emits groups in postorder: [ND(A)] [ND(B)] [separator]; each group becomes >= 1 supernode.
class Dissector {
public:
    Dissector(const Graph& g, const std::vector<char>& skip, int leaf)
        : g_(g), skip_(skip), leaf_(leaf), mark_(g.n, -1), level_(g.n, 0), queue_(g.n) {}

    void run(std::vector<int32_t>& order, std::vector<int32_t>& group_start) {
        order_ = &order;
        groups_ = &group_start;
        std::vector<int32_t> all;
        all.reserve(g_.n);
        for (int32_t v = 0; v < g_.n; ++v)
            if (!skip_[v]) all.push_back(v);
        dissect(std::move(all));
        flush_pending();
    }

private:
    const Graph& g_;
    const std::vector<char>& skip_;
    int leaf_;
    std::vector<int32_t> mark_, level_, queue_;
    int32_t stamp_ = 0;
    std::vector<int32_t>* order_ = nullptr;
    std::vector<int32_t>* groups_ = nullptr;
    std::vector<int32_t> pending_;  // small independent components merged into one leaf group

    void emit(const std::vector<int32_t>& nodes) {
        if (nodes.empty()) return;
        groups_->push_back((int32_t)order_->size());
        order_->insert(order_->end(), nodes.begin(), nodes.end());
    }
    void flush_pending() {
        if (!pending_.empty()) { emit(pending_); pending_.clear(); }
    }

    // BFS inside the set marked `member`; returns number of visited nodes, fills queue_/level_
    int32_t bfs(int32_t start, int32_t member, int32_t visit, int32_t& nlev) {
        int32_t head = 0, tail = 0;
        queue_[tail++] = start;
        mark_[start] = visit;
        level_[start] = 0;
        nlev = 1;
        while (head < tail) {
            int32_t v = queue_[head++];
            int32_t lv = level_[v] + 1;
            for (int64_t p = g_.ap[v]; p < g_.ap[v + 1]; ++p) {
                int32_t w = g_.ai[p];
                if (mark_[w] != member) continue;  // not in set, or already visited this sweep
                mark_[w] = visit;
                level_[w] = lv;
                if (lv + 1 > nlev) nlev = lv + 1;
                queue_[tail++] = w;
            }
        }
        return tail;
    }

    void dissect(std::vector<int32_t> S) {
        const int32_t sz = (int32_t)S.size();
        if (sz == 0) return;
        if (sz <= leaf_) {
            pending_.insert(pending_.end(), S.begin(), S.end());
            if ((int)pending_.size() >= leaf_) flush_pending();
            return;
        }
        // mark members, check connectivity
        int32_t member = ++stamp_;
        for (int32_t v : S) mark_[v] = member;
        int32_t nlev = 0;
        int32_t visit = ++stamp_;
        int32_t reached = bfs(S[0], member, visit, nlev);
        if (reached < sz) {
            // split into connected components; each is dissected independently
            std::vector<std::vector<int32_t>> comps;
            comps.emplace_back(queue_.begin(), queue_.begin() + reached);
            for (int32_t v : S) {
                if (mark_[v] != member) continue;
                int32_t vis = ++stamp_;
                int32_t cnt = bfs(v, member, vis, nlev);
                comps.emplace_back(queue_.begin(), queue_.begin() + cnt);
            }
            S.clear();
            S.shrink_to_fit();
            for (auto& c : comps) dissect(std::move(c));
            return;
        }
        flush_pending();
        // pseudo-peripheral node: farthest node of a sweep, lowest degree in the last level
        int32_t start = S[0];
        for (int it = 0; it < 2; ++it) {
            int32_t best = -1;
            for (int32_t q = 0; q < reached; ++q) {
                int32_t v = queue_[q];
                if (level_[v] != nlev - 1) continue;
                if (best < 0 || g_.ap[v + 1] - g_.ap[v] < g_.ap[best + 1] - g_.ap[best]) best = v;
            }
            for (int32_t v : S) mark_[v] = member;
            visit = ++stamp_;
            int32_t nl2 = 0;
            bfs(best, member, visit, nl2);
            bool improved = nl2 > nlev;
            start = best;
            nlev = nl2;
            if (!improved) break;
        }
        (void)start;
        if (nlev < 3) {  // no separating level: one (possibly wide) group
            emit(S);
            return;
        }
        std::vector<int32_t> cnt(nlev + 1, 0);
        for (int32_t v : S) cnt[level_[v]]++;
        int32_t acc = 0, lmed = 1;
        for (int32_t l = 0; l < nlev; ++l) {
            acc += cnt[l];
            if (2 * acc >= sz) { lmed = l; break; }
        }
        lmed = std::min(std::max(lmed, 1), nlev - 2);
        int32_t best = lmed;
        for (int32_t l = std::max(1, lmed - 3); l <= std::min(nlev - 2, lmed + 3); ++l)
            if (cnt[l] < cnt[best] || (cnt[l] == cnt[best] && std::abs(l - lmed) < std::abs(best - lmed)))
                best = l;
        const int32_t L = best;
        std::vector<int32_t> A, B, sep;
        A.reserve(sz / 2 + 1);
        B.reserve(sz / 2 + 1);
        for (int32_t v : S) {
            int32_t lv = level_[v];
            if (lv < L) A.push_back(v);
            else if (lv > L) B.push_back(v);
            else {
                // keep only separator nodes that touch the far side
                bool touches = false;
                for (int64_t p = g_.ap[v]; p < g_.ap[v + 1] && !touches; ++p) {
                    int32_t w = g_.ai[p];
                    touches = mark_[w] == visit && level_[w] == L + 1;
                }
                (touches ? sep : A).push_back(v);
            }
        }
        S.clear();
        S.shrink_to_fit();
        dissect(std::move(A));
        flush_pending();
        dissect(std::move(B));
        flush_pending();
        emit(sep);
    }
};

}  // namespace

std::string order_pattern(int64_t n, int64_t nnz, const int64_t* row, const int64_t* col,
                          const AnalysisOptions& opt, Pattern& P) {
    P = Pattern();
    if (n < 0 || nnz < 0) return "negative size";
    if (n >= (int64_t(1) << 30) || nnz >= (int64_t(1) << 31) - 1) return "n exceeds 2^30 or nnz exceeds int32 range";
    for (int64_t k = 0; k < nnz; ++k)
        if (row[k] < 0 || row[k] >= n || col[k] < 0 || col[k] >= n)
            return "COO entry " + std::to_string(k) + " out of range";
    P.n = n;
    P.nnz = nnz;
    const int32_t N = (int32_t)n;

    // ---- canonical lower pattern: bucket by min index, sort by (max index, position) ----
    std::vector<int64_t> bstart(n + 1, 0);
    for (int64_t k = 0; k < nnz; ++k) bstart[std::min(row[k], col[k]) + 1]++;
    for (int64_t i = 0; i < n; ++i) bstart[i + 1] += bstart[i];
    std::vector<std::pair<int32_t, int32_t>> pr(nnz);
    {
        std::vector<int64_t> fill(bstart.begin(), bstart.end() - 1);
        for (int64_t k = 0; k < nnz; ++k) {
            int64_t b = std::min(row[k], col[k]), a = std::max(row[k], col[k]);
            pr[fill[b]++] = {(int32_t)a, (int32_t)k};
        }
    }
    P.ur.reserve(nnz);
    P.uc.reserve(nnz);
    P.udp.reserve(nnz + 1);
    P.pos_sorted.resize(nnz);
    for (int64_t b = 0; b < n; ++b) {
        auto first = pr.begin() + bstart[b], last = pr.begin() + bstart[b + 1];
        if (last - first > 1) std::sort(first, last);
        for (auto it = first; it != last; ++it) {
            if (it == first || it->first != (it - 1)->first) {
                P.ur.push_back(it->first);
                P.uc.push_back((int32_t)b);
                P.udp.push_back((int32_t)(it - pr.begin()));
            }
            P.pos_sorted[it - pr.begin()] = it->second;
        }
    }
    P.nu = (int64_t)P.ur.size();
    P.udp.push_back((int32_t)nnz);
    const int64_t nu = P.nu;

    // ---- adjacency (no diagonal) ----
    P.ap.assign(n + 1, 0);
    for (int64_t u = 0; u < nu; ++u)
        if (P.ur[u] != P.uc[u]) { P.ap[P.ur[u] + 1]++; P.ap[P.uc[u] + 1]++; }
    for (int64_t i = 0; i < n; ++i) P.ap[i + 1] += P.ap[i];
    P.ai.resize(P.ap[n]);
    {
        std::vector<int64_t> pos(P.ap.begin(), P.ap.end() - 1);
        for (int64_t u = 0; u < nu; ++u)
            if (P.ur[u] != P.uc[u]) { P.ai[pos[P.ur[u]]++] = P.uc[u]; P.ai[pos[P.uc[u]]++] = P.ur[u]; }
    }
    Graph g;
    g.n = N;
    g.ap.swap(P.ap);
    g.ai.swap(P.ai);

    // ---- ordering: dense nodes last, nested dissection on the rest ----
    std::vector<char> dense(n, 0);
    const double dthr = std::max(16.0, opt.dense_factor * std::sqrt((double)n));
    for (int32_t v = 0; v < N; ++v)
        if ((double)(g.ap[v + 1] - g.ap[v]) > dthr) { dense[v] = 1; P.n_dense++; }
    std::vector<int32_t> order;
    order.reserve(n);
    std::vector<int32_t> group_start;
    Dissector(g, dense, std::max(1, opt.leaf_size)).run(order, group_start);
    if (P.n_dense) {
        group_start.push_back((int32_t)order.size());
        for (int32_t v = 0; v < N; ++v) if (dense[v]) order.push_back(v);
    }
    g.ap.swap(P.ap);
    g.ai.swap(P.ai);
    if ((int64_t)order.size() != n) return "internal: ordering is not a permutation";
    group_start.push_back(N);
    P.perm.swap(order);

    // ---- supernodes: each group cut into blocks of at most max_block (long groups: wide_block) columns ----
    for (size_t gi = 0; gi + 1 < group_start.size(); ++gi) {
        int32_t s = group_start[gi], e = group_start[gi + 1];
        int32_t len = e - s;
        if (len <= 0) continue;
        const int32_t wmax = len > opt.wide_group ? std::max(opt.max_block, opt.wide_block) : opt.max_block;
        int32_t nb = (len + wmax - 1) / wmax;
        for (int32_t b = 0; b < nb; ++b) P.bfirst.push_back(s + (int32_t)((int64_t)len * b / nb));
    }
    P.bfirst.push_back(N);
    return "";
}

std::string build_structure(const Pattern& P, Symbolic& S) {
    S = Symbolic();
    const int64_t n = P.n, nnz = P.nnz, nu = P.nu;
    S.n = n;
    S.nnz = nnz;
    S.nu = nu;
    S.n_dense = P.n_dense;
    S.perm = P.perm;
    S.iperm.assign(n, -1);
    for (int32_t q = 0; q < (int32_t)n; ++q) S.iperm[S.perm[q]] = q;
    const std::vector<int32_t>& bfirst = P.bfirst;
    const int32_t nf = (int32_t)bfirst.size() - 1;
    S.nf = nf;
    std::vector<int32_t> blk(n);
    for (int32_t b = 0; b < nf; ++b)
        for (int32_t j = bfirst[b]; j < bfirst[b + 1]; ++j) blk[j] = b;

    // ---- block symbolic factorization (struct = rows beyond the block, new numbering) ----
    std::vector<int64_t> soff(nf + 1, 0);
    std::vector<int32_t> sidx;
    S.f_parent.assign(nf, -1);
    std::vector<std::vector<int32_t>> children(nf);
    {
        std::vector<int32_t> mark(n, -1), buf;
        buf.reserve(1024);
        for (int32_t b = 0; b < nf; ++b) {
            const int32_t first = bfirst[b], last = bfirst[b + 1] - 1;
            buf.clear();
            for (int32_t j = first; j <= last; ++j) {
                int32_t v = S.perm[j];
                for (int64_t p = P.ap[v]; p < P.ap[v + 1]; ++p) {
                    int32_t i = S.iperm[P.ai[p]];
                    if (i > last && mark[i] != b) { mark[i] = b; buf.push_back(i); }
                }
            }
            for (int32_t c : children[b])
                for (int64_t q = soff[c]; q < soff[c + 1]; ++q) {
                    int32_t i = sidx[q];
                    if (i > last && mark[i] != b) { mark[i] = b; buf.push_back(i); }
                }
            std::sort(buf.begin(), buf.end());
            sidx.insert(sidx.end(), buf.begin(), buf.end());
            soff[b + 1] = (int64_t)sidx.size();
            if (!buf.empty()) {
                int32_t par = blk[buf[0]];
                S.f_parent[b] = par;
                children[par].push_back(b);
            }
        }
    }

    // ---- front descriptors ----
    S.f_m.resize(nf);
    S.f_p.resize(nf);
    S.f_level.assign(nf, 0);
    S.f_rows_off.assign(nf + 1, 0);
    S.f_L_off.assign(nf + 1, 0);
    S.f_cb_off.assign(nf + 1, 0);
    S.f_child_off.assign(nf + 1, 0);
    for (int32_t b = 0; b < nf; ++b) {
        int64_t p = bfirst[b + 1] - bfirst[b];
        int64_t m = p + (soff[b + 1] - soff[b]);
        if (m > 65535) return "front order exceeds 65535";
        if (p > 32767) return "supernode wider than 32767 columns";
        S.f_m[b] = (int32_t)m;
        S.f_p[b] = (int32_t)p;
        S.max_m = std::max<int64_t>(S.max_m, m);
        S.f_rows_off[b + 1] = S.f_rows_off[b] + m;
        S.f_L_off[b + 1] = S.f_L_off[b] + p * m - p * (p - 1) / 2;
        int64_t cm = m - p;
        // 128-byte-aligned blocks: no cache line holds two fronts' contribution blocks (the dataflow
        // factorization hands them over inside one launch, kkt_kernels.hip k_factor_df)
        S.f_cb_off[b + 1] = (S.f_cb_off[b] + cm * (cm + 1) / 2 + 15) & ~(int64_t)15;
        S.nnz_L += p * (m - p) + p * (p - 1) / 2;
        for (int64_t k = 0; k < p; ++k) {
            double r = (double)(m - k - 1);
            S.flops += r + r * (r + 1.0);
        }
        for (int32_t c : children[b]) S.f_level[b] = std::max(S.f_level[b], S.f_level[c] + 1);
        S.f_child_off[b + 1] = S.f_child_off[b] + (int32_t)children[b].size();
    }
    S.L_size = S.f_L_off[nf];
    S.cb_size = S.f_cb_off[nf];
    S.rows.resize(S.f_rows_off[nf]);
    for (int32_t b = 0; b < nf; ++b) {
        int64_t o = S.f_rows_off[b];
        for (int32_t j = bfirst[b]; j < bfirst[b + 1]; ++j) S.rows[o++] = S.perm[j];
        for (int64_t q = soff[b]; q < soff[b + 1]; ++q) S.rows[o++] = S.perm[sidx[q]];
    }
    S.child.reserve(S.f_child_off[nf]);
    for (int32_t b = 0; b < nf; ++b) S.child.insert(S.child.end(), children[b].begin(), children[b].end());

    // local row of new index i inside front b
    auto local_row = [&](int32_t b, int32_t i) -> int32_t {
        if (i >= bfirst[b] && i < bfirst[b + 1]) return i - bfirst[b];
        auto first = sidx.begin() + soff[b], last = sidx.begin() + soff[b + 1];
        auto it = std::lower_bound(first, last, i);
        if (it == last || *it != i) return -1;
        return (int32_t)(S.f_p[b] + (it - first));
    };

    // ---- extend-add maps: contribution-block row of child -> parent local row ----
    S.f_relmap_off.assign(nf + 1, 0);
    for (int32_t b = 0; b < nf; ++b) S.f_relmap_off[b + 1] = S.f_relmap_off[b] + (soff[b + 1] - soff[b]);
    S.relmap.resize(S.f_relmap_off[nf]);
    for (int32_t b = 0; b < nf; ++b) {
        int32_t par = S.f_parent[b];
        for (int64_t q = soff[b]; q < soff[b + 1]; ++q) {
            int32_t lr = par >= 0 ? local_row(par, sidx[q]) : -1;
            if (lr < 0) return "internal: contribution row missing from parent front";
            S.relmap[S.f_relmap_off[b] + (q - soff[b])] = lr;
        }
    }

    // ---- packed value slots, front-major ----
    S.f_ent_off.assign(nf + 1, 0);
    std::vector<int32_t> ublk(nu);
    for (int64_t u = 0; u < nu; ++u) {
        int32_t a = S.iperm[P.ur[u]], c = S.iperm[P.uc[u]];
        ublk[u] = blk[std::min(a, c)];
        S.f_ent_off[ublk[u] + 1]++;
    }
    for (int32_t b = 0; b < nf; ++b) S.f_ent_off[b + 1] += S.f_ent_off[b];
    S.ent_r.resize(nu);
    S.ent_c.resize(nu);
    S.ent_lpos.resize(nu);
    S.identity_dups = (nu == nnz);
    S.dup_ptr.assign(S.identity_dups ? 0 : nu + 1, 0);
    S.dup_pos.resize(nnz);
    {
        // slots ordered by (column, row) in the new numbering: fronts are contiguous column ranges,
        // so this is front-major and column i of the permuted lower triangle is contiguous
        std::vector<int64_t> ccount(n + 1, 0);
        for (int64_t u = 0; u < nu; ++u) ccount[std::min(S.iperm[P.ur[u]], S.iperm[P.uc[u]]) + 1]++;
        for (int64_t i = 0; i < n; ++i) ccount[i + 1] += ccount[i];
        S.cptr.assign(ccount.begin(), ccount.end());
        std::vector<int32_t> slot_of(nu);
        {
            std::vector<std::pair<int32_t, int32_t>> key(nu);  // (col, row) new numbering
            std::vector<int64_t> cf(ccount.begin(), ccount.end() - 1);
            std::vector<int32_t> bycol(nu);
            for (int64_t u = 0; u < nu; ++u) {
                int32_t a = S.iperm[P.ur[u]], c = S.iperm[P.uc[u]];
                bycol[cf[std::min(a, c)]++] = (int32_t)u;
            }
            for (int64_t i = 0; i < n; ++i) {
                auto first = bycol.begin() + ccount[i], last = bycol.begin() + ccount[i + 1];
                std::sort(first, last, [&](int32_t x, int32_t y) {
                    return std::max(S.iperm[P.ur[x]], S.iperm[P.uc[x]]) < std::max(S.iperm[P.ur[y]], S.iperm[P.uc[y]]);
                });
            }
            for (int64_t q = 0; q < nu; ++q) slot_of[bycol[q]] = (int32_t)q;
        }
        // row part: entries (i, c), c < i, listed per row i
        S.rptr.assign(n + 1, 0);
        for (int64_t u = 0; u < nu; ++u) {
            int32_t a = S.iperm[P.ur[u]], c = S.iperm[P.uc[u]];
            if (a != c) S.rptr[std::max(a, c) + 1]++;
        }
        for (int64_t i = 0; i < n; ++i) S.rptr[i + 1] += S.rptr[i];
        S.rslot.resize(S.rptr[n]);
        {
            std::vector<int32_t> rf(S.rptr.begin(), S.rptr.end() - 1);
            std::vector<int32_t> uof(nu);
            for (int64_t u = 0; u < nu; ++u) uof[slot_of[u]] = (int32_t)u;
            for (int64_t q = 0; q < nu; ++q) {
                int32_t u = uof[q];
                int32_t a = S.iperm[P.ur[u]], c = S.iperm[P.uc[u]];
                if (a != c) S.rslot[rf[std::max(a, c)]++] = (int32_t)q;
            }
        }
        // row-major symmetric layout (kkt_kernels.hip k_rowscanR): row i = its column part, then its row
        // part, at [cptr[i] + rptr[i], ...); the partner's original id per entry (filled below)
        S.rowpartner.assign((size_t)(S.cptr[n] + S.rptr[n]), 0);
        for (int64_t u = 0; u < nu; ++u) {
            int32_t s = slot_of[u], b = ublk[u];
            int32_t a = S.iperm[P.ur[u]], c = S.iperm[P.uc[u]];
            int32_t hi = std::max(a, c), lo = std::min(a, c);
            int32_t lc = lo - bfirst[b];
            int32_t lr = local_row(b, hi);
            if (lr < 0) return "internal: entry row missing from its front";
            S.ent_r[s] = S.perm[hi];
            S.ent_c[s] = S.perm[lo];
            // bit 15: the column's original id is the larger one, so the oracle's scaled value
            // (s[larger] * v) * s[smaller] is (s_col * v) * s_row (kkt_kernels.hip assemble_front)
            const uint32_t flip = S.perm[lo] > S.perm[hi] ? 0x8000u : 0u;
            S.ent_lpos[s] = ((uint32_t)lr << 16) | flip | (uint32_t)lc;
            if (!S.identity_dups) S.dup_ptr[s + 1] = P.udp[u + 1] - P.udp[u];
        }
        for (int64_t i = 0; i < n; ++i) {
            int64_t t = (int64_t)S.cptr[i] + S.rptr[i];
            const int32_t o = S.perm[i];
            auto code = [&](int32_t partner) { return (S.iperm[partner] << 1) | (o > partner ? 1 : 0); };
            for (int32_t q = S.cptr[i]; q < S.cptr[i + 1]; ++q) S.rowpartner[t++] = code(S.ent_r[q]);
            for (int32_t r = S.rptr[i]; r < S.rptr[i + 1]; ++r) S.rowpartner[t++] = code(S.ent_c[S.rslot[r]]);
        }
        if (S.identity_dups) {
            for (int64_t u = 0; u < nu; ++u) S.dup_pos[slot_of[u]] = P.pos_sorted[P.udp[u]];
        } else {
            for (int64_t s = 0; s < nu; ++s) S.dup_ptr[s + 1] += S.dup_ptr[s];
            for (int64_t u = 0; u < nu; ++u) {
                int64_t o = S.dup_ptr[slot_of[u]];
                for (int32_t q = P.udp[u]; q < P.udp[u + 1]; ++q) S.dup_pos[o++] = P.pos_sorted[q];
            }
        }
    }

    // ---- level schedule ----
    int32_t maxlev = 0;
    for (int32_t b = 0; b < nf; ++b) maxlev = std::max(maxlev, S.f_level[b]);
    S.nlevels = nf ? maxlev + 1 : 0;
    S.level_off.assign(S.nlevels + 1, 0);
    for (int32_t b = 0; b < nf; ++b) S.level_off[S.f_level[b] + 1]++;
    for (int l = 0; l < S.nlevels; ++l) S.level_off[l + 1] += S.level_off[l];
    S.level_fronts.resize(nf);
    {
        std::vector<int32_t> fill(S.level_off.begin(), S.level_off.end() - 1);
        for (int32_t b = 0; b < nf; ++b) S.level_fronts[fill[S.f_level[b]]++] = b;
        for (int l = 0; l < S.nlevels; ++l)
            std::stable_sort(S.level_fronts.begin() + S.level_off[l], S.level_fronts.begin() + S.level_off[l + 1],
                             [&](int32_t a, int32_t b) { return S.f_m[a] > S.f_m[b]; });
    }
    return "";
}

int64_t delay_columns(Pattern& P, const Symbolic& S, const std::vector<int32_t>& delayed_vars) {
    const int32_t nf = (int32_t)S.nf;
    std::vector<int32_t> blk(P.n), iperm(P.n);
    for (int32_t b = 0; b < nf; ++b)
        for (int32_t j = P.bfirst[b]; j < P.bfirst[b + 1]; ++j) blk[j] = b;
    for (int32_t q = 0; q < (int32_t)P.n; ++q) iperm[P.perm[q]] = q;
    std::vector<char> moved(P.n, 0);
    std::vector<std::vector<int32_t>> into(nf);  // new indices delayed into each block
    int64_t count = 0;
    if ((int64_t)P.delay_count.size() != P.n) P.delay_count.assign(P.n, 0);
    for (int32_t v : delayed_vars) {
        if (v < 0 || v >= P.n) continue;
        int32_t j = iperm[v];
        if (moved[j]) continue;
        int32_t par = S.f_parent[blk[j]];
        if (par < 0) continue;  // roots cannot delay
        if (P.delay_count[v] < 255) P.delay_count[v]++;
        if (P.delay_count[v] >= 2)  // failed again after a delay: the cascade would climb level by level
            while (S.f_parent[par] >= 0) par = S.f_parent[par];
        moved[j] = 1;
        into[par].push_back(j);
        count++;
    }
    if (!count) return 0;
    std::vector<int32_t> perm, bfirst;
    perm.reserve(P.n);
    for (int32_t b = 0; b < nf; ++b) {
        std::sort(into[b].begin(), into[b].end());
        size_t start = perm.size();
        for (int32_t j : into[b]) perm.push_back(P.perm[j]);
        for (int32_t j = P.bfirst[b]; j < P.bfirst[b + 1]; ++j)
            if (!moved[j]) perm.push_back(P.perm[j]);
        if (perm.size() > start) bfirst.push_back((int32_t)start);
    }
    bfirst.push_back((int32_t)perm.size());
    P.perm.swap(perm);
    P.bfirst.swap(bfirst);
    return count;
}

int64_t amalgamate(Pattern& P, const Symbolic& S, const std::vector<char>& merge) {
    const int32_t nf = (int32_t)S.nf;
    // final target of every front: follow merged fronts up to the first kept ancestor
    std::vector<int32_t> target(nf);
    int64_t merged = 0;
    for (int32_t b = nf - 1; b >= 0; --b) {  // parents have larger ids
        if (merge[b] && S.f_parent[b] >= 0) {
            target[b] = target[S.f_parent[b]];
            merged++;
        } else {
            target[b] = b;
        }
    }
    if (!merged) return 0;
    std::vector<std::vector<int32_t>> pending(nf);
    std::vector<int32_t> perm, bfirst;
    perm.reserve(P.n);
    for (int32_t b = 0; b < nf; ++b) {
        if (target[b] != b) {
            auto& q = pending[target[b]];
            for (int32_t j = P.bfirst[b]; j < P.bfirst[b + 1]; ++j) q.push_back(P.perm[j]);
            continue;
        }
        bfirst.push_back((int32_t)perm.size());
        perm.insert(perm.end(), pending[b].begin(), pending[b].end());  // delayed columns first
        for (int32_t j = P.bfirst[b]; j < P.bfirst[b + 1]; ++j) perm.push_back(P.perm[j]);
        std::vector<int32_t>().swap(pending[b]);
    }
    bfirst.push_back((int32_t)perm.size());
    P.perm.swap(perm);
    P.bfirst.swap(bfirst);
    return merged;
}

// Greedy top-down cut: repeatedly move the heaviest candidate subtree's root into the top set (its
// children become candidates), pack the candidates onto the ranks longest-first, and keep the cut
// with the smallest estimated critical path = makespan of the packed subtrees + serial top work.
void partition_tree(const Symbolic& S, int world, Partition& out) {
    const int32_t nf = (int32_t)S.nf;
    out = Partition();
    out.world = world;
    out.owner.assign(nf, 0);
    if (world <= 1 || nf == 0) return;
    // per-front cost estimate: factor flops + assembly + a per-pivot-step latency term
    std::vector<double> work(nf), sub(nf, 0.0);
    std::vector<std::vector<int32_t>> kids(nf);
    for (int32_t f = 0; f < nf; ++f) {
        const double m = S.f_m[f], p = S.f_p[f];
        double fl = 0.0;
        for (int k = 0; k < (int)p; ++k) {
            const double r = m - k - 1;
            fl += r + r * (r + 1.0);
        }
        work[f] = fl + m * m + 2000.0 * p;
    }
    for (int32_t f = 0; f < nf; ++f) {  // children have smaller ids
        sub[f] += work[f];
        if (S.f_parent[f] >= 0) {
            sub[S.f_parent[f]] += sub[f];
            kids[S.f_parent[f]].push_back(f);
        }
    }
    std::vector<int32_t> cand;
    double total = 0.0;
    for (int32_t f = 0; f < nf; ++f)
        if (S.f_parent[f] < 0) { cand.push_back(f); total += sub[f]; }
    out.total_work = total;
    auto pack = [&](const std::vector<int32_t>& c, std::vector<int32_t>* assign) {
        std::vector<int32_t> order(c.begin(), c.end());
        std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) { return sub[a] > sub[b]; });
        std::vector<double> load(world, 0.0);
        if (assign) assign->assign(nf, -1);
        for (int32_t r : order) {
            int best = 0;
            for (int q = 1; q < world; ++q)
                if (load[q] < load[best]) best = q;
            load[best] += sub[r];
            if (assign) (*assign)[r] = best;
        }
        return *std::max_element(load.begin(), load.end());
    };
    std::vector<char> top(nf, 0);
    double top_work = 0.0;
    double best_cost = pack(cand, nullptr);
    std::vector<char> best_top = top;
    std::vector<int32_t> best_cand = cand;
    double best_top_work = 0.0;
    const int max_cuts = 64 * world;
    int since_best = 0;
    for (int cut = 0; cut < max_cuts && since_best < 8 * world; ++cut) {
        // split the heaviest candidate that has children
        int pick = -1;
        for (size_t q = 0; q < cand.size(); ++q)
            if (!kids[cand[q]].empty() && (pick < 0 || sub[cand[q]] > sub[cand[pick]])) pick = (int)q;
        if (pick < 0) break;
        const int32_t f = cand[pick];
        cand.erase(cand.begin() + pick);
        for (int32_t c : kids[f]) cand.push_back(c);
        top[f] = 1;
        top_work += work[f];
        const double cost = pack(cand, nullptr) + top_work;
        if (cost < best_cost * (1.0 - 1e-9)) {
            best_cost = cost;
            best_top = top;
            best_cand = cand;
            best_top_work = top_work;
            since_best = 0;
        } else {
            ++since_best;
        }
    }
    std::vector<int32_t> root_owner;
    out.max_rank_work = pack(best_cand, &root_owner);
    out.top_work = best_top_work;
    out.n_subtrees = (int64_t)best_cand.size();
    // owner of every front: top fronts -1, others inherit the rank of their subtree root
    for (int32_t f = nf - 1; f >= 0; --f) {
        if (best_top[f]) { out.owner[f] = -1; out.n_top++; continue; }
        if (root_owner[f] >= 0) { out.owner[f] = root_owner[f]; continue; }
        out.owner[f] = out.owner[S.f_parent[f]];  // parent id is larger: already set
    }
    for (int32_t r : best_cand) {
        if (S.f_parent[r] >= 0) {
            out.send_roots.push_back(r);
            out.root_rank.push_back(root_owner[r]);
        }
    }
}

}  // namespace ukkt
