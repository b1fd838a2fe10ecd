// Host-only front statistics of the symbolic analysis (no GPU): per level, fronts, mean rows m, mean
// pivots p, nnz_L share and flops.  build: g++ -O2 -std=c++17 -fopenmp tools/front_stats.cpp
//   uno_amd/csrc/analysis.cpp /tmp/arrowband.o -o /tmp/front_stats   (gcc -O2 -c uno_amd/csrc/arrowband.c -o /tmp/arrowband.o)
// usage: /tmp/front_stats [n] [leaf_size] [max_block] [world] [seed]
//   world > 1: also the multi-GPU partition (analysis.cpp::partition_tree): subtrees per rank, the top
//   fronts rank 0 factors after the exchange, their levels / sizes and the cost model's work shares
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../uno_amd/csrc/analysis.hpp"

extern "C" int64_t arrowband_size(int64_t N, int64_t* nv_out, int64_t* m_out);
extern "C" int64_t arrowband_generate(int64_t N, uint64_t seed, int64_t* row, int64_t* col, double* val);

int main(int argc, char** argv) {
    const int64_t n = argc > 1 ? atoll(argv[1]) : 1000000;
    ukkt::AnalysisOptions opt;
    if (argc > 2) opt.leaf_size = atoi(argv[2]);
    if (argc > 3) opt.max_block = atoi(argv[3]);
    int64_t nv, m;
    const int64_t nnz = arrowband_size(n, &nv, &m);
    std::vector<int64_t> r(nnz), c(nnz);
    std::vector<double> v(nnz);
    const int world = argc > 4 ? atoi(argv[4]) : 1;
    const unsigned long long seed = argc > 5 ? strtoull(argv[5], nullptr, 0) : 0x5EED0003ULL;
    arrowband_generate(n, seed, r.data(), c.data(), v.data());
    ukkt::Pattern P;
    ukkt::Symbolic S;
    std::string e = ukkt::analyze(n, nnz, r.data(), c.data(), opt, P, S);
    if (!e.empty()) { fprintf(stderr, "%s\n", e.c_str()); return 1; }
    printf("n %lld nnz %lld fronts %lld levels %d nnz_L %lld flops %.3e max_m %lld\n", (long long)n, (long long)nnz,
           (long long)S.nf, S.nlevels, (long long)S.nnz_L, S.flops, (long long)S.max_m);
    for (int l = 0; l < S.nlevels; ++l) {
        double cnt = 0, sm = 0, sp = 0, L = 0, fl = 0;
        int mx = 0;
        for (int t = S.level_off[l]; t < S.level_off[l + 1]; ++t) {
            const int f = S.level_fronts[t];
            const double fm = S.f_m[f], fp = S.f_p[f];
            cnt++; sm += fm; sp += fp; mx = std::max(mx, (int)fm);
            L += fp * fm - fp * (fp - 1) / 2;
            for (int k = 0; k < fp; ++k) { const double rk = fm - k - 1; fl += rk + rk * (rk + 1); }
        }
        printf("level %2d fronts %6.0f m %6.1f (max %3d) p %5.1f  L %5.1f%%  flops %5.1f%%\n", l, cnt, sm / cnt, mx,
               sp / cnt, 100 * L / S.nnz_L, 100 * fl / S.flops);
    }
    if (world > 1) {
        ukkt::Partition Pt;
        ukkt::partition_tree(S, world, Pt);
        printf("partition world %d: subtrees %lld, top fronts %lld, work total %.4e, max rank %.4e (%.1f%%), top %.4e (%.1f%%)\n",
               world, (long long)Pt.n_subtrees, (long long)Pt.n_top, Pt.total_work, Pt.max_rank_work,
               100 * Pt.max_rank_work / Pt.total_work, Pt.top_work, 100 * Pt.top_work / Pt.total_work);
        // the top fronts per level: count, rows, pivots, and the longest chain of top fronts (critical path)
        std::vector<int> depth(S.nf, 0);
        int maxd = 0;
        for (int32_t f = 0; f < (int32_t)S.nf; ++f) {  // children have smaller ids
            if (Pt.owner[f] >= 0) continue;
            int d = 1;
            for (int32_t c = 0; c < f; ++c) (void)c;  // (kids scanned below)
            depth[f] = std::max(depth[f], d);
            const int32_t par = S.f_parent[f];
            if (par >= 0 && Pt.owner[par] < 0) depth[par] = std::max(depth[par], depth[f] + 1);
            maxd = std::max(maxd, depth[f]);
        }
        double sm = 0, sp = 0, chainp = 0;
        int mx = 0;
        for (int32_t f = 0; f < (int32_t)S.nf; ++f)
            if (Pt.owner[f] < 0) { sm += S.f_m[f]; sp += S.f_p[f]; mx = std::max(mx, (int)S.f_m[f]); }
        // pivots along the deepest top chain (the serial pivot steps rank 0 runs after the exchange)
        int32_t best = -1;
        for (int32_t f = 0; f < (int32_t)S.nf; ++f)
            if (Pt.owner[f] < 0 && S.f_parent[f] < 0 && (best < 0 || depth[f] > depth[best])) best = f;
        (void)best;
        for (int32_t f = 0; f < (int32_t)S.nf; ++f)
            if (Pt.owner[f] < 0 && depth[f] == 1) {
                double cp = 0;
                for (int32_t g = f; g >= 0 && Pt.owner[g] < 0; g = S.f_parent[g]) cp += S.f_p[g];
                chainp = std::max(chainp, cp);
            }
        printf("top fronts: mean m %.1f (max %d), mean p %.1f, depth %d, pivots on the longest top chain %.0f\n",
               sm / std::max<double>(1, Pt.n_top), mx, sp / std::max<double>(1, Pt.n_top), maxd, chainp);
    }
    return 0;
}
