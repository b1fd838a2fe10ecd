// Host-only front statistics of the symbolic analysis (no GPU): per level, fronts, mean rows m, mean
// pivots p, nnz_L share and flops.  build: g++ -O2 -std=c++17 -fopenmp tools/front_stats.cpp
//   uno_amd/csrc/analysis.cpp uno_amd/csrc/arrowband.c -o /tmp/front_stats
// usage: /tmp/front_stats [n] [leaf_size] [max_block]
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
    arrowband_generate(n, 0x5EED0003ULL, r.data(), c.data(), v.data());
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
    return 0;
}
