// sanitize_main.cpp -- TEST INFRASTRUCTURE ONLY: host-code sanitizer run (race detection /
// sanitizers).  Built by `make -C oracle asan` with -fsanitize=address,undefined and run by
// tests/test_sanitizers.py: the product's host symbolic analysis (uno_amd/csrc/analysis.cpp: ordering,
// supernodes, device layout, delayed-column moves, amalgamation, subtree partition) through the CPU
// baseline (oracle/cpu_mf.cpp), and the oracle (oracle/kkt_oracle.c), on the MUMPSSolverTests.cpp:14-61
// known answer, random sparse indefinite systems and a small arrowband KKT.  Exit status 0 = clean run
// with matching inertias.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <vector>

#include "../uno_amd/csrc/analysis.hpp"
#include "kkt_oracle.h"

extern "C" {
void* cpu_mf_create();
void cpu_mf_destroy(void*);
int cpu_mf_analyze(void*, int64_t, int64_t, const int64_t*, const int64_t*);
int cpu_mf_factorize(void*, const double*);
int cpu_mf_inertia(void*, int64_t*, int64_t*, int64_t*);
int cpu_mf_solve(void*, const double*, double*);
int64_t arrowband_size(int64_t N, int64_t* nv_out, int64_t* m_out);
int64_t arrowband_generate(int64_t N, uint64_t seed, int64_t* row, int64_t* col, double* val);
}

static int check(const char* name, int64_t n, const std::vector<int64_t>& r, const std::vector<int64_t>& c,
                 const std::vector<double>& v) {
    oracle_kkt_t o = oracle_kkt_create();
    void* g = cpu_mf_create();
    int bad = 0;
    if (oracle_kkt_analyze(o, n, (int64_t)r.size(), r.data(), c.data()) || oracle_kkt_factorize(o, v.data())) bad = 1;
    if (cpu_mf_analyze(g, n, (int64_t)r.size(), r.data(), c.data()) || cpu_mf_factorize(g, v.data())) bad = 1;
    int64_t a[3] = {0, 0, 0}, b[3] = {0, 0, 0};
    if (!bad) {
        oracle_kkt_inertia(o, a, a + 1, a + 2);
        cpu_mf_inertia(g, b, b + 1, b + 2);
        std::vector<double> rhs(n, 1.0), x1(n), x2(n);
        oracle_kkt_solve(o, rhs.data(), x1.data());
        cpu_mf_solve(g, rhs.data(), x2.data());
        if (a[0] != b[0] || a[1] != b[1] || a[2] != b[2]) bad = 1;
    }
    // the rest of the host analysis: column delays, amalgamation, subtree partitions
    ukkt::Pattern P;
    ukkt::Symbolic S;
    if (ukkt::analyze(n, (int64_t)r.size(), r.data(), c.data(), ukkt::AnalysisOptions(), P, S).empty() && S.nf > 1) {
        std::vector<int32_t> dv;
        for (int64_t i = 0; i < n; i += 7) dv.push_back((int32_t)i);
        ukkt::delay_columns(P, S, dv);
        ukkt::build_structure(P, S);
        std::vector<char> merge(S.nf, 0);
        for (int64_t f = 0; f < S.nf; f += 3) merge[f] = 1;
        ukkt::amalgamate(P, S, merge);
        ukkt::build_structure(P, S);
        for (int w : {2, 3, 8}) {
            ukkt::Partition part;
            ukkt::partition_tree(S, w, part);
        }
    }
    std::printf("%s: n=%lld oracle (%lld,%lld,%lld) cpu_mf (%lld,%lld,%lld) %s\n", name, (long long)n, (long long)a[0],
                (long long)a[1], (long long)a[2], (long long)b[0], (long long)b[1], (long long)b[2], bad ? "MISMATCH" : "ok");
    cpu_mf_destroy(g);
    oracle_kkt_destroy(o);
    return bad;
}

int main() {
    int bad = 0;
    // MUMPSSolverTests.cpp:14-61 known answer (inertia (3,2,0))
    bad |= check("kat5x5", 5, {0, 0, 1, 1, 2, 2, 4}, {0, 1, 2, 4, 2, 3, 4}, {2, 3, 4, 6, 1, 5, 1});
    // random sparse symmetric indefinite (LCG): diagonally dominant with random signs (nonsingular, so the
    // inertia does not depend on the pivot order), both triangles and duplicate diagonal entries
    uint64_t s = 12345;
    auto rnd = [&]() { s = s * 6364136223846793005ULL + 1442695040888963407ULL; return (double)(s >> 11) / 9007199254740992.0; };
    for (int t = 0; t < 6; ++t) {
        const int64_t n = 50 + 60 * t;
        std::vector<int64_t> r, c;
        std::vector<double> v, rowabs(n, 0.0);
        for (int64_t i = 0; i < n; ++i)
            for (int64_t j = 0; j < i; ++j)
                if (rnd() < 4.0 / (double)n) {
                    const double x = 2.0 * rnd() - 1.0;
                    const bool upper = rnd() < 0.5;
                    r.push_back(upper ? j : i); c.push_back(upper ? i : j); v.push_back(x);
                    rowabs[i] += std::fabs(x); rowabs[j] += std::fabs(x);
                }
        for (int64_t i = 0; i < n; ++i) {
            const double d = (rnd() < 0.5 ? -1.0 : 1.0) * (1.0 + rowabs[i]);
            r.push_back(i); c.push_back(i); v.push_back(0.25 * d);  // duplicates summed
            r.push_back(i); c.push_back(i); v.push_back(0.75 * d);
        }
        char name[32];
        std::snprintf(name, sizeof(name), "random%d", t);
        bad |= check(name, n, r, c, v);
    }
    // configs[1]-shaped arrowband KKT (dense arrow rows, duplicates on the diagonal)
    const int64_t N = 4000;
    const int64_t nnz = arrowband_size(N, nullptr, nullptr);
    std::vector<int64_t> r(nnz), c(nnz);
    std::vector<double> v(nnz);
    arrowband_generate(N, 0x5EED0002ULL, r.data(), c.data(), v.data());
    bad |= check("arrowband4000", N, r, c, v);
    return bad;
}
