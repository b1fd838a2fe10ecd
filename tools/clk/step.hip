// The one-wave pivot step of factor_front (kkt_kernels.hip, REG && W == 1, MR = 8) in isolation: 17 steps on a
// register-resident 8 x 8 lane grid, shader cycles per step for the full step and for variants without one of its
// parts (DIV: reciprocal by division; LDS: column publish + read-back; TEST: ballot + branch; FMA: rank-1 update).
// Build: hipcc --offload-arch=gfx950 -O3 step.hip -o step
#include <hip/hip_runtime.h>
#include <cstdio>
__device__ __forceinline__ double rl(double x, int l) {
    unsigned long long b = __double_as_longlong(x);
    unsigned lo = __builtin_amdgcn_readlane((int)(unsigned)b, l), hi = __builtin_amdgcn_readlane((int)(unsigned)(b >> 32), l);
    return __longlong_as_double(((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
}
template <bool DIV, bool LDS, bool TEST, bool FMA, bool STEPS = false>
__global__ __launch_bounds__(64) void k(unsigned long long* out, double* sink, double seed, double u, int p) {
    __shared__ double colw[72];
    constexpr int G = 8, RM = 8;
    const int tid = threadIdx.x, ty = tid / G, tx = tid % G;
    double R[RM][RM];
#pragma unroll
    for (int a = 0; a < RM; ++a)
#pragma unroll
        for (int b = 0; b <= a; ++b) R[a][b] = (a == b && tx == ty) ? 40.0 + seed : 0.01 * ((ty + 3 * a + 5 * tx + 7 * b) % 11);
    int k = 0, nfail = 0;
    unsigned long long ts[9];
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    ts[0] = t0;
    const int bk = 0;
    while (k < p) {
        const int kk = k;
        const bool owner = tx == kk;
        const double akk = rl(R[bk][bk], kk * G + kk);
        const double aak = fabs(akk);
        wsync();
        if (LDS) {
            if (owner) {
#pragma unroll
                for (int a = bk; a < RM; ++a) colw[ty + G * a] = R[a][bk];
            }
            wsync();
        }
        double lv[RM], cw[RM], t0v;
        if (LDS) {
            t0v = colw[tid];
#pragma unroll
            for (int a = bk; a < RM; ++a) { lv[a] = colw[ty + G * a]; cw[a] = colw[tx + G * a]; }
        } else {
            t0v = R[7][bk];
#pragma unroll
            for (int a = bk; a < RM; ++a) { lv[a] = R[a][bk] * 0.5; cw[a] = R[a][bk] * 0.25; }
        }
        double dinv = DIV ? 1.0 / akk : 0.025;
        asm volatile("" : "+v"(dinv));
        bool need = false;
        if (TEST) {
            const bool bad = (tid > k) & (u * fabs(t0v) > aak);
            need = __ballot(bad) != 0;
        }
        if (!need) {
            double cv[RM];
#pragma unroll
            for (int a = bk; a < RM; ++a) cv[a] = cw[a] * dinv;
            if (tx <= kk) cv[bk] = 0.0;
            if (FMA) {
#pragma unroll
                for (int a = bk; a < RM; ++a)
#pragma unroll
                    for (int b = bk; b <= a; ++b) R[a][b] -= lv[a] * cv[b];
            } else {
                R[bk][bk] -= lv[bk] * cv[bk];
            }
        } else {
            ++nfail;
        }
        k += 1;
        if (STEPS) ts[k < 9 ? k : 8] = __builtin_amdgcn_s_memtime();
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    double acc = nfail;
#pragma unroll
    for (int a = 0; a < RM; ++a)
#pragma unroll
        for (int b = 0; b <= a; ++b) acc += R[a][b];
    sink[tid] = acc;
    if (tid == 0) {
        out[0] = t1 - t0;
        if (STEPS) for (int q = 0; q < 8; ++q) out[1 + q] = ts[q + 1] - ts[q];
    }
}
template <bool D, bool L, bool T, bool F>
void run(const char* name, unsigned long long* o, double* s) {
    unsigned long long h = 0, best = ~0ull;
    for (int r = 0; r < 5; ++r) {
        hipLaunchKernelGGL((k<D, L, T, F>), dim3(1), dim3(64), 0, 0, o, s, 1.0 + r, 0.01, 8);
        (void)hipMemcpy(&h, o, 8, hipMemcpyDeviceToHost);
        if (r > 0 && h < best) best = h;
    }
    printf("%-34s %7.1f cycles per step (8 steps, best of 4)\n", name, best / 8.0);
}
// per-step cycles of one launch on a fresh CU (cold instruction cache) and of the launch right after on the same CU
void steps(unsigned long long* o, double* s) {
    for (int r = 0; r < 3; ++r) {
        hipLaunchKernelGGL((k<true, true, true, true, true>), dim3(1), dim3(64), 0, 0, o, s, 1.0 + r, 0.01, 8);
        unsigned long long h[9];
        (void)hipMemcpy(h, o, 72, hipMemcpyDeviceToHost);
        printf("launch %d per-step cycles:", r);
        for (int q = 1; q < 9; ++q) printf(" %llu", h[q]);
        printf("\n");
    }
}
int main() {
    unsigned long long* o; double* s;
    (void)hipMalloc(&o, 256); (void)hipMalloc(&s, 64 * 8);
    run<true, true, true, true>("full step", o, s);
    run<false, true, true, true>("no division", o, s);
    run<true, false, true, true>("no LDS publish/read", o, s);
    run<true, true, false, true>("no ballot/branch", o, s);
    run<true, true, true, false>("no rank-1 FMAs (one)", o, s);
    run<false, false, false, true>("FMAs only", o, s);
    run<false, false, false, false>("skeleton", o, s);
    steps(o, s);
    return 0;
}
