// Latency probes on one wave (shader cycles, s_memtime = 2.4 GHz on MI355X, tools/clk/clk.hip): a dependent
// chain of 64 DP FMAs, of 16 IEEE divisions (1.0 / x), of 32 LDS write->read round trips, of 32 readlanes of a
// DP value, and the one-wave pivot step's skeleton.  Build: hipcc --offload-arch=gfx950 -O3 lat.hip -o lat
#include <hip/hip_runtime.h>
#include <cstdio>
__device__ __forceinline__ double rl(double x, int l) {
    unsigned long long b = __double_as_longlong(x);
    unsigned lo = __builtin_amdgcn_readlane((int)(unsigned)b, l), hi = __builtin_amdgcn_readlane((int)(unsigned)(b >> 32), l);
    return __longlong_as_double(((unsigned long long)hi << 32) | lo);
}
__global__ void k(unsigned long long* out, double* sink, double seed) {
    __shared__ double sm[64];
    const int lane = threadIdx.x;
    double x = seed + lane * 1e-9, y = 1.0000001;
    unsigned long long t0, t1;
    // FMA chain
    t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < 64; ++i) x = fma(x, y, 1e-9);
    asm volatile("" : "+v"(x));
    t1 = __builtin_amdgcn_s_memtime();
    out[0] = t1 - t0;
    // division chain
    t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < 16; ++i) x = 1.0 / (x + 1.0);
    asm volatile("" : "+v"(x));
    t1 = __builtin_amdgcn_s_memtime();
    out[1] = t1 - t0;
    // LDS write -> read of another lane's word
    t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < 32; ++i) {
        sm[lane] = x;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
        x = sm[(lane + 1) & 63] + 1e-9;
    }
    asm volatile("" : "+v"(x));
    t1 = __builtin_amdgcn_s_memtime();
    out[2] = t1 - t0;
    // readlane chain (VALU result -> SGPR -> VALU)
    t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int i = 0; i < 32; ++i) x = rl(x, i & 63) + 1e-9;
    asm volatile("" : "+v"(x));
    t1 = __builtin_amdgcn_s_memtime();
    out[3] = t1 - t0;
    sink[lane] = x;
}
int main() {
    unsigned long long* o; double* s;
    (void)hipMalloc(&o, 64); (void)hipMalloc(&s, 64 * 8);
    for (int r = 0; r < 3; ++r) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, o, s, 1.0 + r);
        unsigned long long h[4];
        (void)hipMemcpy(h, o, 32, hipMemcpyDeviceToHost);
        printf("cycles: fma %.1f per dependent op, div %.1f per 1/x, lds write->read %.1f per round trip, readlane %.1f per hop\n",
               h[0] / 64.0, h[1] / 16.0, h[2] / 32.0, h[3] / 32.0);
    }
    return 0;
}
