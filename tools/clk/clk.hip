// s_memtime vs s_memrealtime (100 MHz) over a dependent FMA chain in one wave: the shader clock the per-step
// cycle stamps (UKKT_STEP_STAMPS) are counted in.  Build: hipcc --offload-arch=gfx950 -O3 clk.hip -o clk
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned long long* out, double* sink, int iters) {
    double x = threadIdx.x * 1e-3, y = 1.0000001;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; ++i) x = fma(x, y, 1e-9);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    sink[threadIdx.x] = x;
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = r1 - r0; }
}
int main() {
    unsigned long long* o; double* s;
    hipMalloc(&o, 16); hipMalloc(&s, 64 * 8);
    for (int it : {100000, 1000000, 4000000}) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, o, s, it);
        unsigned long long h[2];
        hipMemcpy(h, o, 16, hipMemcpyDeviceToHost);
        printf("iters %d memtime %llu realtime %llu (10 ns) -> %.3f GHz, %.2f memtime per dependent fma\n", it, h[0], h[1],
               h[0] / (h[1] * 10.0), (double)h[0] / it);
    }
    return 0;
}
