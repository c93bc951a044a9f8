// Micro-benchmarks (single wave) to calibrate per-operation latency on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
template <int CTRL, int RM, int BM>
__device__ __forceinline__ int dpp_mov(int old, int v) { return __builtin_amdgcn_update_dpp(old, v, CTRL, RM, BM, false); }
__device__ __forceinline__ int dpp_incl_max(int v, int ident) {
    v = max(v, dpp_mov<0x111, 0xf, 0xf>(ident, v)); v = max(v, dpp_mov<0x112, 0xf, 0xf>(ident, v));
    v = max(v, dpp_mov<0x114, 0xf, 0xf>(ident, v)); v = max(v, dpp_mov<0x118, 0xf, 0xf>(ident, v));
    v = max(v, dpp_mov<0x142, 0xa, 0xf>(ident, v)); v = max(v, dpp_mov<0x143, 0xc, 0xf>(ident, v));
    return v;
}
__global__ void k(long long *out, int iters, int *gsink) {
    __shared__ int lds[4096];
    const int lane = threadIdx.x;
    for (int i = lane; i < 4096; i += 64) lds[i] = (i * 7 + 1) & 4095;
    __syncthreads();
    long long t0 = clock64();
    int x = lane;
    for (int i = 0; i < iters; ++i) x = lds[x];            // dependent LDS chain
    long long t1 = clock64();
    int y = lane;
    for (int i = 0; i < iters; ++i) y = dpp_incl_max(y, -1000000) + 1;  // DPP scan chain
    long long t2 = clock64();
    int z = lane;
    for (int i = 0; i < iters; ++i) z = __builtin_amdgcn_readlane(z, i & 63) + lane;  // readlane chain
    long long t3 = clock64();
    int u = lane;
    for (int i = 0; i < iters; ++i) u = u * 3 + (u >> 2) + 7;  // plain VALU chain (3 ops)
    long long t4 = clock64();
    int w = lane;
    for (int i = 0; i < iters; ++i) { int xx = lds[(w + i) & 4095]; lds[(w * 3 + i) & 4095] = xx + 1; w = xx; }  // LDS write+read
    long long t5 = clock64();
    unsigned long long bsum = 0; int v = lane;
    for (int i = 0; i < iters; ++i) { bsum += __ballot(v > i); v = v + (int)(bsum & 1); }
    long long t6 = clock64();
    if (lane == 0) { out[0] = t1 - t0; out[1] = t2 - t1; out[2] = t3 - t2; out[3] = t4 - t3; out[4] = t5 - t4; out[5] = t6 - t5; }
    gsink[lane] = x + y + z + u + w + (int)bsum + v;
}
int main() {
    long long *d; int *g; hipMalloc(&d, 64); hipMalloc(&g, 4096);
    const int it = 10000;
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, it, g);
        hipDeviceSynchronize();
    }
    long long h[6]; hipMemcpy(h, d, 48, hipMemcpyDeviceToHost);
    const char *nm[6] = {"LDS dependent read", "DPP 6-step incl max scan", "readlane chain", "3-op VALU chain", "LDS read+write dep", "ballot chain"};
    for (int i = 0; i < 6; ++i) printf("%-28s %.1f cycles/iter\n", nm[i], (double)h[i] / it);
    return 0;
}
