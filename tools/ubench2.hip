// Micro-benchmark (single wave): dependent-chain latency of the DPP forms the POA kernel uses.
#include <hip/hip_runtime.h>
#include <cstdio>
#define CHAIN(expr) { long long t0 = clock64(); for (int i = 0; i < iters; ++i) { x = (expr); } out[k++] = clock64() - t0; }
__global__ void k(long long *out, int iters, int *gsink) {
    const int lane = threadIdx.x;
    int x = lane, k = 0;
    CHAIN(__builtin_amdgcn_update_dpp(x, x, 0x111, 0xf, 0xf, false) + 1)   // row_shr:1
    CHAIN(__builtin_amdgcn_update_dpp(x, x, 0x138, 0xf, 0xf, false) + 1)   // wave_shr:1
    CHAIN(__builtin_amdgcn_update_dpp(x, x, 0x130, 0xf, 0xf, false) + 1)   // wave_shl:1
    CHAIN(__builtin_amdgcn_update_dpp(x, x, 0x142, 0xa, 0xf, false) + 1)   // row_bcast:15
    CHAIN(__builtin_amdgcn_update_dpp(x, x, 0x143, 0xc, 0xf, false) + 1)   // row_bcast:31
    CHAIN(__builtin_amdgcn_update_dpp(x, x, 0x121, 0xf, 0xf, false) + 1)   // row_ror:1
    CHAIN(__builtin_amdgcn_ds_bpermute(((lane + 1) & 63) * 4, x) + 1)     // ds_bpermute
    CHAIN(x * 3 + 1)                                                        // plain VALU pair
    CHAIN(__builtin_amdgcn_readlane(x, 5) + lane)                           // readlane + add
    if (lane == 0) for (int i = 0; i < k; ++i) out[i] = out[i];
    gsink[lane] = x;
}
int main() {
    long long *d; int *g; hipMalloc(&d, 256); hipMalloc(&g, 4096);
    const int it = 20000;
    for (int rep = 0; rep < 2; ++rep) { hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, it, g); hipDeviceSynchronize(); }
    long long h[9]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    const char *nm[9] = {"row_shr:1 +add", "wave_shr:1 +add", "wave_shl:1 +add", "row_bcast:15 +add", "row_bcast:31 +add",
                         "row_ror:1 +add", "ds_bpermute +add", "mul+add", "readlane+add"};
    for (int i = 0; i < 9; ++i) printf("%-22s %.1f cycles/iter\n", nm[i], (double)h[i] / it);
    return 0;
}
