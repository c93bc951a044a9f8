// Cross-wave exchange micro-benchmark (gfx950): the cost of the per-row synchronisation a POA row split
// over the waves of one workgroup would pay.  Cycles per iteration (s_memtime), one workgroup on one CU:
//   0: one wave, LDS write -> wait -> read -> wait chain (the LDS round trip a lone wave pays anyway)
//   1: two waves, each iteration: write own word, s_barrier, read the other's word (dependent chain)
//   2: the same with two barriers per iteration (exchange + ring visibility)
//   3: two waves, s_barrier only (no LDS traffic)
// usage: ubench_xwave [iters]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

template <int KIND>
__global__ __launch_bounds__(128) void k(long long *out, int iters) {
    __shared__ int x[2][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    x[w][lane] = lane;
    __syncthreads();
    int v = lane;
    const long long t0 = clock64();
    for (int i = 0; i < iters; ++i) {
        if (KIND == 0) {
            if (w == 0) {
                x[0][lane] = v + 1;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                __builtin_amdgcn_wave_barrier();
                v = x[0][(lane + 1) & 63];
            }
        } else if (KIND == 1) {
            x[w][lane] = v + 1;
            __syncthreads();
            v = x[w ^ 1][lane];
        } else if (KIND == 2) {
            x[w][lane] = v + 1;
            __syncthreads();
            v = x[w ^ 1][lane];
            __syncthreads();
        } else {
            __syncthreads();
            v += 1;
        }
    }
    const long long t1 = clock64();
    if (lane == 0) out[w] = t1 - t0;
    if (v == -12345) out[2] = v;
}

template <int KIND>
static void run(const char *name, int iters, int threads) {
    long long *d, h[3] = {0, 0, 0};
    (void)hipMalloc(&d, 3 * sizeof(long long));
    (void)hipMemset(d, 0, 3 * sizeof(long long));
    hipLaunchKernelGGL(k<KIND>, dim3(1), dim3(threads), 0, 0, d, 16);
    hipLaunchKernelGGL(k<KIND>, dim3(1), dim3(threads), 0, 0, d, iters);
    (void)hipMemcpy(h, d, 3 * sizeof(long long), hipMemcpyDeviceToHost);
    printf("%-44s %8.1f cycles per iteration\n", name, (double)h[0] / iters);
    (void)hipFree(d);
}

int main(int argc, char **argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 100000;
    run<0>("1 wave: LDS write -> read chain", iters, 64);
    run<1>("2 waves: write, s_barrier, read other", iters, 128);
    run<2>("2 waves: write, s_barrier, read, s_barrier", iters, 128);
    run<3>("2 waves: s_barrier only", iters, 128);
    run<3>("1 wave: barrier (wave-local)", iters, 64);
    return 0;
}
