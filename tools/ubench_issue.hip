// Issue-rate micro-benchmark (gfx950): cycles per instruction of independent VALU (packed i16), SALU
// and mixed VALU+SALU streams, with W waves per SIMD (one workgroup of 4W waves on one CU).
// Answers: does one wave issue a VALU and a SALU in the same slot, and how many waves does it take to
// saturate the SIMD's VALU / the CU's SALU?
#include <hip/hip_runtime.h>
#include <cstdio>

#define R8(x) x x x x x x x x
template <int KIND>
__global__ void k(long long *out, int iters) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    unsigned a0 = lane, a1 = lane + 1, a2 = lane + 2, a3 = lane + 3, a4 = lane + 4, a5 = lane + 5, a6 = lane + 6,
             a7 = lane + 7;
    int s0 = 1, s1 = 2, s2 = 3, s3 = 4, s4 = 5, s5 = 6, s6 = 7, s7 = 8;
    __syncthreads();
    long long t0 = clock64();
    for (int i = 0; i < iters; ++i) {
        if (KIND == 0) {  // 64 independent packed VALU ops
            asm volatile(R8("v_pk_max_i16 %0, %0, %1\n v_pk_max_i16 %1, %1, %2\n v_pk_max_i16 %2, %2, %3\n "
                            "v_pk_max_i16 %3, %3, %4\n v_pk_max_i16 %4, %4, %5\n v_pk_max_i16 %5, %5, %6\n "
                            "v_pk_max_i16 %6, %6, %7\n v_pk_max_i16 %7, %7, %0\n")
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
        } else if (KIND == 1) {  // 64 independent SALU ops
            asm volatile(R8("s_add_u32 %0, %0, %1\n s_add_u32 %1, %1, %2\n s_add_u32 %2, %2, %3\n "
                            "s_add_u32 %3, %3, %4\n s_add_u32 %4, %4, %5\n s_add_u32 %5, %5, %6\n "
                            "s_add_u32 %6, %6, %7\n s_add_u32 %7, %7, %0\n")
                         : "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3), "+s"(s4), "+s"(s5), "+s"(s6), "+s"(s7) : : "scc");
        } else if (KIND == 2) {  // 32 VALU + 32 SALU interleaved
            asm volatile(R8("v_pk_max_i16 %0, %0, %1\n s_add_u32 %8, %8, %9\n v_pk_max_i16 %1, %1, %2\n "
                            "s_add_u32 %9, %9, %10\n v_pk_max_i16 %2, %2, %3\n s_add_u32 %10, %10, %11\n "
                            "v_pk_max_i16 %3, %3, %0\n s_add_u32 %11, %11, %8\n")
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7),
                           "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3) : : "scc");
        } else if (KIND == 3) {  // 64 independent 32-bit VALU ops (v_max_i32)
            asm volatile(R8("v_max_i32 %0, %0, %1\n v_max_i32 %1, %1, %2\n v_max_i32 %2, %2, %3\n "
                            "v_max_i32 %3, %3, %4\n v_max_i32 %4, %4, %5\n v_max_i32 %5, %5, %6\n "
                            "v_max_i32 %6, %6, %7\n v_max_i32 %7, %7, %0\n")
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
        } else if (KIND == 4) {  // 64 v_mov_b32_dpp row_shr:1 (independent)
            asm volatile(R8("v_mov_b32_dpp %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf\n "
                            "v_mov_b32_dpp %2, %3 row_shr:1 row_mask:0xf bank_mask:0xf\n "
                            "v_mov_b32_dpp %4, %5 row_shr:1 row_mask:0xf bank_mask:0xf\n "
                            "v_mov_b32_dpp %6, %7 row_shr:1 row_mask:0xf bank_mask:0xf\n "
                            "v_mov_b32_dpp %1, %0 row_shr:1 row_mask:0xf bank_mask:0xf\n "
                            "v_mov_b32_dpp %3, %2 row_shr:1 row_mask:0xf bank_mask:0xf\n "
                            "v_mov_b32_dpp %5, %4 row_shr:1 row_mask:0xf bank_mask:0xf\n "
                            "v_mov_b32_dpp %7, %6 row_shr:1 row_mask:0xf bank_mask:0xf\n")
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
        } else if (KIND == 5) {  // 64 v_perm_b32 (independent)
            asm volatile(R8("v_perm_b32 %0, %0, %1, %2\n v_perm_b32 %1, %1, %2, %3\n v_perm_b32 %2, %2, %3, %4\n "
                            "v_perm_b32 %3, %3, %4, %5\n v_perm_b32 %4, %4, %5, %6\n v_perm_b32 %5, %5, %6, %7\n "
                            "v_perm_b32 %6, %6, %7, %0\n v_perm_b32 %7, %7, %0, %1\n")
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
        } else {  // 64 dependent v_pk_max_i16 (one chain): latency
            asm volatile(R8("v_pk_max_i16 %0, %0, %1\n v_pk_max_i16 %0, %0, %2\n v_pk_max_i16 %0, %0, %3\n "
                            "v_pk_max_i16 %0, %0, %4\n v_pk_max_i16 %0, %0, %5\n v_pk_max_i16 %0, %0, %6\n "
                            "v_pk_max_i16 %0, %0, %7\n v_pk_max_i16 %0, %0, %1\n")
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
        }
    }
    long long t1 = clock64();
    if (lane == 0) out[wv] = t1 - t0;
    if ((a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ s0 ^ s1 ^ s2 ^ s3 ^ s4 ^ s5 ^ s6 ^ s7) == 0x7fffffff) out[63] = 1;
}

int main() {
    long long *d;
    hipMalloc(&d, 64 * 8);
    const int it = 2000;
    const char *nm[] = {"v_pk_max_i16 indep", "s_add_u32 indep", "32 VALU + 32 SALU", "v_max_i32 indep",
                        "v_mov_b32_dpp indep", "v_perm_b32 indep", "v_pk_max_i16 dep chain"};
    void (*ks[])(long long *, int) = {k<0>, k<1>, k<2>, k<3>, k<4>, k<5>, k<6>};
    for (int kind = 0; kind < 7; ++kind) {
        for (int w : {1, 2, 3, 4}) {
            for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(ks[kind], dim3(1), dim3(64 * 4 * w), 0, 0, d, it);
            hipDeviceSynchronize();
            long long h[64];
            hipMemcpy(h, d, 8 * 4 * w, hipMemcpyDeviceToHost);
            double mx = 0;
            for (int i = 0; i < 4 * w; ++i) mx = h[i] > mx ? h[i] : mx;
            printf("%-24s waves/SIMD %d: %.2f cycles per instruction per wave, %.2f per SIMD\n", nm[kind], w,
                   mx / (64.0 * it), mx / (64.0 * it * w));
        }
    }
    return 0;
}
