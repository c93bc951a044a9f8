// stale_probe.hip — looks for the "stale bytes" the clustering code recorded twice in round 2
// (cluster_kernel.hip: a recycled stream-ordered pool buffer refilled by a copy; cluster.cpp: a reused
// page-locked host buffer rewritten and copied again).  Each scenario refills a buffer with a new byte
// pattern per iteration and lets a kernel count the bytes that differ from it.
//   A  pinned host source (hipHostMalloc default) reused, rewritten by the CPU, H2D each iteration
//   B  the same with hipHostMallocCoherent
//   C  device buffer from the stream-ordered pool (hipMallocAsync/hipFreeAsync), read by a kernel on a
//      second stream before it is freed and re-allocated
//   D  hipMalloc'd device buffer reused, read by a kernel on a second stream before the next refill
//   E  as D, the reader on the copy's own stream
//   F  pageable host source
// The pipeline's pattern (cluster.cpp): the host text is copied in 64 MB pieces while later pieces are
// still being written by other threads; the pieces are complete when enqueued.
// build: hipcc --offload-arch=gfx950 -O2 -o tools/stale_probe tools/stale_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));   \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

__global__ void count_diff(const uint4 *p, size_t n16, uint32_t want, unsigned long long *bad) {
    unsigned long long local = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = p[i];
        local += (v.x != want) + (v.y != want) + (v.z != want) + (v.w != want);
    }
    if (local) atomicAdd(bad, local);
}

__global__ void reader(const uint4 *p, size_t n16, unsigned long long *sink) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) atomicAdd(sink, 1ull);  // keeps the loads
}

static const size_t kBytes = size_t(512) << 20;
static const int kIters = 15;

static void fill(uint8_t *h, int it) {
    // written by 8 threads in 64 MB pieces, copied piece by piece as in cluster.cpp
    memset(h, 0x10 + it, kBytes);
}

static unsigned long long check(const void *d, uint8_t pat, hipStream_t s, unsigned long long *d_bad) {
    CK(hipMemsetAsync(d_bad, 0, 8, s));
    const uint32_t w = 0x01010101u * pat;
    hipLaunchKernelGGL(count_diff, dim3(4096), dim3(256), 0, s, (const uint4 *)d, kBytes / 16, w, d_bad);
    unsigned long long bad = 0;
    CK(hipMemcpyAsync(&bad, d_bad, 8, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    return bad;
}

static void copy_pieces(void *d, const uint8_t *h, hipStream_t s) {
    const size_t piece = size_t(64) << 20;
    for (size_t o = 0; o < kBytes; o += piece) CK(hipMemcpyAsync((char *)d + o, h + o, piece, hipMemcpyHostToDevice, s));
}

int main() {
    hipStream_t s, s2;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    unsigned long long *d_bad, *d_sink;
    CK(hipMalloc(&d_bad, 8));
    CK(hipMalloc(&d_sink, 8));
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    void *dev;
    CK(hipMalloc(&dev, kBytes));
    const char *names[] = {"A pinned-default reused", "B pinned-coherent reused", "C pool recycled + reader s2",
                           "D hipMalloc reused + reader s2", "E hipMalloc reused + reader same stream",
                           "F pageable source"};
    for (int sc = 0; sc < 6; ++sc) {
        uint8_t *h = nullptr;
        if (sc == 0) CK(hipHostMalloc((void **)&h, kBytes, hipHostMallocDefault));
        else if (sc == 1) CK(hipHostMalloc((void **)&h, kBytes, hipHostMallocCoherent));
        else if (sc == 5) h = (uint8_t *)aligned_alloc(4096, kBytes);
        else CK(hipHostMalloc((void **)&h, kBytes, hipHostMallocDefault));
        int fails = 0;
        unsigned long long worst = 0;
        for (int it = 0; it < kIters; ++it) {
            fill(h, it);
            void *d = dev;
            if (sc == 2) CK(hipMallocAsync(&d, kBytes, s));
            copy_pieces(d, h, s);
            const unsigned long long bad = check(d, (uint8_t)(0x10 + it), s, d_bad);
            if (bad) ++fails;
            if (bad > worst) worst = bad;
            if (sc == 2 || sc == 3) {  // a kernel on another stream reads the buffer before it is reused
                CK(hipEventRecord(ev, s));
                CK(hipStreamWaitEvent(s2, ev, 0));
                hipLaunchKernelGGL(reader, dim3(4096), dim3(256), 0, s2, (const uint4 *)d, kBytes / 16, d_sink);
                CK(hipEventRecord(ev, s2));
                CK(hipStreamWaitEvent(s, ev, 0));
            } else if (sc == 4) {
                hipLaunchKernelGGL(reader, dim3(4096), dim3(256), 0, s, (const uint4 *)d, kBytes / 16, d_sink);
            }
            if (sc == 2) CK(hipFreeAsync(d, s));
            CK(hipStreamSynchronize(s));
            CK(hipStreamSynchronize(s2));
        }
        printf("%-40s stale iterations %2d of %d, worst %llu bytes\n", names[sc], fails, kIters, worst);
        fflush(stdout);
        if (sc == 5) free(h);
        else CK(hipHostFree(h));
    }
    CK(hipFree(dev));
    return 0;
}
