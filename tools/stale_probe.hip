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

struct Scn {
    const char *name;
    int src;        // 0 pinned default, 1 pinned coherent, 2 pageable
    bool pool;      // device buffer from hipMallocAsync / hipFreeAsync on s (else one hipMalloc, reused)
    int reader;     // 0 none, 1 kernel on s2 (event-ordered both ways), 2 kernel on s
    bool pieces;    // 64 MB copies (else one copy)
    bool sync_copy; // hipStreamSynchronize between the copy and the check kernel
    bool sync_free; // hipDeviceSynchronize before the hipFreeAsync (no reliance on events)
};

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
    const Scn scn[] = {
        {"A pinned-default reused", 0, false, 0, true, false, false},
        {"B pinned-coherent reused", 1, false, 0, true, false, false},
        {"C pool recycled + reader s2", 0, true, 1, true, false, false},
        {"D hipMalloc reused + reader s2", 0, false, 1, true, false, false},
        {"E hipMalloc reused + reader s", 0, false, 2, true, false, false},
        {"F pageable source", 2, false, 0, true, false, false},
        {"C1 pool recycled, no reader", 0, true, 0, true, false, false},
        {"C2 pool recycled + reader s", 0, true, 2, true, false, false},
        {"C3 pool + reader s2, one copy", 0, true, 1, false, false, false},
        {"C4 pool + reader s2, pageable src", 2, true, 1, true, false, false},
        {"C5 pool + reader s2, sync after copy", 0, true, 1, true, true, false},
        {"C6 pool + reader s2, device sync before free", 0, true, 1, true, false, true},
    };
    for (const Scn &c : scn) {
        uint8_t *h = nullptr;
        if (c.src == 0) CK(hipHostMalloc((void **)&h, kBytes, hipHostMallocDefault));
        else if (c.src == 1) CK(hipHostMalloc((void **)&h, kBytes, hipHostMallocCoherent));
        else h = (uint8_t *)aligned_alloc(4096, kBytes);
        int fails = 0;
        unsigned long long worst = 0;
        for (int it = 0; it < kIters; ++it) {
            fill(h, it);
            void *d = dev;
            if (c.pool) CK(hipMallocAsync(&d, kBytes, s));
            if (c.pieces) copy_pieces(d, h, s);
            else CK(hipMemcpyAsync(d, h, kBytes, hipMemcpyHostToDevice, s));
            if (c.sync_copy) CK(hipStreamSynchronize(s));
            const unsigned long long bad = check(d, (uint8_t)(0x10 + it), s, d_bad);
            if (bad) ++fails;
            if (bad > worst) worst = bad;
            if (c.reader == 1) {
                CK(hipEventRecord(ev, s));
                CK(hipStreamWaitEvent(s2, ev, 0));
                hipLaunchKernelGGL(reader, dim3(4096), dim3(256), 0, s2, (const uint4 *)d, kBytes / 16, d_sink);
                CK(hipEventRecord(ev, s2));
                CK(hipStreamWaitEvent(s, ev, 0));
            } else if (c.reader == 2) {
                hipLaunchKernelGGL(reader, dim3(4096), dim3(256), 0, s, (const uint4 *)d, kBytes / 16, d_sink);
            }
            if (c.sync_free) CK(hipDeviceSynchronize());
            if (c.pool) CK(hipFreeAsync(d, s));
            CK(hipStreamSynchronize(s));
            CK(hipStreamSynchronize(s2));
        }
        printf("%-46s stale iterations %2d of %d, worst %llu bytes\n", c.name, fails, kIters, worst);
        fflush(stdout);
        if (c.src == 2) free(h);
        else CK(hipHostFree(h));
    }
    // G: D2H into a reused pinned host buffer (the K2 output path): the kernel writes a new pattern, the
    // copy brings it back, the CPU checks every byte
    {
        uint8_t *h = nullptr;
        CK(hipHostMalloc((void **)&h, kBytes, hipHostMallocDefault));
        int fails = 0;
        for (int it = 0; it < kIters; ++it) {
            CK(hipMemsetAsync(dev, 0x40 + it, kBytes, s));
            CK(hipMemcpyAsync(h, dev, kBytes, hipMemcpyDeviceToHost, s));
            CK(hipStreamSynchronize(s));
            size_t bad = 0;
            for (size_t i = 0; i < kBytes; i += 64) bad += h[i] != (uint8_t)(0x40 + it);
            fails += bad != 0;
        }
        printf("%-46s stale iterations %2d of %d\n", "G D2H into reused pinned host", fails, kIters);
        CK(hipHostFree(h));
    }
    CK(hipFree(dev));
    return 0;
}
