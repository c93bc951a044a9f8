// queue_probe.hip — which HIP streams of one process share a hardware queue (GPU_MAX_HW_QUEUES).
//
// Two streams on one hardware queue run their kernels one after the other whatever the stream API
// promises; the D pipeline needs its POA lanes, its orientation context and the clustering streams on
// distinct queues to overlap them.  For every pair of the streams created below the probe launches a
// one-wave spin kernel of `ms` milliseconds on each and times both: ≈ms means the pair ran
// concurrently, ≈2·ms that it shares a queue.
//
// Streams: N plain non-blocking streams (N > GPU_MAX_HW_QUEUES, so the pool wraps), then one of each
// other kind: high priority, low priority, full CU mask.
//
// build: hipcc --offload-arch=gfx950 -O2 -o tools/queue_probe tools/queue_probe.hip
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

// spins for `ticks` of the 100 MHz constant clock; every wave leaves when its own clock passes the mark
__global__ void spin(unsigned long long ticks, int *out) {
    const unsigned long long t0 = wall_clock64();
    unsigned long long t = t0;
    int n = 0;
    while (t - t0 < ticks) {
        t = wall_clock64();
        ++n;
    }
    if (threadIdx.x == 0) out[blockIdx.x] = n;
}

int main(int argc, char **argv) {
    const int n_plain = argc > 1 ? std::atoi(argv[1]) : 6;
    const double ms = argc > 2 ? std::atof(argv[2]) : 40.0;
    CK(hipSetDevice(0));
    int lo = 0, hi = 0;
    CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    const char *env = std::getenv("GPU_MAX_HW_QUEUES");
    std::printf("GPU_MAX_HW_QUEUES=%s priority range least %d greatest %d\n", env ? env : "(unset)", lo, hi);

    std::vector<hipStream_t> s;
    std::vector<std::string> name;
    for (int i = 0; i < n_plain; ++i) {
        hipStream_t x;
        CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
        s.push_back(x);
        name.push_back("plain" + std::to_string(i));
    }
    {
        hipStream_t x;
        CK(hipStreamCreateWithPriority(&x, hipStreamNonBlocking, hi));
        s.push_back(x);
        name.push_back("high");
        CK(hipStreamCreateWithPriority(&x, hipStreamNonBlocking, lo));
        s.push_back(x);
        name.push_back("low");
        hipDeviceProp_t p;
        CK(hipGetDeviceProperties(&p, 0));
        std::vector<uint32_t> mask((size_t)(p.multiProcessorCount + 31) / 32, 0xffffffffu);
        if (p.multiProcessorCount % 32) mask.back() = (1u << (p.multiProcessorCount % 32)) - 1;
        CK(hipExtStreamCreateWithCUMask(&x, (uint32_t)mask.size(), mask.data()));
        s.push_back(x);
        name.push_back("cumask");
    }
    int *out = nullptr;
    CK(hipMalloc(&out, 64 * sizeof(int)));
    const unsigned long long ticks = (unsigned long long)(ms * 1e5);  // 100 MHz
    // warm every stream once
    for (auto x : s) hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, x, 1000ull, out);
    CK(hipDeviceSynchronize());
    const int n = (int)s.size();
    std::printf("pair time / single time (1.0 = concurrent, 2.0 = one queue)\n%8s", "");
    for (int j = 0; j < n; ++j) std::printf(" %7s", name[(size_t)j].c_str());
    std::printf("\n");
    for (int i = 0; i < n; ++i) {
        std::printf("%8s", name[(size_t)i].c_str());
        for (int j = 0; j < n; ++j) {
            if (j <= i) {
                std::printf(" %7s", "");
                continue;
            }
            CK(hipDeviceSynchronize());
            auto t0 = std::chrono::steady_clock::now();
            hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s[(size_t)i], ticks, out);
            hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s[(size_t)j], ticks, out + 1);
            CK(hipStreamSynchronize(s[(size_t)i]));
            CK(hipStreamSynchronize(s[(size_t)j]));
            const double dt = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            std::printf(" %7.2f", dt / ms);
        }
        std::printf("\n");
    }
    CK(hipFree(out));
    for (auto x : s) CK(hipStreamDestroy(x));
    return 0;
}
