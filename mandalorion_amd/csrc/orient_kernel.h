// orient_kernel.h — internal interface between capi.hip and orient_kernel.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mando {

constexpr int kOrientCap = 2048;  // minimizers per sequence and anchors per read held in LDS

struct OrientArgs {
    const uint8_t *seq;       // ASCII reads
    const int64_t *seq_off;
    const int64_t *grp_off;
    int32_t n_groups;
    int8_t *hits;             // n_reads * max_hits
    int32_t *n_hits;          // n_reads
    int32_t max_hits;
    int32_t *status;          // per group: 0 ok, -1 over kOrientCap
    int32_t *counter;         // work-queue head (zeroed before launch)
};

hipError_t launch_orient(const OrientArgs &a, int n_slots, hipStream_t stream);

}  // namespace mando
