// orient_kernel.h — internal interface between capi.hip and orient_kernel.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mando {

constexpr int kOrientCap = 2048;     // largest per-read capacity held in LDS
constexpr int kOrientCapMax = 1 << 22;  // HBM-slab variant beyond it (a read of ~40 Mb)

struct OrientArgs {
    const uint8_t *seq;       // ASCII reads
    const int64_t *seq_off;
    const int64_t *grp_off;
    int32_t n_groups;
    int8_t *hits;             // n_reads * max_hits
    int32_t *n_hits;          // n_reads
    int32_t max_hits;
    int32_t *status;          // per group: 0 ok, -1 over this launch's cap
    int32_t *counter;         // work-queue head (zeroed before launch)
    const int32_t *gidx;      // optional: the group indices to process (a re-run of overflowed groups)
    int32_t cap;              // per-read capacity of this launch (power of two; > kOrientCap: HBM slabs)
    uint64_t *gscratch;       // per launched block an HBM slab of orient_slab_words(cap, cap_fb) words:
                              // the reference keys and the chain table (cap <= kOrientCap), or every array
    int32_t cap_fb;           // cap <= kOrientCap: a group over `cap` is re-run at once in the kernel with
                              // every array in the slab at this capacity (0: left to a host re-run)
};

size_t orient_dyn_bytes(int cap);
int orient_blocks_per_cu(int cap);
size_t orient_slab_words(int cap, int cap_fb);
hipError_t launch_orient(const OrientArgs &a, int n_slots, hipStream_t stream);

}  // namespace mando
