// seed_kernel.h — internal interface between capi.hip and seed_kernel.hip (the -S window partition).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mando {

constexpr int kSeedMaxOcc = 8;       // t hashes occurring more often are not anchored (oracle SEED_MAX_OCC)
constexpr int kSeedCapMax = 8192;    // largest per-read minimizer capacity (2 x 64 KB of LDS)

struct SeedArgs {
    const uint8_t *seq;       // encoded bases 0..4
    const int64_t *seq_off;   // per read
    const int32_t *items;     // n_items pairs (t read, q read): q is aligned after t, its predecessor
    const int32_t *redo;      // optional: the item indices to process (re-run at a larger cap)
    int32_t n_items;
    int32_t k, w, min_w, max_occ;
    int32_t pc;               // kept-anchor capacity per item
    int32_t *par_n;           // per item: kept anchors, -1 over capacity
    int32_t *par_t, *par_q;   // item * pc + x: k-mer starts in t and in q
    uint64_t *scratch;        // per block: scratch_words words
    int64_t scratch_words;
    int32_t max_len;          // longest read of any item
    int32_t *counter;         // work-queue head (zeroed before launch)
    int32_t cap;              // per-read minimizer capacity of this launch (power of two)
};

size_t seed_dyn_bytes(int cap);
int64_t seed_scratch_words(int max_len, int cap);
hipError_t launch_seed(const SeedArgs &a, int n_blocks, hipStream_t stream);

}  // namespace mando
