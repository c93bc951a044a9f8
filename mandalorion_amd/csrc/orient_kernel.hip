// orient_kernel.hip — read orientation (mappy map-ont strand / primary-hit replacement).
// Placeholder until the minimizer-chain kernel lands: reports MANDO_E_UNSUPPORTED (no CPU fallback).
#include <hip/hip_runtime.h>
#include "../../include/mando.h"

extern "C" int mando_orient_batch(mando_ctx *ctx, const uint8_t *seqs, const int64_t *seq_off,
                                  const int64_t *grp_off, int64_t n_groups, int8_t *hit_strands,
                                  int32_t max_hits, int32_t *n_hits) {
    (void)ctx; (void)seqs; (void)seq_off; (void)grp_off; (void)n_groups; (void)hit_strands;
    (void)max_hits; (void)n_hits;
    return MANDO_E_UNSUPPORTED;
}
