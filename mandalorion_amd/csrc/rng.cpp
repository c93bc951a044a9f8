// rng.cpp — numpy legacy RandomState replay for the D module's subsampling draws.
//
// The reference draws `np.random.choice(np.arange(n), min(n, k), replace=False)` from the
// process-global legacy RandomState at /root/reference/utils/SpliceDefineConsensus.py:505 (k=500),
// :818 (k=10000) and :884 (k=100).  For p=None and replace=False numpy returns
// permutation(n)[:k]; permutation shuffles arange(n) by Fisher-Yates from i = n-1 down to 1 with
// j = random_interval(i) (mask-and-reject on 32-bit MT19937 outputs).  Because every locus worker is
// forked from the same parent state (defineIsoforms.py:130), each locus replays the stream of a
// fresh RandomState(seed) — this file reproduces exactly that stream.
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/mando.h"

#include "mt19937.h"

using mando::MT19937;

extern "C" int mando_mt_permutation(uint32_t seed, const int64_t *ns, const int64_t *ks,
                                    int64_t n_draws, int64_t *out, int64_t out_cap) {
    if (n_draws < 0 || (n_draws > 0 && (!ns || !ks))) return MANDO_E_ARG;
    int64_t need = 0;
    for (int64_t d = 0; d < n_draws; ++d) {
        if (ns[d] < 0 || ks[d] < 0 || ks[d] > ns[d]) return MANDO_E_ARG;
        need += ks[d];
    }
    if (need > out_cap || (need > 0 && !out)) return MANDO_E_CAP;
    MT19937 mt(seed);
    std::vector<int64_t> perm;
    int64_t used = 0;
    for (int64_t d = 0; d < n_draws; ++d) {
        const int64_t n = ns[d];
        perm.resize((size_t)n);
        for (int64_t i = 0; i < n; ++i) perm[(size_t)i] = i;
        for (int64_t i = n - 1; i >= 1; --i) {
            const int64_t j = (int64_t)mt.interval((uint64_t)i);
            const int64_t t = perm[(size_t)i];
            perm[(size_t)i] = perm[(size_t)j];
            perm[(size_t)j] = t;
        }
        for (int64_t t = 0; t < ks[d]; ++t) out[used + t] = perm[(size_t)t];
        used += ks[d];
    }
    return MANDO_OK;
}
