// mt19937_ref.h — (oracle copy) numpy legacy RandomState stream (MT19937 + random_interval + permutation).
// Shared by rng.cpp (mando_mt_permutation) and cluster.cpp (per-locus RNG replay).  See rng.cpp for
// the reference call sites this replays.
#pragma once
#include <cstdint>
#include <vector>

namespace mando_ref {


struct MT19937 {
    uint32_t key[624];
    int pos;
    explicit MT19937(uint32_t seed) {
        for (int i = 0; i < 624; ++i) {
            key[i] = seed;
            seed = 1812433253u * (seed ^ (seed >> 30)) + (uint32_t)i + 1u;
        }
        pos = 624;
    }
    void refill() {
        static const uint32_t mag01[2] = {0u, 0x9908b0dfu};
        int kk = 0;
        for (; kk < 624 - 397; ++kk) {
            uint32_t y = (key[kk] & 0x80000000u) | (key[kk + 1] & 0x7fffffffu);
            key[kk] = key[kk + 397] ^ (y >> 1) ^ mag01[y & 1u];
        }
        for (; kk < 623; ++kk) {
            uint32_t y = (key[kk] & 0x80000000u) | (key[kk + 1] & 0x7fffffffu);
            key[kk] = key[kk + (397 - 624)] ^ (y >> 1) ^ mag01[y & 1u];
        }
        uint32_t y = (key[623] & 0x80000000u) | (key[0] & 0x7fffffffu);
        key[623] = key[396] ^ (y >> 1) ^ mag01[y & 1u];
        pos = 0;
    }
    uint32_t next32() {
        if (pos == 624) refill();
        uint32_t y = key[pos++];
        y ^= (y >> 11);
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= (y >> 18);
        return y;
    }
    uint64_t next64() {
        uint64_t hi = next32();
        uint64_t lo = next32();
        return (hi << 32) | lo;
    }
    uint64_t interval(uint64_t max) {
        if (max == 0) return 0;
        uint64_t mask = max;
        mask |= mask >> 1;
        mask |= mask >> 2;
        mask |= mask >> 4;
        mask |= mask >> 8;
        mask |= mask >> 16;
        mask |= mask >> 32;
        uint64_t v;
        if (max <= 0xffffffffull) {
            while ((v = (next32() & mask)) > max) {
            }
        } else {
            while ((v = (next64() & mask)) > max) {
            }
        }
        return v;
    }
};


// numpy `RandomState.permutation(n)[:k]` == `choice(arange(n), k, replace=False)` (p=None)
inline void mt_choice(MT19937 &mt, int64_t n, int64_t k, std::vector<int64_t> &perm, std::vector<int64_t> &out) {
    perm.resize((size_t)n);
    for (int64_t i = 0; i < n; ++i) perm[(size_t)i] = i;
    for (int64_t i = n - 1; i >= 1; --i) {
        const int64_t j = (int64_t)mt.interval((uint64_t)i);
        const int64_t t = perm[(size_t)i];
        perm[(size_t)i] = perm[(size_t)j];
        perm[(size_t)j] = t;
    }
    out.assign(perm.begin(), perm.begin() + k);
}

}  // namespace mando
