// orient_kernel.hip — read orientation on gfx950 (replaces mappy map-ont strand / primary calls).
//
// Reference: SpliceDefineConsensus.py:895-907 maps every subsampled read of an isoform against a
// one-sequence minimap2 index of the first subsampled read and keeps, per primary hit, the read
// (reverse-complemented for strand -1).  The specification followed here — and by the CPU checker
// oracle/orient_ref.c, bit for bit — is the map-ont subset that decides strand and primary status:
// (15,10) minimizers, a one-sequence index with a max-occurrence filter, chaining DP, greedy chain
// extraction and mask_level-0.5 primary selection (see oracle/orient_ref.c for the exact rules and
// the known differences from minimap2; parity with mappy itself is unpinned).
//
// Layout: one 64-lane wave per isoform group (persistent over groups).  Two per-read arrays hold `cap`
// entries (a power of two chosen per launch, 1024 for R2C2-length reads; groups that overflow are
// re-run by the host at the next capacity):
//   refk  sorted reference minimizer keys  (h << 33 | pos << 1 | strand)   8 B x cap, the wave's HBM slab
//   an    anchor keys (rev << 62 | x << 31 | y), bitonic-sorted in LDS; after the chaining DP each
//         slot is rewritten as used << 63 | f << 48 | (p + 1) << 32 | rev << 31 | y   8 B x cap, dynamic LDS
// With the keys in HBM (a bucket index over their top hash bits stays in LDS) a wave takes 10 KB of
// LDS and 16 waves fit per CU, the VGPR limit (both arrays in LDS: 20 KB, 8 waves; 1.47x slower).
// The query's minimizers are not stored: each 64-position batch of them is looked up in refk as it is
// found and its anchors appended.  Beyond kOrientCap (2048, ~10 kb reads) the same code runs with the
// anchors in the HBM slab too (orient_kernel<true>), with f[] / p[] and a used bitmap of their own,
// so long reads are oriented instead of refused.
// Minimizers are computed in 128-position tiles (k-mer hashes -> window minima -> marks -> ballot
// compaction); the chaining DP is sequential over anchors with the 64-anchor look-back spread over the
// 64 lanes and a DPP max-reduction per anchor.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "orient_kernel.h"

namespace mando {
namespace {

constexpr int K = 15, W = 10, MAX_OCC = 10, MAX_GAP = 5000, BW = 500, MIN_CNT = 3, MIN_SCORE = 40;
// 128-position minimizer tiles: the tile buffers are half of a 256-position tile's, which with the
// keys in HBM brings a wave to 10 KB of LDS (16 waves per CU; 256: 14, 62.0 against 58.0 ms)
constexpr int TILE = 128;
constexpr int MAXCH = 64;
constexpr int kChWords = 4 * MAXCH / 2;  // the chain table in 64-bit words (slabs of the LDS variant: cap + kChWords)
constexpr int kBucketShift = 2 * K - 8, kBuckets = 1 << 8;  // refk index over the top 8 hash bits
constexpr uint64_t INF = ~0ull;
constexpr uint32_t INF32 = ~0u;

// bases one tile's k-mers touch (k-mer starts h0 .. h0 + TILE + 2W - 2), staged once per tile as
// 2-bit codes, 16 per word with the first base in the top bits, plus a 1-bit-per-base mask of
// non-ACGT bases (and of positions outside the read)
constexpr int TB = TILE + 2 * W - 1 + K - 1;
constexpr int NPK = ((TB + 15) / 16 + 1 + 3) / 4 * 4;  // + the second word of the last window; x4 lanes
constexpr int NNM = NPK / 4 + 1;                       // 64-bit words; +1 read (masked) past the end
static_assert(NPK * 16 >= TB + 16 && (NPK * 16) % 64 == 0, "tile staging size");

// fixed-size part (static LDS); the cap-sized arrays live in dynamic LDS (see OrientDyn)
struct OrientLds {
    int cap;
    uint64_t *gdyn;  // the cap-sized arrays in HBM (the long-read variant), else null
    uint32_t pk[NPK];           // staged 2-bit codes
    uint64_t nm[NNM];           // staged non-ACGT mask
    uint32_t hb[TILE + 2 * W];  // (hash << 1 | z) of the tile's k-mers (30-bit hashes), INF32 when invalid
    uint32_t mb[TILE + W];      // window minima (hash only)
    int32_t misc[8];
    uint16_t bst[kBuckets + 1];  // LDS variant: first refk index of each top-8-bit hash bucket
#ifdef MANDO_ORIENT_PROF
    uint64_t prof[8], tlast;
#endif
};
#ifdef MANDO_ORIENT_PROF
// dev builds: per-phase wall cycles summed over waves, printed by the last wave of each launch
__device__ unsigned long long g_oprof[8];
__device__ unsigned int g_odone;
#define OPROF(i)                                     \
    if (lane == 0) {                                 \
        const uint64_t t_ = wall_clock64();          \
        sh.prof[i] += t_ - sh.tlast;                 \
        sh.tlast = t_;                               \
    }
#else
#define OPROF(i)
#endif
extern __shared__ __attribute__((aligned(16))) uint64_t g_orient_dyn[];  // 2 * cap words
// views into the dynamic buffer (LDS address space kept: the base is the LDS symbol itself)
// G: the arrays live in a per-wave HBM slab (reads beyond the LDS capacity) instead of dynamic LDS
__device__ __forceinline__ int o_cap(const OrientLds &sh) { return __builtin_amdgcn_readfirstlane(sh.cap); }
// the reference keys: always in the wave's HBM slab (read by the query lookups, a few dependent loads
// per 64 query positions); the anchors: in dynamic LDS, or (G) in the slab past the keys.  With only
// the anchors in LDS a wave takes 10 KB instead of 20 KB: 16 waves per CU instead of 8 (orientation
// kernel 85.6 -> 58 ms on 32,000 groups x 25 reads x 3 kb, profiles/r06f_ab_orient_ref_hbm.txt)
template <bool G>
__device__ __forceinline__ uint64_t *o_refk(const OrientLds &sh) { return sh.gdyn; }
template <bool G>
__device__ __forceinline__ uint64_t *o_an(const OrientLds &sh) { return G ? sh.gdyn + 2 * o_cap(sh) : g_orient_dyn; }
// HBM variant only: f[] / p[] of the chaining DP and the used bitmap
__device__ __forceinline__ int32_t *o_f(const OrientLds &sh) { return reinterpret_cast<int32_t *>(sh.gdyn + o_cap(sh)); }
__device__ __forceinline__ int32_t *o_p(const OrientLds &sh) { return o_f(sh) + o_cap(sh); }
__device__ __forceinline__ uint64_t *o_used(const OrientLds &sh) { return sh.gdyn + 3 * o_cap(sh); }
// LDS variant: the DP's results packed into the anchor slot (f < 2^15 and p + 1 < 2^16 for cap <= kOrientCap)
constexpr uint64_t kUsed = 1ull << 63;
__device__ __forceinline__ int slot_f(uint64_t s) { return (int)((s >> 48) & 0x7fff); }
__device__ __forceinline__ int slot_p(uint64_t s) { return (int)((s >> 32) & 0xffff) - 1; }
static_assert(kOrientCap * K < (1 << 15) && kOrientCap < (1 << 16), "packed f / p fields");

__device__ __forceinline__ int lane_id() { return (int)__lane_id(); }
// words of a wave's HBM slab: every array at `cap` (cap > kOrientCap), else the keys at cap, plus the
// arrays of the in-kernel fallback at cap_fb (0: none) and the chain table
__host__ __device__ __forceinline__ int64_t slab_words(int cap, int cap_fb) {
    if (cap > kOrientCap) return 3 * (int64_t)cap + cap / 64;
    const int64_t keys = cap_fb > 0 ? 3 * (int64_t)cap_fb + cap_fb / 64 : (int64_t)cap;
    return keys + kChWords;
}
// the workgroup is one wave, and a wave's LDS accesses complete in order: waiting for its own LDS
// traffic (with a compiler memory barrier) is the whole sync.  __syncthreads() would also wait for
// every outstanding global load (its workgroup-scope fence), e.g. the next tile's bases.
__device__ __forceinline__ void wsync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// A/a 0, C/c 1, G/g 2, T/t 3, anything else 4, without branches: ((c >> 1) ^ (c >> 2)) & 3 maps the
// eight letters to their codes
__device__ __forceinline__ int enc(uint8_t c) {
    const uint32_t u = c & 0xdfu;
    const bool ok = u == 'A' || u == 'C' || u == 'G' || u == 'T';
    return ok ? (int)(((c >> 1) ^ (c >> 2)) & 3u) : 4;
}

// hash64(key, 2^30 - 1) in 32-bit arithmetic: every step is masked to 30 bits (the low bits of a sum
// depend only on the low bits of its terms) and the last step's key << 31 is masked away entirely
__device__ __forceinline__ uint32_t hash30(uint32_t key) {
    constexpr uint32_t mask = (1u << (2 * K)) - 1;
    key = (~key + (key << 21)) & mask;
    key = key ^ key >> 24;
    key = ((key + (key << 3)) + (key << 8)) & mask;
    key = key ^ key >> 14;
    key = ((key + (key << 2)) + (key << 4)) & mask;
    key = key ^ key >> 28;
    return key;
}

__device__ __forceinline__ int wave_sum(int v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
    for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o, 64));
    return v;
}
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t u = __shfl_xor(v, o, 64);
        v = u > v ? u : v;
    }
    return v;
}
// wave-wide max of a non-negative int (every lane gets it): DPP inclusive max, then lane 63
__device__ __forceinline__ int wave_max_dpp(int v) {
    asm volatile("s_nop 1\n"
                 "v_max_i32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf\n s_nop 1\n"
                 "v_max_i32_dpp %0, %0, %0 row_shr:2 row_mask:0xf bank_mask:0xf\n s_nop 1\n"
                 "v_max_i32_dpp %0, %0, %0 row_shr:4 row_mask:0xf bank_mask:0xf\n s_nop 1\n"
                 "v_max_i32_dpp %0, %0, %0 row_shr:8 row_mask:0xf bank_mask:0xf\n s_nop 1\n"
                 "v_max_i32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n s_nop 1\n"
                 "v_max_i32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf\n"
                 : "+v"(v));
    return __builtin_amdgcn_readlane(v, 63);
}
// the same max with DPP builtins, so the compiler may fill the DPP wait states with independent work
__device__ __forceinline__ int wave_max_dpp_sched(int v) {
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false));  // row_shr:1
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false));  // row_shr:2
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false));  // row_shr:4
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false));  // row_shr:8
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false));  // row_bcast:15
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false));  // row_bcast:31
    return __builtin_amdgcn_readlane(v, 63);
}
// inclusive prefix sum over the wave (DPP row scans, then the row carries)
__device__ __forceinline__ int wave_incl_sum(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);  // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);  // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);  // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);  // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);  // row_bcast:15
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return v;
}
// lane l receives lane l+1's value; lane 63 receives `fill`
__device__ __forceinline__ int wave_shl1(int v, int fill) {
    return __builtin_amdgcn_update_dpp(fill, v, 0x130, 0xf, 0xf, false);
}

__device__ __forceinline__ unsigned long long lanemask_lt(int lane) {
    return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

// minimizers of s[0, L) in position order, handed to sink(mark, key) one 64-position batch at a time
// (the whole wave calls it; key = h << 33 | pos << 1 | strand on the marked lanes); a sink returning
// false (over capacity) ends the scan and minimizers() returns false
template <class Sink>
__device__ bool minimizers(OrientLds &sh, const uint8_t *s, int64_t L, int lane, Sink &&sink) {
    if (L < K) return true;
    const int64_t np = L - K + 1;
    const int64_t nw = np <= W ? 1 : np - W + 1;
    const int ww = np <= W ? (int)np : W;
    const uint32_t mask30 = (1u << (2 * K)) - 1;
    // the bases of the next tile are loaded while this one is processed (NPK / 4 bytes per lane)
    constexpr int NST = NPK * 16 / 64;
    uint8_t nxt[NST];
#pragma unroll
    for (int j = 0; j < NST; ++j) {
        const int64_t p = -(W - 1) + 64 * j + lane;
        nxt[j] = (p >= 0 && p < L) ? s[p] : (uint8_t)'N';
    }
    for (int64_t t0 = 0; t0 < np; t0 += TILE) {
        const int64_t h0 = t0 - (W - 1);  // position of hb[0] and of window mb[0]
        uint8_t cur[NST];
#pragma unroll
        for (int j = 0; j < NST; ++j) cur[j] = nxt[j];
        if (t0 + TILE < np) {
#pragma unroll
            for (int j = 0; j < NST; ++j) {
                const int64_t p = h0 + TILE + 64 * j + lane;
                nxt[j] = p < L ? s[p] : (uint8_t)'N';
            }
        }
        // stage the tile's bases: 16 two-bit codes OR-reduced per word
#pragma unroll
        for (int j = 0; j < NST; ++j) {
            const int e0 = 64 * j;
            const int e = e0 + lane;
            const int c = enc(cur[j]);
            int v = c > 3 ? 0 : c << (2 * (15 - (lane & 15)));
            // OR over each row of 16 lanes (DPP inclusive scan): lane 15 of the row holds the word
            v |= __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);
            v |= __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);
            v |= __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);
            v |= __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);
            const unsigned long long bad = __ballot(c > 3);
            if ((lane & 15) == 15) sh.pk[e >> 4] = (uint32_t)v;
            if (lane == 0) sh.nm[e0 >> 6] = bad;
        }
        if (lane == 0) sh.nm[NNM - 1] = ~0ull;
        wsync();
        // (hash << 1 | z) of each k-mer: a 30-bit window of two staged words; the reverse complement
        // by complementing and reversing the 2-bit groups
        for (int e = lane; e < TILE + 2 * W - 1; e += 64) {
            const int64_t p = h0 + e;
            uint32_t hz = INF32;
            if (p >= 0 && p < np) {
                uint64_t m = sh.nm[e >> 6] >> (e & 63);
                if ((e & 63) > 64 - K) m |= sh.nm[(e >> 6) + 1] << (64 - (e & 63));
                if (!(m & ((1ull << K) - 1))) {
                    const int q = e >> 4, o = e & 15;
                    const uint64_t w = ((uint64_t)sh.pk[q] << 32) | sh.pk[q + 1];
                    const uint32_t f = (uint32_t)(w >> (2 * (32 - o - K))) & mask30;
                    const uint32_t x = __builtin_bitreverse32(f ^ mask30) >> (32 - 2 * K);
                    const uint32_t r = ((x >> 1) & 0x15555555u) | ((x & 0x15555555u) << 1);
                    if (f != r) hz = (hash30(f < r ? f : r) << 1) | (f < r ? 0u : 1u);
                }
            }
            sh.hb[e] = hz;
        }
        wsync();
        for (int e = lane; e < TILE + W - 1; e += 64) {
            const int64_t w0 = h0 + e;
            uint32_t m = INF32;
            if (w0 >= 0 && w0 < nw) {
                if (ww == W) {
#pragma unroll
                    for (int t = 0; t < W; ++t) {
                        const uint32_t v = sh.hb[e + t];
                        const uint32_t hv = v == INF32 ? INF32 : v >> 1;
                        m = hv < m ? hv : m;
                    }
                } else {
                    for (int t = 0; t < ww; ++t) {
                        const uint32_t v = sh.hb[e + t];
                        const uint32_t hv = v == INF32 ? INF32 : v >> 1;
                        m = hv < m ? hv : m;
                    }
                }
            }
            sh.mb[e] = m;
        }
        wsync();
        for (int i0 = 0; i0 < TILE; i0 += 64) {
            const int64_t p = t0 + i0 + lane;
            bool mark = false;
            uint32_t v = INF32;
            if (p < np) {
                v = sh.hb[i0 + lane + (W - 1)];
                if (v != INF32) {
                    const int64_t slo = p - ww + 1 > 0 ? p - ww + 1 : 0;
                    const int64_t shi = p < nw - 1 ? p : nw - 1;
                    if (ww == W) {
                        // every window holding p has minimum <= h(p), so p is some window's minimum
                        // iff h(p) <= the largest of those minima: W independent LDS reads, no break
                        uint32_t mx = 0;
#pragma unroll
                        for (int t = 0; t < W; ++t) {
                            const int64_t w0 = p - (W - 1) + t;
                            const uint32_t mv = sh.mb[i0 + lane + t];  // mb index of window w0
                            if (w0 >= slo && w0 <= shi) mx = mv > mx ? mv : mx;
                        }
                        mark = (v >> 1) <= mx;
                    } else {
                        for (int64_t w0 = slo; w0 <= shi; ++w0)
                            if (sh.mb[w0 - h0] == (v >> 1)) {
                                mark = true;
                                break;
                            }
                    }
                }
            }
            const uint64_t key = ((uint64_t)(v >> 1) << 33) | ((uint64_t)(p + K - 1) << 1) | (uint64_t)(v & 1u);
            if (!sink(mark, key)) return false;
        }
        wsync();
    }
    return true;
}

// bitonic sort of a[0, n) held in registers: lane l owns elements l * P .. l * P + P - 1 (INF past n),
// so strides below P are compare-exchanges inside a lane and larger ones one 64-bit lane swap per
// element; no LDS traffic or barriers between stages (n <= 64 * P)
__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m) {
    const int lo = __shfl_xor((int)(uint32_t)v, m, 64), hi = __shfl_xor((int)(uint32_t)(v >> 32), m, 64);
    return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}
template <int P, int S>
__device__ __forceinline__ void cx_lane(uint64_t (&v)[P], int lane, int size) {
#pragma unroll
    for (int k = 0; k < P; ++k) {
        if (k & S) continue;
        const bool asc = ((lane * P + k) & size) == 0;
        const uint64_t x = v[k], y = v[k | S];
        const bool sw = (x > y) == asc;
        v[k] = sw ? y : x;
        v[k | S] = sw ? x : y;
    }
}
template <int P>
__device__ void sort_regs(uint64_t *a, int n, int lane) {
    uint64_t v[P];
#pragma unroll
    for (int k = 0; k < P; ++k) {
        const int i = lane * P + k;
        v[k] = i < n ? a[i] : INF;
    }
    int n2 = 64 * P;
    while (n2 / 2 >= n && n2 > P) n2 >>= 1;  // stages past the padded size are no-ops
    for (int size = 2; size <= n2; size <<= 1)
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            if (stride >= P) {
                const int lm = stride / P;
                const bool keep_min = ((lane & lm) == 0) == (((lane * P) & size) == 0);
#pragma unroll
                for (int k = 0; k < P; ++k) {
                    const uint64_t o = shfl_xor64(v[k], lm);
                    v[k] = ((v[k] > o) == keep_min) ? o : v[k];
                }
            } else if (stride == 1) {
                cx_lane<P, 1>(v, lane, size);
            } else if (stride == 2) {
                if constexpr (P > 2) cx_lane<P, 2>(v, lane, size);
            } else if (stride == 4) {
                if constexpr (P > 4) cx_lane<P, 4>(v, lane, size);
            } else if (stride == 8) {
                if constexpr (P > 8) cx_lane<P, 8>(v, lane, size);
            }
        }
#pragma unroll
    for (int k = 0; k < P; ++k) {
        const int i = lane * P + k;
        if (i < n) a[i] = v[k];
    }
    wsync();
}

__device__ void bitonic_sort_lds(uint64_t *a, int n, int lane) {
    int n2 = 1;
    while (n2 < n) n2 <<= 1;
    for (int i = n + lane; i < n2; i += 64) a[i] = INF;
    wsync();
    for (int size = 2; size <= n2; size <<= 1)
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int t = lane; t < n2 / 2; t += 64) {
                const int i = 2 * t - (t & (stride - 1));
                const int j = i + stride;
                const bool asc = (i & size) == 0;
                const uint64_t x = a[i], y = a[j];
                if ((x > y) == asc) {
                    a[i] = y;
                    a[j] = x;
                }
            }
            wsync();
        }
}

// sort a[0, n) ascending: registers up to 1024 elements, the LDS/HBM network beyond
__device__ void bitonic_sort(uint64_t *a, int n, int lane) {
    if (n <= 1) return;
    if (n <= 256) {
        sort_regs<4>(a, n, lane);
    } else if (n <= 512) {
        sort_regs<8>(a, n, lane);
    } else if (n <= 1024) {
        sort_regs<16>(a, n, lane);
    } else {
        bitonic_sort_lds(a, n, lane);
    }
}

__device__ __forceinline__ int lower_bound_h(const uint64_t *a, int lo, int hi, uint64_t h) {
    const uint64_t key = h << 33;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (a[mid] < key)
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo;
}

__device__ __forceinline__ int ilog2_u32(uint32_t v) { return 31 - __clz((int)v); }

// one query read; returns 0 or -1 (over CAP)
// ch: the extracted chains' score / strand / query start / query end, MAXCH each (LDS, or the wave's
// HBM slab: lane 0 alone writes and reads them)
template <bool G>
__device__ int orient_read(OrientLds &sh, int32_t *ch, int nref, const uint8_t *q, int64_t qlen, int8_t *hits,
                           int max_hits, int32_t *n_hits, int lane) {
    int32_t *ch_score = ch, *ch_rev = ch + MAXCH, *ch_qs = ch + 2 * MAXCH, *ch_qe = ch + 3 * MAXCH;
    const uint64_t *refk = o_refk<G>(sh);
    uint64_t *an = o_an<G>(sh);
    const int cap = o_cap(sh);
    // anchors, one batch of query minimizers at a time: count per minimizer, wave scan, scatter
    int na = 0;
    OPROF(7)
    const bool fits = minimizers(sh, q, qlen, lane, [&](bool mark, uint64_t key) -> bool {
        if (!__ballot(mark)) return true;
        int lo = 0, cnt = 0;
        if (mark) {
            const uint64_t h = key >> 33;
            if constexpr (G) {
                lo = lower_bound_h(refk, 0, nref, h);
            } else {  // within h's bucket (~2 entries for R2C2 reads) instead of all of refk
                const int b = (int)(h >> kBucketShift);
                lo = lower_bound_h(refk, sh.bst[b], sh.bst[b + 1], h);
            }
            while (lo + cnt < nref && (refk[lo + cnt] >> 33) == h && cnt <= MAX_OCC) ++cnt;
            if (cnt > MAX_OCC) cnt = 0;
        }
        const int incl = wave_incl_sum(cnt);
        const int tot = __builtin_amdgcn_readlane(incl, 63);
        if (na + tot > cap) return false;
        const int base = na + incl - cnt;
        const int64_t qpos = (int64_t)((key >> 1) & 0xffffffffull);
        const int qz = (int)(key & 1);
        for (int t = 0; t < cnt; ++t) {
            const uint64_t r = refk[lo + t];
            const int64_t rpos = (int64_t)((r >> 1) & 0xffffffffull);
            const int rev = qz ^ (int)(r & 1);
            const int64_t y = rev ? qlen - 1 - (qpos - K + 1) : qpos;
            an[base + t] = ((uint64_t)rev << 62) | ((uint64_t)rpos << 31) | (uint64_t)y;
        }
        na += tot;
        return true;
    });
    if (!fits) return -1;
    wsync();
    OPROF(1)
    bitonic_sort(an, na, lane);
    OPROF(2)
    // chaining DP: lane l looks at predecessor j = i - 64 + l.  The 64-anchor look-back window (x, y,
    // strand, f) lives in registers and slides one lane per anchor (DPP wave_shl); the best
    // predecessor is one DPP max-reduction.  Software-pipelined by one anchor: the reduction for
    // anchor i covers lanes 0..62 (anchors i-64 .. i-2, whose f are known one anchor early) and runs
    // while anchor i-1's f is being decided; anchor i-1 (lane 63, f = f_prev) joins as one scalar
    // max, so the loop-carried chain is a few scalar ops.  Only lane 0 stores f / p (for the chain
    // walk below): in the LDS variant into anchor i's own slot, which the DP has read by then.
    // window x is rev << 30 | x (positions < 2^30), so a strand mismatch puts dr far outside
    // (0, MAX_GAP]; an empty slot (j < 0) has x = INT_MAX.  wf lane 63 is unused.
    int wx = 0x7fffffff, wy = 0, wf = 0;
    // best key of lanes 0..62 for the anchor at (xa, ya) and lane 63's score term (0: no predecessor)
    auto reduce = [&](int xa, int ya, int &t63) -> int {
        const int dr = xa - wx, dq = ya - wy;
        const uint32_t dd = __usad((uint32_t)dr, (uint32_t)dq, 0u);  // |dr - dq| where both are > 0
        const bool valid = min(dr, dq) > 0 && max(dr, dq) <= MAX_GAP && dd <= (uint32_t)BW;
        // min(dq, dr, K) - (dd * 15 / 100 + ilog2(dd) / 2): dd * 15 / 100 == dd * 157287 >> 20 for
        // dd <= BW, and ilog2(dd | 1) == ilog2(dd) with 0 for dd == 0
        const int sc = min(min(dq, dr), K) - (int)((dd * 157287u) >> 20) - ((31 - __clz((int)(dd | 1u))) >> 1);
        const int kv = valid ? sc + 65536 : 0;
        t63 = __builtin_amdgcn_readlane(kv, 63);
        return wave_max_dpp_sched(valid && lane != 63 ? ((wf + kv) << 6) | lane : 0);
    };
    // anchor fields, wave-uniform (every lane read the same slot)
    auto uload = [&](uint64_t v, int &x, int &y, int &r) {
        const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
        const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
        r = (int)(hi >> 30);
        x = (int)((((hi << 1) | (lo >> 31)) & 0x3fffffffu) | ((hi & 0x40000000u)));
        y = (int)(lo & 0x7fffffffu);
    };
    int xi = 0, yi = 0, ri = 0;
    if (na > 0) uload(an[0], xi, yi, ri);
    uint64_t an_next = na > 1 ? an[1] : 0;  // one anchor ahead: the LDS read leaves the DP chain
    int t63 = 0;
    int part = na > 0 ? reduce(xi, yi, t63) : 0;
    int f_prev = 0;
    for (int i = 0; i < na; ++i) {
        // anchor i: lanes 0..62 (part) and lane 63 = anchor i-1 with f_prev
        const int k63 = t63 ? ((f_prev + t63) << 6) | 63 : 0;
        const int best = part > k63 ? part : k63;
        const int cand = (best >> 6) - 65536;
        const bool take = best != 0 && cand > K;
        const int fi = take ? cand : K;
        if (lane == 0) {
            const int pi = take ? i - 64 + (best & 63) : -1;
            if constexpr (G) {
                o_f(sh)[i] = fi;
                o_p(sh)[i] = pi;
            } else {
                an[i] = ((uint64_t)fi << 48) | ((uint64_t)(pi + 1) << 32) | ((uint64_t)ri << 31) | (uint64_t)yi;
            }
        }
        // the window for anchor i+1: anchor i enters lane 63, f of anchor i-1 lands in lane 62
        wx = wave_shl1(wx, xi);
        wy = wave_shl1(wy, yi);
        {
            const int sh1 = wave_shl1(wf, 0);
            wf = lane == 62 ? f_prev : sh1;
        }
        if (i + 1 < na) {
            uload(an_next, xi, yi, ri);
            if (i + 2 < na) an_next = an[i + 2];
            part = reduce(xi, yi, t63);
        }
        f_prev = fi;
    }
    wsync();
    OPROF(3)
    // greedy chain extraction: highest f first (ties: lowest index), walk back to a used anchor
    if constexpr (G) {
        for (int t = lane; t < cap / 64; t += 64) o_used(sh)[t] = 0;
        wsync();
    }
    int nch = 0;
    for (int it = 0;; ++it) {
        if (it > na) return -1;  // each pass marks its best anchor used: never reached
        uint64_t bk = 0;  // (f + 2^20) << 32 | (2^31 - 1 - i): max picks highest f, then lowest i
        for (int c0 = 0; c0 < na; c0 += 64) {
            const int i = c0 + lane;
            if (i >= na) continue;
            int fv;
            if constexpr (G) {
                if ((o_used(sh)[i >> 6] >> (i & 63)) & 1) continue;
                fv = o_f(sh)[i];
            } else {
                const uint64_t sl = an[i];
                if (sl & kUsed) continue;
                fv = slot_f(sl);
            }
            const uint64_t k = ((uint64_t)(uint32_t)(fv + (1 << 20)) << 32) | (uint64_t)(0x7fffffff - i);
            bk = k > bk ? k : bk;
        }
        bk = wave_max_u64(bk);
        if (bk == 0) break;
        const int fbest = (int)(bk >> 32) - (1 << 20);
        const int bi = 0x7fffffff - (int)(bk & 0xffffffffull);
        if (fbest < MIN_SCORE) break;
        if (lane == 0) {
            int k = bi, first = bi, cnt = 0, fk = 0;
            if constexpr (G) {
                while (k >= 0 && !((o_used(sh)[k >> 6] >> (k & 63)) & 1)) {
                    o_used(sh)[k >> 6] |= 1ull << (k & 63);
                    ++cnt;
                    first = k;
                    k = o_p(sh)[k];
                }
                fk = k >= 0 ? o_f(sh)[k] : 0;
            } else {
                // one LDS read per step: the slot holds the used flag, p and f
                uint64_t sl = an[k];
                while (!(sl & kUsed)) {
                    an[k] = sl | kUsed;
                    ++cnt;
                    first = k;
                    k = slot_p(sl);
                    if (k < 0) break;
                    sl = an[k];
                }
                fk = k >= 0 ? slot_f(sl) : 0;
            }
            const int score = fbest - fk;
            int ok = 0;
            if (cnt >= MIN_CNT && score >= MIN_SCORE) {
                if (nch >= MAXCH) {
                    ok = -1;
                } else {
                    // G: anchor keys (rev << 62 | x << 31 | y); LDS: slots (rev << 31 | y)
                    const uint64_t sb = an[bi], sf = an[first];
                    const int rev = G ? (int)(sb >> 62) : (int)((sb >> 31) & 1);
                    ch_score[nch] = score;
                    ch_rev[nch] = rev;
                    const int ys = (int)(sf & 0x7fffffff) - K + 1, ye = (int)(sb & 0x7fffffff) + 1;
                    ch_qs[nch] = rev ? (int)qlen - ye : ys;
                    ch_qe[nch] = rev ? (int)qlen - ys : ye;
                    ok = 1;
                }
            }
            sh.misc[0] = ok;
        }
        wsync();
        const int ok = sh.misc[0];
        wsync();
        if (ok < 0) return -1;
        nch += ok;
    }
    OPROF(4)
    // primary selection (lane 0): decreasing score, extraction order on ties (stable insertion sort)
    if (lane == 0) {
        int idx[MAXCH];
        for (int c = 0; c < nch; ++c) {
            int t = c;
            while (t > 0 && ch_score[idx[t - 1]] < ch_score[c]) {
                idx[t] = idx[t - 1];
                --t;
            }
            idx[t] = c;
        }
        int np = 0;
        // one primary past max_hits (<= 8) is still counted: n_hits == max_hits + 1 reports the
        // overflow, and the host re-runs with room for more (the reference writes every primary)
        int pqs[9], pqe[9];
        for (int c = 0; c < nch && np <= max_hits && np < 9; ++c) {
            const int id = idx[c];
            const int qs = ch_qs[id], qe = ch_qe[id];
            bool prim = true;
            for (int t = 0; t < np; ++t) {
                const int ov = min(qe, pqe[t]) - max(qs, pqs[t]);
                const int l0 = qe - qs, l1 = pqe[t] - pqs[t];
                if (2 * ov > min(l0, l1)) {
                    prim = false;
                    break;
                }
            }
            if (!prim) continue;
            pqs[np] = qs;
            pqe[np] = qe;
            if (np < max_hits) hits[np] = ch_rev[id] ? -1 : 1;
            ++np;
        }
        *n_hits = np;
    }
    wsync();
    OPROF(5)
    return 0;
}

// one group: 0, or -1 when a read is over the capacity o_cap(sh) (its outputs are then rewritten in full
// by the re-run)
template <bool G>
__device__ int orient_group(OrientLds &sh, int32_t *ch, const OrientArgs &a, int g, int lane) {
    const int64_t r0 = a.grp_off[g], r1 = a.grp_off[g + 1];
    if (r1 <= r0) return 0;
    uint64_t *refk = o_refk<G>(sh);
    int nref = 0;
    const bool fits = minimizers(sh, a.seq + a.seq_off[r0], a.seq_off[r0 + 1] - a.seq_off[r0], lane,
                                 [&](bool mark, uint64_t key) -> bool {
                                     const unsigned long long m = __ballot(mark);
                                     const int cnt = __popcll(m);
                                     if (nref + cnt > o_cap(sh)) return false;
                                     if (mark) refk[nref + __popcll(m & lanemask_lt(lane))] = key;
                                     nref += cnt;
                                     return true;
                                 });
    wsync();
    if (!fits) return -1;
    bitonic_sort(o_refk<G>(sh), nref, lane);
    // (HBM keys: the sorted stores complete before any lane reads another lane's keys)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    OPROF(6)
    if constexpr (!G) {
        for (int b = lane; b <= kBuckets; b += 64)
            sh.bst[b] = (uint16_t)lower_bound_h(refk, 0, nref, (uint64_t)b << kBucketShift);
        wsync();
    }
    for (int64_t r = r0; r < r1; ++r) {
        const int rc = orient_read<G>(sh, ch, nref, a.seq + a.seq_off[r], a.seq_off[r + 1] - a.seq_off[r],
                                      a.hits + r * a.max_hits, a.max_hits, a.n_hits + r, lane);
        if (rc < 0) return -1;
    }
    return 0;
}

template <bool G>
// at most 128 VGPRs: the orientation runs beside the POA grids of the chunk before (cluster_kernel.hip,
// cluster_locus)
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4))) void orient_kernel(OrientArgs a) {
    __shared__ OrientLds sh;
    const int lane = lane_id();
    // the wave's HBM slab: G's arrays at a.cap; the LDS variant's keys, its fallback's arrays at a.cap_fb
    // and the chain table at the end
    const int64_t slab = slab_words(a.cap, G ? 0 : a.cap_fb);
    if (lane == 0) {
#ifdef MANDO_ORIENT_PROF
        for (int k = 0; k < 8; ++k) sh.prof[k] = 0;
        sh.tlast = wall_clock64();
#endif
        sh.cap = a.cap;
        sh.gdyn = a.gscratch + (int64_t)blockIdx.x * slab;
    }
    int32_t *ch;
    if constexpr (G) {
        __shared__ int32_t ch_lds[4 * MAXCH];
        ch = ch_lds;
    } else {
        ch = reinterpret_cast<int32_t *>(a.gscratch + (int64_t)blockIdx.x * slab + slab - kChWords);
    }
    wsync();
    for (;;) {
        int gi = 0;
        if (lane == 0) gi = atomicAdd(a.counter, 1);
        gi = __builtin_amdgcn_readfirstlane(gi);
        if (gi >= a.n_groups) break;
        const int g = a.gidx ? __builtin_amdgcn_readfirstlane(a.gidx[gi]) : gi;
        int st = orient_group<G>(sh, ch, a, g, lane);
        if constexpr (!G) {
            // over the LDS capacity: the group again at once with every array in the slab (capacity
            // a.cap_fb), instead of in a re-run launch after this one (a few long-read groups, one wave
            // each: 10-30 ms per config-4 chunk on the pipeline's critical path)
            if (st != 0 && a.cap_fb > a.cap) {
                if (lane == 0) sh.cap = a.cap_fb;
                wsync();
                st = orient_group<true>(sh, ch, a, g, lane);
                if (lane == 0) sh.cap = a.cap;
                wsync();
            }
        }
        if (lane == 0) a.status[g] = st;
        wsync();
    }
#ifdef MANDO_ORIENT_PROF
    if (lane == 0) {
        for (int k = 0; k < 8; ++k) atomicAdd(&g_oprof[k], (unsigned long long)sh.prof[k]);
        __threadfence();
        if (atomicAdd(&g_odone, 1u) % gridDim.x == gridDim.x - 1)
            printf("[orient prof] Mcyc of the 100 MHz clock over all waves: ref %.1f misc %.1f q-min+anchors %.1f sort %.1f dp %.1f extract %.1f primary %.1f\n",
                   g_oprof[6] * 1e-6, g_oprof[7] * 1e-6, g_oprof[1] * 1e-6, g_oprof[2] * 1e-6, g_oprof[3] * 1e-6,
                   g_oprof[4] * 1e-6, g_oprof[5] * 1e-6);
    }
#endif
}

}  // namespace

size_t orient_dyn_bytes(int cap) { return (size_t)cap * sizeof(uint64_t); }

int orient_blocks_per_cu(int cap) {
    int nb = 0;
    const hipError_t e = cap > kOrientCap  // HBM variant: no dynamic LDS
                             ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, orient_kernel<true>, 64, 0)
                             : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, orient_kernel<false>, 64,
                                                                            orient_dyn_bytes(cap));
    if (e != hipSuccess || nb < 1) nb = 1;
    return nb;
}


size_t orient_slab_words(int cap, int cap_fb) { return (size_t)slab_words(cap, cap_fb); }

hipError_t launch_orient(const OrientArgs &a, int n_slots, hipStream_t stream) {
    if (a.cap > kOrientCap) {
        hipLaunchKernelGGL(orient_kernel<true>, dim3(n_slots), dim3(64), 0, stream, a);
    } else {
        hipLaunchKernelGGL(orient_kernel<false>, dim3(n_slots), dim3(64), orient_dyn_bytes(a.cap), stream, a);
    }
    return hipGetLastError();
}

}  // namespace mando
