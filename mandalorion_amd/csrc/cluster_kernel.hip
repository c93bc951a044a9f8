// cluster_kernel.hip — per-locus read clustering of the D module on the GPU (gfx950).
//
// Restates the clustering half of the reference's process_locus (/root/reference/defineIsoforms.py:55-91)
// as two kernels, one 64-lane wave per locus (large loci: a workgroup of kMwWaves waves, whose helper
// waves join wave 0 for the data-parallel phases, see LocusRun::par):
//   cluster_parse  PSL text -> records (SDC:278-331 field use), blocks, and every cs string tokenised
//                  into run-length records (getCSaroundSS, SDC:107-161)
//   cluster_locus  collect_reads (SDC:278-331), make_genome_bins (:392-438), find_peaks /
//                  scan_for_best_bin / determine_cov (:232-275, :163-224), characterize_splicing_event
//                  (:499-550), spliceDict (defineIsoforms.py:71-83), sort_reads_into_splice_junctions
//                  (:714-769), group_mono_exon_transcripts (:772-794), define_start_end_sites / find_ends
//                  (:797-868, :554-711) and determine_consensus's subsample draw (:884-888)
// Control that the reference runs in RNG order (candidate peaks, identities, isoforms) stays in that
// order and is executed wave-uniformly; the data-parallel parts (text scans, per-read work, window
// sums, the coverage merge, the sampled junction queries, sorts) are spread over the lanes.  The
// numpy RandomState stream (MT19937) lives in LDS and is refilled by the wave.
// Semantics follow oracle/cluster_ref.cpp (the host restatement pinned byte-for-byte against the
// reference by tests/golden/*_vectors.json), which the GPU tests compare against locus by locus.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <map>
#include <memory>
#include <mutex>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "cluster_gpu.h"
#include "internal.h"
#include "mt19937.h"

namespace mando {
namespace cl {
namespace {

// ---------------------------------------------------------------------------------------------
// wave helpers (one workgroup == one wave of 64 lanes)
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ int ln() { return (int)(threadIdx.x & 63); }
__device__ __forceinline__ int wv() { return (int)(threadIdx.x >> 6); }

template <class T>
__device__ __forceinline__ T wsum(T v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
template <class T>
__device__ __forceinline__ T wmax(T v) {
    for (int o = 32; o > 0; o >>= 1) {
        const T t = __shfl_xor(v, o);
        v = t > v ? t : v;
    }
    return v;
}
template <class T>
__device__ __forceinline__ T wmin(T v) {
    for (int o = 32; o > 0; o >>= 1) {
        const T t = __shfl_xor(v, o);
        v = t < v ? t : v;
    }
    return v;
}
// inclusive prefix sum over the lanes
template <class T>
__device__ __forceinline__ T wincl(T v) {
    for (int o = 1; o < 64; o <<= 1) {
        const T t = __shfl_up(v, o);
        if (ln() >= o) v += t;
    }
    return v;
}
__device__ __forceinline__ bool wany(bool p) { return __ballot(p) != 0ull; }
// A wave's barrier: its own memory operations complete (lanes exchange data through LDS and the locus
// scratch).  The large-locus kernel's workgroup has several waves; they meet only at gsync().
__device__ __forceinline__ void wsync() { __asm__ volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void gsync() { __syncthreads(); }
// the large-locus kernels' waves per workgroup (K2: loci of kMwMinRecs records or more; K1: kK1MwBytes)
constexpr int kMwWaves = 8;
constexpr int kMwMinRecs = 2048;

__host__ __device__ __forceinline__ int64_t al256(int64_t x) { return (x + 255) & ~int64_t(255); }

__device__ __forceinline__ bool is_space6(uint8_t c) { return c == ' ' || (c >= 9 && c <= 13); }  // C isspace
__device__ __forceinline__ bool is_trim4(uint8_t c) { return c == ' ' || c == '\t' || c == '\r' || c == '\n'; }
__device__ __forceinline__ bool is_digit(uint8_t c) { return c >= '0' && c <= '9'; }
__device__ __forceinline__ bool is_op(uint8_t c) {
    return c == '=' || c == '+' || c == '-' || c == '*' || c == '~' || c == '\\';
}

// Python int() as the host restatement parses it: surrounding ' ' '\t' '\r' '\n', a sign, digits, '_'
__device__ int64_t to_i64(const uint8_t *s, int a, int b, bool &ok) {
    while (a < b && is_trim4(s[a])) ++a;
    while (b > a && is_trim4(s[b - 1])) --b;
    if (a == b) {
        ok = false;
        return 0;
    }
    bool neg = false;
    if (s[a] == '+' || s[a] == '-') {
        neg = s[a] == '-';
        ++a;
    }
    if (a == b) {
        ok = false;
        return 0;
    }
    int64_t v = 0;
    for (int i = a; i < b; ++i) {
        const uint8_t c = s[i];
        if (c == '_') continue;
        if (!is_digit(c)) {
            ok = false;
            return 0;
        }
        v = v * 10 + (c - '0');
    }
    return neg ? -v : v;
}

// float(accuracy) < 0.9 (SDC:321), decided exactly on the decimal text: the double nearest the text
// is below 0.9 iff the text is <= the midpoint between 0.9 and its predecessor (ties go to the even
// predecessor).  Accepts what float() accepts in a PSL column: sign, digits with an optional point,
// an exponent, inf / nan; anything else is a parse error.
__device__ bool acc_below_09(const uint8_t *s, int a, int b, bool &ok) {
    const char *kMid = "899999999999999966693309261245303787291049957275390625";  // digits of 0.8999...625
    constexpr int kMidN = 54;
    int i = a;
    while (i < b && is_space6(s[i])) ++i;
    int e_ = b;
    while (e_ > i && is_space6(s[e_ - 1])) --e_;
    b = e_;
    bool neg = false;
    if (i < b && (s[i] == '+' || s[i] == '-')) {
        neg = s[i] == '-';
        ++i;
    }
    auto low = [&](int k) -> uint8_t {
        const uint8_t c = s[k];
        return (c >= 'A' && c <= 'Z') ? (uint8_t)(c + 32) : c;
    };
    if (i + 3 <= b && low(i) == 'i' && low(i + 1) == 'n' && low(i + 2) == 'f') {
        if (!((b == i + 3) || (b == i + 8 && low(i + 3) == 'i' && low(i + 4) == 'n' && low(i + 5) == 'i' &&
                               low(i + 6) == 't' && low(i + 7) == 'y')))
            ok = false;
        return neg;
    }
    if (i + 3 == b && low(i) == 'n' && low(i + 1) == 'a' && low(i + 2) == 'n') return false;
    const int is0 = i;
    while (i < b && (is_digit(s[i]) || (s[i] == '_' && i > is0 && i + 1 < b && is_digit(s[i - 1]) && is_digit(s[i + 1])))) ++i;
    const int ie = i;
    int fs = -1, fe = -1;
    if (i < b && s[i] == '.') {
        ++i;
        fs = i;
        while (i < b && (is_digit(s[i]) || (s[i] == '_' && i > fs && i + 1 < b && is_digit(s[i - 1]) && is_digit(s[i + 1])))) ++i;
        fe = i;
    }
    // digits only (underscores skipped)
    auto ndig = [&](int x, int y) {
        int c = 0;
        for (int k = x; k < y; ++k) c += is_digit(s[k]);
        return c;
    };
    const int ni = ndig(is0, ie), nf = fs >= 0 ? ndig(fs, fe) : 0;
    if (ni + nf == 0) {
        ok = false;
        return false;
    }
    int64_t ex = 0;
    if (i < b && (s[i] == 'e' || s[i] == 'E')) {
        int j = i + 1;
        bool en = false;
        if (j < b && (s[j] == '+' || s[j] == '-')) {
            en = s[j] == '-';
            ++j;
        }
        if (j < b && is_digit(s[j])) {
            while (j < b && (is_digit(s[j]) || (s[j] == '_' && j + 1 < b && is_digit(s[j + 1])))) {
                if (is_digit(s[j]) && ex < 100000000) ex = ex * 10 + (s[j] - '0');
                ++j;
            }
            if (en) ex = -ex;
            i = j;
        } else {
            ok = false;
            return false;
        }
    }
    if (i != b) {  // trailing characters: ValueError in float()
        ok = false;
        return false;
    }
    // k-th digit of the concatenated integer and fraction digits
    auto dig = [&](int k) -> int {
        int x = is0, y = ie;
        if (k >= ni) {
            k -= ni;
            x = fs;
            y = fe;
        }
        for (int p = x; p < y; ++p)
            if (is_digit(s[p])) {
                if (k == 0) return s[p] - '0';
                --k;
            }
        return 0;
    };
    const int nd = ni + nf;
    int z = 0;
    while (z < nd && dig(z) == 0) ++z;
    if (z == nd || neg) return true;  // zero, or negative
    const int64_t P = (int64_t)ni - z + ex;  // value = 0.d_z d_z+1 ... x 10^P
    if (P > 0) return false;
    if (P < 0) return true;
    for (int k = 0;; ++k) {
        if (k >= kMidN) {
            for (int q = z + k; q < nd; ++q)
                if (dig(q) != 0) return false;
            return true;
        }
        if (z + k >= nd) return true;
        const int vd = dig(z + k), md = kMid[k] - '0';
        if (vd != md) return vd < md;
    }
}

__device__ __forceinline__ bool bytes_eq(const uint8_t *x, const uint8_t *y, int n) {
    for (int i = 0; i < n; ++i)
        if (x[i] != y[i]) return false;
    return true;
}

// 0x80 in the bytes of x that are zero (exact in every byte, not only the lowest)
__device__ __forceinline__ uint32_t zero_bytes(uint32_t x) {
    return ~(((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x | 0x7f7f7f7fu);
}
// bits 0..3 <- the 0x80 bits of bytes 0..3 (no two partial products share a bit, so no carries)
__device__ __forceinline__ uint32_t byte_bits(uint32_t z) { return ((z >> 7) * 0x00204081u) >> 21 & 0xfu; }
// 16-bit masks of the tabs and the cs operators among the 16 bytes of v
__device__ __forceinline__ uint32_t byte_mask16(const uint4 v, uint32_t K) {  // K: the byte in all four lanes
    return byte_bits(zero_bytes(v.x ^ K)) | byte_bits(zero_bytes(v.y ^ K)) << 4 |
           byte_bits(zero_bytes(v.z ^ K)) << 8 | byte_bits(zero_bytes(v.w ^ K)) << 12;
}
__device__ __forceinline__ uint32_t tab_mask16(const uint4 v) { return byte_mask16(v, 0x09090909u); }
__device__ __forceinline__ uint32_t op_mask16(const uint4 v) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint32_t om = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) om |= (uint32_t)is_op((uint8_t)(w[k >> 2] >> ((k & 3) * 8))) << k;
    return om;
}
__device__ __forceinline__ uint8_t byte_of(const uint4 v, int k) {
    const uint32_t w = k < 8 ? (k < 4 ? v.x : v.y) : (k < 12 ? v.z : v.w);
    return (uint8_t)(w >> ((k & 3) * 8));
}
// bits [lo, hi) of a 16-bit chunk mask, lo in [0, 16), hi clamped to 16
__device__ __forceinline__ uint32_t span_mask16(int64_t lo, int64_t hi) {
    const uint32_t h = hi >= 16 ? 0xffffu : hi <= 0 ? 0u : (1u << hi) - 1u;
    return h & ~((1u << (lo > 0 ? lo : 0)) - 1u);
}
// one cs operation of build_cs (cluster.cpp, getCSaroundSS SDC:107-161): operator `op` at p, its text
// up to q; returns whether it is a run (n != 0); `bad` is set for a malformed intron token
__device__ __forceinline__ bool cs_run(const uint8_t *T, int p, int q, uint8_t op, Run &u, int &bad) {
    const int len = q - p - 1;
    u = Run{};
    u.st = (char)op;
    switch (op) {
        case '=':
        case '-':
            u.n = len;
            u.step = 1;
            break;
        case '+':
            u.n = len;
            u.step = 0;
            break;
        case '*':
            u.n = (len + 1) / 2;
            u.step = 1;
            break;
        case '~': {
            u.n = 1;
            u.st = '|';
            if (len < 4) {
                bad = 1;
                u.n = 0;
                break;
            }
            bool ok = true;
            const int64_t il = to_i64(T, p + 3, q - 2, ok);
            if (!ok) {
                bad = 1;
                u.n = 0;
                break;
            }
            u.step = (int32_t)il;
            u.motif[0] = (char)T[p + 1];
            u.motif[1] = (char)T[p + 2];
            u.motif[2] = (char)T[q - 2];
            u.motif[3] = (char)T[q - 1];
            break;
        }
        default:  // '\\'
            u.n = 0;
    }
    return u.n != 0;
}
__device__ __forceinline__ bool run_advances(const Run &u) { return u.step > 0 || u.st == '|'; }

// ---------------------------------------------------------------------------------------------
// K1: parse
// ---------------------------------------------------------------------------------------------
struct ALayout {
    int32_t *line_end;
    Rec *recs;
    int64_t *blk;  // (size, start) pairs
    int32_t *ops;
    Run *runs;
    int32_t *adv_run;
    int64_t *adv_first;
};

__device__ __forceinline__ ALayout a_layout(uint8_t *base, const Locus &L) {
    ALayout A;
    uint8_t *p = base;
    A.line_end = (int32_t *)p;
    p += al256((int64_t)L.line_cap * 4);
    A.recs = (Rec *)p;
    p += al256((int64_t)L.line_cap * (int64_t)sizeof(Rec));
    A.blk = (int64_t *)p;
    p += al256((int64_t)L.blk_cap * 16);
    A.ops = (int32_t *)p;
    p += al256((int64_t)L.op_cap * 4);
    A.runs = (Run *)p;
    p += al256((int64_t)L.op_cap * (int64_t)sizeof(Run));
    A.adv_run = (int32_t *)p;
    p += al256((int64_t)L.op_cap * 4);
    A.adv_first = (int64_t *)p;
    return A;
}

// K1 for a locus file of kK1MwBytes or more runs on a workgroup of kMwWaves waves: wave w scans the
// w-th share of the text and parses the w-th share of the records, the offsets of each share (line ends,
// blocks) continuing those of the shares before it (one exchange each), so the results are the one-wave
// kernel's.  The parse is then two passes over a wave's records: fields (the block columns' starts
// parked in the record's op / run offsets, which steps 3-4 set later), then the blocks at their offsets.
constexpr int64_t kK1MwBytes = int64_t(4) << 20;
struct K1X {
    int64_t part[2][kMwWaves][4];
};

template <int NW>
__global__ __launch_bounds__(64 * NW) void cluster_parse(Args G) {
    __shared__ K1X kx;
    const int w = NW > 1 ? wv() : 0;
    const int li = G.order[blockIdx.x];
    const Locus L = G.loci[li];
    Stats *st = G.stats + li;
    // the locus' statistics start from zero here rather than by a memset on the stream: a fill kernel
    // queued behind a running POA grid waited ~0.28 s for CUs
    if (w == 0 && ln() == 0) *st = Stats{};
    // exchanges between the waves: each posts up to four values; after one barrier every wave reads all
    // posts (banks alternate, so no wave overwrites a post another has yet to read)
    int ph = 0;
    auto post = [&](int64_t v0, int64_t v1 = 0, int64_t v2 = 0, int64_t v3 = 0) {
        if (ln() == 0) {
            kx.part[ph][w][0] = v0;
            kx.part[ph][w][1] = v1;
            kx.part[ph][w][2] = v2;
            kx.part[ph][w][3] = v3;
        }
        gsync();
        const int b = ph;
        ph ^= 1;
        return b;
    };
    const uint8_t *T = G.text + L.text_off;
    const int64_t n = L.text_len;
    ALayout A = a_layout(G.scratch_a + L.a_off, L);
    const uint8_t *lchrom = G.chroms + L.chrom_off;

#ifdef MANDO_CL_PHASES
    const uint64_t k1t0 = clock64();
#endif
    // 1. line ends: coalesced 16-byte chunks, newline masks compacted in text order; kLineUnroll
    //    chunks per lane are loaded before any is scanned (one load in flight per lane left the wave
    //    waiting on HBM latency: ~55 M cycles for a 22 MB config-2 locus)
    constexpr int kLineUnroll = 16;
    const uintptr_t base = (uintptr_t)T & ~(uintptr_t)15;
    const int pad0 = (int)((uintptr_t)T - base);
    const int64_t nch = (pad0 + n + 15) >> 4;
    // this wave's chunks; several waves: their newlines counted first, the line ends of the waves
    // before come first
    const int64_t c_lo = nch * w / NW, c_hi = nch * (w + 1) / NW;
    int32_t nl = 0, nl_all = 0;
    if (NW > 1) {
        int64_t cnt = 0;
        for (int64_t c00 = c_lo; c00 < c_hi; c00 += 64 * kLineUnroll) {
            uint4 vv[kLineUnroll];
#pragma unroll
            for (int u = 0; u < kLineUnroll; ++u) {
                const int64_t c = c00 + u * 64 + ln();
                vv[u] = c < c_hi ? ((const uint4 *)base)[c] : uint4{0, 0, 0, 0};
            }
#pragma unroll
            for (int u = 0; u < kLineUnroll; ++u) {
                const int64_t c = c00 + u * 64 + ln();
                cnt += c < c_hi ? __popc(byte_mask16(vv[u], 0x0a0a0a0au) & span_mask16(pad0 - c * 16, pad0 + n - c * 16)) : 0;
            }
        }
        const int bk = post(wsum(cnt));
        for (int v = 0; v < NW; ++v) {
            if (v < w) nl += (int32_t)kx.part[bk][v][0];
            nl_all += (int32_t)kx.part[bk][v][0];
        }
    }
    for (int64_t c00 = c_lo; c00 < c_hi; c00 += 64 * kLineUnroll) {
        uint4 vv[kLineUnroll];
#pragma unroll
        for (int u = 0; u < kLineUnroll; ++u) {
            const int64_t c = c00 + u * 64 + ln();
            vv[u] = c < c_hi ? ((const uint4 *)base)[c] : uint4{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < kLineUnroll; ++u) {
            const int64_t c = c00 + u * 64 + ln();
            // newline bytes at text positions [0, n) of the chunk (bytes k with 0 <= c * 16 + k - pad0 < n)
            uint32_t m = c < c_hi ? byte_mask16(vv[u], 0x0a0a0a0au) & span_mask16(pad0 - c * 16, pad0 + n - c * 16) : 0u;
            const int cnt = __popc(m);
            const int incl = wincl(cnt);
            int idx = nl + incl - cnt;
            while (m) {
                const int k = __ffs(m) - 1;
                m &= m - 1;
                if (idx < L.line_cap) A.line_end[idx] = (int32_t)(c * 16 + k - pad0);
                ++idx;
            }
            nl += __shfl(incl, 63);
        }
    }
    if (NW > 1) nl = nl_all;
    const bool tail = n > 0 && T[n - 1] != '\n';
    const int32_t nrec = nl + (tail ? 1 : 0);
    if (tail && nl < L.line_cap && w == 0 && ln() == 0) A.line_end[nl] = (int32_t)n;
    if (nrec > L.line_cap) {
        if (w == 0 && ln() == 0) {
            st->status = kCapacity;
            st->n_rec = nrec;
            st->n_ops = 0;
            st->n_blk = 0;
        }
        return;
    }
    wsync();
    if (NW > 1) gsync();  // every line end written

#ifdef MANDO_CL_PHASES
    const uint64_t k1t1 = clock64();
#endif
    // 2. fields 0-21 and the blocks, one record per lane
    int err = 0;
    int64_t blk_carry = 0, cov_cap = 0, ident_cap = 0;
    int64_t span_lo = INT64_MAX, span_hi = INT64_MIN;
    int32_t hist_l = 0, hist_r = 0, max_nblk = 0;
    const int r_lo = (int)((int64_t)nrec * w / NW), r_hi = (int)((int64_t)nrec * (w + 1) / NW);
    // the fields of record r (act: a record of this lane); the block columns' starts and their count
    auto fields = [&](int r, bool act, Rec &R, int &nb, int &f18a, int &f20a) {
        int f18b = 0, f20b = 0;
        if (act) {
            int a = r == 0 ? 0 : A.line_end[r - 1] + 1, b = A.line_end[r];
            while (a < b && is_space6(T[a])) ++a;
            while (b > a && is_space6(T[b - 1])) --b;
            R.line_lo = a;
            R.line_hi = b;
            // field k = [fs, fe); we need 8-13, 15, 16, 18, 20, 21 and the start of 22
            int k = 0, fs = a;
            // starts / ends of the columns the clustering reads (8-13, 15, 16, 18, 20, 21)
            int f8a = 0, f8b = 0, f9a = 0, f9b = 0, f10a = 0, f10b = 0, f11a = 0, f11b = 0, f12a = 0, f12b = 0;
            int f13a = 0, f13b = 0, f15a = 0, f15b = 0, f16a = 0, f16b = 0, f21a = 0, f21b = 0;
            bool done = false;
            // the tabs of [a, b) in order, from aligned 16-byte chunks (the chunks the line scan read)
            for (uintptr_t ch = ((uintptr_t)(T + a)) & ~(uintptr_t)15; ch < (uintptr_t)(T + b) && !done; ch += 16) {
                const int64_t c0 = (int64_t)(ch - (uintptr_t)T);
                uint32_t tm = tab_mask16(*(const uint4 *)ch) & span_mask16(a - c0, b - c0);
                while (tm && !done) {
                    const int i = (int)(c0 + __ffs(tm) - 1);
                    tm &= tm - 1;
                    switch (k) {
                        case 8: f8a = fs; f8b = i; break;
                        case 9: f9a = fs; f9b = i; break;
                        case 10: f10a = fs; f10b = i; break;
                        case 11: f11a = fs; f11b = i; break;
                        case 12: f12a = fs; f12b = i; break;
                        case 13: f13a = fs; f13b = i; break;
                        case 15: f15a = fs; f15b = i; break;
                        case 16: f16a = fs; f16b = i; break;
                        case 18: f18a = fs; f18b = i; break;
                        case 20: f20a = fs; f20b = i; break;
                        case 21: f21a = fs; f21b = i; break;
                        default: break;
                    }
                    ++k;
                    fs = i + 1;
                    if (k == 22) {
                        R.cs_off = fs;
                        done = true;
                    }
                }
            }
            if (!done) {
                err = 1;
            } else {
                bool ok = true;
                R.dirn = (f8b - f8a == 1 && T[f8a] == '+') ? 0 : (f8b - f8a == 1 && T[f8a] == '-') ? 1 : 2;
                R.name_off = f9a;
                R.name_len = f9b - f9a;
                R.qsize = to_i64(T, f10a, f10b, ok);
                R.qstart = to_i64(T, f11a, f11b, ok);
                R.qend = to_i64(T, f12a, f12b, ok);
                R.chrom_off = f13a;
                R.chrom_len = f13b - f13a;
                R.same_chrom = R.chrom_len == L.chrom_len && bytes_eq(T + R.chrom_off, lchrom, L.chrom_len);
                R.tstart = to_i64(T, f15a, f15b, ok);
                R.tend = to_i64(T, f16a, f16b, ok);
                // commas of columns 18 and 20, from aligned 16-byte chunks
                auto commas = [&](int lo, int hi) {
                    int c = 0;
                    for (uintptr_t ch = ((uintptr_t)(T + lo)) & ~(uintptr_t)15; ch < (uintptr_t)(T + hi); ch += 16) {
                        const int64_t c0 = (int64_t)(ch - (uintptr_t)T);
                        c += __popc(byte_mask16(*(const uint4 *)ch, 0x2c2c2c2cu) & span_mask16(lo - c0, hi - c0));
                    }
                    return c;
                };
                const int c18 = commas(f18a, f18b), c20 = commas(f20a, f20b);
                if (c18 != c20) ok = false;
                nb = c18;
                R.acc_lt = acc_below_09(T, f21a, f21b, ok);
                if (!ok) err = 1;
            }
        }
    };
    // the blocks of record r at boff, and its statistics
    auto blocks = [&](int r, bool act, Rec &R, int nb, int f18a, int f20a, int64_t boff) {
        if (act && !err) {
            // blocks: str.split(',')[:-1] of columns 18 (sizes) and 20 (starts)
            const bool room = boff + nb <= L.blk_cap;
            int64_t cc = 0, lo_cnt = 0, up_cnt = 0;
            bool ok = true;
            int pa = f18a, qa = f20a;
            for (int x = 0; x < nb; ++x) {
                int pe = pa;
                while (T[pe] != ',') ++pe;
                int qe = qa;
                while (T[qe] != ',') ++qe;
                const int64_t sz = to_i64(T, pa, pe, ok), bs = to_i64(T, qa, qe, ok);
                pa = pe + 1;
                qa = qe + 1;
                if (room) {
                    A.blk[2 * (boff + x)] = sz;
                    A.blk[2 * (boff + x) + 1] = bs;
                }
                cc += (sz > 0 ? (sz + 9) / 10 : 0) + 11;
                lo_cnt += (bs + sz) != R.tend;
                up_cnt += bs != R.tstart;
            }
            if (!ok) err = 1;
            if (R.same_chrom) {
                cov_cap += cc;
                span_lo = R.tstart < span_lo ? R.tstart : span_lo;
                span_hi = R.tend > span_hi ? R.tend : span_hi;
                if (!R.acc_lt) {
                    hist_l += (int32_t)lo_cnt;
                    hist_r += (int32_t)up_cnt;
                }
            }
            ident_cap += (R.chrom_len + 2 + (int64_t)(nb > 0 ? nb - 1 : 0) * 28 + 7) & ~int64_t(7);
            max_nblk = nb > max_nblk ? nb : max_nblk;
            A.recs[r] = R;
        }
    };
    if (NW == 1) {
        for (int r0 = 0; r0 < nrec; r0 += 64) {
            const int r = r0 + ln();
            const bool act = r < nrec;
            Rec R = {};
            int nb = 0, f18a = 0, f20a = 0;
            fields(r, act, R, nb, f18a, f20a);
            // block offsets: prefix over the lanes
            const int nbi = act && !err ? nb : 0;
            const int incl = wincl(nbi);
            const int64_t boff = blk_carry + incl - nbi;
            blk_carry += __shfl(incl, 63);
            R.blk_off = (int32_t)boff;
            R.nblk = nbi;
            blocks(r, act, R, nb, f18a, f20a, boff);
        }
    } else {
        // pass 1: fields of this wave's records, block counts summed
        int64_t nbs = 0;
        for (int r0 = r_lo; r0 < r_hi; r0 += 64) {
            const int r = r0 + ln();
            const bool act = r < r_hi;
            Rec R = {};
            int nb = 0, f18a = 0, f20a = 0;
            fields(r, act, R, nb, f18a, f20a);
            if (act) {
                R.nblk = !err ? nb : 0;
                R.op_off = f18a;
                R.run_off = f20a;
                A.recs[r] = R;
                nbs += R.nblk;
            }
        }
        const int bk = post(wsum(nbs), wany(err != 0) ? 1 : 0);
        int64_t all_blk = 0, any_err = 0;
        for (int v = 0; v < NW; ++v) {
            if (v < w) blk_carry += kx.part[bk][v][0];
            all_blk += kx.part[bk][v][0];
            any_err |= kx.part[bk][v][1];
        }
        if (any_err) {
            if (w == 0 && ln() == 0) st->status = kParse;
            return;
        }
        // pass 2: the blocks at the offsets after the waves before this one
        for (int r0 = r_lo; r0 < r_hi; r0 += 64) {
            const int r = r0 + ln();
            const bool act = r < r_hi;
            Rec R = act ? A.recs[r] : Rec{};
            const int nb = R.nblk, f18a = R.op_off, f20a = R.run_off;
            R.op_off = R.run_off = 0;
            const int nbi = act && !err ? nb : 0;
            const int incl = wincl(nbi);
            const int64_t boff = blk_carry + incl - nbi;
            blk_carry += __shfl(incl, 63);
            R.blk_off = (int32_t)boff;
            R.nblk = nbi;
            blocks(r, act, R, nb, f18a, f20a, boff);
        }
        blk_carry = all_blk;
    }
    {
        int64_t e = wany(err != 0) ? 1 : 0;
        if (NW > 1) {
            const int bk = post(e);
            e = 0;
            for (int v = 0; v < NW; ++v) e |= kx.part[bk][v][0];
        }
        if (e) {
            if (w == 0 && ln() == 0) st->status = kParse;
            return;
        }
    }
    const int64_t n_blk = blk_carry;
    if (n_blk > L.blk_cap) {
        if (w == 0 && ln() == 0) {
            st->status = kCapacity;
            st->n_rec = nrec;
            st->n_blk = (int32_t)n_blk;
            st->n_ops = 0;
        }
        return;
    }
    wsync();

#ifdef MANDO_CL_PHASES
    const uint64_t k1t2 = clock64();
#endif
    // 3-4 (the cs and seq columns, the runs) follow in cluster_cs_count / _scan / _runs, several waves
    //    per large locus
#ifdef MANDO_CL_PHASES
    if (ln() == 0)
        printf("[K1 phases] n %d: lines %.2f fields %.2f Mcyc\n", nrec, (k1t1 - k1t0) * 1e-6, (k1t2 - k1t1) * 1e-6);
#endif
    // 5. statistics for the host (scratch B sizing) and K2
    cov_cap = wsum(cov_cap);
    ident_cap = wsum(ident_cap);
    hist_l = wsum(hist_l);
    hist_r = wsum(hist_r);
    span_lo = wmin(span_lo);
    span_hi = wmax(span_hi);
    max_nblk = wmax(max_nblk);
    if (NW > 1) {
        const int b1 = post(cov_cap, ident_cap, hist_l, hist_r);
        int64_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
        for (int v = 0; v < NW; ++v) {
            s0 += kx.part[b1][v][0];
            s1 += kx.part[b1][v][1];
            s2 += kx.part[b1][v][2];
            s3 += kx.part[b1][v][3];
        }
        const int b2 = post(span_lo, span_hi, max_nblk);
        for (int v = 0; v < NW; ++v) {
            span_lo = kx.part[b2][v][0] < span_lo ? kx.part[b2][v][0] : span_lo;
            span_hi = kx.part[b2][v][1] > span_hi ? kx.part[b2][v][1] : span_hi;
            max_nblk = (int32_t)kx.part[b2][v][2] > max_nblk ? (int32_t)kx.part[b2][v][2] : max_nblk;
        }
        cov_cap = s0;
        ident_cap = s1;
        hist_l = (int32_t)s2;
        hist_r = (int32_t)s3;
    }
    if (w == 0 && ln() == 0) {
        st->status = kOk;
        st->n_rec = nrec;
        st->n_ops = 0;  // cluster_cs_scan
        st->n_blk = (int32_t)n_blk;
        st->n_hist_l = hist_l;
        st->n_hist_r = hist_r;
        st->max_nblk = max_nblk;
        st->span_lo = span_lo;
        st->span_hi = span_hi;
        st->cov_cap = cov_cap;
        st->ident_cap = ident_cap;
    }
}


// ---------------------------------------------------------------------------------------------
// K1 steps 3-4: the cs column (field 22) up to its tab, the seq column (23) up to the next tab or the
// line end, and the run-length cs records (cluster.cpp build_cs; getCSaroundSS SDC:107-161).  One record
// per lane: each lane streams its own record's text in 16-byte chunks.  A large locus (config 2: ~7k
// records, ~20 MB) is spread over up to kCsMaxWaves one-wave workgroups, each taking every nmem-th batch
// of 64 records; its offsets come from a per-locus prefix in between.
//   cluster_cs_count  pass 1: the two tabs; counts of operators, runs (operations of non-zero length)
//                     and advancing runs per record
//   cluster_cs_scan   one wave per locus: record offsets by prefix sums, the operator capacity check
//   cluster_cs_runs   pass 2: every run with its first record index and genome position, and the
//                     advancing runs with the genome position of their first record
// ---------------------------------------------------------------------------------------------
constexpr int64_t kCsTextPerWave = 512 << 10;
constexpr int kCsMaxWaves = 64;

__global__ __launch_bounds__(64) void cluster_cs_count(Args G) {
    const int li = G.work[2 * blockIdx.x], mem = G.work[2 * blockIdx.x + 1] & 0xffff,
              nmem = G.work[2 * blockIdx.x + 1] >> 16;
    Stats *st = G.stats + li;
    if (st->status != kOk) return;  // K1 stopped on this locus
    const Locus L = G.loci[li];
    const uint8_t *T = G.text + L.text_off;
    ALayout A = a_layout(G.scratch_a + L.a_off, L);
    const int nrec = st->n_rec;
    int err = 0;
    for (int r0 = 64 * mem; r0 < nrec; r0 += 64 * nmem) {
        const int r = r0 + ln();
        if (r >= nrec) break;
        const int a = A.recs[r].cs_off, b = A.recs[r].line_hi;
        int t1 = -1, t2 = -1, nop = 0, nrun = 0, nadv = 0, bad = 0;
        int64_t nrc = 0;
        const int64_t first = (int64_t)(((uintptr_t)(T + a) & ~(uintptr_t)15) - (uintptr_t)T);
        int pp = -1;
        uint8_t pop = 0;
        auto count = [&](int q) {
            Run u;
            if (cs_run(T, pp, q, pop, u, bad)) {
                ++nrun;
                nrc += u.n;
                nadv += run_advances(u) ? 1 : 0;
            }
        };
        for (int64_t c = first; c < b && t2 < 0; c += 16) {
            const uint4 v = *(const uint4 *)(T + c);
            const uint32_t in = span_mask16(a - c, b - c);
            uint32_t tm = tab_mask16(v) & in;
            if (t1 < 0) {
                uint32_t om = op_mask16(v) & in;
                if (tm) om &= (1u << (__ffs(tm) - 1)) - 1u;
                while (om) {
                    const int k = __ffs(om) - 1;
                    om &= om - 1;
                    if (pp >= 0) count((int)c + k);
                    pp = (int)c + k;
                    pop = byte_of(v, k);
                    ++nop;
                }
                if (tm) {
                    t1 = (int)c + __ffs(tm) - 1;
                    if (pp >= 0) count(t1);
                    tm &= tm - 1;
                }
            }
            if (t1 >= 0 && tm) t2 = (int)c + __ffs(tm) - 1;
        }
        if (t1 < 0) {
            err = 1;  // fewer than 24 columns
            continue;
        }
        Rec &W = A.recs[r];
        W.cs_len = t1 - a;
        W.seq_off = t1 + 1;
        W.seq_len = (t2 >= 0 ? t2 : b) - (t1 + 1);
        W.nop = nop;
        W.nrun = nrun;
        W.nadv = nadv;
        W.nrec_cs = (int32_t)nrc;
        W.cs_bad = bad ? 1 : 0;
    }
    if (wany(err != 0) && ln() == 0) atomicOr(&st->cs_err, 1);
}

__global__ __launch_bounds__(64) void cluster_cs_scan(Args G) {
    const int li = G.order[blockIdx.x];
    Stats *st = G.stats + li;
    if (st->status != kOk) return;
    if (st->cs_err) {
        if (ln() == 0) st->status = kParse;
        return;
    }
    const Locus L = G.loci[li];
    ALayout A = a_layout(G.scratch_a + L.a_off, L);
    const int nrec = st->n_rec;
    int64_t op_carry = 0, run_carry = 0, adv_carry = 0;
    for (int r0 = 0; r0 < nrec; r0 += 64) {
        const int r = r0 + ln();
        int nop = 0, nrun = 0, nadv = 0;
        if (r < nrec) {
            nop = A.recs[r].nop;
            nrun = A.recs[r].nrun;
            nadv = A.recs[r].nadv;
        }
        const int op_in = wincl(nop), run_in = wincl(nrun), adv_in = wincl(nadv);
        if (r < nrec) {
            Rec &W = A.recs[r];
            W.op_off = (int32_t)(op_carry + op_in - nop);
            W.run_off = (int32_t)(run_carry + run_in - nrun);
            W.adv_off = (int32_t)(adv_carry + adv_in - nadv);
        }
        op_carry += __shfl(op_in, 63);
        run_carry += __shfl(run_in, 63);
        adv_carry += __shfl(adv_in, 63);
    }
    if (ln() == 0) {
        st->n_ops = (int32_t)op_carry;
        if (op_carry > L.op_cap) st->status = kCapacity;
    }
}

__global__ __launch_bounds__(64) void cluster_cs_runs(Args G) {
    const int li = G.work[2 * blockIdx.x], mem = G.work[2 * blockIdx.x + 1] & 0xffff,
              nmem = G.work[2 * blockIdx.x + 1] >> 16;
    const Stats *st = G.stats + li;
    if (st->status != kOk) return;
    const Locus L = G.loci[li];
    const uint8_t *T = G.text + L.text_off;
    ALayout A = a_layout(G.scratch_a + L.a_off, L);
    const int nrec = st->n_rec;
    for (int r0 = 64 * mem; r0 < nrec; r0 += 64 * nmem) {
        const int r = r0 + ln();
        if (r >= nrec) break;
        const Rec R = A.recs[r];
        const int a = R.cs_off, b = R.cs_off + R.cs_len;
        const int64_t first = (int64_t)(((uintptr_t)(T + a) & ~(uintptr_t)15) - (uintptr_t)T);
        int pp = -1, bad = 0;
        uint8_t pop = 0;
        int64_t ri = R.run_off, ai = R.adv_off, rec_c = 0, g_c = 0;
        auto emit = [&](int q) {
            Run u;
            if (cs_run(T, pp, q, pop, u, bad)) {
                u.rec0 = (int32_t)rec_c;
                u.g0 = R.tstart + g_c;
                A.runs[ri] = u;
                if (run_advances(u)) {
                    A.adv_run[ai] = (int32_t)(ri - R.run_off);
                    A.adv_first[ai] = u.g0 + u.step;
                    ++ai;
                }
                ++ri;
                rec_c += u.n;
                g_c += (int64_t)u.step * u.n;
            }
        };
        for (int64_t c = first; c < b; c += 16) {
            const uint4 v = *(const uint4 *)(T + c);
            uint32_t om = op_mask16(v) & span_mask16(a - c, b - c);
            while (om) {
                const int k = __ffs(om) - 1;
                om &= om - 1;
                if (pp >= 0) emit((int)c + k);
                pp = (int)c + k;
                pop = byte_of(v, k);
            }
        }
        if (pp >= 0) emit(b);
    }
}

// ---------------------------------------------------------------------------------------------
// K2 scratch layout; the host sizes it with the same carve (base == nullptr)
// ---------------------------------------------------------------------------------------------
__host__ __device__ __forceinline__ int64_t pow2ge(int64_t x) {
    int64_t p = 64;
    while (p < x) p <<= 1;
    return p;
}

struct Side {          // one side's splice-bound histogram (histo_left_bases / histo_right_bases)
    uint64_t *sk;      // entry sort keys: (position + bias) << 24 | insertion rank
    int32_t *erec;     // record of each entry, in sorted (position, insertion) order
    int32_t *etmp;     // insertion rank -> record; later: first insertion rank -> key index
    int64_t *ukey;     // distinct positions, ascending
    int32_t *ulo, *ucnt, *ufirst;
    int32_t *upmb;     // per key: reads on '+', on '-', on anything else
    uint64_t *cand;    // candidate order: count descending, then insertion order
    int32_t H, P, nkeys, ncand;
};

struct BPtr {
    int64_t *cov;
    Side s[2];
    int32_t *names, *cur, *perm;
    int64_t *hv;    // determine_cov: each winner's head value
    int32_t *hcb;   // histo_cov over the map: records whose coverage set holds the bin at map index 10k..10k+9
    int64_t *win;
    uint8_t *areas[2];
    int32_t *splice, *sc, *ec, *sp, *ep;
    int64_t *ann;
    int32_t *lab;
    uint8_t *ibuf;
    int32_t *ioff, *ilen;
    uint64_t *ihash;
    int8_t *ikind;
    int32_t *grp;
    uint64_t *isort;
    int32_t *msuf, *id_lo, *id_hi, *id_rep, *id_m, *idsort, *msort;
    uint64_t *ss;
    int32_t *pa, *pb;
    int8_t *asg;
    int32_t *mem_tmp;
    int64_t total;
};

struct OPtr {
    Peak *peaks;
    int32_t *iso_nmem, *mem, *iso_nsub, *sub;
    int32_t peak_cap;
    int64_t total;
};

__host__ __device__ inline int32_t n_ann_of(const Locus &L) { return L.ann_off[4] - L.ann_off[0]; }
__host__ __device__ inline int32_t peak_cap_of(const Stats &S, const Locus &L) {
    return S.n_hist_l + S.n_hist_r + n_ann_of(L) + 8;
}

// Large loci (>= kMwMinRecs records: config 2's SIRV-sized loci) run on a workgroup of kMwWaves waves.
// Wave 0 runs the locus exactly as the one-wave kernel does; the helper waves wait in
// LocusRun::helper() and join it for the data-parallel phases (coverage sets, the coverage merge),
// each wave taking a contiguous share of the records / winners.  MwX is their LDS exchange: the phase
// and its arguments, and per-wave partials in two banks that alternate between exchanges (a wave that
// runs ahead cannot overwrite a partial another wave has yet to read).
constexpr int kOpExit = 0, kOpCovSets = 1, kOpDetCov = 2, kOpCountSort = 3, kOpKeys = 4;
// waves of a locus's K2 workgroup (the host splits the launch on the same rule)
__host__ __device__ inline int mw_waves(const Stats &S) { return S.n_rec >= kMwMinRecs ? kMwWaves : 1; }

__host__ __device__ inline void carve_b(uint8_t *base, const Stats &S, const Locus &L, int w, BPtr &B) {
    int64_t off = 0;
    auto take = [&](int64_t bytes) -> uint8_t * {
        uint8_t *p = base ? base + off : nullptr;
        off += al256(bytes > 0 ? bytes : 1);
        return p;
    };
    const int64_t n = S.n_rec > 0 ? S.n_rec : 1;
    const int64_t pn = pow2ge(n);
    B.cov = (int64_t *)take(S.cov_cap * 8);
    int64_t hmax = 1;
    for (int k = 0; k < 2; ++k) {
        Side &d = B.s[k];
        d.H = k == 0 ? S.n_hist_l : S.n_hist_r;
        d.P = (int32_t)pow2ge(d.H);
        d.nkeys = d.ncand = 0;
        hmax = d.H > hmax ? d.H : hmax;
        d.sk = (uint64_t *)take((int64_t)d.P * 8);
        d.erec = (int32_t *)take((int64_t)d.H * 4);
        d.etmp = (int32_t *)take((int64_t)d.H * 4);
        d.ukey = (int64_t *)take((int64_t)d.H * 8);
        d.ulo = (int32_t *)take((int64_t)d.H * 4);
        d.ucnt = (int32_t *)take((int64_t)d.H * 4);
        d.ufirst = (int32_t *)take((int64_t)d.H * 4);
        d.upmb = (int32_t *)take((int64_t)d.H * 12);
        d.cand = (uint64_t *)take((int64_t)d.P * 8);
    }
    B.names = (int32_t *)take(hmax * 4);
    B.cur = (int32_t *)take(hmax * 4);
    B.hv = (int64_t *)take(hmax * 8);
    B.hcb = (int32_t *)take((L.map_n / 10 + 2) * 4);
    B.perm = (int32_t *)take((n > hmax ? n : hmax) * 4);
    B.win = (int64_t *)take(4 * (4 * (int64_t)w + 1) * 8);
    B.areas[0] = take(L.map_n);
    B.areas[1] = take(L.map_n);
    B.splice = (int32_t *)take(L.map_n * 4);
    B.sc = (int32_t *)take(L.map_n * 4 * mw_waves(S));  // several waves: one count column per wave
    B.ec = (int32_t *)take(L.map_n * 4);
    B.sp = (int32_t *)take(L.map_n * 4);
    B.ep = (int32_t *)take(L.map_n * 4);
    B.ann = (int64_t *)take((int64_t)n_ann_of(L) * 8);
    B.lab = (int32_t *)take((int64_t)peak_cap_of(S, L) * 4);
    B.ibuf = take(S.ident_cap);
    B.ioff = (int32_t *)take(n * 4);
    B.ilen = (int32_t *)take(n * 4);
    B.ihash = (uint64_t *)take(n * 8);
    B.ikind = (int8_t *)take(n);
    B.grp = (int32_t *)take(n * 4);
    B.isort = (uint64_t *)take(pn * 8);
    B.msuf = (int32_t *)take(n * 4);
    B.id_lo = (int32_t *)take(n * 4);
    B.id_hi = (int32_t *)take(n * 4);
    B.id_rep = (int32_t *)take(n * 4);
    B.id_m = (int32_t *)take(n * 4);
    B.idsort = (int32_t *)take(pn * 4);
    B.msort = (int32_t *)take(pn * 4);
    B.ss = (uint64_t *)take(pn * 8);
    B.pa = (int32_t *)take(n * 4);
    B.pb = (int32_t *)take(n * 4);
    B.asg = (int8_t *)take(n);
    B.mem_tmp = (int32_t *)take(n * 4);
    B.total = off;
}

__host__ __device__ inline void carve_o(uint8_t *base, const Stats &S, const Locus &L, OPtr &O) {
    int64_t off = 0;
    auto take = [&](int64_t bytes) -> uint8_t * {
        uint8_t *p = base ? base + off : nullptr;
        off += al256(bytes > 0 ? bytes : 1);
        return p;
    };
    const int64_t n = S.n_rec > 0 ? S.n_rec : 1;
    O.peak_cap = peak_cap_of(S, L);
    O.peaks = (Peak *)take((int64_t)O.peak_cap * (int64_t)sizeof(Peak));
    O.iso_nmem = (int32_t *)take(n * 4);
    O.mem = (int32_t *)take(n * 4);
    O.iso_nsub = (int32_t *)take(n * 4);
    O.sub = (int32_t *)take(n * 4);
    O.total = off;
}

// ---------------------------------------------------------------------------------------------
// wave sorts (bitonic, in global scratch; P a power of two >= 64)
// ---------------------------------------------------------------------------------------------
// The bitonic network's exchanges with partner distance j < the tile stay inside aligned tiles of
// that many keys (kSortTile at most), so they run in LDS (cluster_locus's dynamic LDS): a tile is loaded once, takes every
// such pass of the current stage, and is written back; only the passes with j >= kSortTile go through
// global memory (for 2^17 keys: 10 global passes instead of 153).
constexpr int64_t kSortTile = 4096;
extern __shared__ uint64_t g_sort_lds[];  // kSortTile keys

// One compare-exchange pass of the network over keys [0, T) of `a` (LDS or global): the T/2 pairs
// (i, i + j), bit j of i clear, are enumerated directly (no idle half-wave), four per lane per step with
// their loads issued together; a pair sorts ascending where ((base + i) & k) == 0.
template <class K>
__device__ __forceinline__ void bitonic_pass(K *a, int64_t T, int64_t base, int64_t k, int64_t j) {
    const int64_t np = T >> 1;
    for (int64_t p0 = 0; p0 < np; p0 += 4 * 64) {
        uint64_t x[4], y[4];
        int64_t ii[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t q = p0 + u * 64 + ln();
            ii[u] = q < np ? ((q & ~(j - 1)) << 1) | (q & (j - 1)) : -1;
            if (ii[u] >= 0) {
                x[u] = a[ii[u]];
                y[u] = a[ii[u] + j];
            }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (ii[u] >= 0 && (x[u] > y[u]) == (((base + ii[u]) & k) == 0)) {
                a[ii[u]] = y[u];
                a[ii[u] + j] = x[u];
            }
        }
    }
}

__device__ void sort_tile_lds(uint64_t *a, int64_t t0, int64_t T, int64_t k, int64_t j_hi) {
    for (int64_t i = ln(); i < T; i += 64) g_sort_lds[i] = a[t0 + i];
    wsync();
    for (int64_t j = j_hi; j > 0; j >>= 1) {
        bitonic_pass(g_sort_lds, T, t0, k, j);
        wsync();
    }
    for (int64_t i = ln(); i < T; i += 64) a[t0 + i] = g_sort_lds[i];
    wsync();
}

// tile: the keys the launch's dynamic LDS holds (Args::sort_tile, at most kSortTile)
__device__ void sort_u64(uint64_t *a, int64_t P, int64_t tile) {
    const int64_t T = P < tile ? P : tile;
    // stages k <= T: every pass inside the tile
    for (int64_t t0 = 0; t0 < P; t0 += T) {
        for (int64_t i = ln(); i < T; i += 64) g_sort_lds[i] = a[t0 + i];
        wsync();
        for (int64_t k = 2; k <= T; k <<= 1)
            for (int64_t j = k >> 1; j > 0; j >>= 1) {
                bitonic_pass(g_sort_lds, T, t0, k, j);
                wsync();
            }
        for (int64_t i = ln(); i < T; i += 64) a[t0 + i] = g_sort_lds[i];
        wsync();
    }
    // stages k > T: passes j >= T in global memory, then the rest of the stage per tile in LDS
    for (int64_t k = 2 * T; k <= P; k <<= 1) {
        for (int64_t j = k >> 1; j >= T; j >>= 1) {
            bitonic_pass(a, P, 0, k, j);
            wsync();
        }
        for (int64_t t0 = 0; t0 < P; t0 += T) sort_tile_lds(a, t0, T, k, T >> 1);
    }
}

// indices with a strict-weak "less"; padding entries are -1 and sort last
template <class Less>
__device__ void sort_idx(int32_t *a, int64_t P, Less less) {
    for (int64_t k = 2; k <= P; k <<= 1)
        for (int64_t j = k >> 1; j > 0; j >>= 1) {
            for (int64_t i = ln(); i < P; i += 64) {
                const int64_t l = i ^ j;
                if (l > i) {
                    const int32_t x = a[i], y = a[l];
                    const bool gt = (x < 0) ? (y >= 0) : (y >= 0 && less(y, x));  // x > y
                    if (gt == ((i & k) == 0)) {
                        a[i] = y;
                        a[l] = x;
                    }
                }
            }
            wsync();
        }
}

// ---------------------------------------------------------------------------------------------
// numpy RandomState (MT19937) in LDS; the refill is spread over the wave
// ---------------------------------------------------------------------------------------------
__device__ void mt_refill(uint32_t *key) {
    auto twist = [&](int lo, int hi, int src_off) {  // key[kk] = key[kk + src_off] ^ f(key[kk], key[kk + 1])
        for (int k0 = lo; k0 < hi; k0 += 64) {
            const int kk = k0 + ln();
            uint32_t v = 0;
            if (kk < hi) {
                const uint32_t y = (key[kk] & 0x80000000u) | (key[kk + 1] & 0x7fffffffu);
                v = key[kk + src_off] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
            }
            wsync();
            if (kk < hi) key[kk] = v;
            wsync();
        }
    };
    twist(0, 227, 397);
    twist(227, 454, -227);
    twist(454, 623, -227);
    uint32_t v = 0;
    if (ln() == 0) {
        const uint32_t y = (key[623] & 0x80000000u) | (key[0] & 0x7fffffffu);
        v = key[396] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    wsync();
    if (ln() == 0) key[623] = v;
    wsync();
}

struct MT {
    uint32_t *key;
    int pos;
#ifdef MANDO_CL_PHASES  // dev build: where a permutation's cycles go
    uint64_t pq_acc = 0, pq_swap = 0;
    int32_t pq_blocks = 0, pq_arounds = 0, pq_srounds = 0;
#endif
    __device__ static uint32_t temper(uint32_t y) {
        y ^= (y >> 11);
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= (y >> 18);
        return y;
    }
    __device__ uint32_t next32() {
        if (pos == 624) {
            mt_refill(key);
            pos = 0;
        }
        return temper(key[pos++]);
    }
    // random_interval(max) for max < 2^32 (every draw here)
    __device__ uint32_t interval(uint32_t max) {
        if (max == 0) return 0;
        uint32_t mask = max;
        mask |= mask >> 1;
        mask |= mask >> 2;
        mask |= mask >> 4;
        mask |= mask >> 8;
        mask |= mask >> 16;
        uint32_t v;
        while ((v = (next32() & mask)) > max) {
        }
        return v;
    }
    // permutation(n): Fisher-Yates from the top (numpy's shuffle: for i = n-1 .. 1, j = interval(i),
    // swap(perm[i], perm[j])), 64 stream outputs at a time, one per lane.
    // Draws: lane t's output serves draw i - (outputs accepted before t); random_interval accepts it iff
    // (output & mask(i)) <= i.  A block takes mf <= 64 lanes such that the draws it can serve,
    // i - mf + 1 .. i, stay at or above the top power of two of i, so one mask serves them all: an
    // output u = y & mask with u > i is rejected whatever draw it serves, u <= i - mf + 1 accepted
    // whatever draw it serves; only the rare u in between depend on how many lanes before them were
    // accepted, and they are settled in lane order on the scalar unit.  Every lane of the block is
    // consumed (no draw index falls below 1 inside it), exactly the outputs interval() would consume.
    // Swaps: the accepted lanes' swaps (d, v) run in lane order; a prefix of lanes that touch no
    // position an earlier pending lane touches (v_s == d_t or v_s == v_t for s < t; d_s == v_t is
    // impossible since v_t <= d_t < d_s) runs at once, then the rest.  Conflicts are found through a
    // table of `slots` words in free LDS (tab): every pending lane posts its lane into slot v & (slots-1)
    // with an atomic min (tagged by round, so the table is cleared once per permutation), and lane t
    // conflicts when slot(d_t) or slot(v_t) holds an earlier lane of this round -- a hash collision can
    // only split a round early, never hide a conflict.
    __device__ void permutation(int32_t n, int32_t *perm, uint32_t *tab, int slots) {
        for (int i = ln(); i < n; i += 64) perm[i] = i;
        for (int i = ln(); i < slots; i += 64) tab[i] = 0xffffffffu;
        wsync();
        const uint64_t below = (1ull << ln()) - 1;  // (lane 0: 0)
        uint32_t round = 0;
        int32_t i = n - 1;
        while (i >= 1) {
#ifdef MANDO_CL_PHASES
            const uint64_t tq0 = clock64();
            ++pq_blocks;
#endif
            if (pos == 624) {
                mt_refill(key);
                pos = 0;
            }
            const int m = 624 - pos < 64 ? 624 - pos : 64;
            const uint32_t y = ln() < m ? temper(key[pos + ln()]) : 0u;
            int start = 0, cur = i;
            int32_t dl = 0, vl = 0;
            uint64_t acc = 0;
            const uint32_t mask = 0xffffffffu >> __clz(cur);
            // the block's lanes: at most the draws down to the top power of two of i, so that one mask
            // serves them all (the next block starts under it with the next mask)
            const int mf = min(m, cur - (int)((mask >> 1) + 1) + 1);
            {
                const uint64_t livef = mf >= 64 ? ~0ull : ((1ull << mf) - 1);
                const uint32_t u = y & mask;
                acc = __ballot(u <= (uint32_t)(cur - (mf - 1))) & livef;
                uint64_t amb = __ballot(u > (uint32_t)(cur - (mf - 1)) && u <= (uint32_t)cur) & livef;
                while (amb) {  // lane order: each one's draw index counts the accepted lanes before it
                    const int l = (int)__ffsll((unsigned long long)amb) - 1;
                    const uint32_t ul = (uint32_t)__builtin_amdgcn_readlane((int)u, l);
                    if (ul <= (uint32_t)(cur - __popcll(acc & ((1ull << l) - 1)))) acc |= 1ull << l;
                    amb &= amb - 1;
                }
                dl = cur - __popcll(acc & below);
                vl = (int32_t)u;
                start = mf;
                cur -= __popcll(acc);
#ifdef MANDO_CL_PHASES
                ++pq_arounds;
#endif
            }
            pos += start;
            i = cur;
#ifdef MANDO_CL_PHASES
            const uint64_t tq1 = clock64();
            pq_acc += tq1 - tq0;
#endif
            uint64_t rem = acc;
            const uint32_t hm = (uint32_t)slots - 1;
            while (rem) {
#ifdef MANDO_CL_PHASES
                ++pq_srounds;
#endif
                ++round;
                const uint32_t tag = (0xffffffu - round) << 8;
                const bool pend = (rem >> ln()) & 1ull;
                if (pend) atomicMin(&tab[(uint32_t)vl & hm], tag | (uint32_t)ln());
                wsync();
                bool conf = false;
                if (pend) {
                    const uint32_t a = tab[(uint32_t)dl & hm], b = tab[(uint32_t)vl & hm];
                    conf = ((a >> 8) == (tag >> 8) && (int)(a & 255u) < ln()) ||
                           ((b >> 8) == (tag >> 8) && (int)(b & 255u) < ln());
                }
                const uint64_t cb = __ballot(conf);
                const int c = cb ? (int)__ffsll((unsigned long long)cb) - 1 : 64;
                const bool mine = pend && ln() < c;
                int32_t pa = 0, pb = 0;
                if (mine) {
                    pa = perm[dl];
                    pb = perm[vl];
                }
                if (mine) {
                    perm[vl] = pa;
                    perm[dl] = pb;
                }
                rem &= c >= 64 ? 0ull : ~((1ull << c) - 1);
                if (rem) wsync();
            }
            wsync();
#ifdef MANDO_CL_PHASES
            pq_swap += clock64() - tq1;
#endif
        }
    }
};

// Python round(best / cov, 3) for positive integers: q * 1000 rounded half-even on its exact binary
// value, then k / 1000 correctly rounded (the double Python's round returns)
__device__ double round3(int64_t best, int64_t cov) {
    const double q = (double)best / (double)cov;
    const uint64_t bits = (uint64_t)__double_as_longlong(q);
    const int ex = (int)((bits >> 52) & 0x7ff);
    uint64_t mant = bits & ((1ull << 52) - 1);
    int e2;
    if (ex == 0) {
        e2 = -1074;
    } else {
        mant |= 1ull << 52;
        e2 = ex - 1075;
    }
    const uint64_t Pm = mant * 1000ull;  // < 2^63
    uint64_t k;
    if (e2 >= 0) {
        if (e2 > 8) return q;  // q >= 2^52 is an integer already
        k = Pm << e2;
    } else {
        const int s = -e2;
        if (s >= 64) {
            k = 0;
        } else {
            k = Pm >> s;
            const uint64_t rem = Pm & ((1ull << s) - 1), half = 1ull << (s - 1);
            if (rem > half || (rem == half && (k & 1ull))) ++k;
        }
    }
    return (double)k / 1000.0;
}

// ---------------------------------------------------------------------------------------------
// K2: one locus
// ---------------------------------------------------------------------------------------------
// the static permutation buffer: 2 KB in the one-wave kernel (its LDS limits how many loci share a CU
// with the POA grids), 16 KB in the large-locus kernel (whose permutations reach 7k entries)
// (one-wave: the large loci whose permutations need more run on several waves; a longer one goes to the
// sort tile's LDS or to global scratch)
constexpr int kLdsPerm = 512, kLdsPermBig = 4096;

struct MwX {
    int32_t op;
    int32_t i32[4];
    int64_t i64[4];
    int64_t part[2][kMwWaves][4];
};
constexpr int64_t kPosBias = int64_t(1) << 39;  // sort keys hold position + bias in 40 bits

struct LocusRun {
    const uint8_t *T;
    Locus L;
    Stats S;
    const Params *P;
    ALayout A;
    BPtr B;
    OPtr O;
    MT mt;
    int32_t *lperm;
    int lperm_cap;  // its entries
    int64_t tile;   // keys of the dynamic LDS (g_sort_lds)
    int n;
    int status;
    int64_t bin_lo, bin_hi, nbins;
    int32_t n_peaks;
    int32_t ctr[2];  // spliceDict per-side counters
    int32_t n_iso, n_mem, n_sub;
    int32_t hcb_ok;  // every coverage bin lies in the map, so B.hcb answers histo_cov
    int W;           // waves of the workgroup (1: the one-wave kernel)
    MwX *X;          // their exchange (LDS)
    int64_t xcov;    // determine_cov's result (wave 0)
#ifdef MANDO_CL_PHASES  // dev build: cycles inside find_peaks (coverage merge, permutation, cs queries)
    uint64_t pc_cov = 0, pc_perm = 0, pc_cs = 0, pc_csof = 0, pc_bins = 0, pc_side = 0;
    uint64_t pc_sd_sort = 0, pc_sd_keys = 0, pc_sd_cand = 0;
    int32_t pc_cand = 0, pc_char = 0;
#endif

    // a permutation's buffer: static LDS, else the sort tile's dynamic LDS (free between sorts; each
    // permutation is consumed before the next sort), else global scratch
    __device__ int32_t *perm_buf(int32_t m) const {
        return m <= lperm_cap ? lperm : m <= 2 * tile ? reinterpret_cast<int32_t *>(g_sort_lds) : B.perm;
    }
    // the permutation's conflict table: whichever of the two LDS buffers the permutation does not use,
    // as many slots as positions where it fits (no collisions then), cleared once per permutation
    __device__ void permute(int32_t m, int32_t *perm) {
        int slots = 64;
        while (slots < m && slots < (m <= lperm_cap ? 2 * (int)tile : lperm_cap)) slots <<= 1;
        mt.permutation(m, perm, m <= lperm_cap ? reinterpret_cast<uint32_t *>(g_sort_lds) : reinterpret_cast<uint32_t *>(lperm),
                       slots);
    }
    __device__ bool in_map(int64_t p) const { return p >= L.map_lo && p < L.map_lo + L.map_n; }
    __device__ int64_t mi(int64_t p) const { return p - L.map_lo; }

    __device__ void fail(int code) {
        if (status == kOk) status = code;
    }

    // --- several waves per locus ----------------------------------------------------------------
    // wave 0: run a data-parallel phase on every wave of the workgroup (its arguments are in X)
    __device__ void par(int op) {
        if (W > 1) {
            if (ln() == 0) X->op = op;
            gsync();
        }
        exec(op, 0, W);
        if (W > 1)
            gsync();
        else
            wsync();
    }
    __device__ void exec(int op, int w, int nw) {
        if (op == kOpCovSets)
            cov_sets(w, nw);
        else if (op == kOpDetCov)
            det_cov(w, nw);
        else if (op == kOpCountSort)
            count_sort_part(X->i32[0], w, nw);
        else if (op == kOpKeys)
            keys_part(X->i32[0], w, nw);
    }
    // the helper waves: phases until wave 0 posts kOpExit
    __device__ void helper() {
        while (true) {
            gsync();
            const int op = X->op;
            if (op == kOpExit) break;
            exec(op, wv(), W);
            gsync();
        }
    }
    // one exchange between nw waves: wave w posts (a, b); after one barrier every wave holds the sum
    // of the a's and the min (or max) of the b's
    __device__ void xchg(int &ph, int w, int nw, int64_t &a, int64_t &b, bool bmax) {
        if (nw == 1) return;
        if (ln() == 0) {
            X->part[ph][w][0] = a;
            X->part[ph][w][1] = b;
        }
        gsync();
        int64_t sa = 0, sb = bmax ? INT64_MIN : INT64_MAX;
        for (int v = 0; v < nw; ++v) {
            sa += X->part[ph][v][0];
            const int64_t t = X->part[ph][v][1];
            sb = bmax ? (t > sb ? t : sb) : (t < sb ? t : sb);
        }
        a = sa;
        b = sb;
        ph ^= 1;
    }
    // exclusive prefix over the waves of v (excl: the waves before w) and the total
    __device__ void xprefix(int &ph, int w, int nw, int64_t v, int64_t &excl, int64_t &total) {
        if (nw == 1) {
            excl = 0;
            total = v;
            return;
        }
        if (ln() == 0) X->part[ph][w][0] = v;
        gsync();
        excl = total = 0;
        for (int u = 0; u < nw; ++u) {
            const int64_t t = X->part[ph][u][0];
            total += t;
            if (u < w) excl += t;
        }
        ph ^= 1;
    }

    // --- collect_reads (SDC:278-331) -----------------------------------------------------------
    __device__ void collect() {
#ifdef MANDO_CL_PHASES
        const uint64_t tc0 = clock64();
#endif
        // cs_of: the last record with this name on the locus chromosome (csDict[name] = cs)
        for (int r0 = 0; r0 < n; r0 += 64) {
            const int r = r0 + ln();
            if (r < n) {
                const Rec &R = A.recs[r];
                uint64_t h = 1469598103934665603ull;
                for (int i = 0; i < R.name_len; ++i) h = (h ^ T[R.name_off + i]) * 1099511628211ull;
                B.ihash[r] = h;
            }
        }
        // records of the locus chromosome sorted by (40 hash bits, index): a name's records are
        // adjacent and ascending, so each record's cs_of is the last same-name record after it in its
        // run (runs of other names that share the 40 bits are skipped by the name compare)
        const int64_t pn = pow2ge(n);
        for (int64_t r = ln(); r < pn; r += 64)
            B.isort[r] = (r < n && A.recs[r].same_chrom) ? ((B.ihash[r] & ~0xffffffull) | (uint64_t)r) : ~0ull;
        wsync();
        sort_u64(B.isort, pn, tile);
        for (int64_t i0 = 0; i0 < n; i0 += 64) {
            const int64_t i = i0 + ln();
            const uint64_t k = i < n ? B.isort[i] : ~0ull;
            if (k != ~0ull) {
                const int r = (int)(k & 0xffffffu);
                const Rec &R = A.recs[r];
                int32_t of = r;
                for (int64_t j = i + 1; j < n; ++j) {
                    const uint64_t kj = B.isort[j];
                    if (kj == ~0ull || (kj >> 24) != (k >> 24)) break;
                    const int q = (int)(kj & 0xffffffu);
                    const Rec &K = A.recs[q];
                    if (K.name_len == R.name_len && bytes_eq(T + K.name_off, T + R.name_off, R.name_len)) of = q;
                }
                A.recs[r].cs_of = of;
            }
        }
        for (int r0 = 0; r0 < n; r0 += 64) {
            const int r = r0 + ln();
            if (r < n && !A.recs[r].same_chrom) A.recs[r].cs_of = -1;
        }
        wsync();
#ifdef MANDO_CL_PHASES
        const uint64_t tc1 = clock64();
        pc_csof = tc1 - tc0;
#endif
        // coverage bins per record: myround over each block at stride 10 plus the block's tail, sorted
        // and made unique (cov_set); on every wave of the workgroup (cov_sets)
        const int64_t hist_n = L.map_n / 10 + 2;
        const bool hist_lds = hist_n <= 2 * tile;  // the sort tile is free until build_side
        if (hist_lds) {
            for (int64_t i = ln(); i < hist_n; i += 64) reinterpret_cast<int32_t *>(g_sort_lds)[i] = 0;
        }
        if (ln() == 0) X->i32[0] = hist_lds ? 1 : 0;
        wsync();
        par(kOpCovSets);
        int64_t lo = INT64_MAX, hi = INT64_MIN;
        int b = 0, oob = 0;
        for (int v = 0; v < W; ++v) {
            const int64_t *q = X->part[1][v];
            lo = q[0] < lo ? q[0] : lo;
            hi = q[1] > hi ? q[1] : hi;
            b = (int)q[2] > b ? (int)q[2] : b;
            oob |= (int)q[3];
        }
        if (b) {
            fail(b == 1 ? kParse : kRange);
            return;
        }
        bin_lo = lo;
        bin_hi = hi;
        hcb_ok = !oob;
        wsync();
        if (hist_lds)
            for (int64_t i = ln(); i < hist_n; i += 64) B.hcb[i] = reinterpret_cast<int32_t *>(g_sort_lds)[i];
        nbins = bin_lo <= bin_hi ? (bin_hi - bin_lo) / 10 + 1 : 0;
        wsync();
#ifdef MANDO_CL_PHASES
        const uint64_t tc2 = clock64();
        pc_bins = tc2 - tc1;
#endif
        for (int k = 0; k < 2; ++k) build_side(k);
#ifdef MANDO_CL_PHASES
        pc_side = clock64() - tc2;
#endif
    }

    // coverage sets (cov_set), the histogram entries of both sides and histo_cov of wave w's share of
    // the records (collect_reads, SDC:300-331), for nw waves
    __device__ void cov_sets(int w, int nw) {
        const int r_lo = (int)((int64_t)n * w / nw), r_hi = (int)((int64_t)n * (w + 1) / nw);
        const bool hist_lds = X->i32[0] != 0;
        // the coverage-set capacity and histogram entries of a record
        auto sizes = [&](const Rec &R, int64_t &capr, int32_t &nl, int32_t &nr) {
            capr = 0;
            nl = nr = 0;
            for (int x = 0; x < R.nblk; ++x) {
                const int64_t sz = A.blk[2 * (R.blk_off + x)], bs = A.blk[2 * (R.blk_off + x) + 1];
                capr += (sz > 0 ? (sz + 9) / 10 : 0) + 11;
                if (!R.acc_lt) {
                    nl += (bs + sz) != R.tend;
                    nr += bs != R.tstart;
                }
            }
        };
        // offsets continue the shares of the waves before this one (record order, as one wave would)
        int64_t carry = 0;
        int32_t hl_carry = 0, hr_carry = 0;
        if (nw > 1) {
            int64_t sc = 0, sl = 0, sr = 0;
            for (int r0 = r_lo; r0 < r_hi; r0 += 64) {
                const int r = r0 + ln();
                if (r < r_hi && A.recs[r].same_chrom) {
                    int64_t c;
                    int32_t x, y;
                    sizes(A.recs[r], c, x, y);
                    sc += c;
                    sl += x;
                    sr += y;
                }
            }
            sc = wsum(sc);
            sl = wsum(sl);
            sr = wsum(sr);
            if (ln() == 0) {
                X->part[0][w][0] = sc;
                X->part[0][w][1] = sl;
                X->part[0][w][2] = sr;
            }
            gsync();
            for (int v = 0; v < w; ++v) {
                carry += X->part[0][v][0];
                hl_carry += (int32_t)X->part[0][v][1];
                hr_carry += (int32_t)X->part[0][v][2];
            }
        }
        int64_t lo = INT64_MAX, hi = INT64_MIN;
        int bad = 0, oob = 0;
        for (int r0 = r_lo; r0 < r_hi; r0 += 64) {
            const int r = r0 + ln();
            const bool act = r < r_hi && A.recs[r].same_chrom;
            const Rec R = act ? A.recs[r] : Rec{};
            int64_t capr = 0;
            int32_t nl = 0, nr = 0;
            if (act) sizes(R, capr, nl, nr);
            const int64_t ci = wincl(capr);
            const int64_t coff = carry + ci - capr;
            carry += __shfl(ci, 63);
            const int32_t li_ = wincl(nl), ri_ = wincl(nr);
            int32_t el = hl_carry + li_ - nl, er = hr_carry + ri_ - nr;
            hl_carry += __shfl(li_, 63);
            hr_carry += __shfl(ri_, 63);
            if (act) {
                int64_t *v = B.cov + coff;
                int64_t m = 0, y = 0, lastv = INT64_MIN, hadd = -1;
                bool y_set = false, sorted = true;
                // histo_cov as a dense count per bin (the reference's histo_cov dict, SDC:318-320),
                // counted as the set is built while it stays in order (in LDS when the map is small)
                auto hist = [&](int64_t val, int d) {
                    const int64_t x = mi(val);
                    if (x < 0 || x >= L.map_n)
                        oob = 1;
                    else if (hist_lds)
                        atomicAdd(&reinterpret_cast<int32_t *>(g_sort_lds)[x / 10], d);
                    else
                        atomicAdd(&B.hcb[x / 10], d);
                };
                // a value equal to the previous one is dropped at once (the unique pass would drop it)
                auto push = [&](int64_t val) {
                    if (val == lastv) return;
                    if (val < lastv && sorted) {
                        sorted = false;
                        hadd = m;  // v[0, m) are counted; undone before the sort below
                    }
                    v[m++] = val;
                    lastv = val;
                    if (sorted) hist(val, 1);
                };
                for (int x = 0; x < R.nblk && !bad; ++x) {
                    const int64_t sz = A.blk[2 * (R.blk_off + x)], bs = A.blk[2 * (R.blk_off + x) + 1];
                    for (int64_t t = 0; t < sz; t += 10) {
                        push(myround(bs + t));
                        y = t;
                        y_set = true;
                    }
                    if (!y_set) {
                        bad = 1;  // NameError in the reference
                        break;
                    }
                    for (int64_t t = y; t < sz; ++t) push(myround(bs + t));
                    // histogram entries in block order (acc >= 0.9 only)
                    if (!R.acc_lt) {
                        const int64_t be = bs + sz;
                        if (be != R.tend) {
                            B.s[0].sk[el] = ((uint64_t)(be + kPosBias) << 24) | (uint64_t)el;
                            B.s[0].etmp[el] = r;
                            if (be + kPosBias < 0 || be + kPosBias >= (int64_t(1) << 40) || el >= (1 << 24)) bad = 2;
                            ++el;
                        }
                        if (bs != R.tstart) {
                            B.s[1].sk[er] = ((uint64_t)(bs + kPosBias) << 24) | (uint64_t)er;
                            B.s[1].etmp[er] = r;
                            if (bs + kPosBias < 0 || bs + kPosBias >= (int64_t(1) << 40) || er >= (1 << 24)) bad = 2;
                            ++er;
                        }
                    }
                }
                if (!bad) {
                    int64_t u = m;
                    if (!sorted) {  // blocks out of order: sort, unique, count
                        for (int64_t i = 0; i < hadd; ++i) hist(v[i], -1);
                        heap_sort(v, m);
                        u = 0;
                        for (int64_t i = 0; i < m; ++i)
                            if (u == 0 || v[i] != v[u - 1]) v[u++] = v[i];
                        for (int64_t i = 0; i < u; ++i) hist(v[i], 1);
                    }
                    A.recs[r].cov_off = (int32_t)coff;
                    A.recs[r].cov_n = (int32_t)u;
                    if (u > 0) {
                        lo = v[0] < lo ? v[0] : lo;
                        hi = v[u - 1] > hi ? v[u - 1] : hi;
                    }
                }
            } else if (r < r_hi) {
                A.recs[r].cov_off = 0;
                A.recs[r].cov_n = 0;
            }
        }
        lo = wmin(lo);
        hi = wmax(hi);
        bad = wmax(bad);
        oob = wany(oob != 0) ? 1 : 0;
        if (ln() == 0) {
            X->part[1][w][0] = lo;
            X->part[1][w][1] = hi;
            X->part[1][w][2] = bad;
            X->part[1][w][3] = oob;
        }
    }

    __device__ static int64_t myround(int64_t x) {
        if (x >= 0 && x < 0x7fffffff) {  // 32-bit division for genome positions
            const uint32_t ux = (uint32_t)x;
            uint32_t q = ux / 10u;
            const uint32_t r = ux - 10u * q;
            if (r > 5 || (r == 5 && (q & 1))) ++q;
            return 10 * (int64_t)q;
        }
        int64_t q = x >= 0 ? x / 10 : -((-x + 9) / 10);
        const int64_t r = x - 10 * q;
        if (r > 5 || (r == 5 && (q & 1))) ++q;
        return 10 * q;
    }

    __device__ static void heap_sort(int64_t *v, int64_t m) {
        auto sift = [&](int64_t i, int64_t len) {
            while (true) {
                int64_t c = 2 * i + 1;
                if (c >= len) break;
                if (c + 1 < len && v[c + 1] > v[c]) ++c;
                if (v[i] >= v[c]) break;
                const int64_t t = v[i];
                v[i] = v[c];
                v[c] = t;
                i = c;
            }
        };
        for (int64_t i = m / 2 - 1; i >= 0; --i) sift(i, m);
        for (int64_t e = m - 1; e > 0; --e) {
            const int64_t t = v[0];
            v[0] = v[e];
            v[e] = t;
            sift(0, e);
        }
    }

    // histogram of one side: entries sorted by (position, insertion), distinct keys with their
    // first insertion rank, strand counts, and the candidate order of find_peaks
    // Stable counting sort of a side's entries by position (keys are (position + bias) << 24 | rank and
    // the ranks follow the insertion order, so a stable sort by position is the key order): counts per
    // map position in B.sc (zero outside start_end_sites), an exclusive scan over the map, then the
    // entries placed in rank order, ties inside a step ranked by lane.  Returns false (nothing
    // changed) when a position falls outside the map.
    // Over nw waves: wave w takes the entries [H*w/nw, H*(w+1)/nw) and counts them in its own column
    // of B.sc (column v of position x at B.sc[x * nw + v]); the scan turns a position's columns into
    // the waves' cursors (the position's start, then the entries of the waves before), so each wave
    // places its entries in insertion order exactly where one wave would.
    __device__ bool count_sort_part(int side_i, int w, int nw) {
        Side &d = B.s[side_i];
        const int H = d.H;
        int32_t *C = B.sc;
        const int e_lo = (int)((int64_t)H * w / nw), e_hi = (int)((int64_t)H * (w + 1) / nw);
        int oob = 0;
        for (int i0 = e_lo; i0 < e_hi; i0 += 64) {
            const int i = i0 + ln();
            if (i < e_hi) {
                const int64_t x = mi((int64_t)(d.sk[i] >> 24) - kPosBias);
                if (x < 0 || x >= L.map_n)
                    oob = 1;
                else
                    atomicAdd(&C[x * nw + w], 1);
            }
        }
        wsync();
        int ph = 0;
        int64_t nbad = wany(oob != 0) ? 1 : 0, unused = 0;
        xchg(ph, w, nw, nbad, unused, true);
        const bool bad = nbad != 0;
        if (!bad) {
            // exclusive scan of the counts over the map (read with agent-scope loads: they were made by
            // L2 atomics), the map split between the waves: this wave's total first, then its range
            const int64_t m_lo = L.map_n * w / nw, m_hi = L.map_n * (w + 1) / nw;
            auto count_at = [&](int64_t x, int v) {
                return __hip_atomic_load(&C[x * nw + v], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            };
            int64_t carry = 0;
            if (nw > 1) {
                int64_t tot = 0;
                for (int64_t x0 = m_lo; x0 < m_hi; x0 += 64) {
                    const int64_t x = x0 + ln();
                    if (x < m_hi)
                        for (int v = 0; v < nw; ++v) tot += count_at(x, v);
                }
                tot = wsum(tot);
                if (ln() == 0) X->part[ph][w][0] = tot;
                gsync();
                for (int v = 0; v < w; ++v) carry += X->part[ph][v][0];
                ph ^= 1;
            }
            for (int64_t x0 = m_lo; x0 < m_hi; x0 += 64) {
                const int64_t x = x0 + ln();
                int32_t c = 0;
                if (x < m_hi)
                    for (int v = 0; v < nw; ++v) c += count_at(x, v);
                const int32_t ci = wincl(c);
                if (x < m_hi && c) {  // the cursor of each wave's column: the start, then the waves before
                    int32_t at = (int32_t)(carry + ci - c);
                    for (int v = 0; v < nw; ++v) {
                        const int32_t cv = count_at(x, v);
                        C[x * nw + v] = at;
                        at += cv;
                    }
                }
                carry += __shfl(ci, 63);
            }
            wsync();
            if (nw > 1) gsync();
            // this wave's entries, in insertion order, each at its column's cursor
            for (int i0 = e_lo; i0 < e_hi; i0 += 64) {
                const int i = i0 + ln();
                const bool act = i < e_hi;
                const uint64_t k = act ? d.sk[i] : ~0ull;
                const int64_t x = act ? mi((int64_t)(k >> 24) - kPosBias) : -1;
                int32_t rank = 0, later = 0;
                for (int t = 0; t < 64; ++t) {
                    const int64_t xt = __shfl(x, t);
                    const bool same = act && xt == x;
                    rank += (same && t < ln()) ? 1 : 0;
                    later |= (same && t > ln()) ? 1 : 0;
                }
                if (act) {
                    const int32_t dst = C[x * nw + w] + rank;
                    d.cand[dst] = k;
                    if (!later) C[x * nw + w] = dst + 1;
                }
                wsync();
            }
            if (nw > 1) gsync();  // every entry placed before any wave clears the counts
            uint64_t *t = d.sk;
            d.sk = d.cand;
            d.cand = t;
        }
        // B.sc back to zero where this side touched it
        for (int i0 = e_lo; i0 < e_hi; i0 += 64) {
            const int i = i0 + ln();
            if (i < e_hi) {
                const int64_t x = mi((int64_t)(d.sk[i] >> 24) - kPosBias);
                if (x >= 0 && x < L.map_n)
                    for (int v = 0; v < nw; ++v) C[x * nw + v] = 0;
            }
        }
        wsync();
        return !bad;
    }

    // the counting sort of side side_i on every wave of the workgroup; false: a position outside the map
    __device__ bool count_sort_side(int side_i) {
        if (W == 1) return count_sort_part(side_i, 0, 1);
        if (ln() == 0) X->i32[0] = side_i;
        wsync();
        const uint64_t *before = B.s[side_i].sk;
        par(kOpCountSort);
        return B.s[side_i].sk != before;  // sorted: the entries moved to the other buffer
    }

    __device__ void build_side(int side_i) {
        Side &d = B.s[side_i];
        const int H = d.H;
        for (int64_t i = H + ln(); i < d.P; i += 64) d.sk[i] = ~0ull;
        wsync();
        // large sides (config 2's ~35k entries): a counting sort over the map instead of the bitonic
        // network's log^2 passes
#ifdef MANDO_CL_PHASES
        const uint64_t ts0 = clock64();
#endif
        if (H <= kSortTile || !count_sort_side(side_i)) sort_u64(d.sk, d.P, tile);
#ifdef MANDO_CL_PHASES
        const uint64_t ts1 = clock64();
        pc_sd_sort += ts1 - ts0;
#endif
        // records in sorted order; distinct-key flags; strand counts per key (keys_part)
        if (W > 1 && H >= 64 * W) {
            if (ln() == 0) X->i32[0] = side_i;
            wsync();
            par(kOpKeys);
        } else {
            keys_part(side_i, 0, 1);
        }
        const int32_t kc = d.nkeys;
#ifdef MANDO_CL_PHASES
        const uint64_t ts2 = clock64();
        pc_sd_keys += ts2 - ts1;
#endif
        for (int u0 = 0; u0 < kc; u0 += 64) {
            const int u = u0 + ln();
            if (u < kc) d.ucnt[u] = (u + 1 < kc ? d.ulo[u + 1] : H) - d.ulo[u];
        }
        wsync();
        // candidates: count >= min_count, count descending, insertion order on ties
        int32_t cc = 0;
        for (int u0 = 0; u0 < kc; u0 += 64) {
            const int u = u0 + ln();
            const int take = (u < kc && d.ucnt[u] >= P->min_count) ? 1 : 0;
            const int32_t ti = wincl(take);
            if (take) {
                d.cand[cc + ti - 1] = ((uint64_t)(0x7fffffff - d.ucnt[u]) << 32) | (uint64_t)d.ufirst[u];
                d.etmp[d.ufirst[u]] = u;
            }
            cc += __shfl(ti, 63);
        }
        d.ncand = cc;
        for (int64_t i = cc + ln(); i < d.P; i += 64) d.cand[i] = ~0ull;
        wsync();
        sort_u64(d.cand, pow2ge(cc), tile);
#ifdef MANDO_CL_PHASES
        pc_sd_cand += clock64() - ts2;
#endif
    }

    // distinct keys of side side_i's sorted entries, wave w of nw taking the entries [H*w/nw,
    // H*(w+1)/nw): lane per entry, the key index of entry i is the number of distinct keys up to i,
    // minus one (the waves before w count theirs first)
    __device__ void keys_part(int side_i, int w, int nw) {
        Side &d = B.s[side_i];
        const int H = d.H;
        const int e_lo = (int)((int64_t)H * w / nw), e_hi = (int)((int64_t)H * (w + 1) / nw);
        for (int64_t i = 3 * (int64_t)e_lo + ln(); i < 3 * (int64_t)e_hi; i += 64) d.upmb[i] = 0;
        auto pos_of = [&](int i) { return (int64_t)(d.sk[i] >> 24) - kPosBias; };
        int64_t kc = 0, total = 0;
        {
            int64_t f = 0;
            if (nw > 1)
                for (int i0 = e_lo; i0 < e_hi; i0 += 64) {
                    const int i = i0 + ln();
                    if (i < e_hi) f += (i == 0 || pos_of(i - 1) != pos_of(i)) ? 1 : 0;
                }
            int ph = 0;
            xprefix(ph, w, nw, wsum(f), kc, total);  // (one wave: both 0, set below)
        }
        wsync();
        for (int i0 = e_lo; i0 < e_hi; i0 += 64) {
            const int i = i0 + ln();
            int first = 0;
            int64_t pos = 0;
            int32_t seq = 0;
            if (i < e_hi) {
                const uint64_t k = d.sk[i];
                pos = (int64_t)(k >> 24) - kPosBias;
                seq = (int32_t)(k & 0xffffffu);
                d.erec[i] = d.etmp[seq];
                first = (i == 0 || pos_of(i - 1) != pos) ? 1 : 0;
            }
            const int32_t fi = wincl(first);
            if (i < e_hi) {
                const int32_t u = (int32_t)kc + fi - 1;
                if (first) {
                    d.ukey[u] = pos;
                    d.ulo[u] = i;
                    d.ufirst[u] = seq;
                }
                const int8_t dn = A.recs[d.etmp[seq]].dirn;
                atomicAdd(&d.upmb[3 * u + (dn == 0 ? 0 : dn == 1 ? 1 : 2)], 1);
            }
            kc += __shfl(fi, 63);
        }
        d.nkeys = (int32_t)(nw > 1 ? total : kc);
        wsync();
    }

    __device__ int find_key(const Side &d, int64_t pos) const {
        int lo = 0, hi = d.nkeys;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (d.ukey[mid] < pos)
                lo = mid + 1;
            else
                hi = mid;
        }
        return (lo < d.nkeys && d.ukey[lo] == pos) ? lo : -1;
    }

    // --- make_genome_bins (SDC:392-438) -------------------------------------------------------
    __device__ void push_peak(int64_t s, int64_t e, char type, char side, double prop, int side_i) {
        if (n_peaks >= O.peak_cap) {
            fail(kCapacity);
            return;
        }
        if (!in_map(s) || !in_map(e)) {
            fail(kRange);
            return;
        }
        if (ln() == 0) {
            Peak pk;
            pk.start = s;
            pk.end = e;
            pk.prop = prop;
            pk.type = type;
            pk.side = side;
            O.peaks[n_peaks] = pk;
        }
        for (int64_t b = s + ln(); b <= e; b += 64) B.areas[side_i][mi(b)] = 1;
        wsync();
        ++n_peaks;
    }

    __device__ void genome_bins(int side_i) {
        const int w = P->w;
        for (int ti = 0; ti < 2; ++ti) {
            const int s = side_i * 2 + ti;
            const int a = L.ann_off[s] - L.ann_off[0], len = L.ann_off[s + 1] - L.ann_off[s];
            if (len <= 0) continue;
            int64_t *pl = B.ann + a;
            // the host passes each list as is; sort ascending (insertion sort on lane 0: short lists)
            if (ln() == 0) {
                for (int i = 1; i < len; ++i) {
                    const int64_t x = pl[i];
                    int j = i - 1;
                    while (j >= 0 && pl[j] > x) {
                        pl[j + 1] = pl[j];
                        --j;
                    }
                    pl[j + 1] = x;
                }
            }
            wsync();
            int i1 = 0;
            while (i1 < len) {
                int64_t mx = pl[i1], mn = pl[i1];
                int i2 = i1;
                while (i2 < len && pl[i2] - mx <= w) {
                    mx = pl[i2] > mx ? pl[i2] : mx;
                    mn = pl[i2] < mn ? pl[i2] : mn;
                    ++i2;
                }
                push_peak(mn - w, mx + w, ti == 0 ? '5' : '3', side_i == 0 ? 'l' : 'r', -1.0, side_i);
                if (status != kOk) return;
                i1 = i2;
            }
        }
    }

    // --- determine_cov (SDC:200-224) ------------------------------------------------------------
    __device__ int32_t hcov(int64_t pos) {
        // pos is a coverage bin, so inside the map; the counts were made by L2 atomics, so the read is
        // an agent-scope atomic load (never a stale L1 line)
        if (hcb_ok) return __hip_atomic_load(&B.hcb[mi(pos) / 10], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int32_t c = 0;
        for (int r0 = 0; r0 < n; r0 += 64) {
            const int r = r0 + ln();
            if (r < n && A.recs[r].cov_n > 0) {
                const Rec &R = A.recs[r];
                const int64_t *v = B.cov + R.cov_off;
                int lo = 0, hi = R.cov_n;
                while (lo < hi) {
                    const int mid = (lo + hi) >> 1;
                    if (v[mid] < pos)
                        lo = mid + 1;
                    else
                        hi = mid;
                }
                c += (lo < R.cov_n && v[lo] == pos) ? 1 : 0;
            }
        }
        return wsum(c);
    }

    __device__ int64_t determine_cov(int32_t nn, int64_t center, bool reverse) {
        if (ln() == 0) {
            X->i32[0] = nn;
            X->i32[1] = reverse ? 1 : 0;
            X->i64[0] = center;
            X->i64[1] = bin_lo;
            X->i64[2] = nbins;
        }
        wsync();
        if (W > 1 && nn >= 64 * W)
            par(kOpDetCov);
        else
            det_cov(0, 1);
        return xcov;
    }

    // the coverage merge of determine_cov over wave w's share of the nn winners (B.names), nw waves;
    // wave 0 keeps the result in xcov
    __device__ void det_cov(int w, int nw) {
        const int32_t nn = X->i32[0];
        const bool reverse = X->i32[1] != 0;
        const int64_t center = X->i64[0], blo = X->i64[1], nbn = X->i64[2];
        int64_t kstart;
        if (reverse) {
            const int64_t k = center - 1 - blo;
            kstart = k < 0 ? -1 : (k / 10 < nbn - 1 ? k / 10 : nbn - 1);
        } else {
            const int64_t k = center + 1 - blo;
            kstart = k <= 0 ? 0 : (k + 9) / 10;
            if (kstart >= nbn) kstart = -1;
        }
        if (kstart < 0) {
            if (w == 0) xcov = 0;
            return;
        }
        const int c_lo = (int)((int64_t)nn * w / nw), c_hi = (int)((int64_t)nn * (w + 1) / nw);
        const int64_t bound = blo + 10 * kstart;
        const int64_t none = reverse ? INT64_MIN : INT64_MAX;
        // each winner's head: the absolute index of its first set element at / after the bound (the
        // last at / before it for the left side) in B.cur, its value in B.hv
        int64_t best = none;
        for (int c0 = c_lo; c0 < c_hi; c0 += 64) {
            const int c = c0 + ln();
            if (c < c_hi) {
                const Rec &R = A.recs[B.names[c]];
                const int64_t *v = B.cov + R.cov_off;
                int lo = 0, hi = R.cov_n;
                int32_t at = -1;
                if (reverse) {  // last element <= bound
                    while (lo < hi) {
                        const int mid = (lo + hi) >> 1;
                        if (v[mid] <= bound)
                            lo = mid + 1;
                        else
                            hi = mid;
                    }
                    at = lo - 1;
                } else {  // first element >= bound
                    while (lo < hi) {
                        const int mid = (lo + hi) >> 1;
                        if (v[mid] < bound)
                            lo = mid + 1;
                        else
                            hi = mid;
                    }
                    at = lo < R.cov_n ? lo : -1;
                }
                const int64_t h = at >= 0 ? v[at] : none;
                B.cur[c] = at >= 0 ? R.cov_off + at : -1;
                B.hv[c] = h;
                best = reverse ? (h > best ? h : best) : (h < best ? h : best);
            }
        }
        int64_t top = reverse ? wmax(best) : wmin(best);
        int ph = 0;
        {
            int64_t z = 0;
            xchg(ph, w, nw, z, top, reverse);
        }
        wsync();
        int64_t cov = 0;
        int counter = 0;
        // merge step: the winners at the extreme head (`top`) advance; the next extreme is taken in the
        // same pass (count and next extreme exchanged between the waves once per step)
        while (counter < 4 && top != none) {
            int64_t count = 0;
            int64_t nb = none;
            for (int c0 = c_lo; c0 < c_hi; c0 += 64) {
                const int c = c0 + ln();
                if (c < c_hi) {
                    int64_t h = B.hv[c];
                    if (h == top) {
                        ++count;
                        const Rec &R = A.recs[B.names[c]];
                        const int32_t nx = reverse ? B.cur[c] - 1 : B.cur[c] + 1;
                        const bool in = nx >= R.cov_off && nx < R.cov_off + R.cov_n;
                        h = in ? B.cov[nx] : none;
                        B.cur[c] = in ? nx : -1;
                        B.hv[c] = h;
                    }
                    nb = reverse ? (h > nb ? h : nb) : (h < nb ? h : nb);
                }
            }
            count = wsum(count);
            nb = reverse ? wmax(nb) : wmin(nb);
            xchg(ph, w, nw, count, nb, reverse);
            wsync();
            if (count > 1) {
                ++counter;
                if (w == 0) {
                    const int64_t hc = hcov(top);
                    cov = hc > cov ? hc : cov;
                }
            }
            top = nb;
        }
        if (w == 0) xcov = cov;
    }

    // --- getCSaroundSS on the tokenised cs (cluster.cpp cs_around) --------------------------------
    __device__ int run_of(const Rec &R, int32_t t) const {
        int lo = 0, hi = R.nrun - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (A.runs[R.run_off + mid].rec0 <= t)
                lo = mid;
            else
                hi = mid - 1;
        }
        return lo;
    }
    __device__ static int st_slot(char c) {
        return c == '*' ? 0 : c == '+' ? 1 : c == '-' ? 2 : c == '=' ? 3 : 4;
    }
    __device__ void count_range(const Rec &R, int32_t a, int32_t b, int32_t *cnt) const {
        if (a >= b) return;
        int k = run_of(R, a);
        while (a < b) {
            const Run &U = A.runs[R.run_off + k];
            const int32_t e = b < U.rec0 + U.n ? b : U.rec0 + U.n;
            cnt[st_slot(U.st)] += e - a;
            cnt[5] += e - a;
            a = e;
            ++k;
        }
    }
    // returns the junction motif (4 chars packed, 0 for "nnnn"), counts into cl / cr
    __device__ bool cs_around(const Rec &R, int64_t start, int64_t end, char mot[4], int32_t *cl, int32_t *cr,
                              bool &has_l, bool &has_r) const {
        mot[0] = mot[1] = mot[2] = mot[3] = 'n';
        has_l = has_r = false;
        const int32_t nrec = R.nrec_cs;
        int lo = 0, hi = R.nadv;  // upper_bound(adv_first, end) - 1
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (A.adv_first[R.adv_off + mid] <= end)
                lo = mid + 1;
            else
                hi = mid;
        }
        const int ka = lo - 1;
        if (ka < 0) return false;
        const Run U = A.runs[R.run_off + A.adv_run[R.adv_off + ka]];
        int64_t i_in = 0;
        if (U.n != 1) {
            const int64_t q = (end - U.g0) / U.step - 1;
            i_in = q < U.n - 1 ? q : U.n - 1;
        }
        const int64_t pos = U.g0 + (int64_t)U.step * (i_in + 1);
        if (pos < start) return false;
        const int64_t si = U.rec0 + i_in + 1;
        const int64_t wlo = si - 10 > 0 ? si - 10 : 0, whi = si + 10 < nrec ? si + 10 : nrec;
        int64_t idx = -1;
        Run IR = {};
        if (wlo < whi) {
            for (int k = run_of(R, (int32_t)(whi - 1)); k >= 0; --k) {
                const Run &V = A.runs[R.run_off + k];
                if (V.rec0 + V.n <= wlo) break;
                if (V.st == '|') {
                    idx = V.rec0;
                    IR = V;
                    break;
                }
            }
        }
        if (idx < 0) return false;
        mot[0] = IR.motif[0];
        mot[1] = IR.motif[1];
        mot[2] = IR.motif[2];
        mot[3] = IR.motif[3];
        int64_t a = idx - 5, b = idx;
        if (a < 0) a += nrec;
        if (a < 0) a = 0;
        if (a < b) {
            count_range(R, (int32_t)a, (int32_t)(b < nrec ? b : nrec), cl);
            has_l = true;
        }
        const int64_t ra = idx + 1, rb = idx + 6 < nrec ? idx + 6 : nrec;
        if (ra < rb) {
            count_range(R, (int32_t)ra, (int32_t)rb, cr);
            has_r = true;
        }
        return true;
    }

    // --- characterize_splicing_event (SDC:499-550) ----------------------------------------------
    __device__ bool characterize(int64_t left, int64_t right, int32_t nn) {
        const int32_t k = nn < 500 ? nn : 500;
        int32_t *perm = perm_buf(nn);
#ifdef MANDO_CL_PHASES
        const uint64_t tq0 = clock64();
        permute(nn, perm);
        const uint64_t tq1 = clock64();
        pc_perm += tq1 - tq0;
        ++pc_char;
#else
        permute(nn, perm);
#endif
        int32_t allowed = 0, bad = 0;
        int32_t lc[6] = {0, 0, 0, 0, 0, 0}, rc[6] = {0, 0, 0, 0, 0, 0};
        for (int t0 = 0; t0 < k; t0 += 64) {
            const int t = t0 + ln();
            if (t < k) {
                const int32_t ri = A.recs[B.names[perm[t]]].cs_of;
                const Rec R = A.recs[ri];
                if (R.cs_bad) {
                    bad = 1;
                } else {
                    char mot[4];
                    int32_t cl[6] = {0, 0, 0, 0, 0, 0}, cr[6] = {0, 0, 0, 0, 0, 0};
                    bool hl, hr;
                    cs_around(R, left, right, mot, cl, cr, hl, hr);
                    for (int j = 0; j < P->n_junc; ++j)
                        if (P->junc_len4[j] && P->junc[j][0] == mot[0] && P->junc[j][1] == mot[1] &&
                            P->junc[j][2] == mot[2] && P->junc[j][3] == mot[3]) {
                            ++allowed;
                            break;
                        }
                    if (hl)
                        for (int s = 0; s < 6; ++s) lc[s] += cl[s];
                    if (hr)
                        for (int s = 0; s < 6; ++s) rc[s] += cr[s];
                }
            }
        }
        wsync();
#ifdef MANDO_CL_PHASES
        pc_cs += clock64() - tq1;
#endif
        if (wany(bad != 0)) {
            fail(kParse);
            return false;
        }
        allowed = wsum(allowed);
        for (int s = 0; s < 6; ++s) {
            lc[s] = wsum(lc[s]);
            rc[s] = wsum(rc[s]);
        }
        if (k == 0) {
            fail(kZeroDivision);
            return false;
        }
        if (!((double)allowed / (double)k > 0.85)) return false;
        if (lc[5] == 0 || rc[5] == 0) {
            fail(kZeroDivision);
            return false;
        }
        return (double)lc[3] / (double)lc[5] > 0.85 && (double)rc[3] / (double)rc[5] > 0.85;
    }

    // --- find_peaks / scan_for_best_bin (SDC:232-275, :163-197) --------------------------------
    __device__ void find_peaks(int side_i) {
        Side &d = B.s[side_i];
        const bool reverse = side_i == 0;
        const int64_t w = P->w, span = 4 * w + 1;
        int64_t *wc = B.win, *wp = B.win + span, *wm = B.win + 2 * span, *wf = B.win + 3 * span;
        uint8_t *areas = B.areas[side_i];
        for (int ci = 0; ci < d.ncand; ++ci) {
            const int u = d.etmp[(int)(d.cand[ci] & 0xffffffffu)];
            const int64_t entry = d.ukey[u];
            if (!in_map(entry - 2 * w) || !in_map(entry + 2 * w)) {
                fail(kRange);
                return;
            }
            if (areas[mi(entry)]) continue;
#ifdef MANDO_CL_PHASES
            ++pc_cand;
#endif
            for (int64_t dd = ln(); dd < span; dd += 64) {
                const int64_t pos = entry - 2 * w + dd;
                int64_t f = areas[mi(pos)] ? 1 : 0, c = 0, p = 0, m = 0;
                const int k = find_key(d, pos);
                if (k >= 0) {
                    c = d.ucnt[k];
                    p = d.upmb[3 * k];
                    m = d.upmb[3 * k + 1];
                    if (d.upmb[3 * k + 2] > 0) f |= 2;
                }
                wc[dd] = c;
                wp[dd] = p;
                wm[dd] = m;
                wf[dd] = f;
            }
            wsync();
            int64_t best = 0, center = 0, bx = 0, bdp = 0, bdm = 0;
            bool key_err = false;
            for (int64_t xi = 0; xi < 2 * w + 1 && !key_err; ++xi) {
                const int64_t x = xi == 0 ? 0 : ((xi & 1) ? (xi + 1) / 2 : -(xi / 2));
                const int64_t d0 = x + w;
                int64_t fl = 0, cnt = 0, dp = 0, dm = 0;
                for (int64_t q = d0; q < d0 + 2 * w + 1; ++q) fl |= wf[q];
                if (fl & 1) continue;
                if (fl & 2) {
                    key_err = true;
                    break;
                }
                for (int64_t q = d0; q < d0 + 2 * w + 1; ++q) {
                    cnt += wc[q];
                    dp += wp[q];
                    dm += wm[q];
                }
                if (cnt > best) {
                    best = cnt;
                    center = entry + x;
                    bx = x;
                    bdp = dp;
                    bdm = dm;
                }
            }
            if (key_err) {
                fail(kKeyError);
                return;
            }
            int32_t nn = 0;
            int64_t cov = 0;
            if (best > 0) {
                for (int64_t yi = 0; yi < 2 * w + 1; ++yi) {
                    const int64_t y = yi == 0 ? 0 : ((yi & 1) ? (yi + 1) / 2 : -(yi / 2));
                    const int k = find_key(d, entry + bx + y);
                    if (k < 0) continue;
                    const int c = d.ucnt[k], lo = d.ulo[k];
                    for (int i = ln(); i < c; i += 64) B.names[nn + i] = d.erec[lo + i];
                    nn += c;
                }
                wsync();
#ifdef MANDO_CL_PHASES
                const uint64_t tc0 = clock64();
                cov = determine_cov(nn, center, reverse);
                pc_cov += clock64() - tc0;
#else
                cov = determine_cov(nn, center, reverse);
#endif
            }
            if (cov <= 0) continue;
            const double prop = round3(best, cov);
            if (!(prop > P->cutoff)) continue;
            char type = 0;
            if (bdp < bdm)
                type = reverse ? '3' : '5';
            else if (bdp > bdm)
                type = reverse ? '5' : '3';
            if (!type) continue;
            const bool ok = characterize(center - w, center + w, nn);
            if (status != kOk) return;
            if (ok) {
                push_peak(center - w, center + w, type, side_i == 0 ? 'l' : 'r', prop, side_i);
                if (status != kOk) return;
            }
        }
    }

    // --- spliceDict (defineIsoforms.py:71-83): per-side counters, later rows overwrite -------------
    __device__ void splice_dict() {
        ctr[0] = ctr[1] = 0;
        for (int pi = 0; pi < n_peaks; ++pi) {
            const Peak pk = O.peaks[pi];
            const int s = pk.side == 'l' ? 0 : 1;
            ctr[s] += 1;
            if (ln() == 0) B.lab[pi] = ctr[s] | (pk.type == '3' ? (1 << 30) : 0) | (s ? (1 << 29) : 0);
            for (int64_t b = pk.start + ln(); b <= pk.end; b += 64) B.splice[mi(b)] = pi;
            wsync();
        }
    }

    __device__ int put_label(uint8_t *o, int32_t lab) const {
        int len = 0;
        o[len++] = (lab & (1 << 30)) ? '3' : '5';
        o[len++] = (lab & (1 << 29)) ? 'r' : 'l';
        const int32_t c = lab & ((1 << 29) - 1);
        char d[12];
        int nd = 0;
        int32_t v = c;
        do {
            d[nd++] = (char)('0' + v % 10);
            v /= 10;
        } while (v);
        while (nd) o[len++] = (uint8_t)d[--nd];
        return len;
    }

    // --- sort_reads_into_splice_junctions (SDC:714-769): identity text per record -----------------
    __device__ void sort_reads() {
        int64_t carry = 0;
        for (int r0 = 0; r0 < n; r0 += 64) {
            const int r = r0 + ln();
            int64_t cap = 0;
            Rec R = {};
            if (r < n) {
                R = A.recs[r];
                cap = (R.chrom_len + 2 + (int64_t)(R.nblk > 0 ? R.nblk - 1 : 0) * 28 + 7) & ~int64_t(7);
            }
            const int64_t ci = wincl(cap);
            const int64_t off = carry + ci - cap;
            carry += __shfl(ci, 63);
            if (r < n) {
                uint8_t *o = B.ibuf + off;
                int len = 0;
                for (int i = 0; i < R.chrom_len; ++i) o[len++] = T[R.chrom_off + i];
                o[len++] = '_';
                bool failed = false;
                for (int x = 0; x + 1 < R.nblk; ++x) {
                    const int64_t ls = A.blk[2 * (R.blk_off + x) + 1] + A.blk[2 * (R.blk_off + x)];
                    const int64_t rs = A.blk[2 * (R.blk_off + x + 1) + 1];
                    if (rs - ls > 50) {
                        if (!R.same_chrom) {
                            failed = true;
                            break;
                        }
                        const int32_t a = in_map(ls) ? B.splice[mi(ls)] : -1;
                        const int32_t b = in_map(rs) ? B.splice[mi(rs)] : -1;
                        if (a < 0 || b < 0) {
                            failed = true;
                            break;
                        }
                        len += put_label(o + len, B.lab[a]);
                        o[len++] = '-';
                        len += put_label(o + len, B.lab[b]);
                        o[len++] = '~';
                    }
                }
                int8_t kind = 0;
                if (!failed) {
                    // identity.split('_')[1] != ''
                    int u1 = -1;
                    for (int i = 0; i < R.chrom_len; ++i)
                        if (o[i] == '_') {
                            u1 = i;
                            break;
                        }
                    bool spliced;
                    if (u1 < 0) {
                        spliced = len > R.chrom_len + 1;
                    } else {
                        int u2 = R.chrom_len;
                        for (int i = u1 + 1; i < R.chrom_len; ++i)
                            if (o[i] == '_') {
                                u2 = i;
                                break;
                            }
                        spliced = u2 > u1 + 1;
                    }
                    kind = spliced ? 1 : 2;
                }
                uint64_t h = 1469598103934665603ull;
                for (int i = 0; i < len; ++i) h = (h ^ o[i]) * 1099511628211ull;
                B.ioff[r] = (int32_t)off;
                B.ilen[r] = len;
                B.ikind[r] = kind;
                B.ihash[r] = h;
            }
        }
        wsync();
    }

    __device__ bool ident_eq(int32_t a, int32_t b) const {
        return B.ilen[a] == B.ilen[b] && bytes_eq(B.ibuf + B.ioff[a], B.ibuf + B.ioff[b], B.ilen[a]);
    }

    // byte p of identity `id`: the rep record's identity text, then "M<k>" for a mono-exon group
    __device__ int id_char(int32_t id, int p) const {
        const int32_t rep = B.id_rep[id];
        const int L0 = B.ilen[rep];
        if (p < L0) return B.ibuf[B.ioff[rep] + p];
        const int32_t m = B.id_m[id];
        if (m < 0) return -1;
        if (p == L0) return 'M';
        int nd = 1;
        for (int32_t v = m; v >= 10; v /= 10) ++nd;
        const int k = p - L0 - 1;
        if (k >= nd) return -1;
        int32_t v = m;
        for (int i = 0; i < nd - 1 - k; ++i) v /= 10;
        return '0' + v % 10;
    }
    __device__ bool id_less(int32_t a, int32_t b) const {
        for (int p = 0;; ++p) {
            const int x = id_char(a, p), y = id_char(b, p);
            if (x != y) return x < y;  // -1 (end) sorts first
            if (x < 0) return false;
        }
    }

    // the position tuple of group_mono's sort: (start, end, (name, seq), left_extra, right_extra)
    __device__ int bytes_cmp(const uint8_t *x, int nx, const uint8_t *y, int ny) const {
        const int m = nx < ny ? nx : ny;
        for (int i = 0; i < m; ++i)
            if (x[i] != y[i]) return x[i] < y[i] ? -1 : 1;
        return nx < ny ? -1 : nx > ny ? 1 : 0;
    }
    __device__ bool pos_less(int32_t a, int32_t b) const {
        const Rec &X = A.recs[a], &Y = A.recs[b];
        if (X.tstart != Y.tstart) return X.tstart < Y.tstart;
        if (X.tend != Y.tend) return X.tend < Y.tend;
        int c = bytes_cmp(T + X.name_off, X.name_len, T + Y.name_off, Y.name_len);
        if (c) return c < 0;
        c = bytes_cmp(T + X.seq_off, X.seq_len, T + Y.seq_off, Y.seq_len);
        if (c) return c < 0;
        if (X.qstart != Y.qstart) return X.qstart < Y.qstart;
        const int64_t rx = X.qsize - X.qend, ry = Y.qsize - Y.qend;
        if (rx != ry) return rx < ry;
        return a < b;  // stable
    }

    // --- identities: group records by identity text; mono-exon groups split into "M<k>" groups
    //     (group_mono_exon_transcripts, SDC:772-794); all identities sorted by text --------------------
    int32_t n_ids, n_members;
    __device__ void identities() {
        const int64_t pn = pow2ge(n);
        for (int64_t i = ln(); i < pn; i += 64) {
            uint64_t k = ~0ull;
            if (i < n && B.ikind[i] != 0) k = (B.ihash[i] & ~0xffffffull) | (uint64_t)i;
            B.isort[i] = k;
        }
        wsync();
        sort_u64(B.isort, pn, tile);
        // valid entries and hash-run starts (max-scan of run-start flags)
        int32_t nv = 0, carry = 0;
        for (int i0 = 0; i0 < n; i0 += 64) {
            const int i = i0 + ln();
            const uint64_t k = i < n ? B.isort[i] : ~0ull;
            const bool valid = k != ~0ull;
            int32_t st_ = -1;
            if (valid) st_ = (i == 0 || (B.isort[i - 1] >> 24) != (k >> 24)) ? i : -1;
            int32_t m = st_;
            for (int o = 1; o < 64; o <<= 1) {
                const int32_t t = __shfl_up(m, o);
                if (ln() >= o && t > m) m = t;
            }
            m = m > carry ? m : carry;
            if (valid) B.msort[i] = m;
            carry = __shfl(m, 63);
            nv += (int32_t)__popcll(__ballot(valid));
        }
        wsync();
        // group representative: the first record of the run with the same identity text
        for (int i0 = 0; i0 < nv; i0 += 64) {
            const int i = i0 + ln();
            if (i < nv) {
                const int32_t r = (int32_t)(B.isort[i] & 0xffffffu);
                int32_t rep = r;
                for (int j = B.msort[i]; j < i; ++j) {
                    const int32_t q = (int32_t)(B.isort[j] & 0xffffffu);
                    if (ident_eq(q, r)) {
                        rep = q;
                        break;
                    }
                }
                B.grp[r] = rep;
            }
        }
        wsync();
        // members grouped by representative (first occurrence), record order inside
        for (int64_t i = ln(); i < pn; i += 64) {
            uint64_t k = ~0ull;
            if (i < n && B.ikind[i] != 0) k = ((uint64_t)B.grp[i] << 24) | (uint64_t)i;
            B.isort[i] = k;
        }
        wsync();
        sort_u64(B.isort, pn, tile);
        for (int i = ln(); i < nv; i += 64) B.msort[i] = (int32_t)(B.isort[i] & 0xffffffu);
        wsync();
        n_members = nv;
        // walk the groups (uniform): spliced groups are one identity; mono groups are sorted by the
        // position tuple and split by the overlap counter
        n_ids = 0;
        int g0 = 0;
        while (g0 < nv) {
            const int32_t rep = (int32_t)(B.isort[g0] >> 24);
            // group end: first index with another representative (binary search: keys ascend)
            int lo = g0 + 1, hi = nv;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if ((int32_t)(B.isort[mid] >> 24) == rep)
                    lo = mid + 1;
                else
                    hi = mid;
            }
            const int g1 = lo;
            if (B.ikind[rep] == 1) {
                if (ln() == 0) {
                    B.id_lo[n_ids] = g0;
                    B.id_hi[n_ids] = g1;
                    B.id_rep[n_ids] = rep;
                    B.id_m[n_ids] = -1;
                }
                ++n_ids;
            } else {
                const int m = g1 - g0;
                const int64_t pm = pow2ge(m);
                for (int64_t i = ln(); i < pm; i += 64) B.idsort[i] = i < m ? B.msort[g0 + i] : -1;
                wsync();
                sort_idx(B.idsort, pm, [&](int32_t a, int32_t b) { return pos_less(a, b); });
                for (int i = ln(); i < m; i += 64) B.msort[g0 + i] = B.idsort[i];
                wsync();
                // overlap counter (lane 0, in order), then one identity per counter run
                if (ln() == 0) {
                    int64_t prev_end = 0;
                    int32_t counter = 0;
                    for (int i = 0; i < m; ++i) {
                        const Rec &R = A.recs[B.msort[g0 + i]];
                        if (R.tstart > prev_end) {
                            counter += 1;
                            prev_end = R.tend > prev_end ? R.tend : prev_end;
                        } else {
                            prev_end = R.tend;
                        }
                        B.msuf[g0 + i] = counter;
                    }
                }
                wsync();
                int i = 0;
                while (i < m) {
                    const int32_t c = B.msuf[g0 + i];
                    int j = i + 1;
                    while (j < m && B.msuf[g0 + j] == c) ++j;
                    if (ln() == 0) {
                        B.id_lo[n_ids] = g0 + i;
                        B.id_hi[n_ids] = g0 + j;
                        B.id_rep[n_ids] = rep;
                        B.id_m[n_ids] = c;
                    }
                    ++n_ids;
                    i = j;
                }
            }
            wsync();
            g0 = g1;
        }
        const int64_t pi = pow2ge(n_ids);
        for (int64_t i = ln(); i < pi; i += 64) B.idsort[i] = i < n_ids ? (int32_t)i : -1;
        wsync();
        sort_idx(B.idsort, pi, [&](int32_t a, int32_t b) { return id_less(a, b); });
    }

    // --- find_ends (SDC:554-711) with dense position maps ----------------------------------------
    __device__ void extend(int32_t *peaks, const int32_t *cnt, int64_t position, int64_t adjacent, int dir,
                           int64_t best_bin) {
        const int64_t mc = P->min_count;
        bool extended = true;
        while (extended) {
            const int64_t a = adjacent + dir * (int64_t)(ln() + 1);
            const bool mine = ln() < 10;
            const bool rng = wany(mine && !in_map(a));
            if (rng) {
                fail(kRange);
                return;
            }
            const int32_t c = mine ? cnt[mi(a)] : 0;
            const int64_t wc = wsum((int64_t)c);
            if (best_bin > wc && wc >= mc) {
                const bool present = mine && peaks[mi(a)] >= 0;
                wsync();
                if (mine && !present) peaks[mi(a)] = (int32_t)mi(position);
                if (wany(present)) extended = false;
            } else {
                extended = false;
            }
            adjacent += dir * 10;
            wsync();
        }
    }

    // one side of find_ends: sorted positions pos_at(i), i < k, walked in `order` (+1 ascending
    // starts, -1 descending ends)
    __device__ void ends_side(int32_t *pk, const int32_t *cnt, const uint64_t *sorted, int32_t k, bool starts) {
        const int64_t up = P->up, down = P->down, mc = P->min_count;
        int64_t prev = INT64_MIN;
        for (int32_t ii = 0; ii < k; ++ii) {
            const int32_t i = starts ? ii : k - 1 - ii;
            const int64_t position = (int64_t)sorted[i] - kPosBias;
            if (position == prev) continue;  // same answer as the previous visit
            prev = position;
            const int64_t probe = starts ? position - up : position + up - 1;
            if (!in_map(probe)) {
                fail(kRange);
                return;
            }
            if (pk[mi(probe)] >= 0) continue;
            int64_t wc = 0;
            {
                const int64_t q = starts ? position + ln() : position - ln();
                int32_t c = 0;
                if (ln() < 10 && in_map(q)) c = cnt[mi(q)];
                wc = wsum((int64_t)c);
            }
            if (wc < mc) continue;
            const int64_t s_lo = starts ? -up : -down, s_hi = starts ? down : up;
            if (s_lo >= s_hi) {
                fail(kValueError);
                return;
            }
            if (!in_map(position + s_lo) || !in_map(position + s_hi)) {
                fail(kRange);
                return;
            }
            for (int64_t s = s_lo + ln(); s < s_hi; s += 64) pk[mi(position + s)] = (int32_t)mi(position);
            const int64_t ob_min = position + s_lo, ob_max = position + s_hi - 1;
            if (ob_min >= ob_max) {
                fail(kValueError);
                return;
            }
            int64_t bb = INT64_MIN;
            for (int64_t x = ob_min + ln(); x < ob_max; x += 64) {
                int64_t b = 0;
                for (int q = 0; q < 10; ++q)
                    if (in_map(x + q)) b += cnt[mi(x + q)];
                bb = b > bb ? b : bb;
            }
            const int64_t best_bin = wmax(bb);
            wsync();
            extend(pk, cnt, position, position + s_lo, -1, best_bin);
            if (status != kOk) return;
            extend(pk, cnt, position, position + s_hi - 1, +1, best_bin);
            if (status != kOk) return;
        }
    }

    // --- define_start_end_sites (SDC:797-868) + the subsample draw (SDC:884-888) -----------------
    __device__ void start_end_sites() {
        n_iso = n_mem = n_sub = 0;
        for (int t = 0; t < n_ids; ++t) {
            const int32_t id = B.idsort[t];
            const int lo = B.id_lo[id], m = B.id_hi[id] - lo;
            const int32_t k = m < 10000 ? m : 10000;
            int32_t *perm = perm_buf(m);
            permute(m, perm);
            const int64_t pk = pow2ge(k);
            int64_t tlo = INT64_MAX, thi = INT64_MIN;
            for (int64_t i = ln(); i < pk; i += 64) {
                uint64_t s = ~0ull, e = ~0ull;
                if (i < k) {
                    const Rec &R = A.recs[B.msort[lo + perm[i]]];
                    s = (uint64_t)(R.tstart + kPosBias);
                    e = (uint64_t)(R.tend + kPosBias);
                    tlo = R.tstart < tlo ? R.tstart : tlo;
                    tlo = R.tend < tlo ? R.tend : tlo;
                    thi = R.tstart > thi ? R.tstart : thi;
                    thi = R.tend > thi ? R.tend : thi;
                }
                B.ss[i] = s;
                B.isort[i] = e;
            }
            tlo = wmin(tlo);
            thi = wmax(thi);
            if (k > 0 && (!in_map(tlo) || !in_map(thi))) {
                fail(kRange);
                return;
            }
            for (int i = ln(); i < k; i += 64) {
                atomicAdd(&B.sc[mi((int64_t)B.ss[i] - kPosBias)], 1);
                atomicAdd(&B.ec[mi((int64_t)B.isort[i] - kPosBias)], 1);
            }
            wsync();
            sort_u64(B.ss, pk, tile);
            sort_u64(B.isort, pk, tile);
            ends_side(B.sp, B.sc, B.ss, k, true);
            if (status != kOk) return;
            ends_side(B.ep, B.ec, B.isort, k, false);
            if (status != kOk) return;
            wsync();
            // isoforms: (start window, end window) pairs in Pos order, first seen first
            for (int i = ln(); i < m; i += 64) {
                const Rec &R = A.recs[B.msort[lo + i]];
                const int32_t a = in_map(R.tstart) ? B.sp[mi(R.tstart)] : -1;
                const int32_t b = in_map(R.tend) ? B.ep[mi(R.tend)] : -1;
                B.pa[i] = a;
                B.pb[i] = b;
                B.asg[i] = (a >= 0 && b >= 0) ? 0 : 1;
            }
            wsync();
            while (true) {
                int32_t f = INT32_MAX;
                for (int i = ln(); i < m; i += 64)
                    if (!B.asg[i] && i < f) f = i;
                f = wmin(f);
                if (f == INT32_MAX) break;
                const int32_t a0 = B.pa[f], b0 = B.pb[f];
                int32_t cnt = 0;
                for (int i0 = f; i0 < m; i0 += 64) {
                    const int i = i0 + ln();
                    const bool mt_ = i < m && !B.asg[i] && B.pa[i] == a0 && B.pb[i] == b0;
                    const int32_t inc = wincl(mt_ ? 1 : 0);
                    if (mt_) {
                        O.mem[n_mem + cnt + inc - 1] = B.msort[lo + i];
                        B.asg[i] = 1;
                    }
                    cnt += __shfl(inc, 63);
                }
                if (ln() == 0) O.iso_nmem[n_iso] = cnt;
                ++n_iso;
                n_mem += cnt;
                wsync();
            }
            // clear the maps this identity touched
            const int64_t c_lo0 = tlo - P->up - P->down - 32, c_hi0 = thi + P->up + P->down + 32;
            const int64_t c_lo = c_lo0 > L.map_lo ? c_lo0 : L.map_lo;
            const int64_t c_hi = c_hi0 < L.map_lo + L.map_n - 1 ? c_hi0 : L.map_lo + L.map_n - 1;
            for (int64_t p = c_lo + ln(); p <= c_hi; p += 64) {
                B.sc[mi(p)] = 0;
                B.ec[mi(p)] = 0;
                B.sp[mi(p)] = -1;
                B.ep[mi(p)] = -1;
            }
            wsync();
        }
        // determine_consensus subsample per isoform, IsoDict order
        int32_t moff = 0;
        for (int iso = 0; iso < n_iso; ++iso) {
            const int32_t m = O.iso_nmem[iso];
            const int32_t k = m < P->sub_k ? m : P->sub_k;
            int32_t *perm = perm_buf(m);
            permute(m, perm);
            for (int i = ln(); i < k; i += 64) O.sub[n_sub + i] = O.mem[moff + perm[i]];
            if (ln() == 0) O.iso_nsub[iso] = k;
            n_sub += k;
            moff += m;
            wsync();
        }
    }

    __device__ void run(const Args &G) {
        // per-record text offsets for the host (names for reads2isoforms, sequences for the POA)
        for (int r = ln(); r < n; r += 64) {
            const Rec &R = A.recs[r];
            int64_t *o = G.rec_text + 4 * (L.rec_base + r);
            o[0] = L.text_off + R.name_off;
            o[1] = R.name_len;
            o[2] = L.text_off + R.seq_off;
            o[3] = R.seq_len;
        }
        for (int64_t p = ln(); p < L.map_n; p += 64) {
            B.areas[0][p] = 0;
            if (p % 10 == 0) B.hcb[p / 10] = 0;
            B.areas[1][p] = 0;
            B.splice[p] = -1;
            for (int v = 0; v < W; ++v) B.sc[p * W + v] = 0;
            B.ec[p] = 0;
            B.sp[p] = -1;
            B.ep[p] = -1;
        }
        for (int i = ln(); i < n_ann_of(L); i += 64) B.ann[i] = G.ann_pos[L.ann_off[0] + i];
        wsync();
#ifdef MANDO_CL_PHASES  // dev build: cycles per K2 phase of each locus
        uint64_t ph[8];
#define MANDO_PH(i) ph[i] = clock64()
#else
#define MANDO_PH(i)
#endif
        MANDO_PH(0);
        collect();
        if (status != kOk) return;
        MANDO_PH(1);
        genome_bins(0);
        if (status != kOk) return;
        genome_bins(1);
        if (status != kOk) return;
        MANDO_PH(2);
        find_peaks(0);
        if (status != kOk) return;
        find_peaks(1);
        if (status != kOk) return;
        MANDO_PH(3);
        splice_dict();
        sort_reads();
        MANDO_PH(4);
        identities();
        MANDO_PH(5);
        start_end_sites();
        MANDO_PH(6);
#ifdef MANDO_CL_PHASES
        if (ln() == 0)
            printf("[K2 phases] n %d: collect %.2f bins %.2f peaks %.2f dict+sort %.2f identities %.2f ends %.2f Mcyc\n", n,
                   (ph[1] - ph[0]) * 1e-6, (ph[2] - ph[1]) * 1e-6, (ph[3] - ph[2]) * 1e-6, (ph[4] - ph[3]) * 1e-6,
                   (ph[5] - ph[4]) * 1e-6, (ph[6] - ph[5]) * 1e-6);
        if (ln() == 0)
            printf("[K2 peaks] n %d: candidates %d characterized %d | cov %.2f perm %.2f cs %.2f Mcyc | collect: cs_of "
                   "%.2f bins %.2f sides %.2f\n", n, pc_cand, pc_char, pc_cov * 1e-6, pc_perm * 1e-6, pc_cs * 1e-6,
                   pc_csof * 1e-6, pc_bins * 1e-6, pc_side * 1e-6);
        if (ln() == 0)
            printf("[K2 perm] n %d: blocks %d accept rounds %d swap rounds %d | accept %.2f swap %.2f Mcyc\n", n,
                   mt.pq_blocks, mt.pq_arounds, mt.pq_srounds, mt.pq_acc * 1e-6, mt.pq_swap * 1e-6);
        if (ln() == 0)
            printf("[K2 sides] n %d: H %d %d | sort %.2f keys %.2f cand %.2f Mcyc\n", n, B.s[0].H, B.s[1].H,
                   pc_sd_sort * 1e-6, pc_sd_keys * 1e-6, pc_sd_cand * 1e-6);
#endif
#undef MANDO_PH
    }
};

// K2 runs beside the POA grids of the chunk before (config 4): at most 128 VGPRs (a POA wave's share of
// a SIMD) and, one-wave, 9 KB of LDS (a POA workgroup's 10 KB), so a freed POA slot fits a K2
// workgroup: config 4 12.60 -> 12.23 s per step with the orientation kernel's cap
// (profiles/r05l_ab_side_kernels_lite.txt; K2 alone 12.69 -> 12.50 s, r05n_ab_k2_lite.txt)
template <int NW>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(4))) void cluster_locus(Args G) {
    __shared__ uint32_t mtk[624];
    constexpr int kPerm = NW > 1 ? kLdsPermBig : kLdsPerm;
    __shared__ int32_t lperm[kPerm];
    __shared__ MwX mwx;
    const int li = G.order[blockIdx.x];
    Stats *st = G.stats + li;
    LocusRun R;
    R.S = *st;
    if (R.S.status != kOk) return;  // (every wave of the workgroup)
    R.W = NW;
    R.X = &mwx;
    R.xcov = 0;
    R.L = G.loci[li];
    R.T = G.text + R.L.text_off;
    R.P = G.prm;
    R.A = a_layout(G.scratch_a + R.L.a_off, R.L);
    carve_b(G.scratch_b + R.L.b_off, R.S, R.L, R.P->w, R.B);
    carve_o(G.out + R.L.o_off, R.S, R.L, R.O);
    R.n = R.S.n_rec;
    R.status = kOk;
    R.n_peaks = 0;
    R.n_iso = R.n_mem = R.n_sub = 0;
    R.n_ids = R.n_members = 0;
    R.mt.key = mtk;
    R.mt.pos = 624;
    R.lperm = lperm;
    R.lperm_cap = kPerm;
    R.tile = G.sort_tile;
    if (NW > 1 && wv() > 0) {
        R.helper();
        return;
    }
    for (int i = ln(); i < 624; i += 64) mtk[i] = R.P->mt_init[i];
    wsync();
    R.run(G);
    wsync();
    if (NW > 1) {  // the helpers leave their loop
        if (ln() == 0) mwx.op = kOpExit;
        gsync();
    }
    if (ln() == 0) {
        st->status = R.status;
        st->n_peaks = R.n_peaks;
        st->n_iso = R.n_iso;
        st->n_mem = R.n_mem;
        st->n_sub = R.n_sub;
    }
}

}  // namespace

// ---------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------
// K1 over the loci a.order[0, n_blocks): the first n_big (files of kK1MwBytes or more) on several waves each
hipError_t launch_parse(const Args &a, int n_blocks, int n_big, int n_work, hipStream_t s) {
    if (n_blocks <= 0) return hipSuccess;
    if (n_big > 0) hipLaunchKernelGGL(cluster_parse<kMwWaves>, dim3(n_big), dim3(64 * kMwWaves), 0, s, a);
    if (n_blocks > n_big) {
        Args b = a;
        b.order = a.order + n_big;
        hipLaunchKernelGGL(cluster_parse<1>, dim3(n_blocks - n_big), dim3(64), 0, s, b);
    }
    hipLaunchKernelGGL(cluster_cs_count, dim3(n_work), dim3(64), 0, s, a);
    hipLaunchKernelGGL(cluster_cs_scan, dim3(n_blocks), dim3(64), 0, s, a);
    hipLaunchKernelGGL(cluster_cs_runs, dim3(n_work), dim3(64), 0, s, a);
    return hipGetLastError();
}
// K2 over the loci a.order[0, n_big) on kMwWaves-wave workgroups, then a.order[n_big, n_blocks) on
// one wave each
hipError_t launch_locus(const Args &a, int n_blocks, int n_big, hipStream_t s) {
    if (n_big > 0) {
        Args b = a;
        b.sort_tile = kSortTile;
        hipLaunchKernelGGL(cluster_locus<kMwWaves>, dim3(n_big), dim3(64 * kMwWaves), kSortTile * 8, s, b);
    }
    if (n_blocks > n_big) {
        Args b = a;
        b.order = a.order + n_big;
        hipLaunchKernelGGL(cluster_locus<1>, dim3(n_blocks - n_big), dim3(64), b.sort_tile * 8, s, b);
    }
    return hipGetLastError();
}
int64_t b_bytes(const Stats &S, const Locus &L, int w) {
    BPtr B;
    carve_b(nullptr, S, L, w, B);
    return B.total;
}
int64_t o_bytes(const Stats &S, const Locus &L) {
    OPtr O;
    carve_o(nullptr, S, L, O);
    return O.total;
}
// host view of a locus' output region (offsets relative to the region)
void o_offsets(const Stats &S, const Locus &L, int64_t *peaks, int64_t *nmem, int64_t *mem, int64_t *nsub,
               int64_t *sub) {
    OPtr O;
    uint8_t *z = reinterpret_cast<uint8_t *>(uintptr_t(1) << 20);  // any non-null base: offsets only
    carve_o(z, S, L, O);
    *peaks = (uint8_t *)O.peaks - z;
    *nmem = (uint8_t *)O.iso_nmem - z;
    *mem = (uint8_t *)O.mem - z;
    *nsub = (uint8_t *)O.iso_nsub - z;
    *sub = (uint8_t *)O.sub - z;
}


namespace {

// Device buffers are hipMalloc'd and kept per context for reuse (grown, never shrunk).  Never the
// stream-ordered pool (hipMallocAsync / hipFreeAsync): on MI355X / ROCm 7.2 a pool buffer that is freed
// and handed out again shows a kernel the buffer's OLD bytes after a completed host-to-device copy of
// new ones (tools/stale_probe.hip, profiles/r03b_stale_probe.txt: 7-14 of 15 refills stale, 128 MB of
// 512 MB at a time, even with the copy synchronised before the kernel and the device synchronised
// before the free; never with a reused hipMalloc buffer).  That is what round 2 saw as "stale bytes"
// on the recycled text buffer.  A hipFree per call would also wait for the whole device.
std::mutex g_buf_mu;
std::map<std::pair<const mando_ctx *, int>, std::pair<void *, size_t>> g_bufs;
// pinned host buffers per context (the K2 output region comes back through one, reused: a fresh
// pageable vector of that size -- ~25 KB per locus, 0.35 GB per config-3 chunk -- was zero-filled and
// page-faulted on every call, on the path between the clustering kernels and the orientation launch)
std::map<std::pair<const mando_ctx *, int>, std::pair<void *, size_t>> g_pinned;
hipError_t pinned_host(const mando_ctx *ctx, int id, size_t n, uint8_t *&p) {
    std::lock_guard<std::mutex> g(g_buf_mu);
    auto &e = g_pinned[{ctx, id}];
    if (!e.first || e.second < n) {
        if (e.first) (void)hipHostFree(e.first);
        e = {nullptr, 0};
        const size_t cap = n + n / 4;
        void *q = nullptr;
        const hipError_t r = hipHostMalloc(&q, cap, hipHostMallocDefault);
        if (r != hipSuccess) return r;
        e = {q, cap};
    }
    p = static_cast<uint8_t *>(e.first);
    return hipSuccess;
}

struct DevMem {
    const mando_ctx *ctx;
    int id;
    void *p = nullptr;
    DevMem(const mando_ctx *c, int i) : ctx(c), id(i) {}
    hipError_t alloc(size_t n) {
        n = std::max<size_t>(n, 256);
        std::lock_guard<std::mutex> g(g_buf_mu);
        auto &e = g_bufs[{ctx, id}];
        if (e.first && e.second >= n) {
            p = e.first;
            return hipSuccess;
        }
        if (e.first) (void)hipFree(e.first);
        e = {nullptr, 0};
        const size_t cap = n + n / 4;  // headroom: chunk sizes vary from call to call
        hipError_t r = hipMalloc(&p, cap);
        if (r != hipSuccess) {
            p = nullptr;
            return r;
        }
        e = {p, cap};
        return hipSuccess;
    }
    template <class T>
    T *as() const {
        return (T *)p;
    }
};

// the device copy of a result's locus text outlives the call: a small cache of whole buffers, each
// tagged with the device it lives on (a process driving two GPUs must never get the other's buffer)
struct TextBuf {
    void *p;
    size_t cap;
    int dev;
};
std::vector<TextBuf> g_text_free;

// cluster_gpu reuses per-context scratch (g_bufs) and the pinned K2 output buffer (g_pinned): calls on
// one context are serialised here; calls on different contexts run concurrently
std::mutex &ctx_mutex(const mando_ctx *ctx) {
    static std::mutex mu;
    static std::map<const mando_ctx *, std::unique_ptr<std::mutex>> m;
    std::lock_guard<std::mutex> g(mu);
    auto &e = m[ctx];
    if (!e) e = std::make_unique<std::mutex>();
    return *e;
}

#define CL_TRY(expr)                                                                             \
    do {                                                                                         \
        hipError_t _e = (expr);                                                                  \
        if (_e != hipSuccess)                                                                    \
            return mando::set_error(MANDO_E_HIP, std::string("cluster: ") + #expr + ": " +       \
                                                     hipGetErrorString(_e));                     \
    } while (0)

}  // namespace

// Runs both kernels over every locus of `in` (see cluster_gpu.h); fills `out`.
int cluster_gpu(mando_ctx *ctx, const ClusterIn &in, ClusterOut &out) {
    const int64_t nl = in.n_loci;
    out.status.assign((size_t)nl, kOk);
    out.n_rec.assign((size_t)nl, 0);
    out.rec_base.assign((size_t)nl + 1, 0);
    out.peaks.assign((size_t)nl, {});
    out.iso_nmem.assign((size_t)nl, {});
    out.mem.assign((size_t)nl, {});
    out.iso_nsub.assign((size_t)nl, {});
    out.sub.assign((size_t)nl, {});
    out.rec_text.clear();
    if (nl == 0) return MANDO_OK;
    std::lock_guard<std::mutex> ctx_guard(ctx_mutex(ctx));
    CL_TRY(hipSetDevice(mando::ctx_device(ctx)));
    hipStream_t s = cluster_stream(ctx);
    if (in.ready) CL_TRY(hipStreamWaitEvent(s, in.ready, 0));

    // parameters + the RNG state every locus starts from
    Params prm;
    memset(&prm, 0, sizeof prm);
    prm.cutoff = in.cutoff;
    prm.w = in.w;
    prm.min_count = in.min_count;
    prm.up = in.up;
    prm.down = in.down;
    prm.sub_k = in.sub_k;
    prm.n_junc = 0;
    for (const std::string &j : in.junctions) {
        if (prm.n_junc >= 16) break;
        prm.junc_len4[prm.n_junc] = j.size() == 4;
        for (size_t c = 0; c < 4 && c < j.size(); ++c) prm.junc[prm.n_junc][c] = j[c];
        ++prm.n_junc;
    }
    {
        mando::MT19937 mt(in.seed);
        for (int i = 0; i < 624; ++i) prm.mt_init[i] = mt.key[i];
    }
    // locus descriptors; loci whose file could not be read keep their I/O status
    std::vector<Locus> L((size_t)nl);
    std::string chroms;
    std::vector<int32_t> run_order;
    std::vector<int32_t> ann_off_all;
    std::vector<int64_t> ann;
    for (int64_t i = 0; i < nl; ++i) {
        Locus &x = L[(size_t)i];
        memset(&x, 0, sizeof x);
        x.text_off = in.foff[i];
        x.text_len = in.foff[i + 1] - in.foff[i];
        x.chrom_off = (int32_t)chroms.size();
        x.chrom_len = (int32_t)strlen(in.chroms[i]);
        chroms += in.chroms[i];
        x.ann_off[0] = (int32_t)ann.size();
        for (int k = 0; k < 4; ++k) {
            if (in.ann_pos && in.ann_off)
                for (int64_t q = in.ann_off[4 * i + k]; q < in.ann_off[4 * i + k + 1]; ++q) ann.push_back(in.ann_pos[q]);
            x.ann_off[k + 1] = (int32_t)ann.size();
        }
        if (in.fstatus[i] != kOk) {
            out.status[(size_t)i] = in.fstatus[i];
            continue;
        }
        if (x.text_len >= (int64_t(1) << 31) - 64) {
            out.status[(size_t)i] = kRange;
            continue;
        }
        x.line_cap = (int32_t)(x.text_len / 160 + 8);
        x.op_cap = (int32_t)(x.text_len / 32 + 64);
        x.blk_cap = (int32_t)(x.text_len / 96 + 64);
        run_order.push_back((int32_t)i);
    }
    std::stable_sort(run_order.begin(), run_order.end(),
                     [&](int32_t a, int32_t b) { return L[(size_t)a].text_len > L[(size_t)b].text_len; });
    const int nrun = (int)run_order.size();

    DevMem d_chroms(ctx, 0), d_ann(ctx, 1), d_loci(ctx, 2), d_order(ctx, 3), d_stats(ctx, 4), d_a(ctx, 5),
        d_b(ctx, 6), d_o(ctx, 7), d_rec(ctx, 8), d_prm(ctx, 9);
    CL_TRY(d_chroms.alloc(chroms.size() + 1));
    CL_TRY(hipMemcpyAsync(d_chroms.p, chroms.data(), chroms.size() + 1, hipMemcpyHostToDevice, s));
    CL_TRY(d_ann.alloc((ann.size() + 1) * 8));
    if (!ann.empty()) CL_TRY(hipMemcpyAsync(d_ann.p, ann.data(), ann.size() * 8, hipMemcpyHostToDevice, s));
    CL_TRY(d_order.alloc((size_t)(nrun + 1) * 4));
    if (nrun) CL_TRY(hipMemcpyAsync(d_order.p, run_order.data(), (size_t)nrun * 4, hipMemcpyHostToDevice, s));
    // cs waves: up to kCsMaxWaves per locus by text size, the largest loci first
    std::vector<int32_t> work;
    for (int32_t i : run_order) {
        const int64_t nm = std::min<int64_t>(kCsMaxWaves, std::max<int64_t>(1, (L[(size_t)i].text_len + kCsTextPerWave - 1) / kCsTextPerWave));
        for (int64_t m = 0; m < nm; ++m) {
            work.push_back(i);
            work.push_back((int32_t)(m | nm << 16));
        }
    }
    const int n_work = (int)(work.size() / 2);
    DevMem d_work(ctx, 10);
    CL_TRY(d_work.alloc(work.size() * 4 + 8));
    if (n_work) CL_TRY(hipMemcpyAsync(d_work.p, work.data(), work.size() * 4, hipMemcpyHostToDevice, s));
    CL_TRY(d_prm.alloc(sizeof(Params)));
    CL_TRY(hipMemcpyAsync(d_prm.p, &prm, sizeof(Params), hipMemcpyHostToDevice, s));
    CL_TRY(d_loci.alloc((size_t)nl * sizeof(Locus)));
    CL_TRY(d_stats.alloc((size_t)nl * sizeof(Stats)));
    std::vector<Stats> st((size_t)nl);

    Args G;
    G.text = static_cast<const uint8_t *>(in.d_text);
    G.chroms = d_chroms.as<uint8_t>();
    G.ann_pos = d_ann.as<int64_t>();
    G.loci = d_loci.as<Locus>();
    G.order = d_order.as<int32_t>();
    G.work = d_work.as<int32_t>();
    G.stats = d_stats.as<Stats>();
    G.prm = d_prm.as<Params>();

    // run_order is by text size, descending: the large files lead
    int k1_big = 0;
    while (k1_big < nrun && L[(size_t)run_order[(size_t)k1_big]].text_len >= kK1MwBytes) ++k1_big;
    // K1, re-run with the reported sizes while a locus outgrows its scratch
    const bool timing = getenv("MANDO_CL_TIME") != nullptr;
    const auto tk0 = std::chrono::steady_clock::now();
    int k1_runs = 0;
    int64_t a_last = 0;
    for (int attempt = 0; attempt < 3; ++attempt) {
        ++k1_runs;
        int64_t a_tot = 0;
        for (int32_t i : run_order) {
            Locus &x = L[(size_t)i];
            x.a_off = a_tot;
            a_tot += al256(scratch_a_bytes(x.line_cap, x.op_cap, x.blk_cap));
        }
        CL_TRY(d_a.alloc((size_t)a_tot + 256));
        a_last = a_tot;
        CL_TRY(hipMemcpyAsync(d_loci.p, L.data(), (size_t)nl * sizeof(Locus), hipMemcpyHostToDevice, s));
        G.scratch_a = d_a.as<uint8_t>();
        CL_TRY(launch_parse(G, nrun, k1_big, n_work, s));
        CL_TRY(hipMemcpyAsync(st.data(), d_stats.p, (size_t)nl * sizeof(Stats), hipMemcpyDeviceToHost, s));
        CL_TRY(hipStreamSynchronize(s));
        bool again = false;
        for (int32_t i : run_order) {
            const Stats &x = st[(size_t)i];
            if (x.status != kCapacity) continue;
            Locus &y = L[(size_t)i];
            y.line_cap = std::max<int32_t>(y.line_cap, x.n_rec + 8);
            y.op_cap = std::max<int32_t>(y.op_cap, x.n_ops + 64);
            y.blk_cap = std::max<int32_t>(y.blk_cap, x.n_blk + 64);
            // the kernel stops at the first exceeded capacity; later ones are bounded by the text
            if (x.n_rec > 0 && x.n_blk == 0) y.blk_cap = std::max<int64_t>(y.blk_cap, y.text_len / 2 + 64);
            if (x.n_rec > 0 && x.n_ops == 0) y.op_cap = std::max<int64_t>(y.op_cap, y.text_len / 2 + 64);
            again = true;
        }
        if (!again) break;
    }

    const auto tk1 = std::chrono::steady_clock::now();
    if (getenv("MANDO_CL_DEBUG"))
        for (int64_t i = 0; i < nl; ++i) {
            const Stats &x = st[(size_t)i];
            fprintf(stderr, "[K1] %lld st %d rec %d ops %d blk %d hl %d hr %d span %lld %lld cov %lld id %lld\n",
                    (long long)i, x.status, x.n_rec, x.n_ops, x.n_blk, x.n_hist_l, x.n_hist_r, (long long)x.span_lo,
                    (long long)x.span_hi, (long long)x.cov_cap, (long long)x.ident_cap);
        }
    // K2 sizes from K1's statistics: dense position maps over the locus span and its annotation
    const int64_t M = 4 * (int64_t)in.w + in.up + in.down + 256;
    int64_t b_tot = 0, o_tot = 0, recs = 0;
    std::vector<int32_t> k2_order;
    for (int64_t i = 0; i < nl; ++i) {
        out.rec_base[(size_t)i] = recs;
        if (out.status[(size_t)i] != kOk) continue;
        Stats &x = st[(size_t)i];
        if (x.status == kCapacity) x.status = kParse;  // still too big after the re-runs
        out.status[(size_t)i] = x.status;
        if (x.status != kOk) continue;
        out.n_rec[(size_t)i] = x.n_rec;
        recs += x.n_rec;
    }
    out.rec_base[(size_t)nl] = recs;
    for (int32_t i : run_order) {
        if (out.status[(size_t)i] != kOk) continue;
        Locus &x = L[(size_t)i];
        const Stats &y = st[(size_t)i];
        int64_t lo = INT64_MAX, hi = INT64_MIN;
        if (y.span_lo <= y.span_hi) {
            lo = y.span_lo;
            hi = y.span_hi;
        }
        for (int32_t q = x.ann_off[0]; q < x.ann_off[4]; ++q) {
            lo = std::min(lo, ann[(size_t)q]);
            hi = std::max(hi, ann[(size_t)q]);
        }
        if (lo > hi) lo = hi = 0;
        x.map_lo = lo - M;
        x.map_n = hi - lo + 2 * M + 1;
        if (x.map_n > (int64_t(1) << 30)) {
            out.status[(size_t)i] = kRange;
            continue;
        }
        x.rec_base = out.rec_base[(size_t)i];
        x.b_off = b_tot;
        x.b_len = b_bytes(y, x, in.w);
        b_tot += al256(x.b_len);
        x.o_off = o_tot;
        o_tot += al256(o_bytes(y, x));
        k2_order.push_back(i);
    }
    if (!k2_order.empty()) {
        CL_TRY(d_b.alloc((size_t)b_tot + 256));
        CL_TRY(d_o.alloc((size_t)o_tot + 256));
        CL_TRY(d_rec.alloc((size_t)(recs + 1) * 32));
        if (getenv("MANDO_WS_LOG"))  // device bytes of one chunk's clustering (the D driver's HBM plan)
            fprintf(stderr, "[mando ws] cluster: loci %lld text %.3f GB scratch a %.3f b %.3f out %.3f rec %.3f GB\n",
                    (long long)nl, in.foff[nl] / 1e9, a_last / 1e9, b_tot / 1e9, o_tot / 1e9, (recs + 1) * 32 / 1e9);
        // loci not run by K2 must not be: mark them in the stats copy the kernel reads
        for (int64_t i = 0; i < nl; ++i)
            if (out.status[(size_t)i] != kOk && st[(size_t)i].status == kOk) st[(size_t)i].status = out.status[(size_t)i];
        CL_TRY(hipMemcpyAsync(d_stats.p, st.data(), (size_t)nl * sizeof(Stats), hipMemcpyHostToDevice, s));
        CL_TRY(hipMemcpyAsync(d_loci.p, L.data(), (size_t)nl * sizeof(Locus), hipMemcpyHostToDevice, s));
        // loci of kMwMinRecs records or more first: they take the several-wave kernel
        const int n_big = (int)(std::stable_partition(k2_order.begin(), k2_order.end(),
                                                      [&](int32_t i) { return st[(size_t)i].n_rec >= kMwMinRecs; }) -
                                k2_order.begin());
        CL_TRY(hipMemcpyAsync(d_order.p, k2_order.data(), k2_order.size() * 4, hipMemcpyHostToDevice, s));
        G.scratch_b = d_b.as<uint8_t>();
        G.out = d_o.as<uint8_t>();
        G.rec_text = d_rec.as<int64_t>();
        // the one-wave launch's sort tile: 4 KB of dynamic LDS (larger sorts and histograms go through
        // global memory; the large loci's launch keeps kSortTile)
        G.sort_tile = 512;
        CL_TRY(launch_locus(G, (int)k2_order.size(), n_big, s));
        uint8_t *ho = nullptr;
        CL_TRY(pinned_host(ctx, 0, (size_t)o_tot + 256, ho));
        out.rec_text.resize((size_t)recs * 4);
        CL_TRY(hipMemcpyAsync(st.data(), d_stats.p, (size_t)nl * sizeof(Stats), hipMemcpyDeviceToHost, s));
        CL_TRY(hipMemcpyAsync(ho, d_o.p, (size_t)o_tot, hipMemcpyDeviceToHost, s));
        if (recs) CL_TRY(hipMemcpyAsync(out.rec_text.data(), d_rec.p, (size_t)recs * 32, hipMemcpyDeviceToHost, s));
        CL_TRY(hipStreamSynchronize(s));
        if (timing)
            fprintf(stderr, "[cluster] K1 %.3f s (%d runs), K2 %.3f s (%zu loci)\n",
                    std::chrono::duration<double>(tk1 - tk0).count(), k1_runs,
                    std::chrono::duration<double>(std::chrono::steady_clock::now() - tk1).count(), k2_order.size());
        if (getenv("MANDO_CL_DEBUG"))
            for (int32_t i : k2_order) {
                const Stats &x = st[(size_t)i];
                fprintf(stderr, "[K2] %d st %d peaks %d iso %d mem %d sub %d\n", i, x.status, x.n_peaks, x.n_iso,
                        x.n_mem, x.n_sub);
            }
        for (int32_t i : k2_order) {
            const Stats &y = st[(size_t)i];
            out.status[(size_t)i] = y.status;
            if (y.status != kOk) continue;
            const Locus &x = L[(size_t)i];
            int64_t op, onm, om, ons, os;
            o_offsets(y, x, &op, &onm, &om, &ons, &os);
            const uint8_t *base = ho + x.o_off;
            out.peaks[(size_t)i].assign((const Peak *)(base + op), (const Peak *)(base + op) + y.n_peaks);
            out.iso_nmem[(size_t)i].assign((const int32_t *)(base + onm), (const int32_t *)(base + onm) + y.n_iso);
            out.mem[(size_t)i].assign((const int32_t *)(base + om), (const int32_t *)(base + om) + y.n_mem);
            out.iso_nsub[(size_t)i].assign((const int32_t *)(base + ons), (const int32_t *)(base + ons) + y.n_iso);
            out.sub[(size_t)i].assign((const int32_t *)(base + os), (const int32_t *)(base + os) + y.n_sub);
        }
    }
    return MANDO_OK;
}

// (a high-priority stream of its own was measured neutral: profiles/r05v_ab_cluster_priority.txt; so was
// a hardware queue of its own, r05w_ab_hw_queues.txt)
hipStream_t cluster_stream(mando_ctx *ctx) { return mando::ctx_stream(ctx); }

void *acquire_text(mando_ctx *ctx, size_t need, size_t &cap) {
    const int dev = mando::ctx_device(ctx);
    {
        std::lock_guard<std::mutex> g(g_buf_mu);
        size_t best = (size_t)-1;
        for (size_t i = 0; i < g_text_free.size(); ++i)
            if (g_text_free[i].dev == dev && g_text_free[i].cap >= need &&
                (best == (size_t)-1 || g_text_free[i].cap < g_text_free[best].cap))
                best = i;
        if (best != (size_t)-1) {
            const TextBuf e = g_text_free[best];
            g_text_free.erase(g_text_free.begin() + (ptrdiff_t)best);
            cap = e.cap;
            return e.p;
        }
    }
    constexpr size_t kStep = size_t(256) << 20;
    cap = (std::max<size_t>(need, 1) + kStep - 1) / kStep * kStep;
    void *p = nullptr;
    if (hipMalloc(&p, cap) != hipSuccess) return nullptr;
    return p;
}

void release_text(mando_ctx *ctx, void *d_text, size_t cap) {
    if (!d_text) return;
    std::lock_guard<std::mutex> g(g_buf_mu);
    g_text_free.push_back({d_text, cap, mando::ctx_device(ctx)});
    // four: two chunks in flight plus the previous call's two when their release comes late.  A
    // hipFree synchronises the device, so it is kept off the common path
    while (g_text_free.size() > 4) {
        auto it = std::min_element(g_text_free.begin(), g_text_free.end(),
                                   [](const TextBuf &a, const TextBuf &b) { return a.cap < b.cap; });
        (void)hipFree(it->p);
        g_text_free.erase(it);
    }
}

// Frees cached buffers of a device that a larger, earlier call left behind (mando_cache_trim).  The
// scratch of a context whose call is running is skipped (its mutex is held; that call needs it).
int64_t cache_trim(int dev, int64_t text_cap_max, int64_t scratch_max) {
    std::vector<void *> drop;
    std::lock_guard<std::mutex> g(g_buf_mu);
    if (text_cap_max >= 0) {
        for (size_t i = 0; i < g_text_free.size();) {
            if (g_text_free[i].dev == dev && g_text_free[i].cap > (size_t)text_cap_max) {
                drop.push_back(g_text_free[i].p);
                g_text_free.erase(g_text_free.begin() + (ptrdiff_t)i);
            } else {
                ++i;
            }
        }
    }
    size_t scratch = 0;
    for (auto &e : g_bufs)
        if (e.second.first && mando::ctx_device(e.first.first) == dev) scratch += e.second.second;
    if (scratch_max >= 0 && scratch > (size_t)scratch_max)
        for (auto &e : g_bufs) {
            if (!e.second.first || mando::ctx_device(e.first.first) != dev) continue;
            std::unique_lock<std::mutex> lk(ctx_mutex(e.first.first), std::try_to_lock);
            if (!lk.owns_lock()) continue;
            drop.push_back(e.second.first);
            e.second = {nullptr, 0};
        }
    for (void *p : drop) (void)hipFree(p);
    int64_t held = 0;
    for (const TextBuf &t : g_text_free)
        if (t.dev == dev) held += (int64_t)t.cap;
    for (auto &e : g_bufs)
        if (e.second.first && mando::ctx_device(e.first.first) == dev) held += (int64_t)e.second.second;
    return held;
}

}  // namespace cl
}  // namespace mando

extern "C" int mando_cache_trim(int32_t device_ordinal, int64_t text_cap_max, int64_t scratch_max,
                                int64_t *held_bytes) {
    if (device_ordinal < 0) return MANDO_E_ARG;
    if (hipSetDevice(device_ordinal) != hipSuccess) return MANDO_E_HIP;
    const int64_t h = mando::cl::cache_trim(device_ordinal, text_cap_max, scratch_max);
    if (held_bytes) *held_bytes = h;
    return MANDO_OK;
}
