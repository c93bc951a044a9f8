// sam_kernel.hip — SAM -> "Mando PSL" on the GPU: emtrey.py:31-152 (parseLine,
// `-m` mode) + :154-193 (unmapped records skipped, @SQ lengths), the same conversion sam.cpp restates on
// the host, byte for byte (tests/test_sam_gpu.py: the reference-run fixture tests/golden/sam_vectors.json
// and sam.cpp's output).
//
// The host reads the file, splits it into lines and takes the @SQ header (a few hundred lines at most);
// the records go to HBM once and every record is converted by one 64-lane wave, in two launches: the
// first computes each output line's length (and the record's status: the reference's exceptions), the
// host turns the lengths into offsets, the second writes the lines there.  Inside a record:
//   * the strip and the tab split are wave-parallel (64-byte chunks, ballots): column bounds in LDS;
//     the tag patterns emtrey tests with `in` on every column from the 10th ("NM:i:", "nn:i:", "ts:A:",
//     "cs:Z:") are matched in the same pass, one position per lane, into per-column flags;
//   * the CIGAR walk (counters, block lists) and the numeric fields are lane 0's, serial and short;
//   * the long fields (the cs string, the read, reverse-complemented with mappy's table on '-' records)
//     are copied by the whole wave;
//   * the accuracy is printed as Python's repr() prints a float: the shortest decimal that reads back as
//     the same double, found digit count by digit count with exact 128-bit integer comparisons against
//     the double's rounding interval (|x| in [1e-8, 1e9]; outside that the record reports
//     MANDO_E_UNSUPPORTED -- accuracy = matches / aligned bases is never there).
// Every byte-level rule (Python int() on stripped text, the zip that drops a trailing CIGAR number, the
// `third` field of a tag, the strand flip by ts:A:-) follows sam.cpp's restatement.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "internal.h"

namespace mando {
namespace sam {

constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;
constexpr int kMaxCols = 1024;

enum : int32_t { kOk = 0, kSkip = 1, kErrArg = 2, kErrUnsupported = 3 };
enum : int32_t { kFlagNM = 1, kFlagNN = 2, kFlagTS = 4, kFlagCS = 8 };

struct Args {
    const uint8_t *text;
    const int64_t *line_off;
    const int32_t *line_len;
    int64_t n;
    const uint8_t *chrom_text;  // the @SQ names, concatenated
    const int32_t *chrom_off;   // n_chrom + 1 offsets into chrom_text
    const int64_t *chrom_size;
    int32_t n_chrom;
    int32_t mando;
    int32_t *out_len;           // pass 1
    int32_t *status;            // pass 1
    const int64_t *out_off;     // pass 2
    uint8_t *out;               // pass 2
};

struct WaveLds {
    int32_t tabpos[kMaxCols];
    int32_t flags[kMaxCols];
};

__device__ __forceinline__ bool is_space(uint32_t c) { return c == ' ' || (c >= 9 && c <= 13); }
__device__ __forceinline__ uint64_t lanemask_lt(int lane) { return lane ? (~0ull >> (64 - lane)) : 0ull; }
__device__ __forceinline__ int rfl(int x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ int64_t rfl64(int64_t v) {
    return (int64_t)(((uint64_t)(uint32_t)rfl((int)(v >> 32)) << 32) | (uint64_t)(uint32_t)rfl((int)(uint32_t)v));
}

// mappy.revcomp's complement (revcomp.h): IUPAC letters in either case, every other byte kept
__device__ __forceinline__ uint8_t comp(uint8_t c) {
    const uint8_t u = c & 0xDF;  // upper case for letters
    uint8_t r;
    switch (u) {
        case 'A': r = 'T'; break;
        case 'C': r = 'G'; break;
        case 'G': r = 'C'; break;
        case 'T': r = 'A'; break;
        case 'U': r = 'A'; break;
        case 'R': r = 'Y'; break;
        case 'Y': r = 'R'; break;
        case 'K': r = 'M'; break;
        case 'M': r = 'K'; break;
        case 'B': r = 'V'; break;
        case 'V': r = 'B'; break;
        case 'D': r = 'H'; break;
        case 'H': r = 'D'; break;
        case 'S': case 'W': case 'N': r = u; break;
        default: return c;
    }
    return (c >= 'a' && c <= 'z') ? (uint8_t)(r | 0x20) : r;
}

// first position in [a, b) whose byte satisfies pred, or b (wave-parallel, uniform result)
template <class P>
__device__ __forceinline__ int64_t find_first(const uint8_t *t, int64_t a, int64_t b, int lane, P pred) {
    for (int64_t base = a; base < b; base += kWave) {
        const int64_t p = base + lane;
        const bool hit = p < b && pred((uint32_t)t[p]);
        const uint64_t m = __ballot(hit);
        if (m) return base + __ffsll((long long)m) - 1;
    }
    return b;
}

// last position in [a, b) whose byte satisfies pred, or a - 1
template <class P>
__device__ __forceinline__ int64_t find_last(const uint8_t *t, int64_t a, int64_t b, int lane, P pred) {
    for (int64_t top = b; top > a; top -= kWave) {
        const int64_t p = top - 1 - lane;
        const bool hit = p >= a && pred((uint32_t)t[p]);
        const uint64_t m = __ballot(hit);
        if (m) return top - 1 - (__ffsll((long long)m) - 1);  // the lowest lane is the highest position
    }
    return a - 1;
}

// Python int() on the text [a, b) as sam.cpp's to_i64: whitespace stripped, optional sign, decimal digits
// (lane 0, short fields)
__device__ bool to_i64(const uint8_t *t, int64_t a, int64_t b, int64_t &v) {
    while (a < b && is_space(t[a])) ++a;
    while (b > a && is_space(t[b - 1])) --b;
    if (a >= b) return false;
    bool neg = false;
    if (t[a] == '-' || t[a] == '+') {
        neg = t[a] == '-';
        ++a;
    }
    if (a == b) return false;
    int64_t x = 0;
    for (; a < b; ++a) {
        const uint32_t c = t[a];
        if (c < '0' || c > '9') return false;
        x = x * 10 + (int64_t)(c - '0');
    }
    v = neg ? -x : x;
    return true;
}

// ---- output: lane 0 appends short pieces, the wave copies long ones --------------------------------
struct Out {
    uint8_t *p;  // null: count only
    int64_t n;
};

__device__ __forceinline__ void put(Out &o, uint8_t c) {
    if (o.p) o.p[o.n] = c;
    ++o.n;
}

__device__ void put_i64(Out &o, int64_t v) {
    char buf[24];
    int k = 0;
    const bool neg = v < 0;
    uint64_t u = neg ? (uint64_t)0 - (uint64_t)v : (uint64_t)v;
    do {
        buf[k++] = (char)('0' + u % 10);
        u /= 10;
    } while (u);
    if (neg) put(o, '-');
    while (k) put(o, (uint8_t)buf[--k]);
}

__device__ void put_span(Out &o, const uint8_t *t, int64_t a, int64_t b) {
    for (int64_t x = a; x < b; ++x) put(o, t[x]);
}

// ---- Python repr(float) -----------------------------------------------------------------------------
typedef unsigned __int128 u128;

__device__ __forceinline__ u128 pow5(int k) {
    u128 r = 1;
    for (int i = 0; i < k; ++i) r *= 5;
    return r;
}
__device__ __forceinline__ u128 pow10(int k) {
    u128 r = 1;
    for (int i = 0; i < k; ++i) r *= 10;
    return r;
}

// Does the decimal D * 10^k read back as m * 2^e (m in [2^52, 2^53), e < 0)?  Exact: the distance to x
// against half the gap to the neighbour on that side (a quarter below the binade's first value), the
// interval closed when m is even (round-half-even).  All terms scaled by 2^(2 - e) * 5^max(-k, 0).
__device__ bool round_trips(u128 D, int k, uint64_t m, int e) {
    u128 lhs, rhs, thr;
    if (k < 0) {
        lhs = (u128)m * pow5(-k) * 8;                 // x
        const int sh = 3 - e + k;                     // D 10^k in the same units: D 2^(3-e+k)
        if (sh < 0 || sh > 120) return false;
        rhs = D << sh;
        thr = pow5(-k) * 4;                            // 2^(e-1) half gap
    } else {
        lhs = (u128)m * 8;
        const int sh = k + 3 - e;                      // D 5^k 2^(k+3-e)
        if (sh > 100) return false;
        rhs = (D * pow5(k)) << sh;
        thr = 4;
    }
    const bool above = rhs >= lhs;
    const u128 dist = above ? rhs - lhs : lhs - rhs;
    const bool low_edge = m == (1ull << 52);
    const u128 lim = (!above && low_edge) ? thr / 2 : thr;
    return (m & 1) ? dist < lim : dist <= lim;
}

// the n-digit decimal nearest to x = m 2^e with last-digit exponent k (round half even)
__device__ u128 nearest(uint64_t m, int e, int k) {
    if (k < 0) {
        const u128 num = (u128)m * pow5(-k);          // x 10^-k = num 2^(e-k)
        const int s = k - e;                          // right shift
        if (s <= 0) return num << (-s);
        const u128 q = num >> s, r = num - (q << s), half = (u128)1 << (s - 1);
        return (r > half || (r == half && (q & 1))) ? q + 1 : q;
    }
    const u128 den = pow5(k) << (k - e);              // x / 10^k = m / (5^k 2^(k-e))
    const u128 q = (u128)m / den, r = (u128)m - q * den;
    return (2 * r > den || (2 * r == den && (q & 1))) ? q + 1 : q;
}

// 10^E <= m 2^e exactly (E in [-30, 30])
__device__ bool ge_pow10(uint64_t m, int e, int E) {
    if (E < 0) {  // m 5^-E 2^(e-E) >= 1
        const u128 a = (u128)m * pow5(-E);
        const int s = E - e;  // a >= 2^s
        return s <= 0 || (s < 127 && a >= ((u128)1 << s));
    }
    const int s = E - e;      // m >= 5^E 2^(E-e)
    if (s >= 100) return false;
    return (u128)m >= (pow5(E) << s);
}

// repr(x) appended to o; false when |x| is outside [1e-8, 1e9] (not handled on the device)
__device__ bool put_repr(Out &o, double x) {
    if (x == 0.0) {
        if (signbit(x)) put(o, '-');
        put(o, '0'); put(o, '.'); put(o, '0');
        return true;
    }
    const bool neg = x < 0;
    const double ax = neg ? -x : x;
    if (!(ax >= 1e-8 && ax <= 1e9)) return false;
    const uint64_t bits = (uint64_t)__double_as_longlong(ax);
    const uint64_t m = (bits & ((1ull << 52) - 1)) | (1ull << 52);
    const int e = (int)((bits >> 52) & 0x7ff) - 1075;
    // the exponent of the leading digit, exactly: 10^E <= |x| < 10^(E+1)
    int E = (int)floor(log10(ax));
    while (!ge_pow10(m, e, E)) --E;
    while (ge_pow10(m, e, E + 1)) ++E;
    u128 D = 0;
    int ex = E, n;
    for (n = 1; n <= 17; ++n) {
        const int k = E - n + 1;
        const u128 lo = pow10(n - 1), hi = pow10(n);
        const u128 c0 = nearest(m, e, k);  // the nearest n-digit decimal (10^n: x rounds up to 10^(E+1))
        if (c0 >= lo && c0 <= hi && round_trips(c0, k, m, e)) {
            D = c0;
            break;
        }
        // a neighbour: the rounding interval is asymmetric at the bottom of a binade
        if (c0 + 1 < hi && c0 + 1 >= lo && round_trips(c0 + 1, k, m, e)) {
            D = c0 + 1;
            break;
        }
        if (c0 > lo && c0 - 1 < hi && round_trips(c0 - 1, k, m, e)) {
            D = c0 - 1;
            break;
        }
    }
    if (n > 17) return false;
    if (D == pow10(n)) {  // 10^(E+1)
        D = 1;
        ex = E + 1;
    }
    // digits of D, trailing zeros dropped
    char dg[24];
    int nd = 0;
    for (u128 t = D; t; t /= 10) dg[nd++] = (char)('0' + (int)(t % 10));
    for (int a = 0, b = nd - 1; a < b; ++a, --b) {
        const char c = dg[a];
        dg[a] = dg[b];
        dg[b] = c;
    }
    while (nd > 1 && dg[nd - 1] == '0') --nd;
    if (neg) put(o, '-');
    if (ex < -4 || ex >= 16) {
        put(o, (uint8_t)dg[0]);
        if (nd > 1) {
            put(o, '.');
            for (int i = 1; i < nd; ++i) put(o, (uint8_t)dg[i]);
        }
        put(o, 'e');
        put(o, ex < 0 ? '-' : '+');
        const int ae = ex < 0 ? -ex : ex;
        if (ae < 10) put(o, '0');
        put_i64(o, ae);
    } else if (ex >= 0) {
        if (nd <= ex + 1) {
            for (int i = 0; i < nd; ++i) put(o, (uint8_t)dg[i]);
            for (int i = nd; i < ex + 1; ++i) put(o, '0');
            put(o, '.');
            put(o, '0');
        } else {
            for (int i = 0; i <= ex; ++i) put(o, (uint8_t)dg[i]);
            put(o, '.');
            for (int i = ex + 1; i < nd; ++i) put(o, (uint8_t)dg[i]);
        }
    } else {
        put(o, '0');
        put(o, '.');
        for (int i = 0; i < -ex - 1; ++i) put(o, '0');
        for (int i = 0; i < nd; ++i) put(o, (uint8_t)dg[i]);
    }
    return true;
}

// ---- one record -------------------------------------------------------------------------------------
__device__ __forceinline__ bool is_op(uint32_t c) {
    return c == 'M' || c == 'I' || c == 'D' || c == 'N' || c == 'S' || c == 'H' || c == 'P' || c == '=' || c == 'X';
}

struct Cigar {
    int64_t qstart, qend, M, I, nI, D, nD, N, S, H, EQ, X, nops, nblocks;
};

// walks the CIGAR text [a, b) as emtrey's re.split / zip does; list >= 0 emits list `list` (0 block sizes,
// 1 query starts, 2 target starts) into o.  False on a number Python's int() rejects.
__device__ bool walk_cigar(const uint8_t *t, int64_t a, int64_t b, int64_t tstart, int64_t nops, Cigar &c, int list,
                           Out *o) {
    int64_t i = a, op_i = 0, q = 0, tt = tstart;
    while (i < b) {
        int64_t j = i;
        while (j < b && !is_op(t[j])) ++j;
        if (j >= b) break;
        int64_t num;
        if (!to_i64(t, i, j, num)) return false;
        const uint32_t op = t[j];
        if (list < 0) {
            if (op == 'S' || op == 'H') {
                if (op_i == 0)
                    c.qstart = num;
                else if (op_i == nops - 1)
                    c.qend = num;
            }
        }
        if (op_i == 0) q = c.qstart;
        switch (op) {
            case 'M':
                if (list < 0) {
                    c.M += num;
                    c.nblocks += 1;
                } else {
                    put_i64(*o, list == 0 ? num : (list == 1 ? q : tt));
                    put(*o, ',');
                }
                q += num;
                tt += num;
                break;
            case 'I':
                if (list < 0) { c.I += num; c.nI += 1; }
                q += num;
                break;
            case 'D':
                if (list < 0) { c.D += num; c.nD += 1; }
                tt += num;
                break;
            case 'N':
                if (list < 0) c.N += num;
                tt += num;
                break;
            case 'S': if (list < 0) c.S += num; break;
            case 'H': if (list < 0) c.H += num; break;
            case '=': if (list < 0) c.EQ += num; break;
            case 'X': if (list < 0) c.X += num; break;
            default: break;
        }
        ++op_i;
        i = j + 1;
    }
    if (list < 0) c.nops = op_i;
    return true;
}

// emtrey's third(col): the text between the column's second and third ':' (or its end); empty when the
// column has fewer than two ':'
__device__ void third(const uint8_t *t, int64_t a, int64_t b, int lane, int64_t &s, int64_t &f) {
    auto colon = [](uint32_t c) { return c == ':'; };
    const int64_t p1 = find_first(t, a, b, lane, colon);
    const int64_t p2 = p1 < b ? find_first(t, p1 + 1, b, lane, colon) : b;
    if (p2 >= b) {
        s = f = 0;
        return;
    }
    const int64_t p3 = find_first(t, p2 + 1, b, lane, colon);
    s = p2 + 1;
    f = p3;
}

template <bool WRITE>
__device__ void record(const Args &A, WaveLds &L, int64_t r, int lane) {
    const uint8_t *t = A.text;
    const int64_t l0 = A.line_off[r], l1 = l0 + A.line_len[r];
    // strip
    const int64_t a = find_first(t, l0, l1, lane, [](uint32_t c) { return !is_space(c); });
    const int64_t b = find_last(t, a, l1, lane, [](uint32_t c) { return !is_space(c); }) + 1;
    // tab split + tag patterns, one position per lane
    for (int x = lane; x < kMaxCols; x += kWave) L.flags[x] = 0;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the LDS clears before the atomics below
    int ntab = 0;
    for (int64_t base = a; base < b; base += kWave) {
        const int64_t p = base + lane;
        const uint32_t c = p < b ? t[p] : 0;
        const bool tab = p < b && c == '\t';
        const uint64_t mt = __ballot(tab);
        const int col = ntab + __popcll(mt & lanemask_lt(lane));
        if (tab && col < kMaxCols) L.tabpos[col] = (int32_t)(p - a);
        if (p + 5 <= b && t[p + 2] == ':' && t[p + 4] == ':' && col >= 9 && col < kMaxCols) {
            const uint32_t c1 = t[p + 1], c3 = t[p + 3];
            int f = 0;
            if (c == 'N' && c1 == 'M' && c3 == 'i') f = kFlagNM;
            else if (c == 'n' && c1 == 'n' && c3 == 'i') f = kFlagNN;
            else if (c == 't' && c1 == 's' && c3 == 'A') f = kFlagTS;
            else if (c == 'c' && c1 == 's' && c3 == 'Z') f = kFlagCS;
            if (f) atomicOr(&L.flags[col], f);
        }
        ntab += __popcll(mt);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const int ncol = ntab + 1;
    int st = kOk;
    Out o{nullptr, 0};
    if (WRITE) o.p = A.out + A.out_off[r];
    if (ncol > kMaxCols) st = kErrUnsupported;
    auto cb = [&](int k) -> int64_t { return k == 0 ? a : a + L.tabpos[k - 1] + 1; };
    auto ce = [&](int k) -> int64_t { return k == ncol - 1 ? b : a + L.tabpos[k]; };
    if (st == kOk && ncol < 3) st = kErrArg;
    if (st == kOk && ce(2) - cb(2) == 1 && t[cb(2)] == '*') st = kSkip;
    // chromosome -> length (the last @SQ of that name), lanes over the table
    int64_t qsize = 0;
    if (st == kOk) {
        const int64_t c0 = cb(2), clen = ce(2) - c0;
        int hit = -1;
        for (int base = 0; base < A.n_chrom; base += kWave) {
            const int x = base + lane;
            bool eq = false;
            if (x < A.n_chrom && A.chrom_off[x + 1] - A.chrom_off[x] == clen) {
                eq = true;
                const uint8_t *nm = A.chrom_text + A.chrom_off[x];
                for (int64_t y = 0; y < clen && eq; ++y) eq = nm[y] == t[c0 + y];
            }
            const uint64_t m = __ballot(eq);
            if (m) hit = base + 63 - __clzll((long long)m);  // the highest lane: the last definition
        }
        if (hit < 0) st = kErrArg;
        else qsize = A.chrom_size[hit];
    }
    if (st == kOk && ncol < 11) st = kErrArg;
    // the tags' third fields (wave-parallel scans: the cs column is long)
    int64_t NM = 0, ambig = 0, cs_s = 0, cs_f = 0;
    int ts_flips = 0, have_cs = 0;
    if (st == kOk) {
        for (int k = 9; k < ncol && st == kOk; ++k) {
            const int f = L.flags[k];
            if (!f) continue;
            int64_t s, e2;
            third(t, cb(k), ce(k), lane, s, e2);
            if (f & kFlagNM) {
                int64_t v = 0;
                bool ok = false;
                if (lane == 0) ok = to_i64(t, s, e2, v);
                if (!rfl(ok)) st = kErrArg;
                NM = rfl64(v);
            }
            if ((f & kFlagNN) && st == kOk) {
                int64_t v = 0;
                bool ok = false;
                if (lane == 0) ok = to_i64(t, s, e2, v);
                if (!rfl(ok)) st = kErrArg;
                ambig = rfl64(v);
            }
            if (f & kFlagTS) {
                if (e2 - s == 1 && t[s] == '-') ts_flips ^= 1;
            }
            if (f & kFlagCS) {
                cs_s = s;
                cs_f = e2;
                have_cs = 1;
            }
        }
    }
    if (st == kOk && A.mando && !have_cs) st = kErrArg;  // NameError in the reference
    // lane 0: the CIGAR and the numeric fields; the wave: the long copies
    int64_t tstart = 0, flag = 0;
    Cigar c{};
    if (st == kOk) {
        int ok = 1;
        if (lane == 0) {
            ok = to_i64(t, cb(3), ce(3), tstart) && to_i64(t, cb(1), ce(1), flag);
            tstart -= 1;
            if (ok) {
                // ops counted first: qend is the S/H op of the last index
                Cigar c0{};
                ok = walk_cigar(t, cb(5), ce(5), tstart, -1, c0, -1, nullptr);
                c.nops = c0.nops;
                if (ok) ok = walk_cigar(t, cb(5), ce(5), tstart, c.nops, c, -1, nullptr);
            }
        }
        if (!rfl(ok)) st = kErrArg;
    }
    int64_t matches = 0, mismatch = 0, den = 0;
    if (st == kOk && lane == 0) {
        const int64_t ID = c.I + c.D;
        mismatch = NM - ID - ambig;
        if (mismatch < 0) mismatch = 0;
        matches = c.M - mismatch;
        den = matches + mismatch + ID + ambig;
    }
    if (st == kOk && rfl(den == 0)) st = kErrArg;  // ZeroDivisionError in the reference
    flag = rfl64(flag);
    const bool rev0 = (flag >> 4) & 1;                 // the read is reverse-complemented on '-'
    bool minus = rev0;
    if (ts_flips) minus = !minus;
    if (st == kOk) {
        int ok = 1;
        if (lane == 0) {
            const int64_t ID = c.I + c.D;
            const int64_t sLen = c.M + c.I + c.S + c.H + c.EQ + c.X;
            const int64_t tend = tstart + c.M + c.D + c.N + c.EQ + c.X;
            const int64_t end = c.qend == 0 ? sLen : sLen - c.qend;
            (void)ID;
            put_i64(o, matches); put(o, '\t');
            put_i64(o, mismatch); put(o, '\t');
            put(o, '0'); put(o, '\t');
            put_i64(o, c.N); put(o, '\t');
            put_i64(o, c.nI); put(o, '\t');
            put_i64(o, c.I); put(o, '\t');
            put_i64(o, c.nD); put(o, '\t');
            put_i64(o, c.D); put(o, '\t');
            put(o, minus ? '-' : '+'); put(o, '\t');
            put_span(o, t, cb(0), ce(0)); put(o, '\t');
            put_i64(o, sLen); put(o, '\t');
            put_i64(o, c.qstart); put(o, '\t');
            put_i64(o, end); put(o, '\t');
            put_span(o, t, cb(2), ce(2)); put(o, '\t');
            put_i64(o, qsize); put(o, '\t');
            put_i64(o, tstart); put(o, '\t');
            put_i64(o, tend); put(o, '\t');
            put_i64(o, c.nblocks); put(o, '\t');
            Cigar cc = c;
            walk_cigar(t, cb(5), ce(5), tstart, c.nops, cc, 0, &o);
            if (c.nblocks == 0) put(o, ',');
            put(o, '\t');
            walk_cigar(t, cb(5), ce(5), tstart, c.nops, cc, 1, &o);
            if (c.nblocks == 0) put(o, ',');
            put(o, '\t');
            walk_cigar(t, cb(5), ce(5), tstart, c.nops, cc, 2, &o);
            if (c.nblocks == 0) put(o, ',');
            if (A.mando) {
                put(o, '\t');
                ok = put_repr(o, (double)matches / (double)den);
                put(o, '\t');
            }
        }
        if (!rfl(ok)) st = kErrUnsupported;
    }
    int64_t n = rfl64(o.n);
    if (st == kOk && A.mando) {
        // cs (verbatim), tab, the read (reverse-complemented on a '-' record), by the wave
        const int64_t lcs = cs_f - cs_s;
        const int64_t s9 = cb(9), e9 = ce(9), lseq = e9 - s9;
        if (WRITE) {
            uint8_t *d = o.p + n;
            for (int64_t x = lane; x < lcs; x += kWave) d[x] = t[cs_s + x];
            if (lane == 0) d[lcs] = '\t';
            uint8_t *q = d + lcs + 1;
            if (rev0) {
                for (int64_t x = lane; x < lseq; x += kWave) q[x] = comp(t[e9 - 1 - x]);
            } else {
                for (int64_t x = lane; x < lseq; x += kWave) q[x] = t[s9 + x];
            }
        }
        n += lcs + 1 + lseq;
    }
    if (WRITE) {
        if (st == kOk && lane == 0) o.p[n] = '\n';
    } else if (lane == 0) {
        A.status[r] = st;
        A.out_len[r] = st == kOk ? (int32_t)(n + 1) : 0;
    }
}

template <bool WRITE>
__global__ __launch_bounds__(kWave * kWavesPerBlock) void sam_kernel(Args A) {
    __shared__ WaveLds lds[kWavesPerBlock];
    const int w = threadIdx.x / kWave, lane = threadIdx.x % kWave;
    const int64_t nw = (int64_t)gridDim.x * kWavesPerBlock;
    for (int64_t r = (int64_t)blockIdx.x * kWavesPerBlock + w; r < A.n; r += nw) {
        if (WRITE && A.out_len[r] == 0) continue;
        record<WRITE>(A, lds[w], r, lane);
    }
}

// ---- host -----------------------------------------------------------------------------------------
struct Dev {
    void *p = nullptr;
    ~Dev() {
        if (p) (void)hipFree(p);
    }
    int alloc(size_t n) {
        return hipMalloc(&p, n ? n : 1) == hipSuccess ? MANDO_OK : MANDO_E_NOMEM;
    }
};

bool read_file(const char *path, std::string &out) {
    FILE *fh = fopen(path, "rb");
    if (!fh) return false;
    fseek(fh, 0, SEEK_END);
    const long sz = ftell(fh);
    fseek(fh, 0, SEEK_SET);
    out.resize((size_t)(sz > 0 ? sz : 0));
    const size_t got = sz > 0 ? fread(&out[0], 1, (size_t)sz, fh) : 0;
    fclose(fh);
    return (long)got == sz;
}

bool host_space(char c) { return c == ' ' || (c >= 9 && c <= 13); }

}  // namespace sam
}  // namespace mando

#define SAM_TRY(x)                                                                                   \
    do {                                                                                             \
        const hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) return mando::set_error(MANDO_E_HIP, std::string("sam: ") + hipGetErrorString(e_)); \
    } while (0)

extern "C" int mando_sam_to_psl_device(mando_ctx *ctx, const char *sam_path, const char *psl_path, int32_t mando_mode,
                                       int64_t *n_records) {
    using namespace mando::sam;
    if (!ctx || !sam_path || !psl_path) return mando::set_error(MANDO_E_ARG, "mando_sam_to_psl_device: bad argument");
    std::string buf;
    if (!read_file(sam_path, buf)) return mando::set_error(MANDO_E_ARG, std::string("cannot read ") + sam_path);
    // lines: @SQ headers parsed here (emtrey.py:170-176), other header lines skipped, empty lines skipped
    std::vector<int64_t> off;
    std::vector<int32_t> len;
    std::string names;
    std::vector<int32_t> noff{0};
    std::vector<int64_t> nsize;
    size_t p = 0;
    while (p < buf.size()) {
        size_t e = buf.find('\n', p);
        if (e == std::string::npos) e = buf.size();
        const size_t n = e - p;
        if (n > 0) {
            if (buf[p] == '@') {
                if (n >= 3 && buf.compare(p, 3, "@SQ") == 0) {
                    // split(strip(line), '\t'): field 1 = SN:<name>, field 2 = LN:<len>
                    size_t a = p, b = e;
                    while (a < b && host_space(buf[a])) ++a;
                    while (b > a && host_space(buf[b - 1])) --b;
                    std::vector<std::pair<size_t, size_t>> f;
                    size_t s = a;
                    for (size_t x = a; x <= b; ++x)
                        if (x == b || buf[x] == '\t') {
                            f.push_back({s, x});
                            s = x + 1;
                        }
                    if (f.size() < 3) return mando::set_error(MANDO_E_ARG, "malformed @SQ line");
                    const size_t c1 = buf.find(':', f[1].first), c2 = buf.find(':', f[2].first);
                    if (c1 >= f[1].second || c2 >= f[2].second) return mando::set_error(MANDO_E_ARG, "malformed @SQ line");
                    int64_t v = 0;
                    size_t x = c2 + 1, y = f[2].second;
                    while (x < y && host_space(buf[x])) ++x;
                    while (y > x && host_space(buf[y - 1])) --y;
                    bool neg = false, ok = x < y;
                    if (ok && (buf[x] == '-' || buf[x] == '+')) {
                        neg = buf[x] == '-';
                        ++x;
                        ok = x < y;
                    }
                    for (; ok && x < y; ++x) {
                        if (buf[x] < '0' || buf[x] > '9') ok = false;
                        else v = v * 10 + (buf[x] - '0');
                    }
                    if (!ok) return mando::set_error(MANDO_E_ARG, "malformed @SQ length");
                    names.append(buf, c1 + 1, f[1].second - c1 - 1);
                    noff.push_back((int32_t)names.size());
                    nsize.push_back(neg ? -v : v);
                }
            } else {
                off.push_back((int64_t)p);
                len.push_back((int32_t)n);
            }
        }
        p = e + 1;
    }
    const int64_t nrec = (int64_t)off.size();
    if (n_records) *n_records = 0;
    const int dev = mando::ctx_device(ctx);
    hipStream_t s = mando::ctx_stream(ctx);
    SAM_TRY(hipSetDevice(dev));
    Dev d_text, d_off, d_len, d_names, d_noff, d_nsize, d_olen, d_st, d_oof, d_out;
    int rc;
    if ((rc = d_text.alloc(buf.size())) || (rc = d_off.alloc((size_t)nrec * 8)) || (rc = d_len.alloc((size_t)nrec * 4)) ||
        (rc = d_names.alloc(names.size())) || (rc = d_noff.alloc(noff.size() * 4)) ||
        (rc = d_nsize.alloc(nsize.size() * 8)) || (rc = d_olen.alloc((size_t)nrec * 4)) ||
        (rc = d_st.alloc((size_t)nrec * 4)) || (rc = d_oof.alloc((size_t)nrec * 8)))
        return mando::set_error(rc, "sam: device allocation failed");
    SAM_TRY(hipMemcpyAsync(d_text.p, buf.data(), buf.size(), hipMemcpyHostToDevice, s));
    if (nrec) {
        SAM_TRY(hipMemcpyAsync(d_off.p, off.data(), (size_t)nrec * 8, hipMemcpyHostToDevice, s));
        SAM_TRY(hipMemcpyAsync(d_len.p, len.data(), (size_t)nrec * 4, hipMemcpyHostToDevice, s));
    }
    if (!names.empty()) SAM_TRY(hipMemcpyAsync(d_names.p, names.data(), names.size(), hipMemcpyHostToDevice, s));
    SAM_TRY(hipMemcpyAsync(d_noff.p, noff.data(), noff.size() * 4, hipMemcpyHostToDevice, s));
    if (!nsize.empty()) SAM_TRY(hipMemcpyAsync(d_nsize.p, nsize.data(), nsize.size() * 8, hipMemcpyHostToDevice, s));
    Args A{};
    A.text = (const uint8_t *)d_text.p;
    A.line_off = (const int64_t *)d_off.p;
    A.line_len = (const int32_t *)d_len.p;
    A.n = nrec;
    A.chrom_text = (const uint8_t *)d_names.p;
    A.chrom_off = (const int32_t *)d_noff.p;
    A.chrom_size = (const int64_t *)d_nsize.p;
    A.n_chrom = (int32_t)nsize.size();
    A.mando = mando_mode != 0;
    A.out_len = (int32_t *)d_olen.p;
    A.status = (int32_t *)d_st.p;
    A.out_off = (const int64_t *)d_oof.p;
    const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((nrec + kWavesPerBlock - 1) / kWavesPerBlock, 256 * 16));
    std::vector<int32_t> olen((size_t)nrec), st((size_t)nrec);
    if (nrec) {
        hipLaunchKernelGGL(sam_kernel<false>, dim3(blocks), dim3(kWave * kWavesPerBlock), 0, s, A);
        SAM_TRY(hipGetLastError());
        SAM_TRY(hipMemcpyAsync(olen.data(), d_olen.p, (size_t)nrec * 4, hipMemcpyDeviceToHost, s));
        SAM_TRY(hipMemcpyAsync(st.data(), d_st.p, (size_t)nrec * 4, hipMemcpyDeviceToHost, s));
        SAM_TRY(hipStreamSynchronize(s));
    }
    std::vector<int64_t> oof((size_t)nrec);
    int64_t total = 0, written = 0;
    for (int64_t r = 0; r < nrec; ++r) {
        if (st[(size_t)r] == kErrArg)
            return mando::set_error(MANDO_E_ARG, "SAM record " + std::to_string(r) +
                                                     ": emtrey raises here (unknown chromosome, malformed field, no cs "
                                                     "tag with -m, or no aligned base)");
        if (st[(size_t)r] == kErrUnsupported)
            return mando::set_error(MANDO_E_UNSUPPORTED, "SAM record " + std::to_string(r) +
                                                             ": more than 1024 columns, or an accuracy outside [1e-8, 1e9]");
        oof[(size_t)r] = total;
        total += olen[(size_t)r];
        written += st[(size_t)r] == kOk;
    }
    std::string out((size_t)total, '\0');
    if (total > 0) {
        if ((rc = d_out.alloc((size_t)total))) return mando::set_error(rc, "sam: device allocation failed");
        SAM_TRY(hipMemcpyAsync(d_oof.p, oof.data(), (size_t)nrec * 8, hipMemcpyHostToDevice, s));
        A.out = (uint8_t *)d_out.p;
        hipLaunchKernelGGL(sam_kernel<true>, dim3(blocks), dim3(kWave * kWavesPerBlock), 0, s, A);
        SAM_TRY(hipGetLastError());
        SAM_TRY(hipMemcpyAsync(&out[0], d_out.p, (size_t)total, hipMemcpyDeviceToHost, s));
        SAM_TRY(hipStreamSynchronize(s));
    }
    FILE *o = fopen(psl_path, "wb");
    if (!o) return mando::set_error(MANDO_E_ARG, std::string("cannot write ") + psl_path);
    const size_t wr = total > 0 ? fwrite(out.data(), 1, out.size(), o) : 0;
    fclose(o);
    if ((int64_t)wr != total) return mando::set_error(MANDO_E_ARG, std::string("short write to ") + psl_path);
    if (n_records) *n_records = written;
    return MANDO_OK;
}
