// seed_kernel.hip — the -S window partition of abPOA's seeded mode on gfx950 (SURVEY.md Appendix C,
// taken by the reference when the median subsample length is >= 8000: SpliceDefineConsensus.py:915-919).
//
// One item = one read q of a seeded group paired with the previous non-empty read t of that group.
// Per item (one 64-lane wave, persistent over items) the kernel finds the kept partition anchors the
// POA kernel then aligns between (rules: oracle/poa_ref.c "-S", which this follows bit for bit):
//   1. (k, w) minimizers of t: k-mer hashes of every position (lane-parallel, reads staged per 64-
//      position step), window minima, marks (a position is kept when its hash is the minimum of a
//      window holding it), ballot compaction into LDS as sortable keys h << 26 | z << 25 | pos;
//   2. bitonic sort of t's keys in LDS;
//   3. q's minimizers (same steps, position order); per q minimizer a lane binary-searches t's keys for
//      its (hash, strand) run, and runs of 1..max_occ entries emit anchors (q ascending, t descending)
//      into HBM scratch at ballot/prefix-sum offsets;
//   4. longest strictly increasing subsequence of the anchors' t (patience sorting: the pile search is
//      a 64-ary wave-parallel lower bound over the LDS tails; predecessors in LDS);
//   5. trace back the chain, then keep anchors min_w apart (lane 0).
// Work is small next to the POA DP (a few thousand anchors per read pair), so the kernel is written for
// clarity; everything a step re-reads sits in LDS.  An item whose minimizers or anchors exceed the
// launch's LDS capacity reports -1 and the host re-runs it at twice the capacity.
#include "seed_kernel.h"

namespace mando {
namespace {

constexpr uint64_t kInf = ~0ull;

__device__ __forceinline__ int lane_id() { return (int)__lane_id(); }
__device__ __forceinline__ void wsync() { __syncthreads(); }
// this wave's global stores are visible to its own later loads
__device__ __forceinline__ void gfence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup"); }
__device__ __forceinline__ unsigned long long lanemask_lt(int lane) {
    return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

__device__ __forceinline__ uint64_t hash64(uint64_t key, uint64_t mask) {
    key = (~key + (key << 21)) & mask;
    key = key ^ key >> 24;
    key = ((key + (key << 3)) + (key << 8)) & mask;
    key = key ^ key >> 14;
    key = ((key + (key << 2)) + (key << 4)) & mask;
    key = key ^ key >> 28;
    key = (key + (key << 31)) & mask;
    return key;
}

extern __shared__ __attribute__((aligned(16))) uint64_t g_seed_dyn[];  // 2 * cap words

// Minimizers of s[0, L) (codes 0..4) as keys h << 26 | z << 25 | pos, position order, into out[];
// returns the count, or -1 past cap.  H / M: HBM scratch (L words each).
__device__ int sketch(const uint8_t *s, int L, int k, int w, uint64_t *out, int cap, uint64_t *H, uint64_t *M,
                      int lane) {
    if (L < k) return 0;
    const uint64_t mask = (1ull << (2 * k)) - 1;
    const int np = L - k + 1;
    const int nw = np <= w ? 1 : np - w + 1;
    const int ww = np <= w ? np : w;
    // (hash << 1 | z) of every k-mer; kInf when ambiguous or its own reverse complement
    for (int p = lane; p < np; p += 64) {
        uint64_t f = 0, r = 0;
        bool bad = false;
        for (int t = 0; t < k; ++t) {
            const int c = s[p + t];
            bad |= c > 3;
            f = (f << 2) | (uint64_t)(c & 3);
            r |= (uint64_t)(3 - (c & 3)) << (2 * t);
        }
        H[p] = (bad || f == r) ? kInf : ((hash64(f < r ? f : r, mask) << 1) | (f < r ? 0 : 1));
    }
    gfence();
    wsync();
    for (int w0 = lane; w0 < nw; w0 += 64) {
        uint64_t m = kInf;
        for (int t = 0; t < ww; ++t) {
            const uint64_t v = H[w0 + t];
            const uint64_t hv = v == kInf ? kInf : v >> 1;
            m = hv < m ? hv : m;
        }
        M[w0] = m;
    }
    gfence();
    wsync();
    int n = 0;
    for (int p0 = 0; p0 < np; p0 += 64) {
        const int p = p0 + lane;
        bool mark = false;
        uint64_t v = kInf;
        if (p < np) {
            v = H[p];
            if (v != kInf) {
                const int lo = p - ww + 1 > 0 ? p - ww + 1 : 0;
                const int hi = p < nw - 1 ? p : nw - 1;
                for (int w0 = lo; w0 <= hi; ++w0) mark |= M[w0] == (v >> 1);
            }
        }
        const unsigned long long b = __ballot(mark);
        if (n + __popcll(b) > cap) return -1;
        if (mark) out[n + __popcll(b & lanemask_lt(lane))] = ((v >> 1) << 26) | ((v & 1) << 25) | (uint64_t)p;
        n += __popcll(b);
    }
    wsync();
    return n;
}

__device__ void bitonic_sort(uint64_t *a, int n, int lane) {
    int n2 = 1;
    while (n2 < n) n2 <<= 1;
    for (int i = n + lane; i < n2; i += 64) a[i] = kInf;
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

// first index in sorted a[0, n) with a[i] >= x (per lane)
__device__ __forceinline__ int lower_bound_u64(const uint64_t *a, int n, uint64_t x) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (a[mid] < x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// first index in sorted (ascending) tails[0, n) with tails[i] >= x, wave-parallel (64-ary)
__device__ __forceinline__ int wave_lower_bound(const int32_t *tails, int n, int x, int lane) {
    int lo = 0, hi = n;
    while (hi - lo > 64) {
        const int stride = (hi - lo + 63) / 64;
        const int idx = lo + lane * stride;
        const unsigned long long b = __ballot(idx < hi && tails[idx] >= x);
        const int f = b ? __ffsll((long long)b) - 1 : 64;
        const int nlo = f == 0 ? lo : lo + (f - 1) * stride + 1;
        const int nhi = f == 64 ? hi : lo + f * stride;
        lo = nlo;
        hi = nhi;
    }
    const int idx = lo + lane;
    const unsigned long long b = __ballot(idx < hi && tails[idx] >= x);
    return b ? lo + __ffsll((long long)b) - 1 : hi;
}

// one item; returns the number of kept anchors, or -1 over this launch's capacity
__device__ int seed_item(const SeedArgs &a, int item, uint64_t *H, uint64_t *M, int2 *A, int lane) {
    const int cap = a.cap;
    uint64_t *tk = g_seed_dyn;        // t's sorted keys; later tails (t) + tails (anchor index)
    uint64_t *qk = g_seed_dyn + cap;  // q's keys; later the LIS predecessors (int32, 2 * cap)
    const int tr = a.items[2 * item], qr = a.items[2 * item + 1];
    const int64_t to = a.seq_off[tr], qo = a.seq_off[qr];
    const int tlen = (int)(a.seq_off[tr + 1] - to), qlen = (int)(a.seq_off[qr + 1] - qo);
    const int k = a.k;
    const int nt = sketch(a.seq + to, tlen, k, a.w, tk, cap, H, M, lane);
    if (nt < 0) return -1;
    if (nt == 0) return 0;
    bitonic_sort(tk, nt, lane);
    const int nq = sketch(a.seq + qo, qlen, k, a.w, qk, cap, H, M, lane);
    if (nq < 0) return -1;
    // anchors: per q minimizer (ascending position), the t occurrences of its (hash, strand) in
    // descending t position, when there are 1..max_occ of them
    int na = 0;
    for (int i0 = 0; i0 < nq; i0 += 64) {
        const int i = i0 + lane;
        int lo = 0, cnt = 0, qpos = 0;
        if (i < nq) {
            const uint64_t key = qk[i];
            const uint64_t hz = key >> 25;
            qpos = (int)(key & 0x1ffffff);
            lo = lower_bound_u64(tk, nt, hz << 25);
            const int hi = lower_bound_u64(tk, nt, (hz + 1) << 25);
            cnt = hi - lo;
            if (cnt > a.max_occ) cnt = 0;
        }
        // exclusive prefix sum of cnt over the lanes
        int incl = cnt;
        for (int d = 1; d < 64; d <<= 1) {
            const int t = __shfl_up(incl, d, 64);
            if (lane >= d) incl += t;
        }
        const int tot = __shfl(incl, 63, 64);
        if (na + tot > 2 * cap) return -1;
        const int at = na + incl - cnt;
        for (int x = 0; x < cnt; ++x) {
            const int tpos = (int)(tk[lo + cnt - 1 - x] & 0x1ffffff);
            A[at + x] = make_int2(tpos, qpos);
        }
        na += tot;
    }
    gfence();
    wsync();
    if (na == 0) return 0;
    // longest strictly increasing subsequence of t: tails in LDS (t value, anchor index)
    int32_t *tail_t = reinterpret_cast<int32_t *>(tk);
    int32_t *tail_i = tail_t + cap;
    int32_t *prev = reinterpret_cast<int32_t *>(qk);
    int L = 0;
    for (int i0 = 0; i0 < na; i0 += 64) {
        const int2 mine = (i0 + lane < na) ? A[i0 + lane] : make_int2(0, 0);
        const int n = na - i0 < 64 ? na - i0 : 64;
        for (int u = 0; u < n; ++u) {
            const int t = __shfl(mine.x, u, 64);
            const int pile = wave_lower_bound(tail_t, L, t, lane);
            if (lane == 0) {
                prev[i0 + u] = pile > 0 ? tail_i[pile - 1] : -1;
                tail_t[pile] = t;
                tail_i[pile] = i0 + u;
            }
            L += pile == L;
            wsync();
        }
    }
    if (L > cap) return -1;
    // chain (ascending) into tail_t's slots, then the partition walk (lane 0)
    int np = 0;
    if (lane == 0) {
        int c = tail_i[L - 1];
        for (int x = L - 1; x >= 0; --x) {
            tail_t[x] = c;
            c = prev[c];
        }
        int T = 0, Q = 0;
        for (int x = 0; x < L; ++x) {
            const int2 an = A[tail_t[x]];
            if (an.x - T >= a.min_w && an.y - Q >= a.min_w && tlen - (an.x + k) >= a.min_w &&
                qlen - (an.y + k) >= a.min_w) {
                if (np < a.pc) {
                    a.par_t[(int64_t)item * a.pc + np] = an.x;
                    a.par_q[(int64_t)item * a.pc + np] = an.y;
                }
                ++np;
                T = an.x + k;
                Q = an.y + k;
            }
        }
    }
    np = __shfl(np, 0, 64);
    wsync();
    return np;
}

__global__ __launch_bounds__(64) void seed_kernel(SeedArgs a) {
    const int lane = lane_id();
    uint64_t *H = a.scratch + (int64_t)blockIdx.x * a.scratch_words;
    uint64_t *M = H + a.max_len;
    int2 *A = reinterpret_cast<int2 *>(M + a.max_len);
    for (;;) {
        int it = 0;
        if (lane == 0) it = atomicAdd(a.counter, 1);
        it = __shfl(it, 0, 64);
        if (it >= a.n_items) break;
        const int item = a.redo ? a.redo[it] : it;
        const int np = seed_item(a, item, H, M, A, lane);
        if (lane == 0) a.par_n[item] = np < 0 ? -1 : (np > a.pc ? -2 : np);
        wsync();
    }
}

}  // namespace

size_t seed_dyn_bytes(int cap) { return (size_t)2 * (size_t)cap * sizeof(uint64_t); }

int64_t seed_scratch_words(int max_len, int cap) { return 2 * (int64_t)max_len + 2 * (int64_t)cap + 64; }

hipError_t launch_seed(const SeedArgs &a, int n_blocks, hipStream_t stream) {
    hipLaunchKernelGGL(seed_kernel, dim3((unsigned)n_blocks), dim3(64), seed_dyn_bytes(a.cap), stream, a);
    return hipGetLastError();
}

}  // namespace mando
