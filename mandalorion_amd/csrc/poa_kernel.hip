// poa_kernel.hip — persistent, one-wavefront-per-read-group partial-order alignment for gfx950.
//
// Replaces the abPOA v1.4.1 CLI the reference shells out to per isoform
// (/root/reference/utils/SpliceDefineConsensus.py:915-923).  Semantics are those restated in
// oracle/poa_ref.c (the checker); this file is an independent implementation shaped for CDNA4:
//
//   * one 64-lane wavefront owns one read group for its whole life (graph build, every read's
//     banded DP, traceback, graph update, heaviest-bundling consensus): no host round trips, no
//     per-read kernel boundaries, work pulled from a device-side queue (LPT order set by the host);
//   * the banded DP row is spread across the wave, 2 columns per lane, 128-column chunks; the
//     horizontal-gap states (F1/F2) are a wave-wide prefix max (Hillis-Steele over 64 lanes);
//   * the last kRing rows of H/E1/E2 live in LDS indexed by absolute column; rows with a successor
//     further away (or wider than one chunk) are additionally spilled to HBM;
//   * the traceback is one byte per cell in HBM (H source + gap-open flags) plus, only on rows with
//     several predecessors, three predecessor-index bytes; the backtrack never re-reads scores;
//   * the graph lives in HBM in struct-of-arrays form with fixed-stride adjacency (insertion order
//     preserved, capacity overflow reported to the host, which re-runs the group with more room);
//     aligned nodes are kept as per-group base tables;
//   * the topological order is maintained incrementally with every aligned group kept as a
//     contiguous block of rows (see update_graph) — any topological order gives the same DP, so
//     abPOA's per-read BFS re-sort is not needed;
//   * remain (heaviest-edge path length to the sink) is rebuilt per read by 64-row chunks with
//     in-register pointer jumping.
#include "poa_kernel.h"

namespace mando {

struct Slot {
    uint8_t *base;
    int *gid, *gtab, *in_n, *out_n, *in_id, *out_id, *out_w, *sink_in, *src_out, *src_out_w;
    int *order, *order2, *pos, *remrow, *desc, *rinfo;
    uint8_t *tb, *kp;
    int *sv, *qnode, *qtgt, *qflag, *qnb, *qoff, *qmslot, *ins, *insmm, *score, *nxt;
};

__device__ __forceinline__ int lane_id() { return (int)__lane_id(); }

__device__ __forceinline__ int bcast0(int v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ __forceinline__ int readlane(int v, int l) { return __builtin_amdgcn_readlane(v, l); }

// inclusive prefix max over the 64 lanes
__device__ __forceinline__ int wave_incl_max(int v, int lane) {
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        int t = __shfl_up(v, d, kWave);
        if (lane >= d) v = max(v, t);
    }
    return v;
}

// inclusive prefix sum over the 64 lanes
__device__ __forceinline__ int wave_incl_sum(int v, int lane) {
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        int t = __shfl_up(v, d, kWave);
        if (lane >= d) v += t;
    }
    return v;
}

__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) v = max(v, __shfl_xor(v, d, kWave));
    return v;
}

__device__ __forceinline__ unsigned long long lanemask_lt(int lane) {
    return (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
}

__device__ __forceinline__ int score_of(int a, int b, int match, int mismatch) {
    return (a == 4 || b == 4) ? 0 : (a == b ? match : -mismatch);
}

__device__ __forceinline__ int *in_list(const Slot &s, const PoaKArgs &a, int v) {
    return v == kSink ? s.sink_in : s.in_id + (int64_t)v * a.caps.DCAP;
}
__device__ __forceinline__ int in_cap(const PoaKArgs &a, int v) {
    return v == kSink ? a.caps.BIGCAP : a.caps.DCAP;
}
__device__ __forceinline__ int *out_list(const Slot &s, const PoaKArgs &a, int v) {
    return v == kSrc ? s.src_out : s.out_id + (int64_t)v * a.caps.DCAP;
}
__device__ __forceinline__ int *out_wlist(const Slot &s, const PoaKArgs &a, int v) {
    return v == kSrc ? s.src_out_w : s.out_w + (int64_t)v * a.caps.DCAP;
}
__device__ __forceinline__ int out_cap(const PoaKArgs &a, int v) {
    return v == kSrc ? a.caps.BIGCAP : a.caps.DCAP;
}

// wave-level barrier that also orders this wave's global/LDS memory traffic
__device__ __forceinline__ void wave_sync() { __syncthreads(); }

struct RowRec {
    int beg, end, am, soff;
};

struct SharedState {
    int ring[kRing][3][kChunk];
    int4 rrow[kRowRing];
};

// ---------------------------------------------------------------------------------------------
// first read: a chain SRC -> n0 -> ... -> n(L-1) -> SINK
// ---------------------------------------------------------------------------------------------
__device__ int init_chain(const PoaKArgs &a, Slot &s, const uint8_t *q, int L, int lane, int &n) {
    if (L + 2 > a.caps.NC) return kStCap;
    for (int t = lane; t < L; t += kWave) {
        int v = 2 + t;
        s.base[v] = q[t];
        s.gid[v] = -1;
        s.in_n[v] = 1;
        in_list(s, a, v)[0] = (t == 0) ? kSrc : v - 1;
        s.out_n[v] = 1;
        out_list(s, a, v)[0] = (t == L - 1) ? kSink : v + 1;
        out_wlist(s, a, v)[0] = 1;
        s.order[1 + t] = v;
        s.pos[v] = 1 + t;
    }
    for (int t = lane; t < L + 2; t += kWave) {
        s.ins[t] = 0;
        s.insmm[t] = 0;
    }
    if (lane == 0) {
        s.base[kSrc] = 4;
        s.base[kSink] = 4;
        s.gid[kSrc] = -1;
        s.gid[kSink] = -1;
        s.in_n[kSrc] = 0;
        s.out_n[kSrc] = 1;
        s.src_out[0] = 2;
        s.src_out_w[0] = 1;
        s.in_n[kSink] = 1;
        s.sink_in[0] = L + 1;
        s.out_n[kSink] = 0;
        s.order[0] = kSrc;
        s.pos[kSrc] = 0;
        s.order[L + 1] = kSink;
        s.pos[kSink] = L + 1;
    }
    n = L + 2;
    return kStOk;
}

// ---------------------------------------------------------------------------------------------
// row descriptors + remain (heaviest out-edge path length to the sink), 64-row chunks from the end
// desc[r] = {node, base | far<<8 | pre_n<<16, remain, pre_row[0..4]}
// ---------------------------------------------------------------------------------------------
__device__ void build_desc(const PoaKArgs &a, Slot &s, int n, int lane) {
    const int nch = (n + kWave - 1) / kWave;
    int prev_val = 0;
    for (int c = nch - 1; c >= 0; --c) {
        const int r = c * kWave + lane;
        const bool valid = r < n;
        int v = 0, bh = -1, far = 0, pn = 0, vb = 4;
        int pre[kPreInline];
#pragma unroll
        for (int k = 0; k < kPreInline; ++k) pre[k] = -1;
        if (valid) {
            v = s.order[r];
            vb = s.base[v];
            pn = s.in_n[v];
            const int *il = in_list(s, a, v);
#pragma unroll
            for (int k = 0; k < kPreInline; ++k)
                if (k < pn) pre[k] = s.pos[il[k]];
            const int on = s.out_n[v];
            const int *ol = out_list(s, a, v);
            const int *ow = out_wlist(s, a, v);
            int bw = -2147483647 - 1, maxd = 0;
            for (int k = 0; k < on; ++k) {
                int po = s.pos[ol[k]];
                int wg = ow[k];
                if (wg > bw) {
                    bw = wg;
                    bh = po;
                }
                maxd = max(maxd, po - r);
            }
            far = maxd >= kRing ? 1 : 0;
        }
        const int lo_next = (c + 1) * kWave, lo_next2 = (c + 2) * kWave;
        const int idx_prev = (bh >= lo_next && bh < lo_next2) ? bh - lo_next : lane;
        const int from_prev = __shfl(prev_val, idx_prev, kWave);
        int val = 0, ptr = -1;
        if (valid) {
            if (v == kSink) {
                val = -1;
            } else if (bh >= lo_next2) {
                val = s.remrow[bh] + 1;
            } else if (bh >= lo_next) {
                val = from_prev + 1;
            } else {
                val = 1;
                ptr = bh - c * kWave;
            }
        }
#pragma unroll
        for (int it = 0; it < 6; ++it) {
            const int src = ptr >= 0 ? ptr : lane;
            const int pv = __shfl(val, src, kWave);
            const int pp = __shfl(ptr, src, kWave);
            if (ptr >= 0) {
                val += pv;
                ptr = pp;
            }
        }
        if (valid) {
            s.remrow[r] = val;
            int *d = s.desc + (int64_t)r * kDescInts;
            d[0] = v;
            d[1] = vb | (far << 8) | (pn << 16);
            d[2] = val;
#pragma unroll
            for (int k = 0; k < kPreInline; ++k) d[3 + k] = pre[k];
        }
        prev_val = val;
        wave_sync();
    }
}

// predecessor row k of row r (node v); the first kPreInline come from the descriptor
__device__ __forceinline__ int pre_row_slow(const PoaKArgs &a, const Slot &s, int v, int k) {
    return s.pos[in_list(s, a, v)[k]];
}

__device__ __forceinline__ RowRec load_rowrec(const SharedState &sh, const Slot &s, int r, int p) {
    RowRec rr;
    if (r - p < kRowRing) {
        int4 x = sh.rrow[p % kRowRing];
        rr.beg = x.x;
        rr.end = x.y;
        rr.am = x.z;
        rr.soff = x.w;
    } else {
        const int *ri = s.rinfo + (int64_t)p * kRowInfoInts;
        rr.beg = ri[0];
        rr.end = ri[1];
        rr.am = ri[2];
        rr.soff = ri[3];
    }
    return rr;
}

// H (plane 0), E1out (1), E2out (2) of row p at column col, kNegInf outside its band
__device__ __forceinline__ int row_val(const SharedState &sh, const Slot &s, int r, int p,
                                       const RowRec &rr, int plane, int col) {
    if (col < rr.beg || col > rr.end) return kNegInf;
    const int width = rr.end - rr.beg + 1;
    if (r - p < kRing && width <= kChunk) return sh.ring[p % kRing][plane][col & (kChunk - 1)];
    return s.sv[(int64_t)rr.soff + (int64_t)plane * width + (col - rr.beg)];
}

// ---------------------------------------------------------------------------------------------
// banded DP over all rows of the current graph for read q (qlen) — writes traceback bytes and
// returns the start row of the backtrack in *bi (or -1)
// ---------------------------------------------------------------------------------------------
__device__ int run_dp(const PoaKArgs &a, Slot &s, SharedState &sh, const uint8_t *q, int qlen,
                      int n, int lane, int64_t &cells, int &bi_out) {
    const int w = a.band_b + (int)(a.band_f * (float)qlen);
    const int e1 = a.e1, e2 = a.e2, oe1 = a.o1 + a.e1, oe2 = a.o2 + a.e2;
    const int IDENT = -(1 << 30);
    int64_t tb_used = 0, kp_used = 0, sv_used = 0;
    int dreg[kDescInts];
    for (int r = 0; r < n - 1; ++r) {
        if ((r & (kWave - 1)) == 0) {
            const int rr0 = r + lane;
            if (rr0 < n) {
                const int4 *dp4 = reinterpret_cast<const int4 *>(s.desc + (int64_t)rr0 * kDescInts);
                int4 x = dp4[0], y = dp4[1];
                dreg[0] = x.x; dreg[1] = x.y; dreg[2] = x.z; dreg[3] = x.w;
                dreg[4] = y.x; dreg[5] = y.y; dreg[6] = y.z; dreg[7] = y.w;
            }
        }
        const int rl = r & (kWave - 1);
        const int node = readlane(dreg[0], rl);
        const int d1 = readlane(dreg[1], rl);
        const int rem = readlane(dreg[2], rl);
        const int vb = d1 & 0xff;
        const int far = (d1 >> 8) & 0xff;
        const int pn = d1 >> 16;
        int dpre[kPreInline];
#pragma unroll
        for (int k = 0; k < kPreInline; ++k) dpre[k] = readlane(dreg[3 + k], rl);

        // --- band
        int beg, end;
        if (r == 0) {
            beg = 0;
            end = min(qlen, max(0, qlen - rem) + w);
        } else {
            int posL = 2147483647, posR = -2147483647 - 1;
            for (int k = 0; k < pn; ++k) {
                int p;
                if (k < kPreInline) {
                    p = dpre[0];
#pragma unroll
                    for (int kk = 1; kk < kPreInline; ++kk)
                        if (k == kk) p = dpre[kk];
                } else {
                    p = bcast0(pre_row_slow(a, s, node, k));
                }
                RowRec pr = load_rowrec(sh, s, r, p);
                posL = min(posL, pr.am + 1);
                posR = max(posR, pr.am + 1);
            }
            const int x = qlen - rem;
            beg = max(0, min(posL, x) - w);
            end = min(qlen, max(posR, x) + w);
        }
        const int width = end - beg + 1;
        const bool wide = width > kChunk;
        const bool spill = far || wide;
        const int64_t tbw = (width + 3) & ~3;
        const bool multi = pn > 1;
        if (tb_used + tbw > a.caps.TBC) return kStCap;
        if (multi && kp_used + 3 * tbw > a.caps.KPC) return kStCap;
        if (spill && sv_used + 3 * (int64_t)width > a.caps.SVC) return kStCap;
        const int64_t tboff = tb_used, kpoff = multi ? kp_used : -1;
        const int soff = spill ? (int)sv_used : -1;
        tb_used += tbw;
        if (multi) kp_used += 3 * tbw;
        if (spill) sv_used += 3 * (int64_t)width;
        cells += width;

        int best = -2147483647 - 1, besti = beg;
        int carry1 = kNegInf + oe1 + e1 * (beg - 1);
        int carry2 = kNegInf + oe2 + e2 * (beg - 1);
        int *ringrow = &sh.ring[r % kRing][0][0];

        for (int cb = beg; cb <= end; cb += kChunk) {
            const int j0 = cb + 2 * lane, j1 = j0 + 1;
            const bool va = j0 <= end, vbb = j1 <= end;
            int Ha, Hb, E1a, E1b, E2a, E2b;
            uint8_t ta = 0, tbb = 0;
            int mka = 0, mkb = 0, k1a = 0, k1b = 0, k2a = 0, k2b = 0;
            if (r == 0) {
                // source row: H[0][0] = 0, H[0][j] = max(-(o1+e1 j), -(o2+e2 j))
                Ha = (j0 == 0) ? 0 : max(-(a.o1 + e1 * j0), -(a.o2 + e2 * j0));
                Hb = max(-(a.o1 + e1 * j1), -(a.o2 + e2 * j1));
                E1a = Ha - oe1;
                E1b = Hb - oe1;
                E2a = Ha - oe2;
                E2b = Hb - oe2;
            } else {
                int Mva = kNegInf, Mvb = kNegInf, X1a = kNegInf, X1b = kNegInf, X2a = kNegInf,
                    X2b = kNegInf;
                for (int k = 0; k < pn; ++k) {
                    int p;
                    if (k < kPreInline) {
                        p = dpre[0];
#pragma unroll
                        for (int kk = 1; kk < kPreInline; ++kk)
                            if (k == kk) p = dpre[kk];
                    } else {
                        p = bcast0(pre_row_slow(a, s, node, k));
                    }
                    const RowRec pr = load_rowrec(sh, s, r, p);
                    const int hA = row_val(sh, s, r, p, pr, 0, j0 - 1);
                    const int hB = row_val(sh, s, r, p, pr, 0, j0);
                    const int e1A = row_val(sh, s, r, p, pr, 1, j0);
                    const int e1B = row_val(sh, s, r, p, pr, 1, j1);
                    const int e2A = row_val(sh, s, r, p, pr, 2, j0);
                    const int e2B = row_val(sh, s, r, p, pr, 2, j1);
                    if (hA > Mva) { Mva = hA; mka = k; }
                    if (hB > Mvb) { Mvb = hB; mkb = k; }
                    if (e1A > X1a) { X1a = e1A; k1a = k; }
                    if (e1B > X1b) { X1b = e1B; k1b = k; }
                    if (e2A > X2a) { X2a = e2A; k2a = k; }
                    if (e2B > X2b) { X2b = e2B; k2b = k; }
                }
                const int qa = (j0 >= 1 && j0 <= qlen) ? q[j0 - 1] : 4;
                const int qb = (j0 >= 0 && j0 < qlen) ? q[j0] : 4;
                const int Ma = Mva + score_of(vb, qa, a.match, a.mismatch);
                const int Mb = Mvb + score_of(vb, qb, a.match, a.mismatch);
                const int H0a = max(Ma, max(X1a, X2a));
                const int H0b = max(Mb, max(X1b, X2b));
                // horizontal gaps: F[j] = max(C, max_{k<j} H0[k] + e*k) - oe - e*(j-1)
                const int G1a = va ? H0a + e1 * j0 : IDENT;
                const int G1b = vbb ? H0b + e1 * j1 : IDENT;
                const int G2a = va ? H0a + e2 * j0 : IDENT;
                const int G2b = vbb ? H0b + e2 * j1 : IDENT;
                const int inc1 = wave_incl_max(max(G1a, G1b), lane);
                const int inc2 = wave_incl_max(max(G2a, G2b), lane);
                int ex1 = __shfl_up(inc1, 1, kWave);
                int ex2 = __shfl_up(inc2, 1, kWave);
                if (lane == 0) { ex1 = IDENT; ex2 = IDENT; }
                const int P1a = max(ex1, carry1), P1b = max(P1a, G1a);
                const int P2a = max(ex2, carry2), P2b = max(P2a, G2a);
                carry1 = max(carry1, readlane(inc1, kWave - 1));
                carry2 = max(carry2, readlane(inc2, kWave - 1));
                const int F1a = P1a - oe1 - e1 * (j0 - 1), F1b = P1b - oe1 - e1 * (j1 - 1);
                const int F2a = P2a - oe2 - e2 * (j0 - 1), F2b = P2b - oe2 - e2 * (j1 - 1);
                Ha = max(H0a, max(F1a, F2a));
                Hb = max(H0b, max(F1b, F2b));
                auto src_type = [&](int H, int M, int X1, int X2, int F1, int k1, int k2) -> int {
                    if (M == H) return 0;
                    const bool t1 = X1 == H, t2 = X2 == H;
                    if (t1 && t2) return (k1 <= k2) ? 1 : 2;
                    if (t1) return 1;
                    if (t2) return 2;
                    return (F1 == H) ? 3 : 4;
                };
                const int tya = src_type(Ha, Ma, X1a, X2a, F1a, k1a, k2a);
                const int tyb = src_type(Hb, Mb, X1b, X2b, F1b, k1b, k2b);
                E1a = max(X1a - e1, Ha - oe1);
                E1b = max(X1b - e1, Hb - oe1);
                E2a = max(X2a - e2, Ha - oe2);
                E2b = max(X2b - e2, Hb - oe2);
                ta = (uint8_t)(tya | ((Ha - oe1 >= X1a - e1) ? kTbE1Open : 0) |
                               ((Ha - oe2 >= X2a - e2) ? kTbE2Open : 0) |
                               ((G1a >= P1a) ? kTbF1OpenNext : 0) | ((G2a >= P2a) ? kTbF2OpenNext : 0));
                tbb = (uint8_t)(tyb | ((Hb - oe1 >= X1b - e1) ? kTbE1Open : 0) |
                                ((Hb - oe2 >= X2b - e2) ? kTbE2Open : 0) |
                                ((G1b >= P1b) ? kTbF1OpenNext : 0) | ((G2b >= P2b) ? kTbF2OpenNext : 0));
            }
            // store traceback / predecessor indices / row values
            if (va) {
                const int64_t c0 = j0 - beg;
                s.tb[tboff + c0] = ta;
                if (multi) {
                    uint8_t *kpp = s.kp + kpoff + 3 * c0;
                    kpp[0] = (uint8_t)mka;
                    kpp[1] = (uint8_t)k1a;
                    kpp[2] = (uint8_t)k2a;
                }
                if (!wide) {
                    ringrow[0 * kChunk + (j0 & (kChunk - 1))] = Ha;
                    ringrow[1 * kChunk + (j0 & (kChunk - 1))] = E1a;
                    ringrow[2 * kChunk + (j0 & (kChunk - 1))] = E2a;
                }
                if (spill) {
                    int *svp = s.sv + soff;
                    svp[c0] = Ha;
                    svp[width + c0] = E1a;
                    svp[2 * width + c0] = E2a;
                }
            }
            if (vbb) {
                const int64_t c1 = j1 - beg;
                s.tb[tboff + c1] = tbb;
                if (multi) {
                    uint8_t *kpp = s.kp + kpoff + 3 * c1;
                    kpp[0] = (uint8_t)mkb;
                    kpp[1] = (uint8_t)k1b;
                    kpp[2] = (uint8_t)k2b;
                }
                if (!wide) {
                    ringrow[0 * kChunk + (j1 & (kChunk - 1))] = Hb;
                    ringrow[1 * kChunk + (j1 & (kChunk - 1))] = E1b;
                    ringrow[2 * kChunk + (j1 & (kChunk - 1))] = E2b;
                }
                if (spill) {
                    int *svp = s.sv + soff;
                    svp[c1] = Hb;
                    svp[width + c1] = E1b;
                    svp[2 * width + c1] = E2b;
                }
            }
            // leftmost argmax of H over the row
            int lb = -2147483647 - 1, lp = j0;
            if (va) { lb = Ha; lp = j0; }
            if (vbb && Hb > lb) { lb = Hb; lp = j1; }
            const int m = wave_max(lb);
            const unsigned long long hit = __ballot(lb == m && va);
            const int first = __ffsll((long long)hit) - 1;
            const int mpos = __shfl(lp, first < 0 ? 0 : first, kWave);
            if (m > best) {
                best = m;
                besti = mpos;
            }
        }
        if (lane == 0) {
            sh.rrow[r % kRowRing] = make_int4(beg, end, besti, soff);
            int *ri = s.rinfo + (int64_t)r * kRowInfoInts;
            ri[0] = beg;
            ri[1] = end;
            ri[2] = besti;
            ri[3] = soff;
            ri[4] = (int)tboff;
            ri[5] = (int)kpoff;
        }
        // make this row's LDS/HBM values visible to the next rows' loads (same wave)
        wave_sync();
    }

    // best predecessor of the sink at column qlen (first in in-edge order on ties)
    const int sr = n - 1;
    const int nin = s.in_n[kSink];
    int bs = -2147483647 - 1, bi = -1;
    for (int k = 0; k < nin; ++k) {
        const int p = bcast0(s.pos[s.sink_in[k]]);
        const RowRec pr = load_rowrec(sh, s, sr, p);
        if (qlen < pr.beg || qlen > pr.end) continue;
        const int h = bcast0(row_val(sh, s, sr, p, pr, 0, qlen));
        if (h > bs) {
            bs = h;
            bi = p;
        }
    }
    bi_out = bi;
    return kStOk;
}

// ---------------------------------------------------------------------------------------------
// backtrack (lane 0): fills qnode[q] = aligned node or -1 (insertion) for q in [0, qlen)
// ---------------------------------------------------------------------------------------------
__device__ int backtrack(const PoaKArgs &a, Slot &s, int bi, int qlen, int n) {
    int i = bi, j = qlen, st = 0;  // 0 H, 1 E1, 2 E2, 3 F1, 4 F2
    int guard = n + qlen + 8;
    while (i > 0 && j > 0) {
        if (--guard < 0) return kStInternal;
        const int *ri = s.rinfo + (int64_t)i * kRowInfoInts;
        const int rb = ri[0];
        const int64_t tboff = ri[4], kpoff = ri[5];
        const int c = j - rb;
        const int t = s.tb[tboff + c];
        const int *d = s.desc + (int64_t)i * kDescInts;
        const int node = d[0];
        const int pn = d[1] >> 16;
        if (st == 0) {
            const int ty = t & kTbTypeMask;
            if (ty <= 2) {
                const int k = (pn > 1) ? s.kp[kpoff + 3 * c + ty] : 0;
                const int p = (k < kPreInline) ? d[3 + k] : pre_row_slow(a, s, node, k);
                if (ty == 0) {
                    s.qnode[j - 1] = node;
                    i = p;
                    --j;
                } else {
                    const int *pri = s.rinfo + (int64_t)p * kRowInfoInts;
                    const int tp = s.tb[(int64_t)pri[4] + (j - pri[0])];
                    st = (tp & (ty == 1 ? kTbE1Open : kTbE2Open)) ? 0 : ty;
                    i = p;
                }
                continue;
            }
            st = ty;  // 3 or 4: handled below in the same step
        }
        if (st == 1 || st == 2) {
            const int k = (pn > 1) ? s.kp[kpoff + 3 * c + st] : 0;
            const int p = (k < kPreInline) ? d[3 + k] : pre_row_slow(a, s, node, k);
            const int *pri = s.rinfo + (int64_t)p * kRowInfoInts;
            const int tp = s.tb[(int64_t)pri[4] + (j - pri[0])];
            st = (tp & (st == 1 ? kTbE1Open : kTbE2Open)) ? 0 : st;
            i = p;
            continue;
        }
        // F1 / F2: query base j-1 is an insertion at row i
        s.qnode[j - 1] = -1;
        const int tprev = s.tb[tboff + c - 1];
        st = (tprev & (st == 3 ? kTbF1OpenNext : kTbF2OpenNext)) ? 0 : st;
        --j;
    }
    for (int t = 0; t < j; ++t) s.qnode[t] = -1;
    return kStOk;
}

// ---------------------------------------------------------------------------------------------
// graph update for one aligned read (wave-parallel over query positions)
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ int add_edge(const PoaKArgs &a, Slot &s, int from, int to, bool check,
                                        bool from_new, bool to_new) {
    int *ol = out_list(s, a, from);
    int *ow = out_wlist(s, a, from);
    if (check) {
        const int on = s.out_n[from];
        for (int k = 0; k < on; ++k)
            if (ol[k] == to) {
                ow[k] += 1;
                return kStOk;
            }
    }
    const int on = from_new ? 0 : s.out_n[from];
    if (on >= out_cap(a, from)) return kStCap;
    ol[on] = to;
    ow[on] = 1;
    s.out_n[from] = on + 1;
    int *il = in_list(s, a, to);
    const int inn = to_new ? 0 : s.in_n[to];
    if (inn >= in_cap(a, to)) return kStCap;
    il[inn] = from;
    s.in_n[to] = inn + 1;
    return kStOk;
}

__device__ int update_graph(const PoaKArgs &a, Slot &s, const uint8_t *q, int qlen, int &n,
                            int &ng, int lane) {
    // Path kinds per query position: 0 = existing node (matched, or a reused aligned node),
    // 1 = new node aligned to the DP row's node (mismatch), 2 = new inserted node.
    // Topological order invariant kept here: every aligned group occupies a contiguous block of
    // rows.  New mismatch nodes are appended right after their group's block; inserted nodes go
    // right before the block of the next anchored (kind 0/1) node of the path.  Any path of the
    // DP visits blocks in increasing order, so the result is again a valid topological order.
    const int n_old = n;
    int last = kSrc, last_new = 0;
    int err = kStOk;
    const int nch = (qlen + kWave - 1) / kWave;
    // pass 1: targets, new nodes, aligned groups, edges
    for (int c = 0; c < nch; ++c) {
        const int qi = c * kWave + lane;
        const bool valid = qi < qlen;
        const int b = valid ? q[qi] : 0;
        const int v = valid ? s.qnode[qi] : -1;
        int kind = 0, tgt = -1, needgrp = 0, g = -1, aslot = -1, mslot = -1, vbase = 4, gsize = 1;
        if (valid) {
            if (v >= 0) {
                vbase = s.base[v];
                g = s.gid[v];
                const int head = g >= 0 ? s.gtab[g * kGtabInts + 5] : v;
                gsize = g >= 0 ? s.gtab[g * kGtabInts + 6] : 1;
                aslot = s.pos[head];
                if (vbase == b) {
                    tgt = v;
                } else {
                    const int al = g >= 0 ? s.gtab[g * kGtabInts + b] : -1;
                    if (al >= 0) {
                        tgt = al;
                    } else {
                        kind = 1;
                        needgrp = g < 0;
                        mslot = aslot + gsize;
                    }
                }
            } else {
                kind = 2;
            }
        }
        const int isnew = kind != 0;
        const unsigned long long mnew = __ballot(isnew);
        const unsigned long long mgrp = __ballot(needgrp);
        const int nnew = __popcll(mnew), ngrp = __popcll(mgrp);
        if (n + nnew > a.caps.NC || ng + ngrp > a.caps.NC) return kStCap;
        if (isnew) tgt = n + __popcll(mnew & lanemask_lt(lane));
        if (needgrp) g = ng + __popcll(mgrp & lanemask_lt(lane));
        n += nnew;
        ng += ngrp;
        if (isnew) {
            s.base[tgt] = (uint8_t)b;
            if (kind == 2) s.gid[tgt] = -1;
        }
        if (kind == 1) {
            int *gt = s.gtab + (int64_t)g * kGtabInts;
            if (needgrp) {
#pragma unroll
                for (int t = 0; t < 5; ++t) gt[t] = -1;
                gt[vbase] = v;
                gt[5] = v;
                gt[6] = 2;
                s.gid[v] = g;
            } else {
                gt[6] = gsize + 1;
            }
            gt[b] = tgt;
            s.gid[tgt] = g;
        }
        int prev_t = __shfl_up(tgt, 1, kWave);
        int prev_n = __shfl_up(isnew, 1, kWave);
        if (lane == 0) {
            prev_t = last;
            prev_n = last_new;
        }
        int e = kStOk;
        if (valid) e = add_edge(a, s, prev_t, tgt, !prev_n, prev_n != 0, isnew != 0);
        if (__ballot(e != kStOk)) err = kStCap;
        if (valid) {
            s.qtgt[qi] = tgt;
            s.qflag[qi] = kind;
            s.qnb[qi] = aslot;
            s.qmslot[qi] = mslot;
        }
        const int lastl = min(kWave, qlen - c * kWave) - 1;
        last = readlane(tgt, lastl);
        last_new = readlane(isnew, lastl);
    }
    if (err != kStOk) return err;
    if (lane == 0) {
        if (add_edge(a, s, last, kSink, !last_new, last_new != 0, false) != kStOk) err = kStCap;
    }
    err = bcast0(err);
    if (err != kStOk) return err;
    wave_sync();
    // pass 2 (backwards): slot (old row) each new node is inserted in front of
    int nxt_q = qlen, nxt_R = n_old - 1;
    for (int c = nch - 1; c >= 0; --c) {
        const int qi = c * kWave + lane;
        const bool valid = qi < qlen;
        const int kind = valid ? s.qflag[qi] : 0;
        const int aslot = valid ? s.qnb[qi] : -1;
        const bool anch = valid && kind != 2;
        const unsigned long long manch = __ballot(anch);
        const unsigned long long above = (lane == 63) ? 0ull : (manch & ((~0ull) << (lane + 1)));
        const int nl = above ? (__ffsll((long long)above) - 1) : lane;
        const int R_in = __shfl(aslot, nl, kWave);
        const int nq = above ? c * kWave + nl : nxt_q;
        const int R = above ? R_in : nxt_R;
        const int prev_kind = __shfl_up(kind, 1, kWave);
        if (valid && kind == 2) {
            const bool run_start = (qi == 0) || (lane == 0 ? s.qflag[qi - 1] != 2 : prev_kind != 2);
            s.qnb[qi] = R;
            s.qoff[qi] = nq - qi;
            if (run_start) s.ins[R] = nq - qi;
        }
        if (valid && kind == 1) s.insmm[s.qmslot[qi]] = 1;
        if (manch) {
            const int fl = __ffsll((long long)manch) - 1;
            nxt_q = c * kWave + fl;
            nxt_R = readlane(aslot, fl);
        }
    }
    wave_sync();
    // pass 3: shift old rows by the number of new nodes inserted before (and at) them
    int carry = 0;
    for (int c = 0; c * kWave < n_old; ++c) {
        const int r = c * kWave + lane;
        const bool valid = r < n_old;
        const int tot = valid ? s.ins[r] + s.insmm[r] : 0;
        const int inc = wave_incl_sum(tot, lane) + carry;
        carry = readlane(inc, kWave - 1);
        if (valid) {
            const int v = s.order[r];
            const int np = r + inc;
            s.order2[np] = v;
            s.pos[v] = np;
        }
    }
    wave_sync();
    // pass 4: place the new nodes (mismatch node first, then the insertion run, before row R)
    for (int c = 0; c < nch; ++c) {
        const int qi = c * kWave + lane;
        const int kind = qi < qlen ? s.qflag[qi] : 0;
        if (kind == 2) {
            const int x = s.qtgt[qi];
            const int np = s.pos[s.order[s.qnb[qi]]] - s.qoff[qi];
            s.order2[np] = x;
            s.pos[x] = np;
        } else if (kind == 1) {
            const int x = s.qtgt[qi];
            const int R = s.qmslot[qi];
            const int np = s.pos[s.order[R]] - s.ins[R] - 1;
            s.order2[np] = x;
            s.pos[x] = np;
        }
    }
    wave_sync();
    // pass 5: clear the insertion counters for the next read
    for (int t = lane; t < n; t += kWave) {
        s.ins[t] = 0;
        s.insmm[t] = 0;
    }
    int *tmp = s.order;
    s.order = s.order2;
    s.order2 = tmp;
    wave_sync();
    return kStOk;
}

// ---------------------------------------------------------------------------------------------
// heaviest bundling (lane 0): reverse topological sweep, then walk from the source
// ---------------------------------------------------------------------------------------------
__device__ int consensus(const PoaKArgs &a, Slot &s, int n, uint8_t *out, int64_t cap,
                         int &len) {
    for (int r = n - 1; r >= 0; --r) {
        const int v = s.order[r];
        if (v == kSink) {
            s.score[r] = 0;
            s.nxt[r] = -1;
            continue;
        }
        const int on = s.out_n[v];
        const int *ol = out_list(s, a, v);
        const int *ow = out_wlist(s, a, v);
        int maxw = -1, maxr = -1;
        for (int k = 0; k < on; ++k) {
            const int ro = s.pos[ol[k]];
            const int wgt = ow[k];
            if (maxw < wgt) {
                maxw = wgt;
                maxr = ro;
            } else if (maxw == wgt && s.score[maxr] <= s.score[ro]) {
                maxr = ro;
            }
        }
        if (maxr < 0) return kStInternal;
        s.score[r] = maxw + s.score[maxr];
        s.nxt[r] = maxr;
    }
    int r = s.nxt[0];
    int64_t l = 0;
    while (r >= 0 && r != n - 1) {
        if (l < cap) out[l] = s.base[s.order[r]];
        ++l;
        r = s.nxt[r];
        if (l > n) return kStInternal;
    }
    len = (int)l;
    return l <= cap ? kStOk : kStCap;
}

__global__ __launch_bounds__(kWave) void poa_kernel(PoaKArgs a) {
    __shared__ SharedState sh;
    const int lane = lane_id();
    char *ws = a.ws + (int64_t)blockIdx.x * a.slot_bytes;
    Slot s;
    s.base = (uint8_t *)(ws + a.lay.base);
    s.gid = (int *)(ws + a.lay.gid);
    s.gtab = (int *)(ws + a.lay.gtab);
    s.in_n = (int *)(ws + a.lay.in_n);
    s.out_n = (int *)(ws + a.lay.out_n);
    s.in_id = (int *)(ws + a.lay.in_id);
    s.out_id = (int *)(ws + a.lay.out_id);
    s.out_w = (int *)(ws + a.lay.out_w);
    s.sink_in = (int *)(ws + a.lay.sink_in);
    s.src_out = (int *)(ws + a.lay.src_out);
    s.src_out_w = (int *)(ws + a.lay.src_out_w);
    s.pos = (int *)(ws + a.lay.pos);
    s.remrow = (int *)(ws + a.lay.remrow);
    s.desc = (int *)(ws + a.lay.desc);
    s.rinfo = (int *)(ws + a.lay.rinfo);
    s.tb = (uint8_t *)(ws + a.lay.tb);
    s.kp = (uint8_t *)(ws + a.lay.kp);
    s.sv = (int *)(ws + a.lay.sv);
    s.qnode = (int *)(ws + a.lay.qnode);
    s.qtgt = (int *)(ws + a.lay.qtgt);
    s.qflag = (int *)(ws + a.lay.qflag);
    s.qnb = (int *)(ws + a.lay.qnb);
    s.qoff = (int *)(ws + a.lay.qoff);
    s.ins = (int *)(ws + a.lay.ins);
    s.insmm = (int *)(ws + a.lay.insmm);
    s.qmslot = (int *)(ws + a.lay.qmslot);
    s.score = (int *)(ws + a.lay.score);
    s.nxt = (int *)(ws + a.lay.nxt);

    for (;;) {
        int gi = 0;
        if (lane == 0) gi = atomicAdd(a.counter, 1);
        gi = bcast0(gi);
        if (gi >= a.n_groups) break;
        const int g = a.gorder ? a.gorder[gi] : gi;
        s.order = (int *)(ws + a.lay.order0);
        s.order2 = (int *)(ws + a.lay.order1);
        const int64_t r0 = a.grp_off[g], r1 = a.grp_off[g + 1];
        int st = kStOk;
        int n = 0, ng = 0;
        int64_t cells = 0;
        int64_t first = r0;
        while (first < r1 && a.seq_off[first + 1] - a.seq_off[first] <= 0) ++first;
        int clen = 0;
        if (first < r1) {
            const uint8_t *q0 = a.seq + a.seq_off[first];
            const int L0 = (int)(a.seq_off[first + 1] - a.seq_off[first]);
            st = init_chain(a, s, q0, L0, lane, n);
            wave_sync();
            for (int64_t rd = first + 1; rd < r1 && st == kStOk; ++rd) {
                const int qlen = (int)(a.seq_off[rd + 1] - a.seq_off[rd]);
                if (qlen <= 0) continue;
                if (qlen > a.caps.QC) {
                    st = kStCap;
                    break;
                }
                const uint8_t *q = a.seq + a.seq_off[rd];
                build_desc(a, s, n, lane);
                int bi = -1;
                st = run_dp(a, s, sh, q, qlen, n, lane, cells, bi);
                if (st != kStOk) break;
                if (bi < 0) {
                    st = kStInternal;
                    break;
                }
                wave_sync();
                int bst = kStOk;
                if (lane == 0) bst = backtrack(a, s, bi, qlen, n);
                st = bcast0(bst);
                if (st != kStOk) break;
                wave_sync();
                st = update_graph(a, s, q, qlen, n, ng, lane);
                wave_sync();
            }
            if (st == kStOk) {
                int cst = kStOk, len = 0;
                if (lane == 0) {
                    const int64_t cap = a.cons_off[g + 1] - a.cons_off[g];
                    cst = consensus(a, s, n, a.cons + a.cons_off[g], cap, len);
                }
                st = bcast0(cst);
                clen = bcast0(len);
            }
        }
        if (lane == 0) {
            a.status[g] = st;
            a.cons_len[g] = clen;
            a.cells[g] = cells;
        }
        wave_sync();
    }
}

hipError_t launch_poa(const PoaKArgs &a, int n_slots, hipStream_t stream) {
    hipLaunchKernelGGL(poa_kernel, dim3(n_slots), dim3(kWave), 0, stream, a);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// self-test of the wave primitives against serial references
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kWave) void wave_selftest_kernel(int *bad) {
    const int lane = lane_id();
    int errs = 0;
    for (int trial = 0; trial < 64; ++trial) {
        const int v = (int)((lane * 2654435761u + trial * 40503u) % 1000u) - 500;
        const int inc = wave_incl_max(v, lane);
        const int sum = wave_incl_sum(v, lane);
        int rmax = -2147483647 - 1, rsum = 0;
        for (int l = 0; l <= lane; ++l) {
            const int vl = (int)((l * 2654435761u + trial * 40503u) % 1000u) - 500;
            rmax = max(rmax, vl);
            rsum += vl;
        }
        if (inc != rmax) ++errs;
        if (sum != rsum) ++errs;
        int allmax = -2147483647 - 1;
        for (int l = 0; l < kWave; ++l)
            allmax = max(allmax, (int)((l * 2654435761u + trial * 40503u) % 1000u) - 500);
        if (wave_max(v) != allmax) ++errs;
    }
    atomicAdd(bad, errs);
}

hipError_t run_wave_selftest(int *d_bad, hipStream_t stream) {
    hipLaunchKernelGGL(wave_selftest_kernel, dim3(1), dim3(kWave), 0, stream, d_bad);
    return hipGetLastError();
}

}  // namespace mando
