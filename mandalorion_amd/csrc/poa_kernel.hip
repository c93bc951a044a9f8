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

#include <type_traits>

namespace mando {

// Workspace pointers carry the global address space explicitly: they are re-read from LDS per
// phase, and a generic pointer would make every access a flat_* op, which also counts on lgkmcnt and
// so would stall every LDS wait behind this wave's outstanding traceback stores.
#define GLB __attribute__((address_space(1)))
typedef GLB int gint;
typedef GLB uint8_t gu8;

struct Slot {
    gu8 *base;
    gint *gid, *gtab, *in_n, *out_n, *in_id, *out_id, *out_w, *sink_in, *src_out, *src_out_w;
    gint *order, *order2, *pos, *remrow, *desc, *rinfo;
    gu8 *tb, *kp;
    gint *sv, *qnode, *qtgt, *qflag, *qnb, *qoff, *qmslot, *ins, *insmm, *score, *nxt;
    gint *xpre;                                    // extra predecessor rows (> kPreInline), row * DCAP + k
    gint *wdesc, *wxpre, *wmap, *wlist, *wf, *wb;  // -S window rows (see build_window)
    gint *tnode;                                   // -S: node of each position of the previous read
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

// DPP forms (gfx9 DPP: row_shr:1/2/4/8, row_bcast:15/31, wave_shr:1) — VALU-latency wave scans
template <int CTRL, int RM, int BM>
__device__ __forceinline__ int dpp_mov(int old, int v) {
    return __builtin_amdgcn_update_dpp(old, v, CTRL, RM, BM, false);
}

// inclusive prefix max over the wave.  A lane without a DPP source keeps its own value (the
// identity of max), so every step is one v_max_i32_dpp.  Written as inline asm: the compiler does
// not fold update_dpp + max and serialises two scans through one temporary.  The s_nop pads cover
// the 2-wait-state VALU-write -> DPP-read hazard (the asm is opaque to the hazard recognizer).
#define MANDO_DPP_MAX(r, ctl) "v_max_i32_dpp " r ", " r ", " r " " ctl "\n"
#define MANDO_ROW_SHR1 "row_shr:1 row_mask:0xf bank_mask:0xf"
#define MANDO_ROW_SHR2 "row_shr:2 row_mask:0xf bank_mask:0xf"
#define MANDO_ROW_SHR4 "row_shr:4 row_mask:0xf bank_mask:0xf"
#define MANDO_ROW_SHR8 "row_shr:8 row_mask:0xf bank_mask:0xf"
#define MANDO_BCAST15 "row_bcast:15 row_mask:0xa bank_mask:0xf"
#define MANDO_BCAST31 "row_bcast:31 row_mask:0xc bank_mask:0xf"
__device__ __forceinline__ int dpp_incl_max(int v, int /*ident*/) {
    asm volatile("s_nop 1\n" MANDO_DPP_MAX("%0", MANDO_ROW_SHR1) "s_nop 1\n" MANDO_DPP_MAX("%0", MANDO_ROW_SHR2)
                 "s_nop 1\n" MANDO_DPP_MAX("%0", MANDO_ROW_SHR4) "s_nop 1\n" MANDO_DPP_MAX("%0", MANDO_ROW_SHR8)
                 "s_nop 1\n" MANDO_DPP_MAX("%0", MANDO_BCAST15) "s_nop 1\n" MANDO_DPP_MAX("%0", MANDO_BCAST31)
                 : "+v"(v));
    return v;
}
// two independent scans interleaved step by step (each hides part of the other's hazard)
__device__ __forceinline__ void dpp_incl_max2(int &a, int &b) {
    asm volatile("s_nop 1\n"
                 MANDO_DPP_MAX("%0", MANDO_ROW_SHR1) MANDO_DPP_MAX("%1", MANDO_ROW_SHR1) "s_nop 0\n"
                 MANDO_DPP_MAX("%0", MANDO_ROW_SHR2) MANDO_DPP_MAX("%1", MANDO_ROW_SHR2) "s_nop 0\n"
                 MANDO_DPP_MAX("%0", MANDO_ROW_SHR4) MANDO_DPP_MAX("%1", MANDO_ROW_SHR4) "s_nop 0\n"
                 MANDO_DPP_MAX("%0", MANDO_ROW_SHR8) MANDO_DPP_MAX("%1", MANDO_ROW_SHR8) "s_nop 0\n"
                 MANDO_DPP_MAX("%0", MANDO_BCAST15) MANDO_DPP_MAX("%1", MANDO_BCAST15) "s_nop 0\n"
                 MANDO_DPP_MAX("%0", MANDO_BCAST31) MANDO_DPP_MAX("%1", MANDO_BCAST31)
                 : "+v"(a), "+v"(b));
}

__device__ __forceinline__ int dpp_incl_sum(int v) {
    v += dpp_mov<0x111, 0xf, 0xf>(0, v);
    v += dpp_mov<0x112, 0xf, 0xf>(0, v);
    v += dpp_mov<0x114, 0xf, 0xf>(0, v);
    v += dpp_mov<0x118, 0xf, 0xf>(0, v);
    v += dpp_mov<0x142, 0xa, 0xf>(0, v);
    v += dpp_mov<0x143, 0xc, 0xf>(0, v);
    return v;
}

// lane l receives lane l-1's value; lane 0 receives `fill`
__device__ __forceinline__ int dpp_shr1(int v, int fill) { return dpp_mov<0x138, 0xf, 0xf>(fill, v); }

__device__ __forceinline__ unsigned long long lanemask_lt(int lane) {
    return (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
}

__device__ __forceinline__ int score_of(int a, int b, int match, int mismatch) {
    return (a == 4 || b == 4) ? 0 : (a == b ? match : -mismatch);
}

__device__ __forceinline__ gint *in_list(const Slot &s, const PoaRunArgs &a, int v) {
    return v == kSink ? s.sink_in : s.in_id + (int64_t)v * a.caps.DCAP;
}
__device__ __forceinline__ int in_cap(const PoaRunArgs &a, int v) {
    return v == kSink ? a.caps.BIGCAP : a.caps.DCAP;
}
__device__ __forceinline__ gint *out_list(const Slot &s, const PoaRunArgs &a, int v) {
    return v == kSrc ? s.src_out : s.out_id + (int64_t)v * a.caps.DCAP;
}
__device__ __forceinline__ gint *out_wlist(const Slot &s, const PoaRunArgs &a, int v) {
    return v == kSrc ? s.src_out_w : s.out_w + (int64_t)v * a.caps.DCAP;
}
__device__ __forceinline__ int out_cap(const PoaRunArgs &a, int v) {
    return v == kSrc ? a.caps.BIGCAP : a.caps.DCAP;
}

// wave-level barrier that also orders this wave's global/LDS memory traffic.  Wave-local (no s_barrier):
// in a two-wave workgroup (wide launches, below) the serial phases run on wave 0 alone while wave 1 waits
// for DP rows; a one-wave workgroup's __syncthreads() compiles to exactly this (the backend drops the
// s_barrier of a single-wave workgroup).
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
// workgroup barrier of a two-wave workgroup (its waves' LDS and global writes ordered across it)
__device__ __forceinline__ void group_barrier() { __syncthreads(); }

// same-wave RAW through HBM (spilled rows, far row records): drain this wave's stores first
__device__ __forceinline__ void hbm_fence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup"); }

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v2i __attribute__((ext_vector_type(2)));
struct RowRec {
    int beg, end, am, soff;
};

// Predecessor bytes of a multi-predecessor row (the predecessor index of the M, E1 and E2 maxima per
// cell): rows with at most kKpPackMax predecessors pack them into one byte per cell (k0 | k1 << 2 |
// k2 << 4), rows with more keep three bytes per cell.  One byte per cell lets the backtrack's LDS
// window hold three times as many multi-predecessor rows.
constexpr int kKpPackMax = 4;
__device__ __forceinline__ int kp_stride(int pn) { return pn <= kKpPackMax ? 1 : 3; }
constexpr int kNodeKp3 = 1 << 30;  // backtrack window record: the row's predecessor bytes are 3 per cell
#ifndef MANDO_DESC_BATCH
#define MANDO_DESC_BATCH 16
#endif
// row descriptors staged in LDS per refill: 16 rows (512 B) keep a narrow launch with reads up to ~4.6 kb
// at 16 workgroups per CU (10,240 B of LDS each); 32 rows left it at 15 (r04)
constexpr int kDescBatch = MANDO_DESC_BATCH;
constexpr int kTbWin = 4096;          // backtrack: traceback byte window
constexpr int kBtRows = 64;           // backtrack: rows per window
constexpr int kKpWinMax = 2048;       // backtrack: predecessor-byte window (in the read buffer)

// DP phase: the H/E1/E2 ring, carried from row to row
struct DpLds {
    union {
        int ring[kRing][3][kChunk];      // H, E1out, E2out of the last kRing narrow rows, col & 127
        short ring16[kRing16][3][kChunk];  // the same in 16-bit mode (run_dp<SC, true>): twice the rows
    };
};
// backtrack phase (the DP state is dead by then); the predecessor-byte window uses the read's
// dynamic buffer, which the next read's DP re-stages
struct BtLds {
    uint8_t tb[kTbWin];
    int md[kBtRows][8];  // per window row: tb offset, kp offset, node, predecessors 0..4
};

// LDS per wave: ~8.4 KB static + the read (4-bit codes, dynamic: sized by the batch's longest read),
// so 16 waves fit per CU (4 per SIMD) for reads up to ~3.5 kb.
struct alignas(16) SharedState {
    union {
        DpLds dp;
        BtLds bt;
    };
    int4 rrow[kRowRing];            // beg, end, argmax, spill offset of the last kRowRing rows
    int desc[kDescBatch][kDescInts];  // descriptors of the current row batch
    Slot slot;                      // this wave's workspace arrays (read per phase, see slot_of)
    gint *order0, *order1;          // the two topological-order buffers (slot.order swaps them)
    PoaRunArgs args;                  // kernel arguments (read per phase, see args_of)
    // -S window DP: slot.desc / slot.xpre / slot.qnode point at the window's arrays while it runs;
    // the sink of the DP is node win_sink, and a node's row is wmap[pos - win_pb] inside [pb, pe]
    int win_on, win_sink, win_pb, win_pe;
    gint *desc_full, *xpre_full, *qnode_full;
    uint64_t tmark;                 // MANDO_PROF: the last phase boundary of the -S path (prof_mark)
    int slot_idx;                   // this workgroup's workspace slot (one_group launches claim one)

};
static_assert(sizeof(BtLds) <= sizeof(DpLds), "backtrack window must fit the DP scratch");
// -S team leader (seeded launches): the group / read in progress between jobs (seeded_main).  In the
// dynamic LDS after the read's buffer (poa_dyn_lds), so one-wave unseeded workgroups do not carry it.
struct LeadState {
    int64_t r1, rd, cells;
    uint64_t job;
    int g, n, ng, st, pending, active, np, item, qlen;
};
static_assert(sizeof(LeadState) <= kLeadBytes, "poa_kernel.h kLeadBytes");

extern __shared__ __attribute__((aligned(16))) uint8_t g_qnib[];  // dynamic: the read, 4-bit codes
__device__ __forceinline__ LeadState &lead_of(SharedState &sh) {
    return *reinterpret_cast<LeadState *>(g_qnib + ((bcast0(sh.args.qlds) + 15) & ~15));
}

// Ring geometry by launch kind: RW = kChunk keeps the ring in the static LDS (col & 127); a wide launch
// (RW = kWideRing) keeps 256-column rows at the start of the dynamic LDS and the read's nibbles after it.
template <int RW>
__device__ __forceinline__ uint8_t *qnib() {
    if constexpr (RW == kChunk) return g_qnib;
    else return g_qnib + kWideRingBytes;
}
template <int RW>
__device__ __forceinline__ short *ring16_row(const SharedState &sh, int row) {
    if constexpr (RW == kChunk) return const_cast<short *>(&sh.dp.ring16[row][0][0]);
    else return reinterpret_cast<short *>(g_qnib) + row * 3 * RW;
}
// backtrack windows: the traceback bytes in the static BtLds and the predecessor bytes in the read's
// buffer; a wide launch's ring is dead during the backtrack, so its windows are twice / four times as
// large there (predecessor bytes [0, 8 KB), traceback bytes [8 KB, 16 KB) of the dynamic LDS)
template <int RW>
__device__ __forceinline__ constexpr int bt_tb_win() { return RW == kChunk ? 4096 : 8192; }
template <int RW>
__device__ __forceinline__ constexpr int bt_kp_win() { return RW == kChunk ? 2048 : 8192; }
template <int RW>
__device__ __forceinline__ uint8_t *bt_tb(const SharedState &sh) {
    if constexpr (RW == kChunk) return const_cast<uint8_t *>(sh.bt.tb);
    else return g_qnib + bt_kp_win<RW>();
}

template <int RW>
__device__ __forceinline__ int *ring32_row(const SharedState &sh, int row) {
    if constexpr (RW == kChunk) return const_cast<int *>(&sh.dp.ring[row][0][0]);
    else return reinterpret_cast<int *>(g_qnib) + row * 3 * RW;
}

// Each phase re-reads the few workspace pointers it needs from LDS behind a compiler barrier, so
// the ~30 loop-invariant 64-bit pointers are not kept live (and spilled) across the whole
// persistent loop; unused fields of the copy are dead and never loaded.
__device__ __forceinline__ int64_t uni64(int64_t v) {
    const int lo = __builtin_amdgcn_readfirstlane((int)(v & 0xffffffff));
    const int hi = __builtin_amdgcn_readfirstlane((int)(v >> 32));
    return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
template <class T>
__device__ __forceinline__ T *uniptr(T *p) {
    return (T *)(uintptr_t)uni64((int64_t)(uintptr_t)p);
}

// LDS-loaded values are divergent as far as the compiler knows: readfirstlane every field so
// pointer arithmetic, capacity checks and loop bounds stay on the scalar unit.
__device__ __forceinline__ Slot slot_of(SharedState &sh) {
    asm volatile("" ::: "memory");
    Slot s = sh.slot;
    s.base = uniptr(s.base);
    s.gid = uniptr(s.gid);
    s.gtab = uniptr(s.gtab);
    s.in_n = uniptr(s.in_n);
    s.out_n = uniptr(s.out_n);
    s.in_id = uniptr(s.in_id);
    s.out_id = uniptr(s.out_id);
    s.out_w = uniptr(s.out_w);
    s.sink_in = uniptr(s.sink_in);
    s.src_out = uniptr(s.src_out);
    s.src_out_w = uniptr(s.src_out_w);
    s.order = uniptr(s.order);
    s.order2 = uniptr(s.order2);
    s.pos = uniptr(s.pos);
    s.remrow = uniptr(s.remrow);
    s.desc = uniptr(s.desc);
    s.rinfo = uniptr(s.rinfo);
    s.tb = uniptr(s.tb);
    s.kp = uniptr(s.kp);
    s.sv = uniptr(s.sv);
    s.qnode = uniptr(s.qnode);
    s.qtgt = uniptr(s.qtgt);
    s.qflag = uniptr(s.qflag);
    s.qnb = uniptr(s.qnb);
    s.qoff = uniptr(s.qoff);
    s.qmslot = uniptr(s.qmslot);
    s.ins = uniptr(s.ins);
    s.insmm = uniptr(s.insmm);
    s.score = uniptr(s.score);
    s.nxt = uniptr(s.nxt);
    s.xpre = uniptr(s.xpre);
    s.wdesc = uniptr(s.wdesc);
    s.wxpre = uniptr(s.wxpre);
    s.wmap = uniptr(s.wmap);
    s.wlist = uniptr(s.wlist);
    s.wf = uniptr(s.wf);
    s.wb = uniptr(s.wb);
    s.tnode = uniptr(s.tnode);
    return s;
}
__device__ __forceinline__ PoaRunArgs args_of(SharedState &sh) {
    asm volatile("" ::: "memory");
    PoaRunArgs a = sh.args;
    a.caps.NC = bcast0(a.caps.NC);
    a.caps.DCAP = bcast0(a.caps.DCAP);
    a.caps.BIGCAP = bcast0(a.caps.BIGCAP);
    a.caps.QC = bcast0(a.caps.QC);
    a.caps.TBC = uni64(a.caps.TBC);
    a.caps.KPC = uni64(a.caps.KPC);
    a.caps.SVC = uni64(a.caps.SVC);
    a.match = bcast0(a.match);
    a.mismatch = bcast0(a.mismatch);
    a.o1 = bcast0(a.o1);
    a.e1 = bcast0(a.e1);
    a.o2 = bcast0(a.o2);
    a.e2 = bcast0(a.e2);
    a.band_b = bcast0(a.band_b);
    a.band_f = __int_as_float(bcast0(__float_as_int(a.band_f)));
    a.prof = uniptr(a.prof);
    a.dbg = bcast0(a.dbg);
    a.seq = uniptr(a.seq);
    a.seq_off = uniptr(a.seq_off);
    a.grp_off = uniptr(a.grp_off);
    a.gorder = uniptr(a.gorder);
    a.counter = uniptr(a.counter);
    a.cons = uniptr(a.cons);
    a.cons_off = uniptr(a.cons_off);
    a.cons_len = uniptr(a.cons_len);
    a.cells = uniptr(a.cells);
    a.status = uniptr(a.status);
    a.n_groups = bcast0(a.n_groups);
    a.par_item = uniptr(a.par_item);
    a.par_n = uniptr(a.par_n);
    a.par_t = uniptr(a.par_t);
    a.par_q = uniptr(a.par_q);
    a.pc = bcast0(a.pc);
    a.seed_k = bcast0(a.seed_k);
    return a;
}

// ---------------------------------------------------------------------------------------------
// first read: a chain SRC -> n0 -> ... -> n(L-1) -> SINK
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ int init_chain(SharedState &sh, const uint8_t *q, int L, int lane, int &n) {
    const PoaRunArgs a = args_of(sh);
    Slot s = slot_of(sh);
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
// Per-row graph facts of one 64-row chunk.  The loads form three dependent levels (order ->
// node arrays / adjacency rows -> pos), each issued for all edges at once, so a chunk costs three
// memory round trips; build_desc gathers two chunks before using either.
struct DescRow {
    int v, vb, pn, bh, far;
    int pre[kPreInline];
};
constexpr int kOutInline = 4;  // out-edges gathered in the batched levels (more: a serial tail)

__device__ __forceinline__ DescRow desc_gather(const PoaRunArgs &a, const Slot &s, int r, bool valid, int ring) {
    DescRow d;
    d.v = 0;
    d.vb = 4;
    d.pn = 0;
    d.bh = -1;
    d.far = 0;
#pragma unroll
    for (int k = 0; k < kPreInline; ++k) d.pre[k] = -1;
    if (!valid) return d;
    const int v = s.order[r];
    d.v = v;
    // level 2: node arrays and the leading adjacency entries (capacity >= 16, so reading past the
    // list's length stays inside the node's row)
    const int pn = s.in_n[v], on = s.out_n[v];
    d.vb = s.base[v];
    const gint *il = in_list(s, a, v);
    const gint *ol = out_list(s, a, v);
    const gint *ow = out_wlist(s, a, v);
    int iid[kPreInline], oid[kOutInline], owt[kOutInline];
#pragma unroll
    for (int k = 0; k < kPreInline; ++k) iid[k] = il[k];
#pragma unroll
    for (int k = 0; k < kOutInline; ++k) {
        oid[k] = ol[k];
        owt[k] = ow[k];
    }
    d.pn = pn;
    // level 3: topological positions
#pragma unroll
    for (int k = 0; k < kPreInline; ++k)
        if (k < pn) d.pre[k] = s.pos[iid[k]];
    // rare rows with more predecessors: the rest go to the row's xpre list (read by the generic row
    // and the backtrack, which never look predecessors up through the graph)
    for (int k = kPreInline; k < pn; ++k) s.xpre[(int64_t)r * a.caps.DCAP + k] = s.pos[il[k]];
    int opos[kOutInline];
#pragma unroll
    for (int k = 0; k < kOutInline; ++k) opos[k] = (k < on) ? s.pos[oid[k]] : 0;
    int bw = -2147483647 - 1, maxd = 0, bh = -1;
#pragma unroll
    for (int k = 0; k < kOutInline; ++k) {
        if (k < on) {
            if (owt[k] > bw) {
                bw = owt[k];
                bh = opos[k];
            }
            maxd = max(maxd, opos[k] - r);
        }
    }
    for (int k = kOutInline; k < on; ++k) {
        const int po = s.pos[ol[k]];
        const int wg = ow[k];
        if (wg > bw) {
            bw = wg;
            bh = po;
        }
        maxd = max(maxd, po - r);
    }
    d.bh = bh;
    d.far = maxd >= ring ? 1 : 0;
    return d;
}

// remain (pointer jumping within the chunk, the chunk above's values via prev_val) and the
// descriptor store of one chunk
__device__ __forceinline__ void desc_finish(const Slot &s, const DescRow &d, int c, int n, int lane, int ring,
                                            int &prev_val) {
    const int r = c * kWave + lane;
    const bool valid = r < n;
    const int bh = d.bh;
    const int lo_next = (c + 1) * kWave, lo_next2 = (c + 2) * kWave;
    const int idx_prev = (bh >= lo_next && bh < lo_next2) ? bh - lo_next : lane;
    const int from_prev = __shfl(prev_val, idx_prev, kWave);
    int val = 0, ptr = -1;
    if (valid) {
        if (d.v == kSink) {
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
        const int pn = d.pn;
        s.remrow[r] = val;
        gint *dd = s.desc + (int64_t)r * kDescInts;
        dd[0] = d.v;
        // bit 15: the row's predecessor structure allows the fast row (1-2 predecessors, all
        // within the LDS ring); the band-dependent tests are made per read
        const int sfast = (pn == 1 || pn == 2) && r - d.pre[0] < ring && (pn == 1 || r - d.pre[1] < ring);
        // bit 14: 3..kPreInline predecessors, all within the LDS ring (the 16-bit row loop's
        // multi-predecessor fast row)
        bool near = pn >= 3 && pn <= kPreInline;
#pragma unroll
        for (int k = 0; k < kPreInline; ++k) near = near && (k >= pn || r - d.pre[k] < ring);
        dd[1] = d.vb | (d.far << 8) | (near ? (1 << 14) : 0) | (sfast << 15) | (pn << 16);
        dd[2] = val;
#pragma unroll
        for (int k = 0; k < kPreInline; ++k) dd[3 + k] = d.pre[k];
    }
    prev_val = val;
    wave_sync();
}

__device__ __forceinline__ void build_desc(SharedState &sh, int n, int lane, int ring) {
    const PoaRunArgs a = args_of(sh);
    Slot s = slot_of(sh);
    const int nch = (n + kWave - 1) / kWave;
    int prev_val = 0;
    for (int c = nch - 1; c >= 0; c -= 2) {
        const int r = c * kWave + lane, r2 = r - kWave;
        const DescRow d = desc_gather(a, s, r, r < n, ring);
        const DescRow d2 = desc_gather(a, s, r2, c >= 1, ring);
        desc_finish(s, d, c, n, lane, ring, prev_val);
        if (c >= 1) desc_finish(s, d2, c - 1, n, lane, ring, prev_val);
    }
}

// ---------------------------------------------------------------------------------------------
// -S window rows (oracle/poa_ref.c align_window): the topological rows r in [pos B, pos E] that are
// reachable from B and reach E, in order, become window rows 0..m-1 (B the source row, E the sink).
// Built from the whole-graph descriptors of this read (build_desc at the 32-bit ring depth, so their
// `far` bits are safe for both ring depths: a window only shortens row distances).
//   1. forward reachability, 64 rows at a time: a row is reached when a predecessor is; predecessors
//      in earlier chunks are read from wf[], the chunk's own chain is resolved by a scalar walk over
//      the lanes (bit masks of in-chunk predecessors);
//   2. backward reachability from E the same way, descending: reached rows mark their earlier-chunk
//      predecessors in wb[] (idempotent stores), the chunk's own rows by a descending scalar walk;
//   3. compaction (ballot prefix) into wmap (topological -> window row) and wlist (window -> topological);
//   4. window descriptors: predecessors outside the window dropped (in in-edge order), remain taken
//      relative to E (remain[v] - remain[E] - 1), fast-row bits recomputed on window distances.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ int build_window(SharedState &sh, int B, int E, int lane, int ring, int &m_out) {
    const PoaRunArgs a = args_of(sh);
    Slot s = slot_of(sh);
    const int DC = a.caps.DCAP;
    const int pB = bcast0(s.pos[B]), pE = bcast0(s.pos[E]);
    if (pE <= pB) return kStInternal;
    const int span = pE - pB + 1;
    for (int x = lane; x < span; x += kWave) s.wb[x] = 0;
    hbm_fence();
    wave_sync();
    // 1. forward
    for (int c0 = 0; c0 < span; c0 += kWave) {
        const int x = c0 + lane;
        bool ext = false;
        uint64_t pm = 0;
        if (x < span) {
            if (x == 0) {
                ext = true;
            } else {
                const gint *dd = s.desc + (int64_t)(pB + x) * kDescInts;
                const int pn = dd[1] >> 16;
                for (int k = 0; k < pn; ++k) {
                    const int p = (k < kPreInline ? dd[3 + k] : s.xpre[(int64_t)(pB + x) * DC + k]) - pB;
                    if (p < 0) continue;
                    if (p < c0) ext |= s.wf[p] != 0;
                    else pm |= 1ull << (p - c0);
                }
            }
        }
        const uint64_t eb = __ballot(ext);
        uint64_t m = 0;
        const int lim = min(kWave, span - c0);
        for (int l = 0; l < lim; ++l)
            if (((eb >> l) & 1) || (readlane64(pm, l) & m)) m |= 1ull << l;
        if (x < span) s.wf[x] = (int)((m >> lane) & 1);
        hbm_fence();
        wave_sync();
    }
    // 2. backward
    for (int c0 = ((span - 1) / kWave) * kWave; c0 >= 0; c0 -= kWave) {
        const int x = c0 + lane;
        uint64_t pm = 0;
        bool ext = false;
        if (x < span) {
            ext = x == span - 1 || s.wb[x] != 0;
            if (x > 0) {
                const gint *dd = s.desc + (int64_t)(pB + x) * kDescInts;
                const int pn = dd[1] >> 16;
                for (int k = 0; k < pn; ++k) {
                    const int p = (k < kPreInline ? dd[3 + k] : s.xpre[(int64_t)(pB + x) * DC + k]) - pB;
                    if (p >= c0) pm |= 1ull << (p - c0);
                }
            }
        }
        const uint64_t eb = __ballot(ext);
        uint64_t m = 0;
        const int lim = min(kWave, span - c0);
        for (int l = lim - 1; l >= 0; --l)
            if (((eb | m) >> l) & 1) m |= (1ull << l) | readlane64(pm, l);
        const bool on = x < span && ((m >> lane) & 1);
        if (x < span) s.wb[x] = on ? 1 : 0;
        if (on && x > 0) {  // reached: so are its predecessors in earlier chunks
            const gint *dd = s.desc + (int64_t)(pB + x) * kDescInts;
            const int pn = dd[1] >> 16;
            for (int k = 0; k < pn; ++k) {
                const int p = (k < kPreInline ? dd[3 + k] : s.xpre[(int64_t)(pB + x) * DC + k]) - pB;
                if (p >= 0 && p < c0) s.wb[p] = 1;
            }
        }
        hbm_fence();
        wave_sync();
    }
    // 3. compaction
    int m = 0;
    for (int c0 = 0; c0 < span; c0 += kWave) {
        const int x = c0 + lane;
        const bool in = x < span && s.wf[x] != 0 && s.wb[x] != 0;
        const uint64_t b = __ballot(in);
        const int idx = m + __popcll(b & lanemask_lt(lane));
        if (x < span) s.wmap[x] = in ? idx : -1;
        if (in) s.wlist[idx] = pB + x;
        m += __popcll(b);
    }
    hbm_fence();
    wave_sync();
    // 4. window descriptors
    const int remE = bcast0(s.remrow[pE]);
    for (int i0 = 0; i0 < m; i0 += kWave) {
        const int i = i0 + lane;
        if (i < m) {
            const int r = s.wlist[i];
            const gint *dd = s.desc + (int64_t)r * kDescInts;
            const int d1 = dd[1], pn = d1 >> 16;
            int pre[kPreInline];
#pragma unroll
            for (int k = 0; k < kPreInline; ++k) pre[k] = -1;
            int np = 0;
            for (int k = 0; k < pn; ++k) {
                const int p = k < kPreInline ? dd[3 + k] : s.xpre[(int64_t)r * DC + k];
                if (p < pB || p > pE) continue;
                const int wp = s.wmap[p - pB];
                if (wp < 0) continue;
                if (np < kPreInline) {
#pragma unroll
                    for (int t = 0; t < kPreInline; ++t)
                        if (t == np) pre[t] = wp;
                } else {
                    s.wxpre[(int64_t)i * DC + np] = wp;
                }
                ++np;
            }
            const int sfast = (np == 1 || np == 2) && i - pre[0] < ring && (np == 1 || i - pre[1] < ring);
            bool near = np >= 3 && np <= kPreInline;
#pragma unroll
            for (int k = 0; k < kPreInline; ++k) near = near && (k >= np || i - pre[k] < ring);
            gint *wd = s.wdesc + (int64_t)i * kDescInts;
            wd[0] = dd[0];
            wd[1] = (d1 & 0x1ff) | (near ? (1 << 14) : 0) | (sfast << 15) | (np << 16);
            wd[2] = s.remrow[r] - remE - 1;
#pragma unroll
            for (int k = 0; k < kPreInline; ++k) wd[3 + k] = pre[k];
        }
    }
    hbm_fence();
    wave_sync();
#ifdef MANDO_TEAM_DEBUG
    if (m == 0) {
        int nf = 0, nb = 0;
        for (int x = lane; x < span; x += kWave) {
            nf += s.wf[x] != 0;
            nb += s.wb[x] != 0;
        }
        nf = wave_incl_sum(nf, lane);
        nb = wave_incl_sum(nb, lane);
        if (lane == kWave - 1)
            printf("[bw] block %d B %d E %d pB %d pE %d span %d wf %d wb %d ring %d\n", (int)blockIdx.x, B, E, pB, pE, span, nf, nb, ring);
    }
#endif
    m_out = m;
    return kStOk;
}

__device__ __forceinline__ RowRec load_rowrec(const SharedState &sh, const Slot &s, int r, int p) {
    int4 x;
    if (r - p < kRowRing) {
        x = sh.rrow[p % kRowRing];
    } else {
        // rare: record of a row more than kRowRing rows back (written by this wave long ago);
        // consumed (readfirstlane) inside the branch so the common path never waits on vmcnt
        hbm_fence();
        const gint *g = s.rinfo + (int64_t)p * kRowInfoInts;
        x = make_int4(bcast0(g[0]), bcast0(g[1]), bcast0(g[4]), bcast0(g[5]));
    }
    RowRec rr;
    rr.beg = x.x;
    rr.end = x.y;
    rr.am = x.z;
    rr.soff = x.w;
    return rr;
}

// A row's band is processed in 128-column chunks starting at the even column cb0 = beg & ~1.
// "Narrow" rows (one chunk) keep H/E1/E2 in the LDS ring, indexed by absolute column & 127; rows
// that are wider, or that have a successor >= kRing rows later, are (also) spilled to HBM as three
// planes of nchunk*128 ints starting at column cb0; a (rare) predecessor outside the ring is read
// from those planes.
template <int RW = kChunk>
__device__ __forceinline__ bool row_narrow(int beg, int end) { return end - (beg & ~1) < RW; }
// rows of H/E1/E2 the LDS ring holds: the 16-bit ring fits twice as many in the same bytes
template <bool R16>
__device__ __forceinline__ constexpr int ring_rows() { return R16 ? kRing16 : kRing; }
__device__ __forceinline__ int row_spill_width(int beg, int end) {
    return ((end - (beg & ~1)) / kChunk + 1) * kChunk;
}
template <bool R16, int RW>
__device__ __forceinline__ bool pre_in_ring(int r, int p, const RowRec &pr) {
    return (r - p < ring_rows<R16>()) && row_narrow<RW>(pr.beg, pr.end);
}

// Scoring: the reference always runs `abpoa -M 5` with default gaps, so that case is compiled with
// constants (no quarter-rate multiplies, fewer live scalars); any other parameter set uses the
// runtime-valued variant of the same kernel.
struct DefaultScores {
    static constexpr int match = 5, mismatch = 4, o1 = 4, e1 = 2, o2 = 24, e2 = 1;
};
struct RuntimeScores {
    int match, mismatch, o1, e1, o2, e2;
};

struct DpState {
    int tb_used, kp_used, sv_used;
    int r16bad;     // 16-bit mode left its safe range: re-align the read in 32-bit mode
    uint32_t r16acc;  // per-lane min of (H - kR16Low) over valid fast-row columns (16-bit mode)
    int cells;  // DP cells of this read (< 2^31: a read's band cells)
    uint64_t seg[4];
};

#ifdef MANDO_STAMPS
#define STAMP(var) uint64_t var; asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(var)::"memory")
#else
#define STAMP(var) const uint64_t var = 0
#endif

// code of the query base consumed by column j (base j-1): nibble j of the shifted stream, 4 for
// column 0 and every column past the read
template <int RW>
__device__ __forceinline__ int qcol(int j) {
    return (qnib<RW>()[j >> 1] >> ((j & 1) << 2)) & 0xf;
}

// Rare-case predecessor records (more than kPreInline predecessors, or a predecessor whose record
// left the LDS row ring): lane k gathers predecessor k's record from HBM.  The loads are consumed
// inside this uniform branch, so the common path never carries an outstanding load into an s_waitcnt.
__device__ __forceinline__ void pre_records_slow(const PoaRunArgs &a, const Slot &s, SharedState &sh, int r,
                                                 int node, int pn, const int *dl, int lane, int &pP, int &pB,
                                                 int &pE, int &pA, int &pS) {
    hbm_fence();
    if (lane < pn) {
        const int p = (lane < kPreInline) ? dl[3 + lane] : s.xpre[(int64_t)r * a.caps.DCAP + lane];
        int4 x;
        if (r - p < kRowRing) {
            x = sh.rrow[p % kRowRing];
        } else {
            const gint *g = s.rinfo + (int64_t)p * kRowInfoInts;
            x = make_int4(g[0], g[1], g[4], g[5]);
        }
        pP = p;
        pB = x.x;
        pE = x.y;
        pA = x.z;
        pS = x.w;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // consume here (see above)
}

// traceback byte of one cell (layout in poa_kernel.h)
__device__ __forceinline__ int tb_bits(int H, int M, int X1, int X2, int F1, int oe1, int e1, int oe2, int e2, int G1,
                                       int P1, int G2, int P2) {
    return (M != H ? kTbNM : 0) | (X1 != H ? kTbNX1 : 0) | (X2 != H ? kTbNX2 : 0) | (F1 != H ? kTbNF1 : 0) |
           (H - oe1 < X1 - e1 ? kTbE1Ext : 0) | (H - oe2 < X2 - e2 ? kTbE2Ext : 0) | (G1 < P1 ? kTbF1ExtNext : 0) |
           (G2 < P2 ? kTbF2ExtNext : 0);
}

// source of H[i][j] from its traceback byte: 0 M, 1 E1, 2 E2, 3 F1, 4 F2 (k1/k2: predecessor index
// of the E1/E2 maxima, 0 on single-predecessor rows)
__device__ __forceinline__ int tb_type(int t, int k1, int k2) {
    if (!(t & kTbNM)) return 0;
    const bool x1 = !(t & kTbNX1), x2 = !(t & kTbNX2);
    if (x1 && x2) return k1 <= k2 ? 1 : 2;
    if (x1) return 1;
    if (x2) return 2;
    return (t & kTbNF1) ? 4 : 3;
}

__device__ __forceinline__ bool in_band(int col, int b, int e) {
    return (unsigned)(col - b) <= (unsigned)(e - b);
}

// Ring access for the generic row in both modes.  16-bit mode stores values clamped to int16
// (-inf = -32768); the 32-bit mode stores kNegInf.  Columns are absolute & (RW - 1).
__device__ __forceinline__ int clamp16(int v) { return min(max(v, -32768), 32767); }
template <bool R16, int RW>
__device__ __forceinline__ int ring_get(const SharedState &sh, int row, int plane, int col) {
    if constexpr (R16) return ring16_row<RW>(sh, row)[plane * RW + col];
    else return ring32_row<RW>(sh, row)[plane * RW + col];
}
// (col, col+1) of one plane; col even
template <bool R16, int RW>
__device__ __forceinline__ int2 ring_get2(const SharedState &sh, int row, int plane, int col) {
    if constexpr (R16) {
        const uint32_t w = *reinterpret_cast<const uint32_t *>(ring16_row<RW>(sh, row) + plane * RW + col);
        return make_int2((int)(short)(w & 0xffff), (int)w >> 16);
    } else {
        return *reinterpret_cast<const int2 *>(ring32_row<RW>(sh, row) + plane * RW + col);
    }
}
template <bool R16, int RW>
__device__ __forceinline__ void ring_put2(SharedState &sh, int row, int plane, int col, int a, bool va, int b,
                                          bool vb) {
    if constexpr (R16) {
        const uint32_t lo = (uint32_t)(va ? clamp16(a) : -32768) & 0xffff;
        const uint32_t hi = (uint32_t)(vb ? clamp16(b) : -32768) << 16;
        *reinterpret_cast<uint32_t *>(ring16_row<RW>(sh, row) + plane * RW + col) = lo | hi;
    } else {
        *reinterpret_cast<int2 *>(ring32_row<RW>(sh, row) + plane * RW + col) =
            make_int2(va ? a : kNegInf, vb ? b : kNegInf);
    }
}

// 16-bit mode is exact when every finite value fits with room to spare (see kR16Low) and the
// biased score table fits in bytes.  No score exceeds match * qlen, and the gap terms of a row add
// at most (e1 + e2) * RW + o1 + o2 on top; a read whose scores would not fit is shifted down by a
// constant (every value of every row, the source row included: the DP is translation-invariant), as
// long as the shift leaves room above the -inf band for the low scores (8000 or more; a read that
// still leaves the safe range is re-aligned in 32-bit mode).  Reads up to ~6.4 kb (default scores)
// are not shifted.
constexpr int kR16NoBias = 1 << 30;
template <class SC, int RW>
__device__ __forceinline__ int r16_bias(const SC &sc, int qlen) {
    const bool ok = sc.match >= 0 && sc.mismatch >= 0 && sc.match + sc.mismatch <= 255 && sc.e1 >= 0 && sc.e2 >= 0 &&
                    sc.o1 >= 0 && sc.o2 >= 0 && (sc.e1 + sc.e2) * kChunk + sc.o1 + sc.o2 <= 2000;
    const int64_t top = (int64_t)sc.match * qlen + (int64_t)(sc.e1 + sc.e2) * RW + sc.o1 + sc.o2 + 64;
    const int64_t b = top > 32767 ? 32767 - top : 0;
    return ok && b >= -20000 ? (int)b : kR16NoBias;
}
template <class SC, int RW>
__device__ __forceinline__ bool r16_eligible(const SC &sc, int qlen) {
    return r16_bias<SC, RW>(sc, qlen) != kR16NoBias;
}

// 16-bit mode: a finite H must never be confused with a -inf-derived one (those stay below
// kR16Low; every value moves by a bounded step per cell, so one that drifts between the classes
// passes through [kR16Low, kR16High) and is caught); the read is then re-aligned in 32-bit mode.
constexpr int kR16Low = -31000, kR16High = -28000;

// One DP row r.  Predecessor k's record lives in lane k (pP row, pB/pE band, pA argmax, pS spill
// offset); the common case (every predecessor in the LDS ring) reads values with 4 LDS ops per
// predecessor and no global memory traffic except the traceback stores.  RW: ring columns per row
// (a wide launch keeps rows of up to two chunks in the ring; those rows hold only the columns they
// wrote, which the band masks below cover).
template <class SC, bool R16, int RW = kChunk>
__device__ __forceinline__ int dp_row(const PoaRunArgs &a, const SC &sc, Slot &s, SharedState &sh, int qlen,
                                      int w, int r, int lane, DpState &ds) {
    const int e1 = sc.e1, e2 = sc.e2, oe1 = sc.o1 + sc.e1, oe2 = sc.o2 + sc.e2;
    const int IDENT = -(1 << 30);
    STAMP(ts0);
    const int *dl = &sh.desc[r & (kDescBatch - 1)][0];
    const int node = dl[0];
    const int d1 = dl[1];
    const int rem = dl[2];
    const int vb = d1 & 0xff, far = (d1 >> 8) & 1, pn = d1 >> 16;
    if (pn > kWave) return kStUnsupported;
    // ---- predecessor records, lane-parallel
    int pP = 0, pB = 0, pE = -1, pA = 0, pS = -1;
    bool slow = pn > kPreInline;
    if (!slow) {
        if (lane < pn) pP = dl[3 + lane];
        slow = __ballot(lane < pn && r - pP >= kRowRing) != 0;
    }
    if (slow) {
        pre_records_slow(a, s, sh, r, node, pn, dl, lane, pP, pB, pE, pA, pS);
    } else if (lane < pn) {
        const int4 x = sh.rrow[pP % kRowRing];
        pB = x.x;
        pE = x.y;
        pA = x.z;
        pS = x.w;
    }
    // ---- band
    int beg, end;
    if (r == 0) {
        beg = 0;
        end = min(qlen, max(0, qlen - rem) + w);
    } else {
        int posL = 2147483647, posR = -2147483647 - 1;
        for (int k = 0; k < pn; ++k) {
            const int am = readlane(pA, k) + 1;
            posL = min(posL, am);
            posR = max(posR, am);
        }
        const int x = qlen - rem;
        beg = max(0, min(posL, x) - w);
        end = min(qlen, max(posR, x) + w);
    }
    constexpr int kR = ring_rows<R16>();
    const bool pring = (r - pP < kR) && row_narrow<RW>(pB, pE);
    const bool all_ring = __ballot(lane < pn && !pring) == 0;
    const int cb0 = beg & ~1;
    const int span = end - cb0 + 1;
    const int nchunk = (span + kChunk - 1) / kChunk;
    const bool narrow = nchunk <= RW / kChunk;  // kept in the ring
    const bool spill = far || !narrow;
    const int wa = nchunk * kChunk;
    const int tbw = (span + 3) & ~3;
    const bool multi = pn > 1;
    if (ds.tb_used + tbw > (int)a.caps.TBC) return kStCap;
    if (multi && ds.kp_used + 3 * tbw > (int)a.caps.KPC) return kStCap;
    if (spill && ds.sv_used + 3 * wa > (int)a.caps.SVC) return kStCap;
    // 32-bit offsets from the slot's arrays (the stores then use a scalar base + vector offset)
    const int ks = kp_stride(pn);
    const int tbbase = (int)ds.tb_used - cb0;       // traceback byte of column j: tb[tbbase + j]
    const int kpbase = (int)ds.kp_used - ks * cb0;  // predecessor byte(s) of column j: kp[kpbase + ks*j]
    const int soff = spill ? (int)ds.sv_used : -1;
    const int svbase = (int)ds.sv_used - cb0;       // plane pl, column j: sv[svbase + pl*wa + j]
    ds.tb_used += tbw;
    if (multi) ds.kp_used += ks * tbw;
    if (spill) ds.sv_used += 3 * wa;
    ds.cells += end - beg + 1;
    STAMP(ts1);
    uint64_t ts2 = ts1, ts3 = ts1;

    int best = -2147483647 - 1, besti = beg;
    int carry1 = kNegInf + oe1 + e1 * (beg - 1);
    int carry2 = kNegInf + oe2 + e2 * (beg - 1);
    for (int c = 0; c < nchunk; ++c) {
        const int cb = cb0 + c * kChunk;
        const int j0 = cb + 2 * lane, j1 = j0 + 1;
        const bool va = j0 >= beg && j0 <= end, vbb = j1 <= end;
        int Ha, Hb, E1a, E1b, E2a, E2b;
        int tpair = 0;
        if (r == 0) {
            // source row: H[0][0] = 0, H[0][j] = max(-(o1+e1 j), -(o2+e2 j)) (+ the 16-bit bias)
            int B = 0;
            if constexpr (R16) B = r16_bias<SC, RW>(sc, qlen);  // eligible: the caller checked
            Ha = B + ((j0 == 0) ? 0 : max(-(sc.o1 + e1 * j0), -(sc.o2 + e2 * j0)));
            Hb = B + max(-(sc.o1 + e1 * j1), -(sc.o2 + e2 * j1));
            E1a = Ha - oe1;
            E1b = Hb - oe1;
            E2a = Ha - oe2;
            E2b = Hb - oe2;
        } else {
            const int qa = qcol<RW>(j0), qb = qcol<RW>(j1);
            int Mva, Mvb, X1a, X1b, X2a, X2b;
            int mka = 0, mkb = 0, k1a = 0, k1b = 0, k2a = 0, k2b = 0;
            const int ia = (j0 - 1) & (RW - 1), ib = j0 & (RW - 1);
            if (all_ring && pn == 1) {
                // the common row: one predecessor, in the ring
                const int p0 = readlane(pP, 0), b0 = readlane(pB, 0), e0 = readlane(pE, 0);
                const int pr = p0 % kR;
                const int hA = ring_get<R16, RW>(sh, pr, 0, ia), hB = ring_get<R16, RW>(sh, pr, 0, ib);
                const int2 x1 = ring_get2<R16, RW>(sh, pr, 1, ib);
                const int2 x2 = ring_get2<R16, RW>(sh, pr, 2, ib);
                const bool inA = in_band(j0 - 1, b0, e0), inB = in_band(j0, b0, e0),
                           inC = in_band(j1, b0, e0);
                Mva = inA ? hA : kNegInf;
                Mvb = inB ? hB : kNegInf;
                X1a = inB ? x1.x : kNegInf;
                X2a = inB ? x2.x : kNegInf;
                X1b = inC ? x1.y : kNegInf;
                X2b = inC ? x2.y : kNegInf;
            } else {
                Mva = Mvb = X1a = X1b = X2a = X2b = kNegInf;
#pragma unroll 1
                for (int k = 0; k < pn; ++k) {
                    const int pk = readlane(pP, k), bk = readlane(pB, k), ek = readlane(pE, k);
                    int hA, hB;
                    int2 x1, x2;
                    if (all_ring || (r - pk < kR && row_narrow<RW>(bk, ek))) {
                        const int pr = pk % kR;
                        const int iA = (j0 - 1) & (RW - 1), iB = j0 & (RW - 1);
                        hA = ring_get<R16, RW>(sh, pr, 0, iA);
                        hB = ring_get<R16, RW>(sh, pr, 0, iB);
                        x1 = ring_get2<R16, RW>(sh, pr, 1, iB);
                        x2 = ring_get2<R16, RW>(sh, pr, 2, iB);
                    } else {
                        // predecessor outside the ring: its spill planes in HBM (columns clamped to
                        // the spilled width; out-of-band values are masked below)
                        hbm_fence();
                        const int pc0 = bk & ~1, wa_k = row_spill_width(bk, ek);
                        const gint *sp = s.sv + readlane(pS, k);
                        const int cA = min(max(j0 - 1 - pc0, 0), wa_k - 1), cB = min(max(j0 - pc0, 0), wa_k - 1),
                                  cC = min(max(j1 - pc0, 0), wa_k - 1);
                        hA = sp[cA];
                        hB = sp[cB];
                        x1 = make_int2(sp[wa_k + cB], sp[wa_k + cC]);
                        x2 = make_int2(sp[2 * wa_k + cB], sp[2 * wa_k + cC]);
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // consume inside the branch
                    }
                    const bool inA = in_band(j0 - 1, bk, ek), inB = in_band(j0, bk, ek),
                               inC = in_band(j1, bk, ek);
                    const int vA = inA ? hA : kNegInf, vB = inB ? hB : kNegInf;
                    const int v1a = inB ? x1.x : kNegInf, v2a = inB ? x2.x : kNegInf;
                    const int v1b = inC ? x1.y : kNegInf, v2b = inC ? x2.y : kNegInf;
                    if (vA > Mva) { Mva = vA; mka = k; }
                    if (vB > Mvb) { Mvb = vB; mkb = k; }
                    if (v1a > X1a) { X1a = v1a; k1a = k; }
                    if (v1b > X1b) { X1b = v1b; k1b = k; }
                    if (v2a > X2a) { X2a = v2a; k2a = k; }
                    if (v2b > X2b) { X2b = v2b; k2b = k; }
                }
            }
            {
                STAMP(tx);
                ts2 = tx;
            }
            const int Ma = Mva + score_of(vb, qa, sc.match, sc.mismatch);
            const int Mb = Mvb + score_of(vb, qb, sc.match, sc.mismatch);
            const int H0a = max(Ma, max(X1a, X2a));
            const int H0b = max(Mb, max(X1b, X2b));
            // horizontal gaps: F[j] = max(C, max_{k<j} H0[k] + e*k) - oe - e*(j-1)
            const int G1a = va ? H0a + e1 * j0 : IDENT;
            const int G1b = vbb ? H0b + e1 * j1 : IDENT;
            const int G2a = va ? H0a + e2 * j0 : IDENT;
            const int G2b = vbb ? H0b + e2 * j1 : IDENT;
            int inc1 = max(G1a, G1b), inc2 = max(G2a, G2b);
            dpp_incl_max2(inc1, inc2);
            const int ex1 = dpp_shr1(inc1, IDENT);
            const int ex2 = dpp_shr1(inc2, IDENT);
            const int P1a = max(ex1, carry1), P1b = max(P1a, G1a);
            const int P2a = max(ex2, carry2), P2b = max(P2a, G2a);
            if (nchunk > 1) {
                carry1 = max(carry1, readlane(inc1, kWave - 1));
                carry2 = max(carry2, readlane(inc2, kWave - 1));
            }
            const int F1a = P1a - oe1 - e1 * (j0 - 1), F1b = P1b - oe1 - e1 * (j1 - 1);
            const int F2a = P2a - oe2 - e2 * (j0 - 1), F2b = P2b - oe2 - e2 * (j1 - 1);
            Ha = max(H0a, max(F1a, F2a));
            Hb = max(H0b, max(F1b, F2b));
            E1a = max(X1a - e1, Ha - oe1);
            E1b = max(X1b - e1, Hb - oe1);
            E2a = max(X2a - e2, Ha - oe2);
            E2b = max(X2b - e2, Hb - oe2);
            const int ta = tb_bits(Ha, Ma, X1a, X2a, F1a, oe1, e1, oe2, e2, G1a, P1a, G2a, P2a);
            const int tb2 = tb_bits(Hb, Mb, X1b, X2b, F1b, oe1, e1, oe2, e2, G1b, P1b, G2b, P2b);
            tpair = ta | (tb2 << 8);
            if ((va || vbb) && multi) {
                if (ks == 1) {
                    *reinterpret_cast<GLB uint16_t *>(s.kp + (kpbase + j0)) =
                        (uint16_t)((mka | k1a << 2 | k2a << 4) | (mkb | k1b << 2 | k2b << 4) << 8);
                } else {
                    GLB uint16_t *kq = reinterpret_cast<GLB uint16_t *>(s.kp + (kpbase + 3 * j0));
                    kq[0] = (uint16_t)(mka | (k1a << 8));
                    kq[1] = (uint16_t)(k2a | (mkb << 8));
                    kq[2] = (uint16_t)(k1b | (k2b << 8));
                }
            }
            {
                STAMP(tx);
                ts3 = tx;
            }
        }
        if (va || vbb) *reinterpret_cast<GLB uint16_t *>(s.tb + (tbbase + j0)) = (uint16_t)tpair;
        if (narrow) {  // out-of-band columns hold -inf (see dp_row_fast)
            const int ibk = j0 & (RW - 1), rr = r % kR;
            ring_put2<R16, RW>(sh, rr, 0, ibk, Ha, va, Hb, vbb);
            ring_put2<R16, RW>(sh, rr, 1, ibk, E1a, va, E1b, vbb);
            ring_put2<R16, RW>(sh, rr, 2, ibk, E2a, va, E2b, vbb);
        }
        if constexpr (R16) {
            // finite values must stay clear of the -inf band (see kR16Low)
            const bool bad = (va && Ha >= kR16Low && Ha < kR16High) || (vbb && Hb >= kR16Low && Hb < kR16High) ||
                             (va && Ha > 32767 - 256) || (vbb && Hb > 32767 - 256);
            if (__ballot(bad)) ds.r16bad = 1;
        }
        if (spill) {
            gint *sv = s.sv + svbase;
            sv[j0] = Ha;
            sv[j1] = Hb;
            sv[wa + j0] = E1a;
            sv[wa + j1] = E1b;
            sv[2 * wa + j0] = E2a;
            sv[2 * wa + j1] = E2b;
        }
        // leftmost argmax of H in one max-reduction: value (clamped; real values are far inside
        // +-2^23, out-of-band garbage never wins) in the high bits, 127 - column-in-chunk below
        const int ca = va ? (min(max(Ha, -(1 << 23)), (1 << 23)) << 7) | (127 - 2 * lane)
                          : (-2147483647 - 1);
        const int cbk = vbb ? (min(max(Hb, -(1 << 23)), (1 << 23)) << 7) | (126 - 2 * lane)
                            : (-2147483647 - 1);
        const int mp = readlane(dpp_incl_max(max(ca, cbk), -2147483647 - 1), kWave - 1);
        const int m = mp >> 7;
        if (m > best) {
            best = m;
            besti = cb + 127 - (mp & 127);
        }
    }
    {
        STAMP(ts4);
        ds.seg[0] += ts1 - ts0;
        ds.seg[1] += ts2 - ts1;
        ds.seg[2] += ts3 - ts2;
        ds.seg[3] += ts4 - ts3;
    }
    if (lane == 0) {
        sh.rrow[r % kRowRing] = make_int4(beg, end, besti, soff);
        gint *ri = s.rinfo + (int64_t)r * kRowInfoInts;
        *reinterpret_cast<GLB v4i *>(ri) = (v4i){beg, end, tbbase, kpbase};
        *reinterpret_cast<GLB v4i *>(ri + 4) = (v4i){besti, soff, node, pn};
    }
    return kStOk;
}

// Loop-carried state of the row loop: the previous row's band record (forwarded in registers, so
// the common predecessor r-1 costs no LDS round trip) and the next row's prefetched descriptor and
// predecessor records (read from LDS one row ahead, off the critical path).
struct RowPipe {
    int prv_r, prv_beg, prv_end, prv_am;
    int node, d1, rem, p0, p1;
    int4 x0, x1;
};

__device__ __forceinline__ void prefetch_row(const SharedState &sh, int r, RowPipe &rp) {
    const int *dl = &sh.desc[r & (kDescBatch - 1)][0];
    rp.node = dl[0];
    rp.d1 = dl[1];
    rp.rem = dl[2];
    rp.p0 = dl[3];
    rp.p1 = dl[4];
    rp.x0 = sh.rrow[max(rp.p0, 0) % kRowRing];
    rp.x1 = sh.rrow[max(rp.p1, 0) % kRowRing];
}

// Fast path for the common row: 1 or 2 predecessors, both in the LDS ring, band <= 128 columns,
// both records in the row ring.  All row-control values stay in VGPRs (every lane computes them),
// so the row costs a single scalar round trip (the fast-path test) plus the argmax broadcast.
// Returns false (having changed nothing) when the row must take the general path.
template <class SC>
__device__ __forceinline__ bool dp_row_fast(const PoaRunArgs &a, const SC &sc, Slot &s, SharedState &sh, int qlen,
                                           int w, int r, int lane, DpState &ds, RowPipe &pp) {
    const int e1 = sc.e1, e2 = sc.e2, oe1 = sc.o1 + sc.e1, oe2 = sc.o2 + sc.e2;
    const int IDENT = -(1 << 30);
    const int node = pp.node, d1 = pp.d1, rem = pp.rem, p0 = pp.p0, p1 = pp.p1;
    const int vb = d1 & 0xff, pn = d1 >> 16;
    const int4 x0 = (p0 == pp.prv_r) ? make_int4(pp.prv_beg, pp.prv_end, pp.prv_am, 0) : pp.x0;
    const int4 x1 = (p1 == pp.prv_r) ? make_int4(pp.prv_beg, pp.prv_end, pp.prv_am, 0) : pp.x1;
    const bool two = pn == 2;
    const int am0 = x0.z + 1, am1 = two ? x1.z + 1 : am0;
    const int xr = qlen - rem;
    const int beg = max(0, min(min(am0, am1), xr) - w);
    const int end = min(qlen, max(max(am0, am1), xr) + w);
    const int cb0 = beg & ~1;
    const int span = end - cb0 + 1;
    const int tbw = (span + 3) & ~3;
    const bool ring0 = (r - p0 < kRing) && row_narrow(x0.x, x0.y);
    const bool ring1 = !two || ((r - p1 < kRing) && row_narrow(x1.x, x1.y));
    // far / multi come from the descriptor (prefetched a row earlier): cheap scalar tests
    const int d1s = bcast0(d1);
    const bool far = ((d1s >> 8) & 1) != 0;
    const bool multi = (d1s >> 16) > 1;
    const bool ok = pn >= 1 && pn <= 2 && span <= kChunk && ring0 && ring1 &&
                    ds.tb_used + tbw + kChunk <= (int)a.caps.TBC &&
                    (!multi || ds.kp_used + 3 * (tbw + kChunk) <= (int)a.caps.KPC) &&
                    (!far || ds.sv_used + 3 * kChunk <= (int)a.caps.SVC);
    if (!__builtin_amdgcn_readfirstlane((int)ok)) return false;

    const int tbbase = (int)ds.tb_used - cb0;
    const int kpbase = (int)ds.kp_used - cb0;  // at most two predecessors: packed bytes (kp_stride 1)
    const int soff = far ? (int)ds.sv_used : -1;
    const int svbase = (int)ds.sv_used - cb0;
    const int j0 = cb0 + 2 * lane, j1 = j0 + 1;
    const bool va = j0 >= beg && j0 <= end, vbb = j1 <= end;
    // query codes of both columns: one byte of the shifted, padded stream
    const int qbyte = g_qnib[j0 >> 1];
    const int qa = qbyte & 0xf, qb = qbyte >> 4;
    const int ia = (j0 - 1) & (kChunk - 1), ib = j0 & (kChunk - 1);
    // Ring rows hold -inf outside their band (every writer masks its out-of-band columns), so when
    // the columns this row reads, [beg-1, end], lie inside a predecessor's 128-column chunk, the ring
    // values need no band masks.  A single predecessor is read twice (max and first-index ties are
    // unchanged by a duplicate).  Otherwise the masked form below handles chunk aliasing.
    const int pc0 = x0.x & ~1, pc1 = x1.x & ~1;
    const bool nm0 = beg - 1 >= pc0 && end <= pc0 + kChunk - 1;
    const bool nm1 = !two || (beg - 1 >= pc1 && end <= pc1 + kChunk - 1);
    const bool nomask = __builtin_amdgcn_readfirstlane((int)(nm0 && nm1)) != 0;
    const int *r0p = &sh.dp.ring[p0 % kRing][0][0];
    const int *r1p = two ? &sh.dp.ring[max(p1, 0) % kRing][0][0] : r0p;
    const int h0A = r0p[ia], h0B = r0p[ib];
    const int2 y01 = *reinterpret_cast<const int2 *>(r0p + kChunk + ib);
    const int2 y02 = *reinterpret_cast<const int2 *>(r0p + 2 * kChunk + ib);
    const int h1A = r1p[ia], h1B = r1p[ib];
    const int2 y11 = *reinterpret_cast<const int2 *>(r1p + kChunk + ib);
    const int2 y12 = *reinterpret_cast<const int2 *>(r1p + 2 * kChunk + ib);
    int a0, b0, a1, b1, u0, u1, v0, v1, w0, w1, z0, z1;
    if (nomask) {
        a0 = h0A, b0 = h0B, a1 = h1A, b1 = h1B;
        u0 = y01.x, u1 = y11.x, v0 = y01.y, v1 = y11.y;
        w0 = y02.x, w1 = y12.x, z0 = y02.y, z1 = y12.y;
    } else {
        const bool i0A = in_band(j0 - 1, x0.x, x0.y), i0B = in_band(j0, x0.x, x0.y), i0C = in_band(j1, x0.x, x0.y);
        const bool i1A = two && in_band(j0 - 1, x1.x, x1.y), i1B = two && in_band(j0, x1.x, x1.y),
                   i1C = two && in_band(j1, x1.x, x1.y);
        a0 = i0A ? h0A : kNegInf, b0 = i0B ? h0B : kNegInf;
        a1 = i1A ? h1A : kNegInf, b1 = i1B ? h1B : kNegInf;
        u0 = i0B ? y01.x : kNegInf, u1 = i1B ? y11.x : kNegInf;
        v0 = i0C ? y01.y : kNegInf, v1 = i1C ? y11.y : kNegInf;
        w0 = i0B ? y02.x : kNegInf, w1 = i1B ? y12.x : kNegInf;
        z0 = i0C ? y02.y : kNegInf, z1 = i1C ? y12.y : kNegInf;
    }
    // first predecessor attaining the max (strict > keeps the earlier one)
    const int Mva = max(a0, a1), Mvb = max(b0, b1);
    const int mka = a1 > a0, mkb = b1 > b0;
    const int X1a = max(u0, u1), X1b = max(v0, v1), X2a = max(w0, w1), X2b = max(z0, z1);
    const int k1a = u1 > u0, k1b = v1 > v0, k2a = w1 > w0, k2b = z1 > z0;

    const int Ma = Mva + score_of(vb, qa, sc.match, sc.mismatch);
    const int Mb = Mvb + score_of(vb, qb, sc.match, sc.mismatch);
    const int H0a = max(Ma, max(X1a, X2a));
    const int H0b = max(Mb, max(X1b, X2b));
    const int G1a = va ? H0a + e1 * j0 : IDENT;
    const int G1b = vbb ? H0b + e1 * j1 : IDENT;
    const int G2a = va ? H0a + e2 * j0 : IDENT;
    const int G2b = vbb ? H0b + e2 * j1 : IDENT;
    int inc1 = max(G1a, G1b), inc2 = max(G2a, G2b);
    dpp_incl_max2(inc1, inc2);
    const int carry1 = kNegInf + oe1 + e1 * (beg - 1);
    const int carry2 = kNegInf + oe2 + e2 * (beg - 1);
    const int P1a = max(dpp_shr1(inc1, IDENT), carry1), P1b = max(P1a, G1a);
    const int P2a = max(dpp_shr1(inc2, IDENT), carry2), P2b = max(P2a, G2a);
    const int F1a = P1a - oe1 - e1 * (j0 - 1), F1b = P1b - oe1 - e1 * (j1 - 1);
    const int F2a = P2a - oe2 - e2 * (j0 - 1), F2b = P2b - oe2 - e2 * (j1 - 1);
    const int Ha = max(H0a, max(F1a, F2a));
    const int Hb = max(H0b, max(F1b, F2b));
    const int E1a = max(X1a - e1, Ha - oe1), E1b = max(X1b - e1, Hb - oe1);
    const int E2a = max(X2a - e2, Ha - oe2), E2b = max(X2b - e2, Hb - oe2);
    const int ta = tb_bits(Ha, Ma, X1a, X2a, F1a, oe1, e1, oe2, e2, G1a, P1a, G2a, P2a);
    const int tb2 = tb_bits(Hb, Mb, X1b, X2b, F1b, oe1, e1, oe2, e2, G1b, P1b, G2b, P2b);
    // stores: the traceback pair of every lane (lanes past `end` write into slack the next row
    // overwrites; the caller's capacity test keeps one chunk of slack), ring row, optional planes
    *reinterpret_cast<GLB uint16_t *>(s.tb + (tbbase + j0)) = (uint16_t)(ta | (tb2 << 8));
    if (multi)
        *reinterpret_cast<GLB uint16_t *>(s.kp + (kpbase + j0)) =
            (uint16_t)((mka | k1a << 2 | k2a << 4) | (mkb | k1b << 2 | k2b << 4) << 8);
    int *ringrow = &sh.dp.ring[r % kRing][0][0];
    *reinterpret_cast<int2 *>(ringrow + ib) = make_int2(va ? Ha : kNegInf, vbb ? Hb : kNegInf);
    *reinterpret_cast<int2 *>(ringrow + kChunk + ib) = make_int2(va ? E1a : kNegInf, vbb ? E1b : kNegInf);
    *reinterpret_cast<int2 *>(ringrow + 2 * kChunk + ib) = make_int2(va ? E2a : kNegInf, vbb ? E2b : kNegInf);
    if (far) {
        gint *sv = s.sv + svbase;
        sv[j0] = Ha;
        sv[j1] = Hb;
        sv[kChunk + j0] = E1a;
        sv[kChunk + j1] = E1b;
        sv[2 * kChunk + j0] = E2a;
        sv[2 * kChunk + j1] = E2b;
    }
    // leftmost argmax (value << 7 | 127 - column-in-chunk)
    const int ca = va ? (min(max(Ha, -(1 << 23)), (1 << 23)) << 7) | (127 - 2 * lane) : (-2147483647 - 1);
    const int cbk = vbb ? (min(max(Hb, -(1 << 23)), (1 << 23)) << 7) | (126 - 2 * lane) : (-2147483647 - 1);
    const int mp = readlane(dpp_incl_max(max(ca, cbk), -2147483647 - 1), kWave - 1);
    const int besti = cb0 + 127 - (mp & 127);
    // bookkeeping (scalar)
    const int begs = bcast0(beg), ends = bcast0(end), tbws = bcast0(tbw);
    ds.tb_used += tbws;
    if (multi) ds.kp_used += tbws;
    if (far) ds.sv_used += 3 * kChunk;
    ds.cells += ends - begs + 1;
    if (lane == 0) {
        sh.rrow[r % kRowRing] = make_int4(beg, end, besti, soff);
        gint *ri = s.rinfo + (int64_t)r * kRowInfoInts;
        *reinterpret_cast<GLB v4i *>(ri) = (v4i){beg, end, tbbase, kpbase};
        *reinterpret_cast<GLB v4i *>(ri + 4) = (v4i){besti, soff, node, pn};
    }
    pp.prv_r = r;
    pp.prv_beg = beg;
    pp.prv_end = end;
    pp.prv_am = besti;
    return true;
}

// ---- packed 16-bit lane pairs: .lo = column j0 = cb0 + 2*lane, .hi = column j0 + 1 ------------
typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ s16x2 as_s16x2(uint32_t x) { return __builtin_bit_cast(s16x2, x); }
__device__ __forceinline__ uint32_t as_u32(s16x2 x) { return __builtin_bit_cast(uint32_t, x); }
__device__ __forceinline__ uint32_t as_u32(u16x2 x) { return __builtin_bit_cast(uint32_t, x); }
__device__ __forceinline__ u16x2 as_u16x2(uint32_t x) { return __builtin_bit_cast(u16x2, x); }
__host__ __device__ constexpr uint32_t pk2(int v) { return ((uint32_t)v & 0xffffu) * 0x10001u; }
constexpr uint32_t kNeg2 = 0x80008000u;  // (-32768, -32768): -inf of the 16-bit mode
// pk2 of a wave-uniform value, built on the scalar unit (left alone, the compiler splats with a VALU
// multiply per value)
__device__ __forceinline__ uint32_t pk2s(int v) {
    uint32_t r;
    asm("s_pack_ll_b32_b16 %0, %1, %1" : "=s"(r) : "s"(__builtin_amdgcn_readfirstlane(v)));
    return r;
}
__device__ __forceinline__ uint32_t pk_adds(uint32_t a, uint32_t b) {
    return as_u32(__builtin_elementwise_add_sat(as_s16x2(a), as_s16x2(b)));
}
__device__ __forceinline__ uint32_t pk_subs(uint32_t a, uint32_t b) {
    return as_u32(__builtin_elementwise_sub_sat(as_s16x2(a), as_s16x2(b)));
}
__device__ __forceinline__ uint32_t pk_max(uint32_t a, uint32_t b) {
    return as_u32(__builtin_elementwise_max(as_s16x2(a), as_s16x2(b)));
}
__device__ __forceinline__ uint32_t pk_umax(uint32_t a, uint32_t b) {
    return as_u32(__builtin_elementwise_max(as_u16x2(a), as_u16x2(b)));
}
__device__ __forceinline__ uint32_t pk_umin(uint32_t a, uint32_t b) {
    return as_u32(__builtin_elementwise_min(as_u16x2(a), as_u16x2(b)));
}
// 0xffff in the halves where x < 0
__device__ __forceinline__ uint32_t pk_neg_mask(uint32_t x) { return as_u32(as_s16x2(x) >> (s16x2){15, 15}); }
// bit K set in the halves where h != x (h >= x or x is -inf; one saturating subtract + min)
template <int K>
__device__ __forceinline__ uint32_t pk_ne_bit(uint32_t h, uint32_t x) {
    uint32_t r;
    asm("v_pk_min_u16 %0, %1, 1 op_sel_hi:[1,0]" : "=v"(r) : "v"(pk_subs(h, x)));  // (splat 1; the compiler would use compares)
    return K ? as_u32(as_u16x2(r) << (u16x2){K, K}) : r;
}
// bit K set in the halves where a < b
template <int K>
__device__ __forceinline__ uint32_t pk_lt_bit(uint32_t a, uint32_t b) {
    return as_u32((as_u16x2(pk_subs(a, b)) >> (u16x2){15 - K, 15 - K}) & (u16x2){1u << K, 1u << K});
}
// (m & x) | (~m & y) as one v_bfi_b32 (left to itself the compiler turns mask-selects into
// per-half compares + cndmasks + a perm)
__device__ __forceinline__ uint32_t bfi(uint32_t m, uint32_t x, uint32_t y) {
    uint32_t r;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(x), "v"(y));
    return r;
}
// inclusive prefix max over the wave of both halves (unsigned; 0 is the identity, so DPP lanes
// without a source read 0 via bound_ctrl)
// The two row_bcast steps leave the lanes of their masked-off rows at `old`: that is the previous
// step's shifted value, a prefix maximum already folded into u, so no zero-fill is needed.
__device__ __forceinline__ uint32_t pk_scan_umax(uint32_t u) {
    uint32_t t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)u, 0x111, 0xf, 0xf, true);
    u = pk_umax(u, t);
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)u, 0x112, 0xf, 0xf, true);
    u = pk_umax(u, t);
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)u, 0x114, 0xf, 0xf, true);
    u = pk_umax(u, t);
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)u, 0x118, 0xf, 0xf, true);
    u = pk_umax(u, t);
    t = (uint32_t)__builtin_amdgcn_update_dpp((int)t, (int)u, 0x142, 0xa, 0xf, false);
    u = pk_umax(u, t);
    t = (uint32_t)__builtin_amdgcn_update_dpp((int)t, (int)u, 0x143, 0xc, 0xf, false);
    u = pk_umax(u, t);
    return u;
}


// The row's two wave scans in one instruction stream: the inclusive prefix max of the packed F
// input u (unsigned halves; v_mov_dpp + v_pk_max_u16 per step) and of the argmax key a
// (v_max_i32_dpp).  The chains are independent, so each fills the other's VALU-write -> DPP-read
// wait states (two per dependent pair): one s_nop 0 per step instead of two s_nop 1.  The two
// row_bcast steps of u leave the lanes of their masked-off rows at t, the previous step's shifted
// value, which is a prefix maximum already folded into u.
__device__ __forceinline__ void dpp_scan_fa(uint32_t &u, int &a) {
    uint32_t t;
    asm volatile(
        "s_nop 1\n"
        "v_mov_b32_dpp %2, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_max_i32_dpp %1, %1, %1 row_shr:1 row_mask:0xf bank_mask:0xf\n"
        "v_pk_max_u16 %0, %0, %2\n"
        "s_nop 0\n"
        "v_max_i32_dpp %1, %1, %1 row_shr:2 row_mask:0xf bank_mask:0xf\n"
        "v_mov_b32_dpp %2, %0 row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_pk_max_u16 %0, %0, %2\n"
        "v_max_i32_dpp %1, %1, %1 row_shr:4 row_mask:0xf bank_mask:0xf\n"
        "s_nop 0\n"
        "v_mov_b32_dpp %2, %0 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_pk_max_u16 %0, %0, %2\n"
        "s_nop 0\n"
        "v_max_i32_dpp %1, %1, %1 row_shr:8 row_mask:0xf bank_mask:0xf\n"
        "v_mov_b32_dpp %2, %0 row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
        "v_pk_max_u16 %0, %0, %2\n"
        "v_max_i32_dpp %1, %1, %1 row_bcast:15 row_mask:0xa bank_mask:0xf\n"
        "s_nop 0\n"
        "v_mov_b32_dpp %2, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n"
        "v_pk_max_u16 %0, %0, %2\n"
        "v_max_i32_dpp %1, %1, %1 row_bcast:31 row_mask:0xc bank_mask:0xf\n"
        "s_nop 0\n"
        "v_mov_b32_dpp %2, %0 row_bcast:31 row_mask:0xc bank_mask:0xf\n"
        "v_pk_max_u16 %0, %0, %2\n"
        "s_nop 1\n"
        : "+v"(u), "+v"(a), "=&v"(t));
}

// The traceback bytes of a lane's two cells (layout in poa_kernel.h).  Every bit of the layout is
// "a < b" for one pair of values (M < H, X1 < H, X2 < H, F1 < H, Ho1 < X1e, Ho2 < X2e, G1 < P1,
// G2 < P2), i.e. the sign of the saturating difference d_k = a - b, which has the sign of the exact
// one.  v_perm's sign-replicating selectors (8..11: bit 15 / 31 of either source) turn two
// differences into the four bytes [d0.lo, d0.hi, d1.lo, d1.hi] of 0x00 / 0xff; a mask keeps one bit
// of each (even bits in bytes 0-1, odd bits in bytes 2-3) and the two halves are added: the low 16
// bits are [column j0's byte, column j0 + 1's byte].
__device__ __forceinline__ uint32_t tb_pack(uint32_t d0, uint32_t d1, uint32_t d2, uint32_t d3, uint32_t d4,
                                            uint32_t d5, uint32_t d6, uint32_t d7) {
    const uint32_t x01 = __builtin_amdgcn_perm(d1, d0, 0x0B0A0908u);
    const uint32_t x23 = __builtin_amdgcn_perm(d3, d2, 0x0B0A0908u);
    const uint32_t x45 = __builtin_amdgcn_perm(d5, d4, 0x0B0A0908u);
    const uint32_t x67 = __builtin_amdgcn_perm(d7, d6, 0x0B0A0908u);
    uint32_t acc = x01 & 0x02020101u;
    acc |= x23 & 0x08080404u;
    acc |= x45 & 0x20201010u;
    acc |= x67 & 0x80804040u;
    return acc + (acc >> 16);
}

// Leftmost-argmax key of a lane's two 16-bit values hs = (H[j0], H[j0 + 1]): H * 128 + (127 - offset of
// the column), the larger of the two (c_lo = 127 - 2 lane, c_hi = 126 - 2 lane); one v_mad_i32_i16 per
// half (op_sel picks the high half).
__device__ __forceinline__ int pair_key(uint32_t hs, int c_lo, int c_hi) {
    int a, b;
    asm("v_mad_i32_i16 %0, %1, %3, %2" : "=v"(a) : "v"(hs), "v"(c_lo), "s"(128));
    asm("v_mad_i32_i16 %0, %1, %3, %2 op_sel:[1,0,0,0]" : "=v"(b) : "v"(hs), "v"(c_hi), "s"(128));
    return max(a, b);
}

// A lane's store into the current row's range of a slot array: the row's base is scalar (SGPR pair),
// the lane's byte offset an unsigned 32-bit VGPR, so the store takes the global saddr form with no
// per-row address arithmetic on the vector unit.
template <class T>
__device__ __forceinline__ void row_store(gu8 *row_base, uint32_t lane_off, T v) {
    *reinterpret_cast<GLB T *>(uniptr(row_base) + lane_off) = v;
}
// A lane's 16-bit store at byte uoff + lane_off of a slot array (base: the array, loop-invariant in
// SGPRs; uoff: the row's uniform offset).  The per-row offset is folded into the lane's zero-extended
// 32-bit offset, so the compiler selects the saddr form (one v_add per store) instead of building the
// 64-bit row address on the scalar unit (s_ashr + s_add + s_addc) and a 64-bit lane address.  (An
// inline-asm store of the same form faulted: the compiler does not see a VMEM instruction in an asm
// statement, so it places no wait states between a VALU write of the base SGPRs -- v_readlane of a
// spilled SGPR -- and the store's read of them.)
__device__ __forceinline__ void row_store16(gu8 *base, int uoff, uint32_t lane_off, uint32_t v) {
    *reinterpret_cast<GLB uint16_t *>(base + (uint64_t)((uint32_t)uoff + lane_off)) = (uint16_t)v;
}

// A fast row's record in HBM (lane 0): {beg, end, tbbase, kpbase} and, for a row whose successor is
// far, {argmax, spill offset}; stored in the saddr form (the slot's base in SGPRs, the row's 32-bit byte
// offset in a VGPR) instead of through a 64-bit address built on the scalar unit per row: SGPR spills
// 295 -> 267, DP 2,621 -> 2,547 cycles per row, kernel -2 % (profiles/r04x_rinfo_saddr_ab.txt).
__device__ __forceinline__ void row_record(gint *rinfo, int r, int beg, int end, int tbbase, int kpbase, int far,
                                           int besti, int soff) {
    const uint32_t off = (uint32_t)r * (uint32_t)(kRowInfoInts * 4);
    row_store(reinterpret_cast<gu8 *>(rinfo), off, (v4i){beg, end, tbbase, kpbase});
    if (far) row_store(reinterpret_cast<gu8 *>(rinfo), off + 16u, (v2i){besti, soff});
}

// ---- 16-bit mode with scalar row control -------------------------------------------------------
// Everything that is uniform per row (descriptor, predecessor band records, band, fast-path
// tests, allocation) lives in SGPRs: descriptors come straight from HBM through the scalar cache
// (s_load, invalidated once per read: build_desc wrote them with vector stores), the previous row's
// record is forwarded in SGPRs, and other predecessors' records are read from the LDS row ring and
// broadcast.  The vector unit only does the two cells per lane.
typedef __attribute__((address_space(4))) const int cint;

struct Row16 {
    int r, node, vb, pn, beg, end, cb0, tbw;
    int p0slot, p1slot;        // ring rows of the predecessors (p % kRing16)
    int b0, e0, b1, e1;        // their bands
    int two, far, multi, nomask;  // 0/1 (ints: LLVM keeps uniform bools as 64-bit lane masks)
    int pn3;                      // predecessor count when >= 3 (predecessors 2.. are read in row16_vec)
};

// ONE: the row has exactly one predecessor (no second-predecessor merge, no predecessor bytes)
template <class SC, int RW, bool ONE = false>
__device__ __forceinline__ int row16_vec(const SC &sc, gu8 *tb, gu8 *kp, gint *sv, gint *rinfo, SharedState &sh,
                                         int lane, const Row16 &R, DpState &ds) {
    constexpr int HW = RW / 2;  // ring words per plane
    const int e1 = sc.e1, e2 = sc.e2, oe1 = sc.o1 + sc.e1, oe2 = sc.o2 + sc.e2;
    const int beg = R.beg, end = R.end, cb0 = R.cb0;
    const int tbbase = ds.tb_used - cb0;
    const int ks = kp_stride(R.pn);
    const int kpbase = ds.kp_used - ks * cb0;
    const int soff = R.far ? ds.sv_used : -1;
    const int svbase = ds.sv_used - cb0;
    // lane pair index t = j0 / 2 (cb0 is even): one add, and every per-lane position derives from it
    // (16-bit rows: columns < 2^16; the mask lets the LDS offsets fold into the instructions)
    const uint32_t t = (((uint32_t)cb0 >> 1) & 0x7fffu) + ((uint32_t)lane & 63u);
    const int j0 = (int)(2 * t);
    const uint32_t J = __umul24(t, 0x20002u) + 0x10000u;             // (j0, j0 + 1)
    const uint32_t LJ = (uint32_t)(2 * lane) * 0x10001u + 0x10000u;  // (j0, j0 + 1) - cb0
    const uint32_t inv = pk_neg_mask(as_u32(as_s16x2(J) - as_s16x2(pk2s(beg))) |
                                     as_u32(as_s16x2(pk2s(end)) - as_s16x2(J)));
    const uint32_t qbyte = qnib<RW>()[t];
    // perm selector (code of j0, 0x0C, code of j0 + 1, 0x0C): the byte copied to bits 12.. puts the
    // high nibble at bits 16-19
    const uint32_t sel = ((qbyte * 0x1001u) & 0x000F000Fu) | 0x0C000C00u;
    const uint32_t tlo =
        R.vb < 4 ? (uint32_t)(sc.match + sc.mismatch) << (8 * R.vb) : (uint32_t)sc.mismatch * 0x01010101u;
    const uint32_t S = __builtin_amdgcn_perm((uint32_t)sc.mismatch, tlo, sel);
    const uint32_t iw = t & (HW - 1), iwp = (t - 1u) & (HW - 1);
    const uint32_t *w0 = reinterpret_cast<const uint32_t *>(ring16_row<RW>(sh, R.p0slot));
    uint32_t Hd = __builtin_amdgcn_alignbit(w0[iw], w0[iwp], 16);
    uint32_t X1 = w0[HW + iw], X2 = w0[2 * HW + iw];
    const uint32_t JD = as_u32(as_s16x2(J) - (s16x2){1, 1});  // (j0 - 1, j0)
    if (!R.nomask) {
        const uint32_t md = pk_neg_mask(as_u32(as_s16x2(JD) - as_s16x2(pk2s(R.b0))) |
                                        as_u32(as_s16x2(pk2s(R.e0)) - as_s16x2(JD)));
        const uint32_t me = pk_neg_mask(as_u32(as_s16x2(J) - as_s16x2(pk2s(R.b0))) |
                                        as_u32(as_s16x2(pk2s(R.e0)) - as_s16x2(J)));
        Hd = bfi(md, kNeg2, Hd);
        X1 = bfi(me, kNeg2, X1);
        X2 = bfi(me, kNeg2, X2);
    }
    uint32_t MK = 0, K1 = 0, K2 = 0;
    if (!ONE && R.two) {
        const uint32_t *w1 = reinterpret_cast<const uint32_t *>(ring16_row<RW>(sh, R.p1slot));
        uint32_t Hd1 = __builtin_amdgcn_alignbit(w1[iw], w1[iwp], 16);
        uint32_t X11 = w1[HW + iw], X21 = w1[2 * HW + iw];
        if (!R.nomask) {
            const uint32_t md = pk_neg_mask(as_u32(as_s16x2(JD) - as_s16x2(pk2s(R.b1))) |
                                            as_u32(as_s16x2(pk2s(R.e1)) - as_s16x2(JD)));
            const uint32_t me = pk_neg_mask(as_u32(as_s16x2(J) - as_s16x2(pk2s(R.b1))) |
                                            as_u32(as_s16x2(pk2s(R.e1)) - as_s16x2(J)));
            Hd1 = bfi(md, kNeg2, Hd1);
            X11 = bfi(me, kNeg2, X11);
            X21 = bfi(me, kNeg2, X21);
        }
        MK = pk_lt_bit<0>(Hd, Hd1);
        K1 = pk_lt_bit<0>(X1, X11);
        K2 = pk_lt_bit<0>(X2, X21);
        Hd = pk_max(Hd, Hd1);
        X1 = pk_max(X1, X11);
        X2 = pk_max(X2, X21);
    }
    // predecessors 2.. of a multi-predecessor row (records re-read from the LDS row ring; the first
    // strictly larger value names the predecessor, as in dp_row)
    for (int k = 2; k < (ONE ? 0 : R.pn3); ++k) {
        const int p = bcast0(sh.desc[R.r & (kDescBatch - 1)][3 + k]);
        const int4 x = sh.rrow[p & (kRowRing - 1)];
        const int bk = bcast0(x.x), ek = bcast0(x.y);
        const uint32_t *wk = reinterpret_cast<const uint32_t *>(ring16_row<RW>(sh, p & (kRing16 - 1)));
        uint32_t Hdk = __builtin_amdgcn_alignbit(wk[iw], wk[iwp], 16);
        uint32_t X1k = wk[HW + iw], X2k = wk[2 * HW + iw];
        const int pck = bk & ~1;
        if (RW != kChunk || ((beg - 1 - pck) | (pck + kChunk - 1 - end)) < 0) {
            const uint32_t md = pk_neg_mask(as_u32(as_s16x2(JD) - as_s16x2(pk2s(bk))) |
                                            as_u32(as_s16x2(pk2s(ek)) - as_s16x2(JD)));
            const uint32_t me = pk_neg_mask(as_u32(as_s16x2(J) - as_s16x2(pk2s(bk))) |
                                            as_u32(as_s16x2(pk2s(ek)) - as_s16x2(J)));
            Hdk = bfi(md, kNeg2, Hdk);
            X1k = bfi(me, kNeg2, X1k);
            X2k = bfi(me, kNeg2, X2k);
        }
        const uint32_t kk = pk2(k);
        MK = bfi(pk_neg_mask(pk_subs(Hd, Hdk)), kk, MK);
        K1 = bfi(pk_neg_mask(pk_subs(X1, X1k)), kk, K1);
        K2 = bfi(pk_neg_mask(pk_subs(X2, X2k)), kk, K2);
        Hd = pk_max(Hd, Hdk);
        X1 = pk_max(X1, X1k);
        X2 = pk_max(X2, X2k);
    }
    const uint32_t M = pk_subs(pk_adds(Hd, S), pk2(sc.mismatch));
    const uint32_t H0 = bfi(inv, kNeg2, pk_max(M, pk_max(X1, X2)));
    const uint32_t LJ1 = as_u32(as_u16x2(LJ) * (u16x2){(unsigned short)e1, (unsigned short)e1});
    const uint32_t LJ2 = as_u32(as_u16x2(LJ) * (u16x2){(unsigned short)e2, (unsigned short)e2});
    const uint32_t G1 = pk_adds(H0, LJ1), G2 = pk_adds(H0, LJ2);
    const uint32_t Ga = __builtin_amdgcn_perm(G2, G1, 0x05040100u);
    const uint32_t Gb = __builtin_amdgcn_perm(G2, G1, 0x07060302u);
    // the row's leftmost argmax is H0's: F only carries values from the left minus gap penalties, so
    // it never reaches the row maximum (an argmax cell has H = H0, and H >= H0 everywhere)
    uint32_t inc = pk_max(Ga, Gb) ^ kNeg2;
    int amk = pair_key(H0, 127 - 2 * lane, 126 - 2 * lane);
    dpp_scan_fa(inc, amk);
    const int mp = readlane(amk, kWave - 1);
    const uint32_t Pa = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)inc, 0x138, 0xf, 0xf, true) ^ kNeg2;
    const uint32_t Pb = pk_max(Pa, Ga);
    const uint32_t P1 = __builtin_amdgcn_perm(Pb, Pa, 0x05040100u);
    const uint32_t P2 = __builtin_amdgcn_perm(Pb, Pa, 0x07060302u);
    const uint32_t F1 = pk_subs(P1, LJ1 + pk2(oe1 - e1)), F2 = pk_subs(P2, LJ2 + pk2(oe2 - e2));
    const uint32_t H = pk_max(H0, pk_max(F1, F2));
    const uint32_t X1e = pk_subs(X1, pk2(e1)), Ho1 = pk_subs(H, pk2(oe1));
    const uint32_t X2e = pk_subs(X2, pk2(e2)), Ho2 = pk_subs(H, pk2(oe2));
    const uint32_t E1 = pk_max(X1e, Ho1), E2 = pk_max(X2e, Ho2);
    const uint32_t tbv = tb_pack(pk_subs(M, H), pk_subs(X1, H), pk_subs(X2, H), pk_subs(F1, H), pk_subs(Ho1, X1e),
                                 pk_subs(Ho2, X2e), pk_subs(G1, P1), pk_subs(G2, P2));
    // this row's bytes start at ds.tb_used: column j0 = cb0 + 2 lane is at tb_used + 2 lane
    row_store16(tb, ds.tb_used, 2u * (uint32_t)lane, tbv);
    if (!ONE && R.multi) {
        if (ks == 1) {  // packed: k < 8 in each half, so the shifts stay inside the halves
            const uint32_t kb = MK | (K1 << 2) | (K2 << 4);
            row_store16(kp, ds.kp_used, 2u * (uint32_t)lane, __builtin_amdgcn_perm(0u, kb, 0x0C0C0200u));
        } else {
            row_store16(kp, ds.kp_used, 6u * (uint32_t)lane, __builtin_amdgcn_perm(K1, MK, 0x0C0C0400u));
            row_store16(kp, ds.kp_used, 6u * (uint32_t)lane + 2u, __builtin_amdgcn_perm(MK, K2, 0x0C0C0600u));
            row_store16(kp, ds.kp_used, 6u * (uint32_t)lane + 4u, __builtin_amdgcn_perm(K2, K1, 0x0C0C0602u));
        }
    }
    const uint32_t Hs = bfi(inv, kNeg2, H);
    uint32_t *wr = reinterpret_cast<uint32_t *>(ring16_row<RW>(sh, R.r & (kRing16 - 1)));
    wr[iw] = Hs;
    wr[HW + iw] = bfi(inv, kNeg2, E1);
    wr[2 * HW + iw] = bfi(inv, kNeg2, E2);
    if (R.far) {
        gint *svp = sv + svbase;
        svp[j0] = (int)(short)(H & 0xffff);
        svp[j0 + 1] = (int)H >> 16;
        svp[kChunk + j0] = (int)(short)(E1 & 0xffff);
        svp[kChunk + j0 + 1] = (int)E1 >> 16;
        svp[2 * kChunk + j0] = (int)(short)(E2 & 0xffff);
        svp[2 * kChunk + j0 + 1] = (int)E2 >> 16;
    }
    ds.r16acc = pk_umin(ds.r16acc, as_u32(as_u16x2(Hs) - as_u16x2(pk2(kR16Low))));
    const int besti = cb0 + 127 - (mp & 127);
    ds.tb_used += R.tbw;
    if (!ONE && R.multi) ds.kp_used += ks * R.tbw;
    if (R.far) ds.sv_used += 3 * kChunk;
    ds.cells += end - beg + 1;
    if (lane == 0) {
        sh.rrow[R.r & (kRowRing - 1)] = make_int4(beg, end, besti, soff);
        row_record(rinfo, R.r, beg, end, tbbase, kpbase, R.far, besti, soff);
    }
    return besti;
}

// Wide fast row (wide launches only): a band of 129..256 columns as two 128-column halves, lane l
// holding columns cb0 + 128h + 2l and +1 of half h.  The halves are computed side by side; their F
// prefix scans are independent, and the upper half takes the lower half's total as its carry-in.
// Ring rows of a wide launch hold only the columns their row wrote, so the predecessors' values are
// always band-masked.  Predecessors 2.. of a row with up to kPreInline are re-read from the LDS row
// ring, as in row16_vec.
template <class SC>
__device__ __forceinline__ int row16w_vec(const SC &sc, gu8 *tb, gu8 *kp, gint *sv, gint *rinfo, SharedState &sh,
                                          int lane, const Row16 &R, DpState &ds) {
    constexpr int RW = kWideRing, HW = RW / 2;
    const int e1 = sc.e1, e2 = sc.e2, oe1 = sc.o1 + sc.e1, oe2 = sc.o2 + sc.e2;
    const int beg = R.beg, end = R.end, cb0 = R.cb0;
    const int tbbase = ds.tb_used - cb0;
    const int ks = kp_stride(R.pn);
    const int kpbase = ds.kp_used - ks * cb0;
    const int soff = R.far ? ds.sv_used : -1;
    const int svbase = ds.sv_used - cb0;
    const uint32_t *w0 = reinterpret_cast<const uint32_t *>(ring16_row<RW>(sh, R.p0slot));
    const uint32_t *w1 = reinterpret_cast<const uint32_t *>(ring16_row<RW>(sh, R.p1slot));
    const uint32_t tlo =
        R.vb < 4 ? (uint32_t)(sc.match + sc.mismatch) << (8 * R.vb) : (uint32_t)sc.mismatch * 0x01010101u;
    const uint32_t B0 = pk2s(R.b0), E0 = pk2s(R.e0), B1 = pk2s(R.b1), E1b = pk2s(R.e1);
    const uint32_t BEG = pk2s(beg), END = pk2s(end);
    uint32_t H0v[2], Mv[2], X1v[2], X2v[2], MKv[2], K1v[2], K2v[2], G1v[2], G2v[2], Gav[2], incv[2], invv[2];
    uint32_t LJ1v[2], LJ2v[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int j0 = cb0 + kChunk * h + 2 * lane;
        const uint32_t J = (uint32_t)j0 * 0x10001u + 0x10000u;                            // (j0, j0 + 1)
        const uint32_t LJ = (uint32_t)(kChunk * h + 2 * lane) * 0x10001u + 0x10000u;      // the same - cb0
        const uint32_t inv = pk_neg_mask(as_u32(as_s16x2(J) - as_s16x2(BEG)) | as_u32(as_s16x2(END) - as_s16x2(J)));
        const uint32_t qbyte = qnib<RW>()[j0 >> 1];
        const uint32_t sel = ((qbyte * 0x1001u) & 0x000F000Fu) | 0x0C000C00u;
        const uint32_t S = __builtin_amdgcn_perm((uint32_t)sc.mismatch, tlo, sel);
        const int iw = (j0 >> 1) & (HW - 1), iwp = (iw - 1) & (HW - 1);
        const uint32_t JD = as_u32(as_s16x2(J) - (s16x2){1, 1});  // (j0 - 1, j0)
        uint32_t Hd = __builtin_amdgcn_alignbit(w0[iw], w0[iwp], 16);
        uint32_t X1 = w0[HW + iw], X2 = w0[2 * HW + iw];
        {
            const uint32_t md = pk_neg_mask(as_u32(as_s16x2(JD) - as_s16x2(B0)) | as_u32(as_s16x2(E0) - as_s16x2(JD)));
            const uint32_t me = pk_neg_mask(as_u32(as_s16x2(J) - as_s16x2(B0)) | as_u32(as_s16x2(E0) - as_s16x2(J)));
            Hd = bfi(md, kNeg2, Hd);
            X1 = bfi(me, kNeg2, X1);
            X2 = bfi(me, kNeg2, X2);
        }
        uint32_t MK = 0, K1 = 0, K2 = 0;
        if (R.two) {
            uint32_t Hd1 = __builtin_amdgcn_alignbit(w1[iw], w1[iwp], 16);
            uint32_t X11 = w1[HW + iw], X21 = w1[2 * HW + iw];
            const uint32_t md = pk_neg_mask(as_u32(as_s16x2(JD) - as_s16x2(B1)) | as_u32(as_s16x2(E1b) - as_s16x2(JD)));
            const uint32_t me = pk_neg_mask(as_u32(as_s16x2(J) - as_s16x2(B1)) | as_u32(as_s16x2(E1b) - as_s16x2(J)));
            Hd1 = bfi(md, kNeg2, Hd1);
            X11 = bfi(me, kNeg2, X11);
            X21 = bfi(me, kNeg2, X21);
            MK = pk_lt_bit<0>(Hd, Hd1);
            K1 = pk_lt_bit<0>(X1, X11);
            K2 = pk_lt_bit<0>(X2, X21);
            Hd = pk_max(Hd, Hd1);
            X1 = pk_max(X1, X11);
            X2 = pk_max(X2, X21);
        }
        for (int k = 2; k < R.pn3; ++k) {  // the first strictly larger value names the predecessor
            const int p = bcast0(sh.desc[R.r & (kDescBatch - 1)][3 + k]);
            const int4 xr = sh.rrow[p & (kRowRing - 1)];
            const uint32_t Bk = pk2s(xr.x), Ek = pk2s(xr.y);
            const uint32_t *wk = reinterpret_cast<const uint32_t *>(ring16_row<RW>(sh, p & (kRing16 - 1)));
            uint32_t Hdk = __builtin_amdgcn_alignbit(wk[iw], wk[iwp], 16);
            uint32_t X1k = wk[HW + iw], X2k = wk[2 * HW + iw];
            const uint32_t md = pk_neg_mask(as_u32(as_s16x2(JD) - as_s16x2(Bk)) | as_u32(as_s16x2(Ek) - as_s16x2(JD)));
            const uint32_t me = pk_neg_mask(as_u32(as_s16x2(J) - as_s16x2(Bk)) | as_u32(as_s16x2(Ek) - as_s16x2(J)));
            Hdk = bfi(md, kNeg2, Hdk);
            X1k = bfi(me, kNeg2, X1k);
            X2k = bfi(me, kNeg2, X2k);
            const uint32_t kk = pk2(k);
            MK = bfi(pk_neg_mask(pk_subs(Hd, Hdk)), kk, MK);
            K1 = bfi(pk_neg_mask(pk_subs(X1, X1k)), kk, K1);
            K2 = bfi(pk_neg_mask(pk_subs(X2, X2k)), kk, K2);
            Hd = pk_max(Hd, Hdk);
            X1 = pk_max(X1, X1k);
            X2 = pk_max(X2, X2k);
        }
        const uint32_t M = pk_subs(pk_adds(Hd, S), pk2(sc.mismatch));
        const uint32_t H0 = bfi(inv, kNeg2, pk_max(M, pk_max(X1, X2)));
        const uint32_t LJ1 = as_u32(as_u16x2(LJ) * (u16x2){(unsigned short)e1, (unsigned short)e1});
        const uint32_t LJ2 = as_u32(as_u16x2(LJ) * (u16x2){(unsigned short)e2, (unsigned short)e2});
        const uint32_t G1 = pk_adds(H0, LJ1), G2 = pk_adds(H0, LJ2);
        const uint32_t Ga = __builtin_amdgcn_perm(G2, G1, 0x05040100u);
        const uint32_t Gb = __builtin_amdgcn_perm(G2, G1, 0x07060302u);
        incv[h] = pk_scan_umax(pk_max(Ga, Gb) ^ kNeg2);
        H0v[h] = H0;
        Mv[h] = M;
        X1v[h] = X1;
        X2v[h] = X2;
        MKv[h] = MK;
        K1v[h] = K1;
        K2v[h] = K2;
        G1v[h] = G1;
        G2v[h] = G2;
        Gav[h] = Ga;
        invv[h] = inv;
        LJ1v[h] = LJ1;
        LJ2v[h] = LJ2;
    }
    // the lower half's total (both F planes, biased) is the carry into the upper half
    const uint32_t carry = (uint32_t)__builtin_amdgcn_readlane((int)incv[0], kWave - 1);
    uint32_t *wr = reinterpret_cast<uint32_t *>(ring16_row<RW>(sh, R.r & (kRing16 - 1)));
    gint *svp = sv + svbase;
    int amv = -2147483647 - 1;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int j0 = cb0 + kChunk * h + 2 * lane;
        const int iw = (j0 >> 1) & (HW - 1);
        uint32_t Pa = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incv[h], 0x138, 0xf, 0xf, true);
        if (h == 1) Pa = pk_umax(Pa, carry);
        Pa ^= kNeg2;
        const uint32_t Pb = pk_max(Pa, Gav[h]);
        const uint32_t P1 = __builtin_amdgcn_perm(Pb, Pa, 0x05040100u);
        const uint32_t P2 = __builtin_amdgcn_perm(Pb, Pa, 0x07060302u);
        const uint32_t F1 = pk_subs(P1, LJ1v[h] + pk2(oe1 - e1)), F2 = pk_subs(P2, LJ2v[h] + pk2(oe2 - e2));
        const uint32_t X1 = X1v[h], X2 = X2v[h], H0 = H0v[h];
        const uint32_t H = pk_max(H0, pk_max(F1, F2));
        const uint32_t X1e = pk_subs(X1, pk2(e1)), Ho1 = pk_subs(H, pk2(oe1));
        const uint32_t X2e = pk_subs(X2, pk2(e2)), Ho2 = pk_subs(H, pk2(oe2));
        const uint32_t E1 = pk_max(X1e, Ho1), E2 = pk_max(X2e, Ho2);
        const uint32_t tbv = tb_pack(pk_subs(Mv[h], H), pk_subs(X1, H), pk_subs(X2, H), pk_subs(F1, H),
                                     pk_subs(Ho1, X1e), pk_subs(Ho2, X2e), pk_subs(G1v[h], P1), pk_subs(G2v[h], P2));
        row_store<uint16_t>(tb + ds.tb_used, (uint32_t)(kChunk * h + 2 * lane), (uint16_t)tbv);
        if (R.multi) {
            gu8 *kq = kp + ds.kp_used;
            if (ks == 1) {
                const uint32_t kb = MKv[h] | (K1v[h] << 2) | (K2v[h] << 4);
                row_store<uint16_t>(kq, (uint32_t)(kChunk * h + 2 * lane), (uint16_t)__builtin_amdgcn_perm(0u, kb, 0x0C0C0200u));
            } else {
                const uint32_t ko = (uint32_t)(3 * (kChunk * h + 2 * lane));
                row_store<uint16_t>(kq, ko, (uint16_t)__builtin_amdgcn_perm(K1v[h], MKv[h], 0x0C0C0400u));
                row_store<uint16_t>(kq, ko + 2u, (uint16_t)__builtin_amdgcn_perm(MKv[h], K2v[h], 0x0C0C0600u));
                row_store<uint16_t>(kq, ko + 4u, (uint16_t)__builtin_amdgcn_perm(K2v[h], K1v[h], 0x0C0C0602u));
            }
        }
        const uint32_t inv = invv[h];
        const uint32_t Hs = bfi(inv, kNeg2, H);
        wr[iw] = Hs;
        wr[HW + iw] = bfi(inv, kNeg2, E1);
        wr[2 * HW + iw] = bfi(inv, kNeg2, E2);
        if (R.far) {  // spill planes of a two-chunk row: stride RW (row_spill_width)
            svp[j0] = (int)(short)(H & 0xffff);
            svp[j0 + 1] = (int)H >> 16;
            svp[RW + j0] = (int)(short)(E1 & 0xffff);
            svp[RW + j0 + 1] = (int)E1 >> 16;
            svp[2 * RW + j0] = (int)(short)(E2 & 0xffff);
            svp[2 * RW + j0 + 1] = (int)E2 >> 16;
        }
        ds.r16acc = pk_umin(ds.r16acc, as_u32(as_u16x2(Hs) - as_u16x2(pk2(kR16Low))));
        // leftmost argmax: value above 8 bits of (255 - column offset)
        const int c0 = kChunk * h + 2 * lane;
        const int ca = ((int)(short)(Hs & 0xffff) << 8) | (255 - c0);
        const int cbk = (((int)Hs >> 16) << 8) | (254 - c0);
        amv = max(amv, max(ca, cbk));
    }
    const int mp = readlane(dpp_incl_max(amv, -2147483647 - 1), kWave - 1);
    const int besti = cb0 + 255 - (mp & 255);
    ds.tb_used += R.tbw;
    if (R.multi) ds.kp_used += ks * R.tbw;
    if (R.far) ds.sv_used += 3 * RW;
    ds.cells += end - beg + 1;
    if (lane == 0) {
        sh.rrow[R.r & (kRowRing - 1)] = make_int4(beg, end, besti, soff);
        row_record(rinfo, R.r, beg, end, tbbase, kpbase, R.far, besti, soff);
    }
    return besti;
}

// ---- wide rows over two waves (wide launches with two-wave workgroups, PoaKArgs::nw == 2) ----------
// A group of long reads runs on one wave for its whole life, so a launch lasts at least its longest
// group's one-wave latency (config 5's 8.5 kb groups, config 3's 5-6 kb ones, the per-rank floor of the
// multi-GPU split).  In a two-wave workgroup wave 0 runs the group as before (descriptors, one-chunk rows,
// backtrack, graph update, consensus) and wave 1 takes the upper 128-column half of every two-chunk fast
// row: wave 0 posts the row's control (band, predecessors, allocation) in LDS and both waves pass a
// workgroup barrier (B0); each computes its half up to the F prefix scan and its half's argmax key, the
// two exchange the lower half's F total (the upper half's carry-in) and the keys through LDS (barrier BX),
// and each finishes its half: traceback bytes, predecessor bytes, ring and spill columns.  The next row's
// B0 orders the ring halves for both waves' predecessor reads.  A one-chunk or generic row after a split
// row first passes a B0 with a no-op command (wave 0 then reads ring columns wave 1 wrote).  Per split row
// each wave issues one half's VALU work instead of both halves' (row16w_vec), at the cost of two barriers.
// The argmax comes from H0 (before F) in both waves: F only carries values from the left minus gap
// penalties, so it never reaches the row maximum and the leftmost argmax cell of H is that of H0.
constexpr int kW2Row = 1, kW2Nop = 2, kW2End = 3, kW2Exit = 4;
struct W2Cmd {
    int op, r, beg, end, cb0, tbw, vb, pn, b0, e0, b1, e1, p0slot, p1slot, two, far, multi, pn3;
    int tb_used, kp_used, sv_used, pad0, pad1, pad2;
};
static_assert(sizeof(W2Cmd) == 96, "the command is read as six int4");
struct W2Lds {
    W2Cmd cmd;
    int carry, am0, am1, flag;
};
__device__ __forceinline__ W2Lds &w2lds() {
    __shared__ W2Lds v;
    return v;
}

// wave 0: publish a split row's control (and the allocation counters of this read) for wave 1
__device__ __forceinline__ void w2_post_row(const Row16 &R, const DpState &ds, int lane) {
    W2Lds &X = w2lds();
    if (lane == 0) {
        int4 *c = reinterpret_cast<int4 *>(&X.cmd);
        c[0] = make_int4(kW2Row, R.r, R.beg, R.end);
        c[1] = make_int4(R.cb0, R.tbw, R.vb, R.pn);
        c[2] = make_int4(R.b0, R.e0, R.b1, R.e1);
        c[3] = make_int4(R.p0slot, R.p1slot, R.two, R.far);
        c[4] = make_int4(R.multi, R.pn3, ds.tb_used, ds.kp_used);
        c[5] = make_int4(ds.sv_used, 0, 0, 0);
    }
}
__device__ __forceinline__ void w2_post_op(int op, int lane) {
    if (lane == 0) w2lds().cmd.op = op;
}

// One half (h: 0 lower, 1 upper; wave-uniform) of a two-chunk fast row, computed by wave h of a two-wave
// workgroup; the same cells, bytes and ring values as row16w_vec's half h.  Returns the row's argmax.
template <class SC>
__device__ __forceinline__ int row16w_half(const SC &sc, gu8 *tb, gu8 *kp, gint *sv, gint *rinfo, SharedState &sh,
                                           int lane, const Row16 &R, DpState &ds, int h) {
    constexpr int RW = kWideRing, HW = RW / 2;
    W2Lds &X = w2lds();
    const int e1 = sc.e1, e2 = sc.e2, oe1 = sc.o1 + sc.e1, oe2 = sc.o2 + sc.e2;
    const int beg = R.beg, end = R.end, cb0 = R.cb0;
    const int tbbase = ds.tb_used - cb0;
    const int ks = kp_stride(R.pn);
    const int kpbase = ds.kp_used - ks * cb0;
    const int soff = R.far ? ds.sv_used : -1;
    const int svbase = ds.sv_used - cb0;
    const uint32_t *w0 = reinterpret_cast<const uint32_t *>(ring16_row<RW>(sh, R.p0slot));
    const uint32_t *w1 = reinterpret_cast<const uint32_t *>(ring16_row<RW>(sh, R.p1slot));
    const uint32_t tlo =
        R.vb < 4 ? (uint32_t)(sc.match + sc.mismatch) << (8 * R.vb) : (uint32_t)sc.mismatch * 0x01010101u;
    const uint32_t B0 = pk2s(R.b0), E0 = pk2s(R.e0), B1 = pk2s(R.b1), E1b = pk2s(R.e1);
    const uint32_t BEG = pk2s(beg), END = pk2s(end);
    const int c0 = kChunk * h + 2 * lane;  // the lane's first column, relative to cb0
    const int j0 = cb0 + c0;
    const uint32_t J = (uint32_t)j0 * 0x10001u + 0x10000u;  // (j0, j0 + 1)
    const uint32_t LJ = (uint32_t)c0 * 0x10001u + 0x10000u;  // the same - cb0
    const uint32_t inv = pk_neg_mask(as_u32(as_s16x2(J) - as_s16x2(BEG)) | as_u32(as_s16x2(END) - as_s16x2(J)));
    const uint32_t qbyte = qnib<RW>()[j0 >> 1];
    const uint32_t sel = ((qbyte * 0x1001u) & 0x000F000Fu) | 0x0C000C00u;
    const uint32_t S = __builtin_amdgcn_perm((uint32_t)sc.mismatch, tlo, sel);
    const int iw = (j0 >> 1) & (HW - 1), iwp = (iw - 1) & (HW - 1);
    const uint32_t JD = as_u32(as_s16x2(J) - (s16x2){1, 1});  // (j0 - 1, j0)
    uint32_t Hd = __builtin_amdgcn_alignbit(w0[iw], w0[iwp], 16);
    uint32_t X1 = w0[HW + iw], X2 = w0[2 * HW + iw];
    {
        const uint32_t md = pk_neg_mask(as_u32(as_s16x2(JD) - as_s16x2(B0)) | as_u32(as_s16x2(E0) - as_s16x2(JD)));
        const uint32_t me = pk_neg_mask(as_u32(as_s16x2(J) - as_s16x2(B0)) | as_u32(as_s16x2(E0) - as_s16x2(J)));
        Hd = bfi(md, kNeg2, Hd);
        X1 = bfi(me, kNeg2, X1);
        X2 = bfi(me, kNeg2, X2);
    }
    uint32_t MK = 0, K1 = 0, K2 = 0;
    if (R.two) {
        uint32_t Hd1 = __builtin_amdgcn_alignbit(w1[iw], w1[iwp], 16);
        uint32_t X11 = w1[HW + iw], X21 = w1[2 * HW + iw];
        const uint32_t md = pk_neg_mask(as_u32(as_s16x2(JD) - as_s16x2(B1)) | as_u32(as_s16x2(E1b) - as_s16x2(JD)));
        const uint32_t me = pk_neg_mask(as_u32(as_s16x2(J) - as_s16x2(B1)) | as_u32(as_s16x2(E1b) - as_s16x2(J)));
        Hd1 = bfi(md, kNeg2, Hd1);
        X11 = bfi(me, kNeg2, X11);
        X21 = bfi(me, kNeg2, X21);
        MK = pk_lt_bit<0>(Hd, Hd1);
        K1 = pk_lt_bit<0>(X1, X11);
        K2 = pk_lt_bit<0>(X2, X21);
        Hd = pk_max(Hd, Hd1);
        X1 = pk_max(X1, X11);
        X2 = pk_max(X2, X21);
    }
    for (int k = 2; k < R.pn3; ++k) {  // the first strictly larger value names the predecessor
        const int p = bcast0(sh.desc[R.r & (kDescBatch - 1)][3 + k]);
        const int4 xr = sh.rrow[p & (kRowRing - 1)];
        const uint32_t Bk = pk2s(xr.x), Ek = pk2s(xr.y);
        const uint32_t *wk = reinterpret_cast<const uint32_t *>(ring16_row<RW>(sh, p & (kRing16 - 1)));
        uint32_t Hdk = __builtin_amdgcn_alignbit(wk[iw], wk[iwp], 16);
        uint32_t X1k = wk[HW + iw], X2k = wk[2 * HW + iw];
        const uint32_t md = pk_neg_mask(as_u32(as_s16x2(JD) - as_s16x2(Bk)) | as_u32(as_s16x2(Ek) - as_s16x2(JD)));
        const uint32_t me = pk_neg_mask(as_u32(as_s16x2(J) - as_s16x2(Bk)) | as_u32(as_s16x2(Ek) - as_s16x2(J)));
        Hdk = bfi(md, kNeg2, Hdk);
        X1k = bfi(me, kNeg2, X1k);
        X2k = bfi(me, kNeg2, X2k);
        const uint32_t kk = pk2(k);
        MK = bfi(pk_neg_mask(pk_subs(Hd, Hdk)), kk, MK);
        K1 = bfi(pk_neg_mask(pk_subs(X1, X1k)), kk, K1);
        K2 = bfi(pk_neg_mask(pk_subs(X2, X2k)), kk, K2);
        Hd = pk_max(Hd, Hdk);
        X1 = pk_max(X1, X1k);
        X2 = pk_max(X2, X2k);
    }
    const uint32_t M = pk_subs(pk_adds(Hd, S), pk2(sc.mismatch));
    const uint32_t H0 = bfi(inv, kNeg2, pk_max(M, pk_max(X1, X2)));
    const uint32_t LJ1 = as_u32(as_u16x2(LJ) * (u16x2){(unsigned short)e1, (unsigned short)e1});
    const uint32_t LJ2 = as_u32(as_u16x2(LJ) * (u16x2){(unsigned short)e2, (unsigned short)e2});
    const uint32_t G1 = pk_adds(H0, LJ1), G2 = pk_adds(H0, LJ2);
    const uint32_t Ga = __builtin_amdgcn_perm(G2, G1, 0x05040100u);
    const uint32_t Gb = __builtin_amdgcn_perm(G2, G1, 0x07060302u);
    // the half's F prefix scan and its argmax key (H0 << 8 | 255 - column offset) in one DPP stream
    uint32_t inc = pk_max(Ga, Gb) ^ kNeg2;
    int amk = max(((int)(short)(H0 & 0xffff) << 8) | (255 - c0), (((int)H0 >> 16) << 8) | (254 - c0));
    dpp_scan_fa(inc, amk);
    // exchange: the lower half's F total (the upper half's carry-in) and both halves' argmax keys
    const int myam = readlane(amk, kWave - 1);
    if (h == 0) {
        const int tot = readlane((int)inc, kWave - 1);
        if (lane == 0) {
            X.carry = tot;
            X.am0 = myam;
        }
    } else if (lane == 0) {
        X.am1 = myam;
    }
    group_barrier();  // BX
    const int other = bcast0(h ? X.am0 : X.am1);
    const uint32_t carry = h ? (uint32_t)bcast0(X.carry) : 0u;
    const int mp = max(myam, other);
    const int besti = cb0 + 255 - (mp & 255);
    uint32_t Pa = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)inc, 0x138, 0xf, 0xf, true);
    Pa = pk_umax(Pa, carry) ^ kNeg2;  // carry 0 (the identity) in the lower half
    const uint32_t Pb = pk_max(Pa, Ga);
    const uint32_t P1 = __builtin_amdgcn_perm(Pb, Pa, 0x05040100u);
    const uint32_t P2 = __builtin_amdgcn_perm(Pb, Pa, 0x07060302u);
    const uint32_t F1 = pk_subs(P1, LJ1 + pk2(oe1 - e1)), F2 = pk_subs(P2, LJ2 + pk2(oe2 - e2));
    const uint32_t H = pk_max(H0, pk_max(F1, F2));
    const uint32_t X1e = pk_subs(X1, pk2(e1)), Ho1 = pk_subs(H, pk2(oe1));
    const uint32_t X2e = pk_subs(X2, pk2(e2)), Ho2 = pk_subs(H, pk2(oe2));
    const uint32_t E1 = pk_max(X1e, Ho1), E2 = pk_max(X2e, Ho2);
    const uint32_t tbv = tb_pack(pk_subs(M, H), pk_subs(X1, H), pk_subs(X2, H), pk_subs(F1, H), pk_subs(Ho1, X1e),
                                 pk_subs(Ho2, X2e), pk_subs(G1, P1), pk_subs(G2, P2));
    row_store<uint16_t>(tb + ds.tb_used, (uint32_t)c0, (uint16_t)tbv);
    if (R.multi) {
        gu8 *kq = kp + ds.kp_used;
        if (ks == 1) {
            const uint32_t kb = MK | (K1 << 2) | (K2 << 4);
            row_store<uint16_t>(kq, (uint32_t)c0, (uint16_t)__builtin_amdgcn_perm(0u, kb, 0x0C0C0200u));
        } else {
            const uint32_t ko = (uint32_t)(3 * c0);
            row_store<uint16_t>(kq, ko, (uint16_t)__builtin_amdgcn_perm(K1, MK, 0x0C0C0400u));
            row_store<uint16_t>(kq, ko + 2u, (uint16_t)__builtin_amdgcn_perm(MK, K2, 0x0C0C0600u));
            row_store<uint16_t>(kq, ko + 4u, (uint16_t)__builtin_amdgcn_perm(K2, K1, 0x0C0C0602u));
        }
    }
    uint32_t *wr = reinterpret_cast<uint32_t *>(ring16_row<RW>(sh, R.r & (kRing16 - 1)));
    const uint32_t Hs = bfi(inv, kNeg2, H);
    wr[iw] = Hs;
    wr[HW + iw] = bfi(inv, kNeg2, E1);
    wr[2 * HW + iw] = bfi(inv, kNeg2, E2);
    if (R.far) {  // spill planes of a two-chunk row: stride RW (row_spill_width)
        gint *svp = sv + svbase;
        svp[j0] = (int)(short)(H & 0xffff);
        svp[j0 + 1] = (int)H >> 16;
        svp[RW + j0] = (int)(short)(E1 & 0xffff);
        svp[RW + j0 + 1] = (int)E1 >> 16;
        svp[2 * RW + j0] = (int)(short)(E2 & 0xffff);
        svp[2 * RW + j0 + 1] = (int)E2 >> 16;
    }
    ds.r16acc = pk_umin(ds.r16acc, as_u32(as_u16x2(Hs) - as_u16x2(pk2(kR16Low))));
    ds.tb_used += R.tbw;
    if (R.multi) ds.kp_used += ks * R.tbw;
    if (R.far) ds.sv_used += 3 * RW;
    ds.cells += end - beg + 1;
    if (h == 0 && lane == 0) {
        sh.rrow[R.r & (kRowRing - 1)] = make_int4(beg, end, besti, soff);
        row_record(rinfo, R.r, beg, end, tbbase, kpbase, R.far, besti, soff);
    }
    return besti;
}

// Wave 1 of a two-wave workgroup: upper halves of the split rows wave 0 posts, until the exit command.
// At the end of every read's DP (kW2End) it reports whether any of its cells came near the 16-bit -inf
// band (the read is then re-aligned in 32-bit mode, by wave 0 alone).
template <class SC>
__device__ __forceinline__ void w2_helper(SharedState &sh, int lane) {
    W2Lds &X = w2lds();
    gu8 *tb, *kp;
    gint *sv, *rinfo;
    SC sc;
    {
        const Slot s = slot_of(sh);
        tb = s.tb;
        kp = s.kp;
        sv = s.sv;
        rinfo = s.rinfo;
        if constexpr (!std::is_same<SC, DefaultScores>::value) {
            const PoaRunArgs a = args_of(sh);
            sc = SC{a.match, a.mismatch, a.o1, a.e1, a.o2, a.e2};
        }
    }
    DpState ds{0, 0, 0, 0, 0xffffffffu, 0, {0, 0, 0, 0}};
    int spilled = 0;
    for (;;) {
        // a far row's spill columns may be read by wave 0 (a later row whose predecessor left the ring):
        // they are complete before the next barrier (the workgroup barrier orders LDS, not pending stores)
        if (spilled) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        spilled = 0;
        group_barrier();  // B0
        const int4 c0 = *reinterpret_cast<const int4 *>(&X.cmd);
        const int op = bcast0(c0.x);
        if (op == kW2Exit) break;
        if (op == kW2Nop) continue;
        if (op == kW2End) {
            // the read's traceback / predecessor bytes are complete before wave 0's backtrack reads them
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const uint32_t m = min(ds.r16acc & 0xffffu, ds.r16acc >> 16);
            const unsigned long long nearinf = __ballot(m < (uint32_t)(kR16High - kR16Low));
            if (lane == 0) X.flag = nearinf ? 1 : 0;
            ds.r16acc = 0xffffffffu;
            group_barrier();  // the flag is read by wave 0
            continue;
        }
        const int4 *c = reinterpret_cast<const int4 *>(&X.cmd);
        const int4 c1 = c[1], c2 = c[2], c3 = c[3], c4 = c[4], c5 = c[5];
        Row16 R;
        R.r = bcast0(c0.y);
        R.beg = bcast0(c0.z);
        R.end = bcast0(c0.w);
        R.cb0 = bcast0(c1.x);
        R.tbw = bcast0(c1.y);
        R.vb = bcast0(c1.z);
        R.pn = bcast0(c1.w);
        R.b0 = bcast0(c2.x);
        R.e0 = bcast0(c2.y);
        R.b1 = bcast0(c2.z);
        R.e1 = bcast0(c2.w);
        R.p0slot = bcast0(c3.x);
        R.p1slot = bcast0(c3.y);
        R.two = bcast0(c3.z);
        R.far = bcast0(c3.w);
        R.multi = bcast0(c4.x);
        R.pn3 = bcast0(c4.y);
        ds.tb_used = bcast0(c4.z);
        ds.kp_used = bcast0(c4.w);
        ds.sv_used = bcast0(c5.x);
        row16w_half<SC>(sc, tb, kp, sv, rinfo, sh, lane, R, ds, 1);
        spilled = R.far;
    }
}

// ---- fast rows, hand-scheduled (narrow launches, default scores) -------------------------------
// The row loop above, for the rows that make up ~90 % of a narrow launch (config-3/4 rows: one
// predecessor 60 %, two 30 %): fast rows (bit 15 of the descriptor) with one or two predecessors in
// the LDS ring, in batches whose capacity check passed.  Written as one asm loop because the
// compiler's form of the same row spends ~110 scalar instructions on it (bool masks materialised as
// 64-bit lane masks, register copies at the joins of the row kinds, SGPRs reloaded from VGPR lanes,
// lane-0 record stores through exec save / restore) next to ~110 vector ones, and at four waves per
// SIMD both issue ports are saturated (DESIGN.md §3.1 issue model); here the row's control is ~60
// scalar instructions and the vector stream is the same cells as row16_vec.  Every value follows
// run_dp16 / row16_vec exactly (same band, masks, traceback and predecessor bytes, ring and spill
// planes, row records); tests/test_poa_gpu.py compares the bytes with the oracle.
// The loop leaves at the batch end or at the first row it does not take (the C++ row handles it):
// nothing of that row has been written then.  The next row's descriptor words are read from the LDS
// batch once the row's traceback is stored (into the registers the row is done with), so the row head
// finds them loaded instead of waiting on the LDS round trip; at the batch end that read is past the
// batch and unused, and the loop drains it before it leaves.  Hazards (gfx950) are padded inside the string: DPP
// reads two wait states after a VALU write, v_readlane after the scans, VMEM reads of SGPRs written
// by a VALU before the block (s_nop 4).  Exec is the whole wave here (run_dp16 runs wave-uniform; the
// scans need every lane; MANDO_CHECK_EXEC builds trap otherwise); the row records are stored with
// exec = lane 0, exec saved in vcc around them and restored from it.
// A row's head -- descriptor words to SGPRs, the scalar band, the ring addresses and reads up to the
// diagonal of the (first) predecessor -- runs at wave priority 2 (the rest of the row at 0, the serial
// phases at 3): it is the latency-bound start of the row's dependent stream, and a wave there issues
// ahead of the co-resident waves' bulk cell work (kernel -0.7 % / -1.8 % on the config-3 / config-4
// group shapes, profiles/r08ah_*; the scans at 2 as well, or the window up to them, gain less).
typedef __attribute__((address_space(3))) uint8_t lds_u8;
__device__ __forceinline__ uint32_t lds_addr(const void *p) {
    return (uint32_t)(uintptr_t)(lds_u8 *)(const_cast<void *>(p));
}

#define MANDO_FR_OPERANDS \
        : [i] "+s"(i), [pr] "+s"(pr), [pb] "+s"(pb), [pe] "+s"(pe), [pa] "+s"(pa), [tbu] "+s"(tbu), \
          [kpu] "+s"(kpu), [svu] "+s"(svu), [cel] "+s"(cel), [r16] "+v"(r16), \
          [d1] "=&s"(d1), [rem] "=&s"(rem), [p0] "=&s"(p0), [p1] "=&s"(p1), [rb1] "=&s"(rb1), [re1] "=&s"(re1), \
          [ra1] "=&s"(ra1), [x] "=&s"(x), [y] "=&s"(y), [z] "=&s"(z), [beg] "=&s"(beg), [end] "=&s"(end), \
          [cb0] "=&s"(cb0), [spm] "=&s"(spm), [pc0] "=&s"(pc0), [pc1] "=&s"(pc1), [tlo] "=&s"(tlo), [pkb] "=&s"(pkb), \
          [pke] "=&s"(pke), [base1] "=&s"(base1), [mp] "=&s"(mp), [besti] "=&s"(besti), [r] "=&s"(r), \
          [pwb] "=&s"(pwb), [i0] "=&s"(i0), [c20002] "=&s"(c20002), [c128] "=&s"(c128), [cr16] "=&s"(cr16), \
          [cq] "=&s"(cq), [cth] "=&s"(cth), [csel0] "=&s"(csel0), [csel1] "=&s"(csel1), [cseltb] "=&s"(cseltb), \
          [cselkp] "=&s"(cselkp), [m01] "=&s"(m01), [m23] "=&s"(m23), [m45] "=&s"(m45), [m67] "=&s"(m67), \
          [Ga] "=&v"(Ga), [Gb] "=&v"(Gb), [Pa] "=&v"(Pa), [Pb] "=&v"(Pb), [inc] "=&v"(inc), [S] "=&v"(S), \
          [M] "=&v"(M), [H0] "=&v"(H0), [E1] "=&v"(E1), [t1] "=&v"(t1), [F1] "=&v"(F1), [P1] "=&v"(P1), \
          [P2] "=&v"(P2), [iw] "=&v"(iw), [a0] "=&v"(a0), [inv] "=&v"(inv), [m1] "=&v"(m1), [m2] "=&v"(m2), \
          [Hd] "=&v"(Hd), [X1] "=&v"(X1), [X2] "=&v"(X2), [MK] "=&v"(MK), [K1] "=&v"(K1), [K2] "=&v"(K2), \
          [G1] "=&v"(G1), [G2] "=&v"(G2), [amk] "=&v"(amk), [H] "=&v"(H), [X1e] "=&v"(X1e), [Ho1] "=&v"(Ho1), \
          [X2e] "=&v"(X2e), [Ho2] "=&v"(Ho2), [E2] "=&v"(E2), [voff] "=&v"(voff), [vlane] "=&v"(vlane), \
          [vlane2] "=&v"(vlane2), [vlane8] "=&v"(vlane8), [LJ1] "=&v"(LJ1), [LJ2] "=&v"(LJ2), [FJ1] "=&v"(FJ1), \
          [FJ2] "=&v"(FJ2), [clo] "=&v"(clo), [chi] "=&v"(chi), [vkneg] "=&v"(vkneg), [v10000] "=&v"(v10000), \
          [v0c0c] "=&v"(v0c0c) \
        : [iend] "s"(iend), [b0] "s"(b0), [qlen] "s"(qlen), [w] "s"(w), [Ldesc] "s"(Ldesc), [Lrrow] "s"(Lrrow), \
          [Lring] "s"(Lring), [Lq] "s"(Lq), [tbp] "s"(tbp), [kpp] "s"(kpp), [svp] "s"(svp), [rip] "s"(rip) \
        : "memory", "scc", "vcc", "v120", "v121", "v122", "v123", "v124", "v125"

__device__ __forceinline__ int fast_rows_asm(SharedState &sh, int lane, gu8 *tb, gu8 *kp, gint *sv, gint *rinfo,
                                             int b0, int i, int iend, int qlen, int w, int &prv_r, int &prv_beg,
                                             int &prv_end, int &prv_am, DpState &ds) {
    constexpr int RW = kChunk;
    using SC = DefaultScores;
    static_assert(SC::match == 5 && SC::mismatch == 4 && SC::o1 == 4 && SC::e1 == 2 && SC::o2 == 24 && SC::e2 == 1,
                  "the constants below are abPOA's defaults");
    static_assert(kRing16 == 8 && kChunk == 128 && kRowRing == 32 && kDescInts == 8 && kRowInfoInts == 8,
                  "LDS / HBM geometry the block assumes");
    const uint32_t Ldesc = lds_addr(&sh.desc[0][0]), Lrrow = lds_addr(&sh.rrow[0]);
    const uint32_t Lring = lds_addr(ring16_row<RW>(sh, 0)), Lq = lds_addr(qnib<RW>());
    const uint64_t tbp = (uint64_t)uni64((int64_t)tb), kpp = (uint64_t)uni64((int64_t)kp);
    const uint64_t svp = (uint64_t)uni64((int64_t)sv), rip = (uint64_t)uni64((int64_t)rinfo);
    int pr = prv_r, pb = prv_beg, pe = prv_end, pa = prv_am;
    int tbu = ds.tb_used, kpu = ds.kp_used, svu = ds.sv_used, cel = ds.cells;
    uint32_t r16 = ds.r16acc;
    (void)lane;
    // scalar temporaries and constants
    int d1, rem, p0, p1, rb1, re1, ra1, x, y, z, beg, end, cb0, spm, pc0, pc1, tlo, pkb, pke, base1, mp, besti, r, pwb,
        i0, c20002, c128, cr16, cq, cth, csel0, csel1, cseltb, cselkp, m01, m23, m45, m67;
    // vector temporaries (several names of the row share a register where their lifetimes do not
    // overlap: the address and descriptor words of the row head live in the G / P registers of the F
    // scan, the read's code and selector in S, ... -- 34 registers instead of 57, so the block leaves
    // the kernel's other values in registers) and the lane constants, set at the block's entry
    uint32_t Ga, Gb, Pa, Pb, inc, S, M, H0, E1, t1, F1, P1, P2, iw, a0, inv, m1, m2, Hd, X1, X2, MK, K1, K2, G1, G2,
        amk, H, X1e, Ho1, X2e, Ho2, E2, voff, vlane, vlane2, vlane8, LJ1, LJ2, FJ1, FJ2, clo, chi, vkneg, v10000,
        v0c0c;
    {
        asm volatile(
            "s_nop 4\n"
            "s_waitcnt lgkmcnt(0)\n"
            "s_mov_b32 %[c20002], 0x20002\n"
            "s_movk_i32 %[c128], 0x80\n"
            "s_movk_i32 %[cr16], 0x7918\n"
            "s_mov_b32 %[cq], 0xf000f\n"
            "s_mov_b32 %[cth], 0x4040404\n"
            "s_mov_b32 %[csel0], 0x5040100\n"
            "s_mov_b32 %[csel1], 0x7060302\n"
            "s_mov_b32 %[cseltb], 0xb0a0908\n"
            "s_mov_b32 %[cselkp], 0xc0c0200\n"
            "s_mov_b32 %[m01], 0x2020101\n"
            "s_mov_b32 %[m23], 0x8080404\n"
            "s_mov_b32 %[m45], 0x20201010\n"
            "s_mov_b32 %[m67], 0x80804040\n"
            "v_mbcnt_lo_u32_b32 %[vlane], -1, 0\n"
            "v_mbcnt_hi_u32_b32 %[vlane], -1, %[vlane]\n"
            "v_lshlrev_b32 %[vlane2], 1, %[vlane]\n"
            "v_lshlrev_b32 %[vlane8], 3, %[vlane]\n"
            "v_mul_u32_u24 %[LJ2], 0x10001, %[vlane2]\n"
            "v_add_u32 %[LJ2], 0x10000, %[LJ2]\n"
            "v_lshlrev_b32 %[LJ1], 1, %[LJ2]\n"
            "v_add_u32 %[FJ1], 0x40004, %[LJ1]\n"
            "v_add_u32 %[FJ2], 0x180018, %[LJ2]\n"
            "v_sub_u32 %[clo], 0x7f, %[vlane2]\n"
            "v_sub_u32 %[chi], 0x7e, %[vlane2]\n"
            "v_mov_b32 %[vkneg], 0x80008000\n"
            "v_mov_b32 %[v10000], 0x10000\n"
            "v_mov_b32 %[v0c0c], 0xc000c00\n"
            "s_mov_b32 %[i0], %[i]\n"
            "s_and_b32 %[x], %[pr], 7\n"
            "s_mulk_i32 %[x], 0x300\n"
            "s_add_u32 %[pwb], %[x], %[Lring]\n"
            "s_lshl_b32 %[x], %[i], 5\n"
            "s_add_u32 %[x], %[x], %[Ldesc]\n"
            "v_mov_b32 %[Ga], %[x]\n"
            "ds_read_b32 %[Gb], %[Ga] offset:4\n"
            "ds_read_b32 %[Pa], %[Ga] offset:8\n"
            "ds_read_b32 %[Pb], %[Ga] offset:12\n"
            "ds_read_b32 %[inc], %[Ga] offset:16\n"
            "L_top%=:\n"
            "s_cmp_ge_i32 %[i], %[iend]\n"
            "s_cbranch_scc1 L_out%=\n"
            "s_waitcnt lgkmcnt(0)\n"
            "s_setprio 2\n"
            "v_readfirstlane_b32 %[d1], %[Gb]\n"
            "v_readfirstlane_b32 %[p0], %[Pb]\n"
            "v_readfirstlane_b32 %[rem], %[Pa]\n"
            "s_and_b32 %[y], %[d1], 0xffffc000\n"
            "s_cmp_eq_u32 %[y], 0x18000\n"
            "s_cbranch_scc0 L_two%=\n"
            "s_cmp_eq_u32 %[p0], %[pr]\n"
            "s_cbranch_scc1 L_p0ok1%=\n"
            "s_and_b32 %[x], %[p0], 31\n"
            "s_lshl_b32 %[x], %[x], 4\n"
            "s_add_u32 %[x], %[x], %[Lrrow]\n"
            "v_mov_b32 %[Ga], %[x]\n"
            "ds_read_b32 %[Gb], %[Ga]\n"
            "ds_read_b32 %[Pa], %[Ga] offset:4\n"
            "ds_read_b32 %[Pb], %[Ga] offset:8\n"
            "s_and_b32 %[x], %[p0], 7\n"
            "s_mulk_i32 %[x], 0x300\n"
            "s_add_u32 %[pwb], %[x], %[Lring]\n"
            "s_waitcnt lgkmcnt(0)\n"
            "v_readfirstlane_b32 %[pb], %[Gb]\n"
            "v_readfirstlane_b32 %[pe], %[Pa]\n"
            "v_readfirstlane_b32 %[pa], %[Pb]\n"
            "s_mov_b32 %[pr], %[p0]\n"
            "L_p0ok1%=:\n"
            "s_sub_i32 %[x], %[qlen], %[rem]\n"
            "s_add_i32 %[z], %[pa], 1\n"
            "s_min_i32 %[y], %[z], %[x]\n"
            "s_max_i32 %[z], %[z], %[x]\n"
            "s_sub_i32 %[y], %[y], %[w]\n"
            "s_add_i32 %[z], %[z], %[w]\n"
            "s_max_i32 %[beg], %[y], 0\n"
            "s_min_i32 %[end], %[z], %[qlen]\n"
            "s_and_b32 %[cb0], %[beg], -2\n"
            "s_sub_i32 %[spm], %[end], %[cb0]\n"
            "s_and_b32 %[pc0], %[pb], -2\n"
            "s_sub_i32 %[x], %[pe], %[pc0]\n"
            "s_max_i32 %[x], %[x], %[spm]\n"
            "s_cmpk_gt_i32 %[x], 0x7f\n"
            "s_cbranch_scc1 L_out%=\n"
            "s_bfe_u32 %[z], %[d1], 0x80000\n"
            "s_lshl_b32 %[x], %[z], 3\n"
            "s_lshl_b32 %[tlo], 9, %[x]\n"
            "s_cmp_gt_u32 %[z], 3\n"
            "s_cselect_b32 %[tlo], %[cth], %[tlo]\n"
            "s_pack_ll_b32_b16 %[pkb], %[beg], %[beg]\n"
            "s_pack_ll_b32_b16 %[pke], %[end], %[end]\n"
            "s_bfe_u32 %[x], %[cb0], 0xf0001\n"
            "v_add_u32 %[M], %[x], %[vlane]\n"
            "v_mad_u32_u24 %[H0], %[M], %[c20002], %[v10000]\n"
            "v_add_u32 %[Ga], %[Lq], %[M]\n"
            "ds_read_u8 %[S], %[Ga]\n"
            "v_and_b32 %[iw], 63, %[M]\n"
            "v_lshl_add_u32 %[a0], %[iw], 2, %[pwb]\n"
            "ds_read_b32 %[E1], %[a0]\n"
            "ds_read_b32 %[X1], %[a0] offset:256\n"
            "ds_read_b32 %[X2], %[a0] offset:512\n"
            "v_pk_sub_i16 %[m1], %[H0], %[pkb]\n"
            "v_pk_sub_i16 %[m2], %[pke], %[H0]\n"
            "v_or_b32 %[m1], %[m1], %[m2]\n"
            "v_pk_ashrrev_i16 %[inv], 15, %[m1] op_sel_hi:[0,1]\n"
            "s_waitcnt lgkmcnt(3)\n"
            "v_mul_u32_u24 %[S], 0x1001, %[S]\n"
            "v_and_or_b32 %[S], %[S], %[cq], %[v0c0c]\n"
            "v_perm_b32 %[S], 4, %[tlo], %[S]\n"
            "s_waitcnt lgkmcnt(0)\n"
            "v_mov_b32_dpp %[t1], %[E1] wave_ror:1 row_mask:0xf bank_mask:0xf\n"
            "v_alignbit_b32 %[Hd], %[E1], %[t1], 16\n"
            "s_setprio 0\n"
            "s_cmp_le_i32 %[beg], %[pc0]\n"
            "s_cbranch_scc1 L_mask1%=\n"
            "s_add_u32 %[x], %[pc0], 0x7f\n"
            "s_cmp_le_i32 %[end], %[x]\n"
            "s_cbranch_scc1 L_nomask1%=\n"
            "L_mask1%=:\n"
            "s_pack_ll_b32_b16 %[x], %[pb], %[pb]\n"
            "s_pack_ll_b32_b16 %[y], %[pe], %[pe]\n"
            "v_pk_add_u16 %[t1], %[H0], -1\n"
            "v_pk_sub_i16 %[m1], %[t1], %[x]\n"
            "v_pk_sub_i16 %[m2], %[y], %[t1]\n"
            "v_or_b32 %[m1], %[m1], %[m2]\n"
            "v_pk_ashrrev_i16 %[m1], 15, %[m1] op_sel_hi:[0,1]\n"
            "v_pk_sub_i16 %[m2], %[H0], %[x]\n"
            "v_pk_sub_i16 %[t1], %[y], %[H0]\n"
            "v_or_b32 %[m2], %[m2], %[t1]\n"
            "v_pk_ashrrev_i16 %[m2], 15, %[m2] op_sel_hi:[0,1]\n"
            "v_bfi_b32 %[Hd], %[m1], %[vkneg], %[Hd]\n"
            "v_bfi_b32 %[X1], %[m2], %[vkneg], %[X1]\n"
            "v_bfi_b32 %[X2], %[m2], %[vkneg], %[X2]\n"
            "L_nomask1%=:\n"
            "v_pk_add_i16 %[M], %[Hd], %[S] clamp\n"
            "v_pk_add_i16 %[M], %[M], -4 op_sel_hi:[1,0] clamp\n"
            "v_pk_max_i16 %[t1], %[X1], %[X2]\n"
            "v_pk_max_i16 %[t1], %[M], %[t1]\n"
            "v_bfi_b32 %[H0], %[inv], %[vkneg], %[t1]\n"
            "v_pk_add_i16 %[G1], %[H0], %[LJ1] clamp\n"
            "v_pk_add_i16 %[G2], %[H0], %[LJ2] clamp\n"
            "v_perm_b32 %[Ga], %[G2], %[G1], %[csel0]\n"
            "v_perm_b32 %[Gb], %[G2], %[G1], %[csel1]\n"
            "v_pk_max_i16 %[inc], %[Ga], %[Gb]\n"
            "v_xor_b32 %[inc], 0x80008000, %[inc]\n"
            "v_mad_i32_i16 %[amk], %[H0], %[c128], %[clo]\n"
            "v_mad_i32_i16 %[t1], %[H0], %[c128], %[chi] op_sel:[1,0,0,0]\n"
            "v_max_i32 %[amk], %[amk], %[t1]\n"
            "s_nop 1\n"
            "v_mov_b32_dpp %[t1], %[inc] row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
            "v_max_i32_dpp %[amk], %[amk], %[amk] row_shr:1 row_mask:0xf bank_mask:0xf\n"
            "v_pk_max_u16 %[inc], %[inc], %[t1]\n"
            "s_nop 0\n"
            "v_max_i32_dpp %[amk], %[amk], %[amk] row_shr:2 row_mask:0xf bank_mask:0xf\n"
            "v_mov_b32_dpp %[t1], %[inc] row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
            "v_pk_max_u16 %[inc], %[inc], %[t1]\n"
            "v_max_i32_dpp %[amk], %[amk], %[amk] row_shr:4 row_mask:0xf bank_mask:0xf\n"
            "s_nop 0\n"
            "v_mov_b32_dpp %[t1], %[inc] row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
            "v_pk_max_u16 %[inc], %[inc], %[t1]\n"
            "s_nop 0\n"
            "v_max_i32_dpp %[amk], %[amk], %[amk] row_shr:8 row_mask:0xf bank_mask:0xf\n"
            "v_mov_b32_dpp %[t1], %[inc] row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
            "v_pk_max_u16 %[inc], %[inc], %[t1]\n"
            "v_max_i32_dpp %[amk], %[amk], %[amk] row_bcast:15 row_mask:0xa bank_mask:0xf\n"
            "s_nop 0\n"
            "v_mov_b32_dpp %[t1], %[inc] row_bcast:15 row_mask:0xa bank_mask:0xf\n"
            "v_pk_max_u16 %[inc], %[inc], %[t1]\n"
            "v_max_i32_dpp %[amk], %[amk], %[amk] row_bcast:31 row_mask:0xc bank_mask:0xf\n"
            "s_nop 0\n"
            "v_mov_b32_dpp %[t1], %[inc] row_bcast:31 row_mask:0xc bank_mask:0xf\n"
            "v_pk_max_u16 %[inc], %[inc], %[t1]\n"
            "s_nop 1\n"
            "v_readlane_b32 %[mp], %[amk], 63\n"
            "v_xor_b32_dpp %[Pa], %[inc], %[vkneg] wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
            "v_pk_max_i16 %[Pb], %[Pa], %[Ga]\n"
            "v_perm_b32 %[P1], %[Pb], %[Pa], %[csel0]\n"
            "v_perm_b32 %[P2], %[Pb], %[Pa], %[csel1]\n"
            "v_pk_sub_i16 %[F1], %[P1], %[FJ1] clamp\n"
            "v_pk_sub_i16 %[S], %[P2], %[FJ2] clamp\n"
            "v_pk_max_i16 %[H], %[F1], %[S]\n"
            "v_pk_max_i16 %[H], %[H0], %[H]\n"
            "v_pk_add_i16 %[X1e], %[X1], -2 op_sel_hi:[1,0] clamp\n"
            "v_pk_add_i16 %[Ho1], %[H], -6 op_sel_hi:[1,0] clamp\n"
            "v_pk_add_i16 %[X2e], %[X2], -1 clamp\n"
            "v_pk_sub_i16 %[Ho2], %[H], 25 op_sel_hi:[1,0] clamp\n"
            "v_pk_max_i16 %[E1], %[X1e], %[Ho1]\n"
            "v_pk_max_i16 %[E2], %[X2e], %[Ho2]\n"
            "v_pk_sub_i16 %[Ga], %[M], %[H] clamp\n"
            "v_pk_sub_i16 %[Gb], %[X1], %[H] clamp\n"
            "v_perm_b32 %[Pa], %[Gb], %[Ga], %[cseltb]\n"
            "v_pk_sub_i16 %[Ga], %[X2], %[H] clamp\n"
            "v_pk_sub_i16 %[Gb], %[F1], %[H] clamp\n"
            "v_perm_b32 %[Pb], %[Gb], %[Ga], %[cseltb]\n"
            "v_pk_sub_i16 %[Ga], %[Ho1], %[X1e] clamp\n"
            "v_pk_sub_i16 %[Gb], %[Ho2], %[X2e] clamp\n"
            "v_perm_b32 %[inc], %[Gb], %[Ga], %[cseltb]\n"
            "v_pk_sub_i16 %[Ga], %[G1], %[P1] clamp\n"
            "v_pk_sub_i16 %[Gb], %[G2], %[P2] clamp\n"
            "v_perm_b32 %[amk], %[Gb], %[Ga], %[cseltb]\n"
            "v_and_b32 %[amk], %[m67], %[amk]\n"
            "v_and_or_b32 %[amk], %[inc], %[m45], %[amk]\n"
            "v_and_or_b32 %[amk], %[Pb], %[m23], %[amk]\n"
            "v_and_or_b32 %[amk], %[Pa], %[m01], %[amk]\n"
            "v_or_b32_sdwa %[amk], %[amk], %[amk] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n"
            "v_add_u32 %[voff], %[tbu], %[vlane2]\n"
            "global_store_short %[voff], %[amk], %[tbp]\n"
            "s_lshl_b32 %[x], %[i], 5\n"
            "s_add_u32 %[x], %[x], %[Ldesc]\n"
            "v_mov_b32 %[Ga], %[x]\n"
            "ds_read_b32 %[Gb], %[Ga] offset:36\n"
            "ds_read_b32 %[Pa], %[Ga] offset:40\n"
            "ds_read_b32 %[Pb], %[Ga] offset:44\n"
            "ds_read_b32 %[inc], %[Ga] offset:48\n"
            "v_bfi_b32 %[Hd], %[inv], %[vkneg], %[H]\n"
            "v_bfi_b32 %[m1], %[inv], %[vkneg], %[E1]\n"
            "v_bfi_b32 %[m2], %[inv], %[vkneg], %[E2]\n"
            "s_add_u32 %[r], %[b0], %[i]\n"
            "s_and_b32 %[y], %[r], 7\n"
            "s_mulk_i32 %[y], 0x300\n"
            "s_add_u32 %[y], %[y], %[Lring]\n"
            "v_lshl_add_u32 %[a0], %[iw], 2, %[y]\n"
            "ds_write_b32 %[a0], %[Hd]\n"
            "ds_write_b32 %[a0], %[m1] offset:256\n"
            "ds_write_b32 %[a0], %[m2] offset:512\n"
            "v_pk_add_u16 %[t1], %[Hd], %[cr16] op_sel_hi:[1,0]\n"
            "v_pk_min_u16 %[r16], %[r16], %[t1]\n"
            "s_and_b32 %[x], %[mp], 0x7f\n"
            "s_sub_i32 %[besti], %[cb0], %[x]\n"
            "s_addk_i32 %[besti], 0x7f\n"
            "s_bitcmp1_b32 %[d1], 8\n"
            "s_cbranch_scc1 L_far1%=\n"
            "s_sub_i32 %[x], %[tbu], %[cb0]\n"
            "s_sub_i32 %[z], %[kpu], %[cb0]\n"
            "v_mov_b32 v120, %[beg]\n"
            "v_mov_b32 v121, %[end]\n"
            "v_mov_b32 v122, %[x]\n"
            "v_mov_b32 v123, %[z]\n"
            "v_mov_b32 v124, %[besti]\n"
            "s_and_b32 %[x], %[r], 31\n"
            "s_lshl_b32 %[x], %[x], 4\n"
            "s_add_u32 %[x], %[x], %[Lrrow]\n"
            "v_mov_b32 %[a0], %[x]\n"
            "s_lshl_b32 %[x], %[r], 5\n"
            "v_mov_b32 %[voff], %[x]\n"
            "v_mov_b32 v125, -1\n"
            "s_mov_b64 vcc, exec\n"
            "s_mov_b64 exec, 1\n"
            "ds_write2_b64 %[a0], v[120:121], v[124:125] offset1:1\n"
            "global_store_dwordx4 %[voff], v[120:123], %[rip]\n"
            "s_mov_b64 exec, vcc\n"
            "s_sub_i32 %[x], %[end], %[beg]\n"
            "s_add_i32 %[cel], %[cel], %[x]\n"
            "s_add_i32 %[x], %[spm], 4\n"
            "s_and_b32 %[x], %[x], -4\n"
            "s_add_i32 %[tbu], %[tbu], %[x]\n"
            "s_mov_b32 %[pr], %[r]\n"
            "s_mov_b32 %[pb], %[beg]\n"
            "s_mov_b32 %[pe], %[end]\n"
            "s_mov_b32 %[pa], %[besti]\n"
            "s_mov_b32 %[pwb], %[y]\n"
            "s_add_i32 %[i], %[i], 1\n"
            "s_branch L_top%=\n"
            "L_far1%=:\n"
            "s_lshl_b32 %[x], %[svu], 2\n"
            "v_add_u32 %[voff], %[x], %[vlane8]\n"
            "v_bfe_i32 v120, %[H], 0, 16\n"
            "v_ashrrev_i32 v121, 16, %[H]\n"
            "v_bfe_i32 v122, %[E1], 0, 16\n"
            "v_ashrrev_i32 v123, 16, %[E1]\n"
            "v_bfe_i32 v124, %[E2], 0, 16\n"
            "v_ashrrev_i32 v125, 16, %[E2]\n"
            "global_store_dwordx2 %[voff], v[120:121], %[svp]\n"
            "global_store_dwordx2 %[voff], v[122:123], %[svp] offset:512\n"
            "global_store_dwordx2 %[voff], v[124:125], %[svp] offset:1024\n"
            "s_sub_i32 %[x], %[tbu], %[cb0]\n"
            "s_sub_i32 %[z], %[kpu], %[cb0]\n"
            "v_mov_b32 v120, %[beg]\n"
            "v_mov_b32 v121, %[end]\n"
            "v_mov_b32 v122, %[x]\n"
            "v_mov_b32 v123, %[z]\n"
            "v_mov_b32 v124, %[besti]\n"
            "s_and_b32 %[x], %[r], 31\n"
            "s_lshl_b32 %[x], %[x], 4\n"
            "s_add_u32 %[x], %[x], %[Lrrow]\n"
            "v_mov_b32 %[a0], %[x]\n"
            "s_lshl_b32 %[x], %[r], 5\n"
            "v_mov_b32 %[voff], %[x]\n"
            "v_mov_b32 v125, %[svu]\n"
            "s_mov_b64 vcc, exec\n"
            "s_mov_b64 exec, 1\n"
            "ds_write2_b64 %[a0], v[120:121], v[124:125] offset1:1\n"
            "global_store_dwordx4 %[voff], v[120:123], %[rip]\n"
            "global_store_dwordx2 %[voff], v[124:125], %[rip] offset:16\n"
            "s_addk_i32 %[svu], 0x180\n"
            "s_mov_b64 exec, vcc\n"
            "s_sub_i32 %[x], %[end], %[beg]\n"
            "s_add_i32 %[cel], %[cel], %[x]\n"
            "s_add_i32 %[x], %[spm], 4\n"
            "s_and_b32 %[x], %[x], -4\n"
            "s_add_i32 %[tbu], %[tbu], %[x]\n"
            "s_mov_b32 %[pr], %[r]\n"
            "s_mov_b32 %[pb], %[beg]\n"
            "s_mov_b32 %[pe], %[end]\n"
            "s_mov_b32 %[pa], %[besti]\n"
            "s_mov_b32 %[pwb], %[y]\n"
            "s_add_i32 %[i], %[i], 1\n"
            "s_branch L_top%=\n"
            "L_two%=:\n"
            "s_cmp_lg_u32 %[y], 0x28000\n"
            "s_cbranch_scc1 L_out%=\n"
            "v_readfirstlane_b32 %[p1], %[inc]\n"
            "s_cmp_eq_u32 %[p1], %[pr]\n"
            "s_cbranch_scc0 L_p1lds%=\n"
            "s_mov_b32 %[rb1], %[pb]\n"
            "s_mov_b32 %[re1], %[pe]\n"
            "s_mov_b32 %[ra1], %[pa]\n"
            "s_mov_b32 %[base1], %[pwb]\n"
            "s_branch L_p1ok%=\n"
            "L_p1lds%=:\n"
            "s_and_b32 %[x], %[p1], 31\n"
            "s_lshl_b32 %[x], %[x], 4\n"
            "s_add_u32 %[x], %[x], %[Lrrow]\n"
            "v_mov_b32 %[Ga], %[x]\n"
            "ds_read_b32 %[Gb], %[Ga]\n"
            "ds_read_b32 %[Pa], %[Ga] offset:4\n"
            "ds_read_b32 %[Pb], %[Ga] offset:8\n"
            "s_and_b32 %[x], %[p1], 7\n"
            "s_mulk_i32 %[x], 0x300\n"
            "s_add_u32 %[base1], %[x], %[Lring]\n"
            "s_waitcnt lgkmcnt(0)\n"
            "v_readfirstlane_b32 %[rb1], %[Gb]\n"
            "v_readfirstlane_b32 %[re1], %[Pa]\n"
            "v_readfirstlane_b32 %[ra1], %[Pb]\n"
            "L_p1ok%=:\n"
            "s_cmp_eq_u32 %[p0], %[pr]\n"
            "s_cbranch_scc1 L_p0ok2%=\n"
            "s_and_b32 %[x], %[p0], 31\n"
            "s_lshl_b32 %[x], %[x], 4\n"
            "s_add_u32 %[x], %[x], %[Lrrow]\n"
            "v_mov_b32 %[Ga], %[x]\n"
            "ds_read_b32 %[Gb], %[Ga]\n"
            "ds_read_b32 %[Pa], %[Ga] offset:4\n"
            "ds_read_b32 %[Pb], %[Ga] offset:8\n"
            "s_and_b32 %[x], %[p0], 7\n"
            "s_mulk_i32 %[x], 0x300\n"
            "s_add_u32 %[pwb], %[x], %[Lring]\n"
            "s_waitcnt lgkmcnt(0)\n"
            "v_readfirstlane_b32 %[pb], %[Gb]\n"
            "v_readfirstlane_b32 %[pe], %[Pa]\n"
            "v_readfirstlane_b32 %[pa], %[Pb]\n"
            "s_mov_b32 %[pr], %[p0]\n"
            "L_p0ok2%=:\n"
            "s_sub_i32 %[x], %[qlen], %[rem]\n"
            "s_min_i32 %[y], %[pa], %[ra1]\n"
            "s_max_i32 %[z], %[pa], %[ra1]\n"
            "s_add_i32 %[y], %[y], 1\n"
            "s_add_i32 %[z], %[z], 1\n"
            "s_min_i32 %[y], %[y], %[x]\n"
            "s_max_i32 %[z], %[z], %[x]\n"
            "s_sub_i32 %[y], %[y], %[w]\n"
            "s_add_i32 %[z], %[z], %[w]\n"
            "s_max_i32 %[beg], %[y], 0\n"
            "s_min_i32 %[end], %[z], %[qlen]\n"
            "s_and_b32 %[cb0], %[beg], -2\n"
            "s_sub_i32 %[spm], %[end], %[cb0]\n"
            "s_and_b32 %[pc0], %[pb], -2\n"
            "s_sub_i32 %[x], %[pe], %[pc0]\n"
            "s_max_i32 %[x], %[x], %[spm]\n"
            "s_and_b32 %[pc1], %[rb1], -2\n"
            "s_sub_i32 %[y], %[re1], %[pc1]\n"
            "s_max_i32 %[x], %[x], %[y]\n"
            "s_cmpk_gt_i32 %[x], 0x7f\n"
            "s_cbranch_scc1 L_out%=\n"
            "s_bfe_u32 %[z], %[d1], 0x80000\n"
            "s_lshl_b32 %[x], %[z], 3\n"
            "s_lshl_b32 %[tlo], 9, %[x]\n"
            "s_cmp_gt_u32 %[z], 3\n"
            "s_cselect_b32 %[tlo], %[cth], %[tlo]\n"
            "s_pack_ll_b32_b16 %[pkb], %[beg], %[beg]\n"
            "s_pack_ll_b32_b16 %[pke], %[end], %[end]\n"
            "s_bfe_u32 %[x], %[cb0], 0xf0001\n"
            "v_add_u32 %[M], %[x], %[vlane]\n"
            "v_mad_u32_u24 %[H0], %[M], %[c20002], %[v10000]\n"
            "v_add_u32 %[Ga], %[Lq], %[M]\n"
            "ds_read_u8 %[S], %[Ga]\n"
            "v_and_b32 %[iw], 63, %[M]\n"
            "v_lshl_add_u32 %[a0], %[iw], 2, %[pwb]\n"
            "ds_read_b32 %[E1], %[a0]\n"
            "ds_read_b32 %[X1], %[a0] offset:256\n"
            "ds_read_b32 %[X2], %[a0] offset:512\n"
            "v_pk_sub_i16 %[m1], %[H0], %[pkb]\n"
            "v_pk_sub_i16 %[m2], %[pke], %[H0]\n"
            "v_or_b32 %[m1], %[m1], %[m2]\n"
            "v_pk_ashrrev_i16 %[inv], 15, %[m1] op_sel_hi:[0,1]\n"
            "s_waitcnt lgkmcnt(3)\n"
            "v_mul_u32_u24 %[S], 0x1001, %[S]\n"
            "v_and_or_b32 %[S], %[S], %[cq], %[v0c0c]\n"
            "v_perm_b32 %[S], 4, %[tlo], %[S]\n"
            "s_waitcnt lgkmcnt(0)\n"
            "v_mov_b32_dpp %[t1], %[E1] wave_ror:1 row_mask:0xf bank_mask:0xf\n"
            "v_alignbit_b32 %[Hd], %[E1], %[t1], 16\n"
            "s_setprio 0\n"
            "s_max_i32 %[x], %[pc0], %[pc1]\n"
            "s_cmp_le_i32 %[beg], %[x]\n"
            "s_cbranch_scc1 L_mask2%=\n"
            "s_min_i32 %[x], %[pc0], %[pc1]\n"
            "s_addk_i32 %[x], 0x7f\n"
            "s_cmp_le_i32 %[end], %[x]\n"
            "s_cbranch_scc1 L_nomask2%=\n"
            "L_mask2%=:\n"
            "s_pack_ll_b32_b16 %[x], %[pb], %[pb]\n"
            "s_pack_ll_b32_b16 %[y], %[pe], %[pe]\n"
            "v_pk_add_u16 %[t1], %[H0], -1\n"
            "v_pk_sub_i16 %[m1], %[t1], %[x]\n"
            "v_pk_sub_i16 %[m2], %[y], %[t1]\n"
            "v_or_b32 %[m1], %[m1], %[m2]\n"
            "v_pk_ashrrev_i16 %[m1], 15, %[m1] op_sel_hi:[0,1]\n"
            "v_pk_sub_i16 %[m2], %[H0], %[x]\n"
            "v_pk_sub_i16 %[t1], %[y], %[H0]\n"
            "v_or_b32 %[m2], %[m2], %[t1]\n"
            "v_pk_ashrrev_i16 %[m2], 15, %[m2] op_sel_hi:[0,1]\n"
            "v_bfi_b32 %[Hd], %[m1], %[vkneg], %[Hd]\n"
            "v_bfi_b32 %[X1], %[m2], %[vkneg], %[X1]\n"
            "v_bfi_b32 %[X2], %[m2], %[vkneg], %[X2]\n"
            "v_lshl_add_u32 %[a0], %[iw], 2, %[base1]\n"
            "ds_read_b32 %[E1], %[a0]\n"
            "ds_read_b32 %[P1], %[a0] offset:256\n"
            "ds_read_b32 %[P2], %[a0] offset:512\n"
            "s_waitcnt lgkmcnt(0)\n"
            "v_mov_b32_dpp %[t1], %[E1] wave_ror:1 row_mask:0xf bank_mask:0xf\n"
            "v_alignbit_b32 %[F1], %[E1], %[t1], 16\n"
            "s_pack_ll_b32_b16 %[x], %[rb1], %[rb1]\n"
            "s_pack_ll_b32_b16 %[y], %[re1], %[re1]\n"
            "v_pk_add_u16 %[t1], %[H0], -1\n"
            "v_pk_sub_i16 %[m1], %[t1], %[x]\n"
            "v_pk_sub_i16 %[m2], %[y], %[t1]\n"
            "v_or_b32 %[m1], %[m1], %[m2]\n"
            "v_pk_ashrrev_i16 %[m1], 15, %[m1] op_sel_hi:[0,1]\n"
            "v_pk_sub_i16 %[m2], %[H0], %[x]\n"
            "v_pk_sub_i16 %[t1], %[y], %[H0]\n"
            "v_or_b32 %[m2], %[m2], %[t1]\n"
            "v_pk_ashrrev_i16 %[m2], 15, %[m2] op_sel_hi:[0,1]\n"
            "v_bfi_b32 %[F1], %[m1], %[vkneg], %[F1]\n"
            "v_bfi_b32 %[P1], %[m2], %[vkneg], %[P1]\n"
            "v_bfi_b32 %[P2], %[m2], %[vkneg], %[P2]\n"
            "s_branch L_merge2%=\n"
            "L_nomask2%=:\n"
            "v_lshl_add_u32 %[a0], %[iw], 2, %[base1]\n"
            "ds_read_b32 %[E1], %[a0]\n"
            "ds_read_b32 %[P1], %[a0] offset:256\n"
            "ds_read_b32 %[P2], %[a0] offset:512\n"
            "s_waitcnt lgkmcnt(0)\n"
            "v_mov_b32_dpp %[t1], %[E1] wave_ror:1 row_mask:0xf bank_mask:0xf\n"
            "v_alignbit_b32 %[F1], %[E1], %[t1], 16\n"
            "L_merge2%=:\n"
            "v_pk_sub_i16 %[MK], %[Hd], %[F1] clamp\n"
            "v_pk_lshrrev_b16 %[MK], 15, %[MK] op_sel_hi:[0,1]\n"
            "v_pk_sub_i16 %[K1], %[X1], %[P1] clamp\n"
            "v_pk_lshrrev_b16 %[K1], 15, %[K1] op_sel_hi:[0,1]\n"
            "v_pk_sub_i16 %[K2], %[X2], %[P2] clamp\n"
            "v_pk_lshrrev_b16 %[K2], 15, %[K2] op_sel_hi:[0,1]\n"
            "v_pk_max_i16 %[Hd], %[Hd], %[F1]\n"
            "v_pk_max_i16 %[X1], %[X1], %[P1]\n"
            "v_pk_max_i16 %[X2], %[X2], %[P2]\n"
            "v_pk_add_i16 %[M], %[Hd], %[S] clamp\n"
            "v_pk_add_i16 %[M], %[M], -4 op_sel_hi:[1,0] clamp\n"
            "v_pk_max_i16 %[t1], %[X1], %[X2]\n"
            "v_pk_max_i16 %[t1], %[M], %[t1]\n"
            "v_bfi_b32 %[H0], %[inv], %[vkneg], %[t1]\n"
            "v_pk_add_i16 %[G1], %[H0], %[LJ1] clamp\n"
            "v_pk_add_i16 %[G2], %[H0], %[LJ2] clamp\n"
            "v_perm_b32 %[Ga], %[G2], %[G1], %[csel0]\n"
            "v_perm_b32 %[Gb], %[G2], %[G1], %[csel1]\n"
            "v_pk_max_i16 %[inc], %[Ga], %[Gb]\n"
            "v_xor_b32 %[inc], 0x80008000, %[inc]\n"
            "v_mad_i32_i16 %[amk], %[H0], %[c128], %[clo]\n"
            "v_mad_i32_i16 %[t1], %[H0], %[c128], %[chi] op_sel:[1,0,0,0]\n"
            "v_max_i32 %[amk], %[amk], %[t1]\n"
            "s_nop 1\n"
            "v_mov_b32_dpp %[t1], %[inc] row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
            "v_max_i32_dpp %[amk], %[amk], %[amk] row_shr:1 row_mask:0xf bank_mask:0xf\n"
            "v_pk_max_u16 %[inc], %[inc], %[t1]\n"
            "s_nop 0\n"
            "v_max_i32_dpp %[amk], %[amk], %[amk] row_shr:2 row_mask:0xf bank_mask:0xf\n"
            "v_mov_b32_dpp %[t1], %[inc] row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
            "v_pk_max_u16 %[inc], %[inc], %[t1]\n"
            "v_max_i32_dpp %[amk], %[amk], %[amk] row_shr:4 row_mask:0xf bank_mask:0xf\n"
            "s_nop 0\n"
            "v_mov_b32_dpp %[t1], %[inc] row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
            "v_pk_max_u16 %[inc], %[inc], %[t1]\n"
            "s_nop 0\n"
            "v_max_i32_dpp %[amk], %[amk], %[amk] row_shr:8 row_mask:0xf bank_mask:0xf\n"
            "v_mov_b32_dpp %[t1], %[inc] row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
            "v_pk_max_u16 %[inc], %[inc], %[t1]\n"
            "v_max_i32_dpp %[amk], %[amk], %[amk] row_bcast:15 row_mask:0xa bank_mask:0xf\n"
            "s_nop 0\n"
            "v_mov_b32_dpp %[t1], %[inc] row_bcast:15 row_mask:0xa bank_mask:0xf\n"
            "v_pk_max_u16 %[inc], %[inc], %[t1]\n"
            "v_max_i32_dpp %[amk], %[amk], %[amk] row_bcast:31 row_mask:0xc bank_mask:0xf\n"
            "s_nop 0\n"
            "v_mov_b32_dpp %[t1], %[inc] row_bcast:31 row_mask:0xc bank_mask:0xf\n"
            "v_pk_max_u16 %[inc], %[inc], %[t1]\n"
            "s_nop 1\n"
            "v_readlane_b32 %[mp], %[amk], 63\n"
            "v_xor_b32_dpp %[Pa], %[inc], %[vkneg] wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
            "v_pk_max_i16 %[Pb], %[Pa], %[Ga]\n"
            "v_perm_b32 %[P1], %[Pb], %[Pa], %[csel0]\n"
            "v_perm_b32 %[P2], %[Pb], %[Pa], %[csel1]\n"
            "v_pk_sub_i16 %[F1], %[P1], %[FJ1] clamp\n"
            "v_pk_sub_i16 %[S], %[P2], %[FJ2] clamp\n"
            "v_pk_max_i16 %[H], %[F1], %[S]\n"
            "v_pk_max_i16 %[H], %[H0], %[H]\n"
            "v_pk_add_i16 %[X1e], %[X1], -2 op_sel_hi:[1,0] clamp\n"
            "v_pk_add_i16 %[Ho1], %[H], -6 op_sel_hi:[1,0] clamp\n"
            "v_pk_add_i16 %[X2e], %[X2], -1 clamp\n"
            "v_pk_sub_i16 %[Ho2], %[H], 25 op_sel_hi:[1,0] clamp\n"
            "v_pk_max_i16 %[E1], %[X1e], %[Ho1]\n"
            "v_pk_max_i16 %[E2], %[X2e], %[Ho2]\n"
            "v_pk_sub_i16 %[Ga], %[M], %[H] clamp\n"
            "v_pk_sub_i16 %[Gb], %[X1], %[H] clamp\n"
            "v_perm_b32 %[Pa], %[Gb], %[Ga], %[cseltb]\n"
            "v_pk_sub_i16 %[Ga], %[X2], %[H] clamp\n"
            "v_pk_sub_i16 %[Gb], %[F1], %[H] clamp\n"
            "v_perm_b32 %[Pb], %[Gb], %[Ga], %[cseltb]\n"
            "v_pk_sub_i16 %[Ga], %[Ho1], %[X1e] clamp\n"
            "v_pk_sub_i16 %[Gb], %[Ho2], %[X2e] clamp\n"
            "v_perm_b32 %[inc], %[Gb], %[Ga], %[cseltb]\n"
            "v_pk_sub_i16 %[Ga], %[G1], %[P1] clamp\n"
            "v_pk_sub_i16 %[Gb], %[G2], %[P2] clamp\n"
            "v_perm_b32 %[amk], %[Gb], %[Ga], %[cseltb]\n"
            "v_and_b32 %[amk], %[m67], %[amk]\n"
            "v_and_or_b32 %[amk], %[inc], %[m45], %[amk]\n"
            "v_and_or_b32 %[amk], %[Pb], %[m23], %[amk]\n"
            "v_and_or_b32 %[amk], %[Pa], %[m01], %[amk]\n"
            "v_or_b32_sdwa %[amk], %[amk], %[amk] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n"
            "v_add_u32 %[voff], %[tbu], %[vlane2]\n"
            "global_store_short %[voff], %[amk], %[tbp]\n"
            "s_lshl_b32 %[x], %[i], 5\n"
            "s_add_u32 %[x], %[x], %[Ldesc]\n"
            "v_mov_b32 %[Ga], %[x]\n"
            "ds_read_b32 %[Gb], %[Ga] offset:36\n"
            "ds_read_b32 %[Pa], %[Ga] offset:40\n"
            "ds_read_b32 %[Pb], %[Ga] offset:44\n"
            "ds_read_b32 %[inc], %[Ga] offset:48\n"
            "v_lshlrev_b32 %[K1], 2, %[K1]\n"
            "v_lshlrev_b32 %[K2], 4, %[K2]\n"
            "v_or3_b32 %[MK], %[MK], %[K1], %[K2]\n"
            "v_perm_b32 %[MK], 0, %[MK], %[cselkp]\n"
            "v_add_u32 %[voff], %[kpu], %[vlane2]\n"
            "global_store_short %[voff], %[MK], %[kpp]\n"
            "v_bfi_b32 %[Hd], %[inv], %[vkneg], %[H]\n"
            "v_bfi_b32 %[m1], %[inv], %[vkneg], %[E1]\n"
            "v_bfi_b32 %[m2], %[inv], %[vkneg], %[E2]\n"
            "s_add_u32 %[r], %[b0], %[i]\n"
            "s_and_b32 %[y], %[r], 7\n"
            "s_mulk_i32 %[y], 0x300\n"
            "s_add_u32 %[y], %[y], %[Lring]\n"
            "v_lshl_add_u32 %[a0], %[iw], 2, %[y]\n"
            "ds_write_b32 %[a0], %[Hd]\n"
            "ds_write_b32 %[a0], %[m1] offset:256\n"
            "ds_write_b32 %[a0], %[m2] offset:512\n"
            "v_pk_add_u16 %[t1], %[Hd], %[cr16] op_sel_hi:[1,0]\n"
            "v_pk_min_u16 %[r16], %[r16], %[t1]\n"
            "s_and_b32 %[x], %[mp], 0x7f\n"
            "s_sub_i32 %[besti], %[cb0], %[x]\n"
            "s_addk_i32 %[besti], 0x7f\n"
            "s_bitcmp1_b32 %[d1], 8\n"
            "s_cbranch_scc1 L_far2%=\n"
            "s_sub_i32 %[x], %[tbu], %[cb0]\n"
            "s_sub_i32 %[z], %[kpu], %[cb0]\n"
            "v_mov_b32 v120, %[beg]\n"
            "v_mov_b32 v121, %[end]\n"
            "v_mov_b32 v122, %[x]\n"
            "v_mov_b32 v123, %[z]\n"
            "v_mov_b32 v124, %[besti]\n"
            "s_and_b32 %[x], %[r], 31\n"
            "s_lshl_b32 %[x], %[x], 4\n"
            "s_add_u32 %[x], %[x], %[Lrrow]\n"
            "v_mov_b32 %[a0], %[x]\n"
            "s_lshl_b32 %[x], %[r], 5\n"
            "v_mov_b32 %[voff], %[x]\n"
            "v_mov_b32 v125, -1\n"
            "s_mov_b64 vcc, exec\n"
            "s_mov_b64 exec, 1\n"
            "ds_write2_b64 %[a0], v[120:121], v[124:125] offset1:1\n"
            "global_store_dwordx4 %[voff], v[120:123], %[rip]\n"
            "s_mov_b64 exec, vcc\n"
            "s_sub_i32 %[x], %[end], %[beg]\n"
            "s_add_i32 %[cel], %[cel], %[x]\n"
            "s_add_i32 %[x], %[spm], 4\n"
            "s_and_b32 %[x], %[x], -4\n"
            "s_add_i32 %[tbu], %[tbu], %[x]\n"
            "s_add_i32 %[kpu], %[kpu], %[x]\n"
            "s_mov_b32 %[pr], %[r]\n"
            "s_mov_b32 %[pb], %[beg]\n"
            "s_mov_b32 %[pe], %[end]\n"
            "s_mov_b32 %[pa], %[besti]\n"
            "s_mov_b32 %[pwb], %[y]\n"
            "s_add_i32 %[i], %[i], 1\n"
            "s_branch L_top%=\n"
            "L_far2%=:\n"
            "s_lshl_b32 %[x], %[svu], 2\n"
            "v_add_u32 %[voff], %[x], %[vlane8]\n"
            "v_bfe_i32 v120, %[H], 0, 16\n"
            "v_ashrrev_i32 v121, 16, %[H]\n"
            "v_bfe_i32 v122, %[E1], 0, 16\n"
            "v_ashrrev_i32 v123, 16, %[E1]\n"
            "v_bfe_i32 v124, %[E2], 0, 16\n"
            "v_ashrrev_i32 v125, 16, %[E2]\n"
            "global_store_dwordx2 %[voff], v[120:121], %[svp]\n"
            "global_store_dwordx2 %[voff], v[122:123], %[svp] offset:512\n"
            "global_store_dwordx2 %[voff], v[124:125], %[svp] offset:1024\n"
            "s_sub_i32 %[x], %[tbu], %[cb0]\n"
            "s_sub_i32 %[z], %[kpu], %[cb0]\n"
            "v_mov_b32 v120, %[beg]\n"
            "v_mov_b32 v121, %[end]\n"
            "v_mov_b32 v122, %[x]\n"
            "v_mov_b32 v123, %[z]\n"
            "v_mov_b32 v124, %[besti]\n"
            "s_and_b32 %[x], %[r], 31\n"
            "s_lshl_b32 %[x], %[x], 4\n"
            "s_add_u32 %[x], %[x], %[Lrrow]\n"
            "v_mov_b32 %[a0], %[x]\n"
            "s_lshl_b32 %[x], %[r], 5\n"
            "v_mov_b32 %[voff], %[x]\n"
            "v_mov_b32 v125, %[svu]\n"
            "s_mov_b64 vcc, exec\n"
            "s_mov_b64 exec, 1\n"
            "ds_write2_b64 %[a0], v[120:121], v[124:125] offset1:1\n"
            "global_store_dwordx4 %[voff], v[120:123], %[rip]\n"
            "global_store_dwordx2 %[voff], v[124:125], %[rip] offset:16\n"
            "s_addk_i32 %[svu], 0x180\n"
            "s_mov_b64 exec, vcc\n"
            "s_sub_i32 %[x], %[end], %[beg]\n"
            "s_add_i32 %[cel], %[cel], %[x]\n"
            "s_add_i32 %[x], %[spm], 4\n"
            "s_and_b32 %[x], %[x], -4\n"
            "s_add_i32 %[tbu], %[tbu], %[x]\n"
            "s_add_i32 %[kpu], %[kpu], %[x]\n"
            "s_mov_b32 %[pr], %[r]\n"
            "s_mov_b32 %[pb], %[beg]\n"
            "s_mov_b32 %[pe], %[end]\n"
            "s_mov_b32 %[pa], %[besti]\n"
            "s_mov_b32 %[pwb], %[y]\n"
            "s_add_i32 %[i], %[i], 1\n"
            "s_branch L_top%=\n"
            "L_out%=:\n"
            "s_setprio 0\n"
            "s_waitcnt lgkmcnt(0)\n"
            "s_sub_i32 %[x], %[i], %[i0]\n"
            "s_add_i32 %[cel], %[cel], %[x]\n"
            "s_nop 1\n"
            MANDO_FR_OPERANDS);
    }
    prv_r = pr;
    prv_beg = pb;
    prv_end = pe;
    prv_am = pa;
    ds.tb_used = tbu;
    ds.kp_used = kpu;
    ds.sv_used = svu;
    ds.cells = cel;
    ds.r16acc = r16;
    return i;
}

// The row loop of 16-bit mode (same rows, same results as run_dp<SC, true>).  The per-row
// control is written for the scalar unit: tests accumulate as sign bits into one word
// (`bad < 0` = take the generic row) rather than as bools, which the compiler would keep as
// 64-bit lane masks.
template <class SC, int RW, int NW = 1>
__device__ __forceinline__ int run_dp16(SharedState &sh, const SC &sc, int qlen, int n, int lane, int w,
                                        DpState &ds, int &nfast) {
    static_assert(NW == 1 || RW == kWideRing, "two-wave rows: wide launches");
    // NW == 2: the previous row was split over both waves, so wave 1 may still be writing its ring
    // half; a row wave 0 computes alone first passes a B0 with a no-op command
    int split = 0;
    auto sync_alone = [&]() {
        if constexpr (NW > 1) {
            if (split) {
                w2_post_op(kW2Nop, lane);
                group_barrier();
                split = 0;
            }
        }
    };
    gu8 *tb, *kp;
    gint *sv, *rinfo, *desc;
    int tb_lim, kp_lim, sv_lim;
    {
        const Slot s = slot_of(sh);
        const PoaRunArgs a = args_of(sh);
        tb = s.tb;
        kp = s.kp;
        sv = s.sv;
        rinfo = s.rinfo;
        desc = s.desc;
        // a fast row allocates at most tbw + one chunk of slack
        tb_lim = (int)a.caps.TBC - 2 * (RW + 4);
        kp_lim = (int)a.caps.KPC - 6 * (RW + 4);
        sv_lim = (int)a.caps.SVC - 3 * RW;
    }
    int prv_r = -1, prv_beg = 0, prv_end = 0, prv_am = 0;
    // Descriptor batches reach LDS one batch ahead: lane l holds ints [4l, 4l+4) of the next 32 rows
    // (loaded while the current batch's rows run), so the batch refill waits on no HBM round trip.
    static_assert(kDescBatch * kDescInts <= 4 * kWave && kDescInts == 8, "one int4 per lane per descriptor batch");
    const bool pl = (lane >> 1) < kDescBatch;  // the lanes that carry the batch (two per row)
    int4 pf = make_int4(0, 0, 0, 0);
    if (pl && (lane >> 1) < n) {
        const GLB int4 *g = reinterpret_cast<const GLB int4 *>(desc + 4 * lane);
        pf = make_int4(g->x, g->y, g->z, g->w);
    }
    // the current row's descriptor fields, read from the LDS batch one row ahead (an HBM scalar
    // load per row would put a full memory latency on every row: build_desc's stores are long out
    // of L2 by now)
    // Batches of kDescBatch rows; row 0 (the source row) is peeled off the first batch, so the row
    // loop carries no batch-boundary or first-row tests.
    for (int b0 = 0, i0 = 1; b0 < n - 1; b0 += kDescBatch, i0 = 0) {
        if (pl && b0 + (lane >> 1) < n) *reinterpret_cast<int4 *>(&sh.desc[0][0] + 4 * lane) = pf;
        {
            const int rn = b0 + kDescBatch;
            if (pl && rn < n && rn + (lane >> 1) < n) {
                const GLB int4 *g = reinterpret_cast<const GLB int4 *>(desc + (int64_t)rn * kDescInts + 4 * lane);
                pf = make_int4(g->x, g->y, g->z, g->w);
            }
        }
        if (b0 == 0) {
            Slot s = slot_of(sh);
            const PoaRunArgs a = args_of(sh);
            const int st = dp_row<SC, true, RW>(a, sc, s, sh, qlen, w, 0, lane, ds);
            if (st != kStOk) return st;
            const int4 x = sh.rrow[0];
            prv_r = 0;
            prv_beg = bcast0(x.x);
            prv_end = bcast0(x.y);
            prv_am = bcast0(x.z);
        }
        const int iend = min(kDescBatch, n - 1 - b0);
        // the current row's descriptor fields, read from the LDS batch one row ahead (an HBM scalar
        // load per row would put a full memory latency on every row: build_desc's stores are long
        // out of L2 by now); past the batch end the read is harmless and unused
        int4 nA = *reinterpret_cast<const int4 *>(&sh.desc[i0][0]);
        int np1 = sh.desc[i0][4];
        // capacity: when the batch's rows cannot outgrow the traceback / predecessor / spill arrays
        // (the common case), the rows skip the per-row capacity tests (a second copy of the loop)
        const int cap_ok = ((tb_lim - ds.tb_used - kDescBatch * (RW + 4)) |
                            (kp_lim - ds.kp_used - 3 * kDescBatch * (RW + 4)) |
                            (sv_lim - ds.sv_used - 3 * kDescBatch * RW)) >= 0;
        auto rows = [&](auto capchk) -> int {
        constexpr bool CAP = decltype(capchk)::value;
    for (int i = i0; i < iend; ++i) {
        if constexpr (RW == kChunk && NW == 1 && !CAP && std::is_same<SC, DefaultScores>::value) {
            // the one-chunk fast rows with one or two predecessors in the ring, hand-scheduled (~90 % of a
            // narrow launch's rows)
#ifdef MANDO_CHECK_EXEC
            if (__builtin_amdgcn_read_exec() != ~0ull) __builtin_trap();
#endif
            const int j = fast_rows_asm(sh, lane, tb, kp, sv, rinfo, b0, i, iend, qlen, w, prv_r, prv_beg, prv_end,
                                        prv_am, ds);
            if (j != i) {
                nfast += j - i;
                i = j;
                if (i >= iend) break;
                nA = *reinterpret_cast<const int4 *>(&sh.desc[i][0]);
                np1 = sh.desc[i][4];
            }
        }
        const int r = b0 + i;
        const int4 dA = nA;
        const int dp1 = np1;
        nA = *reinterpret_cast<const int4 *>(&sh.desc[(i + 1) & (kDescBatch - 1)][0]);
        np1 = sh.desc[(i + 1) & (kDescBatch - 1)][4];
        const int node = bcast0(dA.x), d1 = bcast0(dA.y), rem = bcast0(dA.z), p0 = bcast0(dA.w);
        const int p1 = bcast0(dp1);
        // one predecessor, in the LDS ring (~60 % of the config-3 rows): its own, shorter band /
        // fast-path computation and row instance (row16_vec<..., ONE>), DP 2,781 -> 2,468 cycles per
        // row with the saddr traceback stores.  Its own row record (Q, not R: sharing one struct with
        // the general path kept R's fields live around the loop, a dozen s_mov per row), and
        // structured if/else only (an early `continue` left the CFG structurizer a per-row dispatch
        // through a VGPR selector).  Measured and dropped (profiles/r03d_poa_kernel_ab.txt): the same
        // specialisation for two-predecessor rows (+7 %: register pressure spilled SGPRs into VGPR
        // lanes on the row path) and the next descriptor's LDS address kept in a VGPR (+4 %).
        const uint32_t shape = (uint32_t)d1 & 0xffff8000u;  // fast-row bit | predecessor count
        bool done = false;
        if (shape == 0x18000u) {
            Row16 Q;
            int bad1;
            int am0;
            if (p0 == prv_r) {
                Q.b0 = prv_beg;
                Q.e0 = prv_end;
                am0 = prv_am;
            } else {
                const int4 x = sh.rrow[p0 & (kRowRing - 1)];
                Q.b0 = bcast0(x.x);
                Q.e0 = bcast0(x.y);
                am0 = bcast0(x.z);
            }
            const int xr = qlen - rem;
            Q.beg = max(0, min(am0 + 1, xr) - w);
            Q.end = min(qlen, max(am0 + 1, xr) + w);
            Q.cb0 = Q.beg & ~1;
            const int span = Q.end - Q.cb0 + 1;
            Q.tbw = (span + 3) & ~3;
            const int pc0 = Q.b0 & ~1;
            bad1 = (RW - span) | (RW - 1 - (Q.e0 - pc0));
            if constexpr (CAP) bad1 |= (tb_lim - ds.tb_used) | (kp_lim - ds.kp_used) | (sv_lim - ds.sv_used);
            Q.nomask = RW == kChunk && ((Q.beg - 1 - pc0) | (pc0 + kChunk - 1 - Q.end)) >= 0;
            Q.r = r;
            Q.node = node;
            Q.vb = d1 & 0xff;
            Q.pn = 1;
            Q.far = (d1 >> 8) & 1;
            Q.two = Q.multi = Q.pn3 = 0;
            Q.p0slot = Q.p1slot = p0 & (kRing16 - 1);
            Q.b1 = Q.b0;
            Q.e1 = Q.e0;
            if (bad1 >= 0) {
#ifdef MANDO_ROW_STATS
                ds.seg[0] += (Q.r - 1) == prv_r && Q.p0slot == (prv_r & (kRing16 - 1));
                ds.seg[2] += Q.nomask;
#endif
                int besti;
                if (RW == kChunk || Q.end - Q.cb0 < kChunk) {
                    sync_alone();
                    besti = row16_vec<SC, RW, true>(sc, tb, kp, sv, rinfo, sh, lane, Q, ds);
                } else if constexpr (NW > 1) {
                    w2_post_row(Q, ds, lane);
                    group_barrier();  // B0
                    split = 1;
                    besti = row16w_half<SC>(sc, tb, kp, sv, rinfo, sh, lane, Q, ds, 0);
                } else {
                    besti = row16w_vec(sc, tb, kp, sv, rinfo, sh, lane, Q, ds);
                }
                prv_r = r;
                prv_beg = Q.beg;
                prv_end = Q.end;
                prv_am = besti;
                ++nfast;
                done = true;
            }
        }
        if (!done) {
        int bad = -1;
        Row16 R;
        {
            if (d1 & 0xC000) {  // 1-kPreInline predecessors, all in the LDS ring (build_desc)
                int am0, am1;
                if (p0 == prv_r) {
                    R.b0 = prv_beg;
                    R.e0 = prv_end;
                    am0 = prv_am;
                } else {
                    const int4 x = sh.rrow[p0 & (kRowRing - 1)];
                    R.b0 = bcast0(x.x);
                    R.e0 = bcast0(x.y);
                    am0 = bcast0(x.z);
                }
                R.two = (d1 >> 16) >= 2;
                if (R.two) {
                    if (p1 == prv_r) {
                        R.b1 = prv_beg;
                        R.e1 = prv_end;
                        am1 = prv_am;
                    } else {
                        const int4 x = sh.rrow[p1 & (kRowRing - 1)];
                        R.b1 = bcast0(x.x);
                        R.e1 = bcast0(x.y);
                        am1 = bcast0(x.z);
                    }
                } else {
                    R.b1 = R.b0;
                    R.e1 = R.e0;
                    am1 = am0;
                }
                int amL = min(am0, am1), amR = max(am0, am1), narrowk = 0;
                R.pn3 = (d1 & 0x4000) ? (d1 >> 16) : 0;
                for (int k = 2; k < R.pn3; ++k) {
                    const int4 x = sh.rrow[bcast0(sh.desc[r & (kDescBatch - 1)][3 + k]) & (kRowRing - 1)];
                    const int amk = bcast0(x.z);
                    amL = min(amL, amk);
                    amR = max(amR, amk);
                    narrowk |= RW - 1 - (bcast0(x.y) - (bcast0(x.x) & ~1));
                }
                const int xr = qlen - rem;
                R.beg = max(0, min(amL + 1, xr) - w);
                R.end = min(qlen, max(amR + 1, xr) + w);
                R.cb0 = R.beg & ~1;
                const int span = R.end - R.cb0 + 1;
                R.tbw = (span + 3) & ~3;
                const int pc0 = R.b0 & ~1, pc1 = R.b1 & ~1;
                // each term is negative exactly when its test fails (a two-chunk row: at most two
                // predecessors)
                bad = (RW - span) | (RW - 1 - (R.e0 - pc0)) | (RW - 1 - (R.e1 - pc1)) | narrowk;
                if constexpr (CAP) bad |= (tb_lim - ds.tb_used) | (kp_lim - ds.kp_used) | (sv_lim - ds.sv_used);
                R.nomask = RW == kChunk && ((R.beg - 1 - pc0) | (pc0 + kChunk - 1 - R.end) | (R.beg - 1 - pc1) |
                                            (pc1 + kChunk - 1 - R.end)) >= 0;
                R.r = r;
                R.node = node;
                R.vb = d1 & 0xff;
                R.pn = d1 >> 16;
                R.far = (d1 >> 8) & 1;
                R.multi = R.two;
                R.p0slot = p0 & (kRing16 - 1);
                R.p1slot = (R.two ? p1 : p0) & (kRing16 - 1);
            }
        }
        if (bad >= 0) {
#ifdef MANDO_ROW_STATS
            // fast rows by shape: chain (one predecessor, the previous row), two predecessors, no band
            // masks, three or more predecessors
            ds.seg[0] += (R.pn == 1 && (R.r - 1) == prv_r && R.p0slot == (prv_r & (kRing16 - 1)));
            ds.seg[1] += R.two;
            ds.seg[2] += R.nomask;
            ds.seg[3] += R.pn3 >= 3;
#endif
            int besti;
            if (RW == kChunk || R.end - R.cb0 < kChunk) {
                sync_alone();
                besti = row16_vec<SC, RW>(sc, tb, kp, sv, rinfo, sh, lane, R, ds);
            } else if constexpr (NW > 1) {
                w2_post_row(R, ds, lane);
                group_barrier();  // B0
                split = 1;
                besti = row16w_half<SC>(sc, tb, kp, sv, rinfo, sh, lane, R, ds, 0);
            } else {
                besti = row16w_vec(sc, tb, kp, sv, rinfo, sh, lane, R, ds);
            }
            prv_r = r;
            prv_beg = R.beg;
            prv_end = R.end;
            prv_am = besti;
            ++nfast;
        } else {
            sync_alone();
            Slot s = slot_of(sh);
            const PoaRunArgs a = args_of(sh);
#ifdef MANDO_GENPROF
            const uint64_t g0 = clock64();
#endif
            const int st = dp_row<SC, true, RW>(a, sc, s, sh, qlen, w, r, lane, ds);
#ifdef MANDO_GENPROF
            ds.seg[0] += clock64() - g0;
            {
                const int *dl = &sh.desc[r & (kDescBatch - 1)][0];
                const int pnn = bcast0(dl[1]) >> 16;
                int md = 0;
                for (int k = 0; k < min(pnn, kPreInline); ++k) md = max(md, r - bcast0(dl[3 + k]));
                if (pnn > 2) ds.seg[1] += 1;
                else if (md < 8) ds.seg[2] += 1;
                else ds.seg[3] += 1;
            }
#endif
            if (st != kStOk) return st;
            const int4 x = sh.rrow[r & (kRowRing - 1)];
            prv_r = r;
            prv_beg = bcast0(x.x);
            prv_end = bcast0(x.y);
            prv_am = bcast0(x.z);
        }
        }
    }
        return kStOk;
        };
        const int rst = cap_ok ? rows(std::false_type{}) : rows(std::true_type{});
        if (rst != kStOk) return rst;
    }
    return kStOk;
}

// ---------------------------------------------------------------------------------------------
// banded DP over all rows of the current graph for read q (qlen): writes the traceback bytes and
// returns the start row of the backtrack in bi_out (or -1)
// ---------------------------------------------------------------------------------------------
template <class SC, bool R16, int RW = kChunk, int NW = 1>
__device__ __forceinline__ int run_dp(SharedState &sh, const SC &sc, const uint8_t *q, int qlen,
                      int n, int lane, int64_t &cells, int &bi_out) {
    const PoaRunArgs a = args_of(sh);
    Slot s = slot_of(sh);
    if ((qlen + kQPad + 2) / 2 > a.qlds) return kStUnsupported;  // the launch sizes the read buffer
    const int w = a.band_b + (int)(a.band_f * (float)qlen);
    DpState ds{0, 0, 0, 0, 0xffffffffu, 0, {0, 0, 0, 0}};
    const int TBC = (int)a.caps.TBC, KPC = (int)a.caps.KPC, SVC = (int)a.caps.SVC;
    (void)TBC; (void)KPC; (void)SVC;
    // stage the read in LDS (4-bit codes): on gfx9 vmcnt orders loads behind every earlier store,
    // so a global load per row would wait for the previous rows' traceback stores to land
    // (shifted by one column: nibble j = base j-1; nibble 0 and the kQPad columns past the read = 4)
    for (int t = 2 * lane; t < qlen + kQPad; t += 2 * kWave) {
        const int lo = (t >= 1 && t <= qlen) ? q[t - 1] : 4, hi = (t < qlen) ? q[t] : 4;
        qnib<RW>()[t >> 1] = (uint8_t)(lo | (hi << 4));
    }
    int nfast = 0;
    if constexpr (R16) {
        const int st = run_dp16<SC, RW, NW>(sh, sc, qlen, n, lane, w, ds, nfast);
        if constexpr (NW > 1) {
            // end of the read's rows: wave 1 has written its last ring half and reports whether its cells
            // came near the 16-bit -inf band
            w2_post_op(kW2End, lane);
            group_barrier();  // B0
            group_barrier();  // wave 1's flag
            if (bcast0(w2lds().flag)) ds.r16bad = 1;
        }
        if (st != kStOk) return st;
    } else {
    RowPipe pp;
    pp.prv_r = -1;
    pp.prv_beg = pp.prv_end = pp.prv_am = 0;
    for (int r = 0; r < n - 1; ++r) {
        if ((r & (kDescBatch - 1)) == 0) {
            // next kDescBatch descriptors -> LDS (one global round trip per batch)
            const int rr0 = r + lane;
            if (lane < kDescBatch && rr0 < n) {
                const gint *dg = s.desc + (int64_t)rr0 * kDescInts;
                int *dl = &sh.desc[lane][0];
#pragma unroll
                for (int k = 0; k < kDescInts; ++k) dl[k] = dg[k];
            }
            prefetch_row(sh, r, pp);
        }
        bool fastok;
        {
            if constexpr (RW == kChunk) fastok = r > 0 && !(a.dbg & 4) && dp_row_fast(a, sc, s, sh, qlen, w, r, lane, ds, pp);
            else fastok = false;
        }
        nfast += fastok;
        if (!fastok) {
            const int st = dp_row<SC, R16, RW>(a, sc, s, sh, qlen, w, r, lane, ds);
            if (st != kStOk) return st;
            const int4 x = sh.rrow[r % kRowRing];
            pp.prv_r = r;
            pp.prv_beg = x.x;
            pp.prv_end = x.y;
            pp.prv_am = x.z;
        }
        if (((r + 1) & (kDescBatch - 1)) != 0) prefetch_row(sh, r + 1, pp);
    }
    }
    if constexpr (R16) {
        const uint32_t m = min(ds.r16acc & 0xffffu, ds.r16acc >> 16);
        const unsigned long long nearinf = __ballot(m < (uint32_t)(kR16High - kR16Low));
        if (nearinf || bcast0(ds.r16bad)) return kStRetry32;
    }
    cells += ds.cells;
    if (a.prof && lane == 0) a.prof[(int64_t)blockIdx.x * kProfPhases + 7] += nfast;
#if defined(MANDO_STAMPS) || defined(MANDO_GENPROF) || defined(MANDO_ROW_STATS)
    if (a.prof && lane == 0) {
        int64_t *pf = a.prof + (int64_t)blockIdx.x * kProfPhases;
        for (int k = 0; k < 4; ++k) pf[8 + k] += (int64_t)ds.seg[k];
    }
#endif

    // best predecessor of the sink at column qlen (first in in-edge order on ties); in a -S window
    // the sink is the window's end node and only its predecessors inside the window count
    hbm_fence();
    const int sr = n - 1;
    const bool win = bcast0(sh.win_on) != 0;
    const int snode = win ? bcast0(sh.win_sink) : kSink;
    const int wpb = bcast0(sh.win_pb), wpe = bcast0(sh.win_pe);
    const int nin = s.in_n[snode];
    const gint *sin = in_list(s, a, snode);
    int bs = -2147483647 - 1, bi = -1;
    for (int k = 0; k < nin; ++k) {
        int p = bcast0(s.pos[sin[k]]);
        if (win) {
            if (p < wpb || p > wpe) continue;
            p = bcast0(s.wmap[p - wpb]);
            if (p < 0) continue;
        }
        const RowRec pr = load_rowrec(sh, s, sr, p);
        if (qlen < pr.beg || qlen > pr.end) continue;
        int hv;
        if (pre_in_ring<R16, RW>(sr, p, pr)) {
            hv = ring_get<R16, RW>(sh, p % ring_rows<R16>(), 0, qlen & (RW - 1));
        } else {
            hv = s.sv[pr.soff + (qlen - (pr.beg & ~1))];
        }
        hv = bcast0(hv);
        if (hv > bs) {
            bs = hv;
            bi = p;
        }
    }
    bi_out = bi;
    return kStOk;
}

// ---------------------------------------------------------------------------------------------
// backtrack: fills qnode[q] = aligned node or -1 (insertion) for q in [0, qlen)
// row record: rinfo[r] = {beg, end, tbbase, kpbase, argmax, soff, node, pre_n}; the fast rows write
// argmax / soff only for far rows (the only ones read back from HBM) and never node / pre_n (the
// backtrack takes those from the row's descriptor).  (Putting argmax / soff first, so that the LDS
// ring and the record share one register tuple, cost the backtrack a second load per window row:
// +9 % backtrack cycles for -1 % DP cycles, measured r03 kab3 v4 / v5.)
//
// The walk is inherently serial, so its cost is the latency chain per step.  Walking HBM directly
// costs three dependent global loads per step (row record -> traceback byte -> predecessor byte).
// Instead the wave copies a window of up to 64 rows -- their records, predecessor lists and the
// contiguous traceback / predecessor-byte ranges the DP allocated for them -- into LDS with a few
// wide loads, and the walk then touches LDS only.  Rows are allocated in DP order, so the rows
// [i-63, i] occupy one contiguous byte range of each array.
// E states are resolved lazily: state E at row i means "at E_out[i][j]", and the open/extend bit
// is read from row i itself, so every step reads only the current row's window entry.
// ---------------------------------------------------------------------------------------------
constexpr int kKpNone = -2147483647 - 1;
// wave priority of the non-DP phases (see the read loop); above the fast rows' head (2, fast_rows_asm),
// which is above the rest of a DP row (0)
constexpr int kSerialPrio = 3;

struct BtWin {
    int lo, hi, glob;  // rows [lo, hi] are in the window; glob: single row read from HBM
};

// binary-lifting tables of the window's first-predecessor chains (the DP's descriptor batch is dead
// during the backtrack): 6 tables of one byte per window row
constexpr int kBtLift = 6;
static_assert(kBtLift * kWave <= kDescBatch * kDescInts * 4, "lifting tables must fit the descriptor batch");
__device__ __forceinline__ uint8_t *bt_lift(const SharedState &sh) {
    return reinterpret_cast<uint8_t *>(const_cast<int *>(&sh.desc[0][0]));
}

template <int RW>
__device__ __forceinline__ void bt_refill(SharedState &sh, const Slot &s, int i, int lane, BtWin &w, int kpwin) {
    constexpr int kTbWinR = bt_tb_win<RW>(), kKpWinR = bt_kp_win<RW>();
    const int rr = i - lane;
    const bool valid = rr >= 0;
    int4 ra = make_int4(0, -1, 0, 0), rb = make_int4(0, 0, 0, 0), da = make_int4(0, 0, 0, 0),
         db = make_int4(0, 0, 0, 0);
    if (valid) {
        const GLB int4 *ri = reinterpret_cast<const GLB int4 *>(s.rinfo + (int64_t)rr * kRowInfoInts);
        const GLB int4 *di = reinterpret_cast<const GLB int4 *>(s.desc + (int64_t)rr * kDescInts);
        ra = make_int4(ri[0].x, ri[0].y, ri[0].z, ri[0].w);
        rb = make_int4(ri[1].x, ri[1].y, ri[1].z, ri[1].w);
        da = make_int4(di[0].x, di[0].y, di[0].z, di[0].w);
        db = make_int4(di[1].x, di[1].y, di[1].z, di[1].w);
    }
    const int beg = ra.x, end = ra.y, tbbase = ra.z, kpbase = ra.w, node = da.x, pn = da.y >> 16;
    const int cb0 = beg & ~1;
    const int tbw = (end - cb0 + 1 + 3) & ~3;
    const bool multi = valid && pn > 1;
    const int ks = kp_stride(pn);
    const int tstart = tbbase + cb0, tend = tstart + tbw;
    const int kstart = kpbase + ks * cb0, kend = kstart + ks * tbw;
    const int TE = readlane(tend, 0);
    const unsigned long long mm = __ballot(multi);
    const int fm = mm ? __ffsll((long long)mm) - 1 : 0;
    const int KE = readlane(kend, fm);
    const bool fit = valid && TE - (tstart & ~15) <= kTbWinR && (!multi || KE - (kstart & ~15) <= kpwin);
    const unsigned long long nf = ~__ballot(fit);
    const int cnt = nf ? __ffsll((long long)nf) - 1 : kWave;
    int *md = &sh.bt.md[lane][0];
    if (cnt == 0) {
        // row i alone does not fit: read it from HBM
        if (lane == 0) {
            md[0] = tbbase;
            md[1] = multi ? kpbase : kKpNone;
            md[2] = node;
            md[3] = da.w;
            md[4] = db.x;
            md[5] = db.y;
            md[6] = db.z;
            md[7] = db.w;
        }
        w.lo = w.hi = i;
        w.glob = 1;
        wave_sync();
        return;
    }
    const int rs16 = readlane(tstart, cnt - 1) & ~15;
    const unsigned long long mw = mm & ((cnt == kWave) ? ~0ull : ((1ull << cnt) - 1));
    const int lm = mw ? 63 - __clzll((long long)mw) : 0;
    const int ks16 = readlane(kstart, lm) & ~15;
    const int tsz = TE - rs16, ksz = mw ? KE - ks16 : 0;
    // wide copies: all loads first, then the LDS stores (one HBM round trip)
    constexpr int kTU = kTbWinR / (16 * kWave), kKU = kKpWinR / (16 * kWave);
    const GLB int4 *tg = reinterpret_cast<const GLB int4 *>(s.tb + rs16);
    const GLB int4 *kg = reinterpret_cast<const GLB int4 *>(s.kp + ks16);
    int4 tv[kTU], kv[kKU];
#pragma unroll
    for (int u = 0; u < kTU; ++u) {
        const int x = u * kWave + lane;
        if (x * 16 < tsz) tv[u] = make_int4(tg[x].x, tg[x].y, tg[x].z, tg[x].w);
    }
#pragma unroll
    for (int u = 0; u < kKU; ++u) {
        const int x = u * kWave + lane;
        if (x * 16 < ksz) kv[u] = make_int4(kg[x].x, kg[x].y, kg[x].z, kg[x].w);
    }
    int4 *tl = reinterpret_cast<int4 *>(bt_tb<RW>(sh));
    int4 *kl = reinterpret_cast<int4 *>(g_qnib);
#pragma unroll
    for (int u = 0; u < kTU; ++u) {
        const int x = u * kWave + lane;
        if (x * 16 < tsz) tl[x] = tv[u];
    }
#pragma unroll
    for (int u = 0; u < kKU; ++u) {
        const int x = u * kWave + lane;
        if (x * 16 < ksz) kl[x] = kv[u];
    }
    if (lane < cnt) {
        md[0] = tbbase - rs16;
        md[1] = multi ? kpbase - ks16 : kKpNone;
        md[2] = node | (multi && ks == 3 ? kNodeKp3 : 0);
        md[3] = da.w;
        md[4] = db.x;
        md[5] = db.y;
        md[6] = db.z;
        md[7] = db.w;
    }
    w.lo = i - cnt + 1;
    w.hi = i;
    w.glob = 0;
    // first-predecessor chains of the window for the diagonal runs: window index x = w.hi - row;
    // table s holds the 2^s-th first-predecessor ancestor of each window row (0xff: leaves the window)
    uint8_t *lift = bt_lift(sh);
    int x1 = 0xff;
    if (lane < cnt && da.w >= w.lo && da.w < rr) x1 = i - da.w;
    lift[lane] = (uint8_t)x1;
#pragma unroll
    for (int t = 1; t < kBtLift; ++t) {
        const int y = lift[(t - 1) * kWave + lane];
        const int z = y != 0xff ? lift[(t - 1) * kWave + y] : 0xff;
        lift[t * kWave + lane] = (uint8_t)z;
    }
    wave_sync();
}

// One walk step read straight from HBM (rows too wide for the window, > kPreInline predecessors).
__device__ __forceinline__ void bt_step_global(const PoaRunArgs &a, const Slot &s, int &i, int &j, int &st) {
    const gint *rb = s.rinfo + (int64_t)i * kRowInfoInts;
    const gint *db = s.desc + (int64_t)i * kDescInts;
    const int tbbase = rb[2], kpbase = rb[3], node = db[0], pn = db[1] >> 16;
    const int t = s.tb[tbbase + j];
    if (st == 1 || st == 2) {
        if (!(t & (st == 1 ? kTbE1Ext : kTbE2Ext))) {
            st = 0;
            return;
        }
    }
    const bool multi = pn > 1;
    // predecessor index of the M / E1 / E2 maximum (field f) of this cell
    auto kp_at = [&](int f) -> int {
        if (kp_stride(pn) == 1) return (s.kp[kpbase + j] >> (2 * f)) & 3;
        return s.kp[kpbase + 3 * j + f];
    };
    const int ty = st == 0 ? tb_type(t, multi ? kp_at(1) : 0, multi ? kp_at(2) : 0) : st;
    if (ty <= 2) {
        const int k = multi ? kp_at(ty) : 0;
        const int p = (k < kPreInline) ? s.desc[(int64_t)i * kDescInts + 3 + k] : s.xpre[(int64_t)i * a.caps.DCAP + k];
        if (ty == 0) {
            s.qnode[j - 1] = node;
            --j;
        }
        st = ty;
        i = p;
        return;
    }
    s.qnode[j - 1] = -1;
    const int tprev = s.tb[tbbase + j - 1];
    st = (tprev & (ty == 3 ? kTbF1ExtNext : kTbF2ExtNext)) ? ty : 0;
    --j;
}

// One walk step from the LDS window, branch-free (every lane computes the same step).  A step that
// cannot be served from the window sets `stall` and changes nothing; finished walks are no-ops.
template <int RW>
__device__ __forceinline__ void bt_step_lds(const SharedState &sh, const Slot &s, int wlo, int whi, int &i,
                                            int &j, int &st, int &stall) {
    const uint8_t *tbw = bt_tb<RW>(sh);
    const bool live = i > 0 && j > 0 && !stall;
    const bool inwin = i >= wlo;
    const int idx = min(max(whi - i, 0), kWave - 1);
    const int4 m0 = *reinterpret_cast<const int4 *>(&sh.bt.md[idx][0]);
    const int4 m1 = *reinterpret_cast<const int4 *>(&sh.bt.md[idx][4]);
    const int woff = m0.x, kof = m0.y, node = m0.z & ~kNodeKp3;
    const bool kp3 = (m0.z & kNodeKp3) != 0;
    const int tix = max(woff + j, 1);
    const int t = tbw[tix], tprev = tbw[tix - 1];
    const bool multi = kof != kKpNone;
    const int kix = multi ? kof + (kp3 ? 3 * j : j) : 0;
    const int kb = g_qnib[kix];
    const int k0 = kp3 ? kb : kb & 3, k1 = kp3 ? g_qnib[kix + 1] : (kb >> 2) & 3,
              k2 = kp3 ? g_qnib[kix + 2] : (kb >> 4) & 3;
    const bool isE = st == 1 || st == 2;
    const bool open = isE && !(t & (st == 1 ? kTbE1Ext : kTbE2Ext));
    const int ty = st == 0 ? tb_type(t, multi ? k1 : 0, multi ? k2 : 0) : st;
    const bool mv = !open && ty <= 2;
    const int k = multi ? (ty == 0 ? k0 : (ty == 1 ? k1 : k2)) : 0;
    const int p = k == 0 ? m0.w : (k == 1 ? m1.x : (k == 2 ? m1.y : (k == 3 ? m1.z : m1.w)));
    const bool blocked = !inwin || (mv && k >= kPreInline);
    const bool go = live && !blocked;
    stall |= (int)(live && blocked);
    const bool isF = !open && ty >= 3;
    const bool wr = go && ((mv && ty == 0) || isF);
    if (wr) s.qnode[j - 1] = mv ? node : -1;
    const int fopen = !(tprev & (ty == 3 ? kTbF1ExtNext : kTbF2ExtNext));
    const int nst = open ? 0 : (mv ? ty : (fopen ? 0 : ty));
    const int ni = mv ? p : i;
    const int nj = j - (int)((mv && ty == 0) || isF);
    i = go ? ni : i;
    j = go ? nj : j;
    st = go ? nst : st;
}

template <int RW>
__device__ __forceinline__ int backtrack(SharedState &sh, int bi, int qlen, int n, int lane) {
    const PoaRunArgs a = args_of(sh);
    Slot s = slot_of(sh);
    int i = bi, j = qlen, st = 0;  // 0 H, 1 E1 (at E1out[i][j]), 2 E2, 3 F1, 4 F2
    constexpr int kUnroll = 8;
    int guard = (2 * (n + qlen) + 8) / kUnroll + 2 * (n + qlen) + 8;
    BtWin w{1, 0, 0};
    int glob_row = -1;
    // predecessor bytes reuse the read's buffer (a wide launch: the dead ring, at least 16 KB in all)
    const int kpwin = RW == kChunk ? min(kKpWinMax, a.qlds & ~15) : bt_kp_win<RW>();
    while (i > 0 && j > 0) {
        if (--guard < 0) return kStInternal;
        if (i == glob_row) {
            bt_step_global(a, s, i, j, st);
            i = bcast0(i);
            j = bcast0(j);
            st = bcast0(st);
            continue;
        }
        if (i < w.lo || i > w.hi) {
            const uint64_t c0 = a.prof ? clock64() : 0;
            bt_refill<RW>(sh, s, i, lane, w, kpwin);
            if (a.prof && !(a.dbg & 16) && lane == 0) {
                int64_t *pf = a.prof + (int64_t)blockIdx.x * kProfPhases;
                pf[12] += (int64_t)(clock64() - c0);
                pf[13] += 1;
            }
            if (w.glob) {
                glob_row = i;
                w.lo = 1;
                w.hi = 0;
                continue;
            }
        }
        if (st == 0) {
            // Diagonal run, wave-parallel: lane k checks the k-th cell of a run of M steps that follows
            // the rows' first predecessors -- row R_k = k-th first-predecessor ancestor of i (binary
            // lifting over the window), column j - k.  The step is taken when the cell is an M step
            // whose source predecessor (the only one, or the one its predecessor byte names) is the
            // first one, i.e. R_{k+1}.  Every step before the first lane that fails is taken at once:
            // runs end at indels, at rows whose M source is another predecessor (that step is taken
            // too, and the next run starts from its row) and at the window's end.
            const uint8_t *lift = bt_lift(sh);
            int x = w.hi - i;
#pragma unroll
            for (int t = 0; t < kBtLift; ++t)
                if ((lane >> t) & 1) x = x != 0xff ? lift[t * kWave + x] : 0xff;
            const int ri = x != 0xff ? w.hi - x : -1, cj = j - lane;
            bool okk = false, okm = false;
            int nd = 0, pr = -1;
            if (ri >= w.lo && ri > 0 && cj > 0) {
                const int4 m0 = *reinterpret_cast<const int4 *>(&sh.bt.md[x][0]);
                const int t = bt_tb<RW>(sh)[m0.x + cj];
                pr = m0.w;
                if (m0.y != kKpNone) {
                    const int4 m1 = *reinterpret_cast<const int4 *>(&sh.bt.md[x][4]);
                    const int k0 = (m0.z & kNodeKp3) ? g_qnib[m0.y + 3 * cj] : g_qnib[m0.y + cj] & 3;
                    pr = k0 == 0 ? m0.w : k0 == 1 ? m1.x : k0 == 2 ? m1.y : k0 == 3 ? m1.z : k0 == 4 ? m1.w : -1;
                }
                okm = pr >= 0 && !(t & kTbNM);
                okk = okm && pr == m0.w;
                nd = m0.z & ~kNodeKp3;
            }
            const unsigned long long bad = ~__ballot(okk);
            const int f = bad ? __ffsll((long long)bad) - 1 : kWave;
#ifdef MANDO_BT_STATS
            if (a.prof && !(a.dbg & 16) && lane == 0) a.prof[(int64_t)blockIdx.x * kProfPhases + 16] += 1;
#endif
            if (f < kWave && ((__ballot(okm) >> f) & 1ull)) {
                // lanes [0, f] are all M steps; lane f's leads to another predecessor (or out of the window)
                if (lane <= f) s.qnode[cj - 1] = nd;
                i = readlane(pr, f);
                j -= f + 1;
                continue;
            }
#ifdef MANDO_BT_STATS
            if (a.prof && f < kWave) {
                int why = 0;
                if (ri >= w.lo && ri > 0 && cj > 0) {
                    const int4 m0 = *reinterpret_cast<const int4 *>(&sh.bt.md[x][0]);
                    const int t = bt_tb<RW>(sh)[m0.x + cj];
                    why = (t & kTbNM) ? 3 : 2;
                }
                why = readlane(why, f);
                if (lane == 0) a.prof[(int64_t)blockIdx.x * kProfPhases + 8 + why] += 1;
            }
#endif
            if (f > 0) {
                // lanes [0, f) are M steps; the walk continues at lane f - 1's source row
                if (lane < f) s.qnode[cj - 1] = nd;
                i = readlane(pr, f - 1);
                j -= f;
                continue;
            }
        }
        int stall = 0;
        int vi = i, vj = j, vst = st;
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) bt_step_lds<RW>(sh, s, w.lo, w.hi, vi, vj, vst, stall);
        if (a.prof && !(a.dbg & 16) && lane == 0) a.prof[(int64_t)blockIdx.x * kProfPhases + 14] += 1;
        i = bcast0(vi);
        j = bcast0(vj);
        st = bcast0(vst);
        if (bcast0(stall) && i >= w.lo && i <= w.hi && i > 0 && j > 0) {
            // in the window but more than kPreInline predecessors: one step from HBM
            bt_step_global(a, s, i, j, st);
            i = bcast0(i);
            j = bcast0(j);
            st = bcast0(st);
        }
    }
    for (int t = lane; t < j; t += kWave) s.qnode[t] = -1;
    return kStOk;
}

// ---------------------------------------------------------------------------------------------
// -S: one read aligned window by window (oracle/poa_ref.c align_read).  The seed kernel's kept
// anchors (k-mer starts t_x in the previous read, q_x in this one) pin q_x + i to the node position
// t_x + i of the previous read joined (tnode); the stretches between pinned k-mers are banded DPs over
// the window rows between their bounding nodes, each writing its slice of qnode.  The whole read's
// path then goes through update_graph at once, exactly like an unseeded read.
// ---------------------------------------------------------------------------------------------
// MANDO_PROF: adds the cycles since the last mark to phase k (k < 0: only sets the mark); a window's
// row count goes to phase 5 and the window to phase 6.  State lives in LDS, not in registers.
__device__ __forceinline__ void prof_mark(SharedState &sh, int lane, int k, int rows = -1) {
    int64_t *prof = sh.args.prof;
    if (prof && lane == 0) {
        prof += (int64_t)blockIdx.x * kProfPhases;
        const uint64_t t = clock64();
        if (k >= 0) prof[k] += (int64_t)(t - sh.tmark);
        if (rows >= 0) {
            prof[5] += rows;
            prof[6] += 1;
        }
        sh.tmark = t;
    }
}

// One -S window x of read q (0 <= x <= np): the rows between the previous pinned k-mer's last node
// (the source for x = 0) and anchor x's first node (the sink for x = np), aligned to the read's
// positions between them; then anchor x's k-mer is pinned to its nodes.  Writes the read's qnode
// entries of those positions only, so windows are independent of each other.
template <class SC>
__device__ __forceinline__ int seeded_window(SharedState &sh, const SC &sc, const uint8_t *q, int qlen, int lane,
                                             int64_t &cells, int item, int np, int x) {
    int k = 0, pc = 0;
    const int32_t *par_t = nullptr, *par_q = nullptr;
    {
        const PoaRunArgs a = args_of(sh);
        k = a.seed_k;
        pc = a.pc;
        par_t = a.par_t;
        par_q = a.par_q;
    }
    int B = kSrc, q0 = 0, E = kSink, q1 = qlen, tx = 0;
    {
        const Slot s = slot_of(sh);
        if (x > 0) {
            const int tp = bcast0(par_t[(int64_t)item * pc + x - 1]);
            B = bcast0(s.tnode[tp + k - 1]);
            q0 = bcast0(par_q[(int64_t)item * pc + x - 1]) + k;
        }
        if (x < np) {
            tx = bcast0(par_t[(int64_t)item * pc + x]);
            q1 = bcast0(par_q[(int64_t)item * pc + x]);
            E = bcast0(s.tnode[tx]);
        }
    }
    if (q1 > q0) {
        const int qw = q1 - q0;
        const bool try16 = r16_eligible<SC, kChunk>(sc, qw) && !(args_of(sh).dbg & 1);
        int m = 0;
        int st = build_window(sh, B, E, lane, try16 ? kRing16 : kRing, m);
#ifdef MANDO_TEAM_DEBUG
        {
            const Slot s = slot_of(sh);
            const int pB = bcast0(s.pos[B]), pE = bcast0(s.pos[E]);
            if (lane == 0 && st != kStOk)
                printf("[win] block %d x %d B %d E %d pB %d pE %d q0 %d q1 %d st %d\n", (int)blockIdx.x, x, B, E, pB, pE, q0, q1, st);
        }
#endif
        if (st != kStOk) return st;
        {
            const Slot s = slot_of(sh);
            const int pB = bcast0(s.pos[B]), pE = bcast0(s.pos[E]);
            if (lane == 0) {
                sh.slot.desc = s.wdesc;
                sh.slot.xpre = s.wxpre;
                sh.slot.qnode = sh.qnode_full + q0;
                sh.win_on = 1;
                sh.win_sink = E;
                sh.win_pb = pB;
                sh.win_pe = pE;
            }
        }
        wave_sync();
        prof_mark(sh, lane, 0, m);
        int bi = -1;
        st = try16 ? run_dp<SC, true>(sh, sc, q + q0, qw, m, lane, cells, bi) : kStRetry32;
        if (st == kStRetry32) {
            if (try16) {  // window descriptors at the 32-bit ring depth
                if (lane == 0) {
                    sh.slot.desc = sh.desc_full;
                    sh.slot.xpre = sh.xpre_full;
                }
                wave_sync();
                st = build_window(sh, B, E, lane, kRing, m);
                if (st != kStOk) return st;
                if (lane == 0) {
                    const Slot s = sh.slot;
                    sh.slot.desc = s.wdesc;
                    sh.slot.xpre = s.wxpre;
                }
                wave_sync();
            }
            st = run_dp<SC, false>(sh, sc, q + q0, qw, m, lane, cells, bi);
        }
        if (st == kStOk && bi < 0) st = kStInternal;
#ifdef MANDO_TEAM_DEBUG
        if (lane == 0 && st != kStOk) printf("[win] block %d x %d dp st %d bi %d m %d qw %d\n", (int)blockIdx.x, x, st, bi, m, qw);
#endif
        prof_mark(sh, lane, 1);
        if (st == kStOk) {
            wave_sync();
            __builtin_amdgcn_s_setprio(kSerialPrio);
            st = backtrack<kChunk>(sh, bi, qw, m, lane);
            __builtin_amdgcn_s_setprio(0);
#ifdef MANDO_TEAM_DEBUG
            if (lane == 0 && st != kStOk) printf("[win] block %d x %d backtrack st %d\n", (int)blockIdx.x, x, st);
#endif
        }
        prof_mark(sh, lane, 2);
        if (lane == 0) {
            sh.slot.desc = sh.desc_full;
            sh.slot.xpre = sh.xpre_full;
            sh.slot.qnode = sh.qnode_full;
            sh.win_on = 0;
        }
        wave_sync();
        if (st != kStOk) return st;
        prof_mark(sh, lane, -1);
    }
    if (x < np) {  // the pinned k-mer
        const Slot s = slot_of(sh);
        hbm_fence();
        for (int i = lane; i < k; i += kWave) s.qnode[q1 + i] = s.tnode[tx + i];
        wave_sync();
    }
    return kStOk;
}

// the read's partition item and anchor count (par_n)
__device__ __forceinline__ int seeded_item(SharedState &sh, int64_t rd, int &np) {
    const PoaRunArgs a = args_of(sh);
    const int item = bcast0(a.par_item[rd]);
    np = item >= 0 ? bcast0(a.par_n[item]) : 0;
    return item;
}

// ---- -S teams -----------------------------------------------------------------------------------
// A seeded launch can give each group a team of a.team one-wave workgroups (consecutive blockIdx,
// member 0 leading).  The leader owns the graph (its slot), builds the read's descriptors and
// publishes the read as a job in the team's box; every member, the leader included, then claims the
// job's windows one at a time (CAS on the box's claim word) and aligns each with its own slot as DP
// scratch (graph and qnode: the leader's).  The leader waits only for windows that were claimed,
// so a team whose helpers are not resident (yet) finishes its read alone.  Hand-offs follow the
// agent-scope release / acquire forms of cdna_hip_programming.md Guideline 16: plain stores, each
// storing wave's s_waitcnt vmcnt(0), a release fence, s_waitcnt again, a relaxed agent-scope flag
// (the claim word, the done counter); the other side polls relaxed, then ONE acquire, then plain
// loads.  The box's own words are read and written only by agent-scope atomics.
constexpr uint64_t kJobExit = 0xffffffull;
// every wait is bounded (s_memrealtime ticks at 100 MHz): a team that stops making progress ends
// with an internal-error status instead of holding the GPU
constexpr uint64_t kTeamWaitTicks = 60ull * 100000000ull;
#define MANDO_RLX_AGENT __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT

__device__ __forceinline__ void team_release() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
__device__ __forceinline__ void team_acquire() {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// next unclaimed window of job `job` (np anchors), or -1 when the job is exhausted or replaced.
// Control stays wave-uniform (every lane loads the word; only the CAS itself is lane 0's): a loop
// inside a lane-0 branch would let the compiler spill other lanes' live values under a one-lane exec.
__device__ __forceinline__ uint64_t box_load64(uint64_t *p) {
    return readlane64(__hip_atomic_load(p, MANDO_RLX_AGENT), 0);
}
__device__ __forceinline__ int box_load32(uint32_t *p) { return bcast0((int)__hip_atomic_load(p, MANDO_RLX_AGENT)); }
__device__ __forceinline__ int team_claim(TeamBox *box, uint64_t job, int lane) {
    for (;;) {
        const uint64_t c = box_load64(&box->claim);
        if ((c >> 40) != job) return -1;
        const int np = (int)((c >> 20) & 0xfffff), nx = (int)(c & 0xfffff);
        if (nx > np) return -1;
        int won = 0;
        if (lane == 0) {
            uint64_t e = c;
            won = __hip_atomic_compare_exchange_strong(&box->claim, &e, c + 1, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT);
        }
        if (bcast0(won)) return nx;
    }
}

// a claimed window is done: its qnode entries are published, then counted
__device__ __forceinline__ void team_report(TeamBox *box, int st, int64_t cells, int lane, bool fence = true) {
    if (lane == 0) {
        if (cells) __hip_atomic_fetch_add(&box->cells, cells, MANDO_RLX_AGENT);
        if (st != kStOk) {
            int z = 0;
            __hip_atomic_compare_exchange_strong(&box->status, &z, st, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    if (fence) team_release();
    if (lane == 0) __hip_atomic_fetch_add(&box->done, 1u, MANDO_RLX_AGENT);
}

// claims and aligns windows of `job` until none is left
template <class SC>
__device__ __forceinline__ void team_windows(SharedState &sh, const SC &sc, TeamBox *box, uint64_t job,
                                             const uint8_t *q, int qlen, int item, int np, int lane) {
#ifdef MANDO_TEAM_DEBUG
    const int dbg = args_of(sh).dbg;
    int xs = 0;
#endif
    for (;;) {
#ifdef MANDO_TEAM_DEBUG
        int x;
        if (dbg & 32) x = xs <= np ? xs++ : -1;
        else x = team_claim(box, job, lane);
#else
        const int x = team_claim(box, job, lane);
#endif
        if (x < 0) break;
        int64_t wc = 0;
        const int st = seeded_window(sh, sc, q, qlen, lane, wc, item, np, x);
#ifdef MANDO_TEAM_DEBUG
        if (lane == 0 && st != kStOk) printf("[team] block %d window %d/%d status %d\n", (int)blockIdx.x, x, np, st);
#endif
#ifdef MANDO_TEAM_DEBUG
        team_report(box, st, wc, lane, !(dbg & 16));
#else
        team_report(box, st, wc, lane);
#endif
    }
}

// ---------------------------------------------------------------------------------------------
// graph update for one aligned read (wave-parallel over query positions)
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ int add_edge(const PoaRunArgs &a, Slot &s, int from, int to, bool check,
                                        bool from_new, bool to_new) {
    gint *ol = out_list(s, a, from);
    gint *ow = out_wlist(s, a, from);
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
    gint *il = in_list(s, a, to);
    const int inn = to_new ? 0 : s.in_n[to];
    if (inn >= in_cap(a, to)) return kStCap;
    il[inn] = from;
    s.in_n[to] = inn + 1;
    return kStOk;
}

__device__ __forceinline__ int update_graph(SharedState &sh, const uint8_t *q, int qlen, int &n,
                            int &ng, int lane) {
    const PoaRunArgs a = args_of(sh);
    Slot s = slot_of(sh);
#ifdef MANDO_UPD_PROF
    // dev build: cycles of the update's passes in prof phases 8..11 (1, 2, 3, 4 + 5)
    uint64_t upd_t = clock64();
#define MANDO_UPD_MARK(k)                                                                \
    do {                                                                                 \
        const uint64_t t_ = clock64();                                                   \
        if (a.prof && lane == 0) a.prof[(int64_t)blockIdx.x * kProfPhases + (k)] += (int64_t)(t_ - upd_t); \
        upd_t = t_;                                                                      \
    } while (0)
#else
#define MANDO_UPD_MARK(k) \
    do {                  \
    } while (0)
#endif
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
            gint *gt = s.gtab + (int64_t)g * kGtabInts;
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
        const int prev_t = dpp_shr1(tgt, last);
        const int prev_n = dpp_shr1(isnew, last_new);
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
    MANDO_UPD_MARK(8);
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
        const int prev_kind = dpp_shr1(kind, 0);
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
    MANDO_UPD_MARK(9);
    // pass 3: shift old rows by the number of new nodes inserted before (and at) them
    int carry = 0;
    for (int c = 0; c * kWave < n_old; ++c) {
        const int r = c * kWave + lane;
        const bool valid = r < n_old;
        const int tot = valid ? s.ins[r] + s.insmm[r] : 0;
        const int inc = dpp_incl_sum(tot) + carry;
        carry = readlane(inc, kWave - 1);
        if (valid) {
            const int v = s.order[r];
            const int np = r + inc;
            s.order2[np] = v;
            s.pos[v] = np;
        }
    }
    wave_sync();
    MANDO_UPD_MARK(10);
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
    if (lane == 0) {
        sh.slot.order = s.order2;
        sh.slot.order2 = s.order;
    }
    wave_sync();
    MANDO_UPD_MARK(11);
#undef MANDO_UPD_MARK
    return kStOk;
}

// ---------------------------------------------------------------------------------------------
// heaviest bundling (lane 0): reverse topological sweep, then walk from the source
// ---------------------------------------------------------------------------------------------
// Heaviest bundling, wave-parallel where it can be: per block of 64 rows (last block first) every lane
// gathers its row's node, out-degree and up to kConsOut (successor row, edge weight) pairs, so the
// sweep itself -- inherently sequential: a row's score is its best successor's plus the edge weight --
// reads them from registers (readlane) and the successors' scores from an LDS ring of the last
// kScRing rows (HBM for successors further ahead), instead of five dependent HBM loads per row.
// Then the walk from the source reads nxt a block of 64 rows at a time, records the path's rows and
// the bases are gathered in parallel.  Same choices as the serial form: the heaviest out-edge, ties
// to the successor with the larger-or-equal score, in out-edge order.
constexpr int kConsOut = 4;
constexpr int kScRing = 1024;
static_assert(kScRing * 4 <= (int)sizeof(DpLds), "score ring must fit the DP scratch");
__device__ __forceinline__ int consensus(SharedState &sh, int n, uint8_t *out, int64_t cap, int &len, int lane) {
    const PoaRunArgs a = args_of(sh);
    Slot s = slot_of(sh);
    int *ring = reinterpret_cast<int *>(&sh.dp);
    int err = kStOk;
    for (int b0 = ((n - 1) / kWave) * kWave; b0 >= 0; b0 -= kWave) {
        const int r = b0 + lane;
        int on = 0, sink = 1, ro[kConsOut], wt[kConsOut];
#pragma unroll
        for (int k = 0; k < kConsOut; ++k) ro[k] = wt[k] = -1;
        if (r < n) {
            const int v = s.order[r];
            sink = v == kSink;
            if (!sink) {
                on = s.out_n[v];
                const gint *ol = out_list(s, a, v);
                const gint *ow = out_wlist(s, a, v);
#pragma unroll
                for (int k = 0; k < kConsOut; ++k)
                    if (k < on) {
                        ro[k] = s.pos[ol[k]];
                        wt[k] = ow[k];
                    }
            }
        }
        int my_sc = 0, my_nx = -1;
        for (int l = min(kWave, n - b0) - 1; l >= 0; --l) {
            const int rr = b0 + l;
            int sc = 0, nx = -1;
            if (!readlane(sink, l)) {
                const int o = readlane(on, l);
                int maxw = -1, maxr = -1, maxs = 0;
                // a successor's score: the ring holds rows (rr, rr + kScRing], HBM the ones further on
                auto score_of = [&](int ro_) -> int {
                    if (ro_ - rr <= kScRing) return bcast0(ring[ro_ & (kScRing - 1)]);
                    hbm_fence();  // this wave's own stores of earlier blocks (rare: an edge > kScRing rows long)
                    return bcast0(s.score[ro_]);
                };
#pragma unroll
                for (int k = 0; k < kConsOut; ++k) {
                    if (k >= o) break;
                    const int rk = readlane(ro[k], l), wk = readlane(wt[k], l);
                    if (maxw < wk) {
                        maxw = wk;
                        maxr = rk;
                        maxs = score_of(rk);
                    } else if (maxw == wk) {
                        const int sk = score_of(rk);
                        if (maxs <= sk) {
                            maxr = rk;
                            maxs = sk;
                        }
                    }
                }
                if (o > kConsOut) {  // rare rows with more out-edges: the rest from HBM
                    const int v = bcast0(s.order[rr]);
                    const gint *ol = out_list(s, a, v);
                    const gint *ow = out_wlist(s, a, v);
                    for (int k = kConsOut; k < o; ++k) {
                        const int rk = bcast0(s.pos[ol[k]]), wk = bcast0(ow[k]);
                        if (maxw < wk) {
                            maxw = wk;
                            maxr = rk;
                            maxs = score_of(rk);
                        } else if (maxw == wk) {
                            const int sk = score_of(rk);
                            if (maxs <= sk) {
                                maxr = rk;
                                maxs = sk;
                            }
                        }
                    }
                }
                if (maxr < 0) err = kStInternal;
                sc = maxw + maxs;
                nx = maxr;
            }
            if (lane == 0) ring[rr & (kScRing - 1)] = sc;
            if (lane == l) {
                my_sc = sc;
                my_nx = nx;
            }
        }
        if (r < n) {
            s.score[r] = my_sc;
            s.nxt[r] = my_nx;
        }
        if (err != kStOk) return err;
    }
    hbm_fence();
    // walk from the source along nxt (a block of 64 rows' successors in registers); the path's rows
    // are listed in the score array (dead now), then the bases gathered
    int r = bcast0(s.nxt[0]);
    int blk = -1, nv = -1;
    int l = 0;
    while (r >= 0 && r != n - 1) {
        if ((r >> 6) != blk) {
            blk = r >> 6;
            const int x = blk * kWave + lane;
            nv = x < n ? s.nxt[x] : -1;
        }
        if (lane == 0) s.score[l] = r;
        ++l;
        if (l > n) return kStInternal;
        r = readlane(nv, r & (kWave - 1));
    }
    hbm_fence();
    const int lim = (int)min<int64_t>(l, cap);
    for (int t = lane; t < lim; t += kWave) out[t] = s.base[s.order[s.score[t]]];
    len = l;
    return (int64_t)l <= cap ? kStOk : kStCap;
}

// SEEDED: the launch holds only -S groups (seeded_main: teams of workgroups over a read's windows);
// the unseeded instantiations carry none of that code, so the hot DP keeps its register allocation.
// ---- the seeded launch's main loop ---------------------------------------------------------------
// Every member of a team runs the same loop, so a window is aligned at one place in the code:
// member 0 first advances the team's group (leader_advance: the serial work between two reads, then
// the next read's descriptors and its job), then every member claims the job's windows
// (team_windows).  The leader's state between jobs lives in LDS (sh.lead).
__device__ __forceinline__ int64_t read_len(SharedState &sh, int64_t rd, const uint8_t *&q) {
    const PoaRunArgs a = args_of(sh);
    const int64_t o0 = uni64(a.seq_off[rd]);
    q = a.seq + o0;
    return uni64(a.seq_off[rd + 1]) - o0;
}

// leader: finishes the job in flight (wait, graph update), moves to the next read or group and
// publishes its job; returns 0 when the queue is empty (the helpers have been told to stop)
template <class SC>
__device__ __forceinline__ int leader_advance(SharedState &sh, TeamBox *box, int lane) {
    __builtin_amdgcn_s_setprio(kSerialPrio);
    for (;;) {
        if (bcast0(lead_of(sh).pending)) {  // every window of the job has been claimed: wait for the rest
            const int np = bcast0(lead_of(sh).np);
            int late = 0;
            {
                const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
                while (box_load32(&box->done) != np + 1) {
                    __builtin_amdgcn_s_sleep(2);
                    if (__builtin_amdgcn_s_memrealtime() - t0 > kTeamWaitTicks) {
                        late = 1;
                        break;
                    }
                }
            }
            team_acquire();
            wave_sync();
            int st = 0;
            int64_t c = 0;
            if (lane == 0) {
                st = late ? kStInternal : __hip_atomic_load(&box->status, MANDO_RLX_AGENT);
                c = __hip_atomic_load(&box->cells, MANDO_RLX_AGENT);
            }
            st = bcast0(st);
            const int64_t cells = uni64(readlane64(c, 0));
            const int64_t rd = uni64(lead_of(sh).rd);
            int n = bcast0(lead_of(sh).n), ng = bcast0(lead_of(sh).ng);
            if (st == kStOk) {
                const uint8_t *q;
                const int qlen = (int)read_len(sh, rd, q);
                prof_mark(sh, lane, -1);
                st = update_graph(sh, q, qlen, n, ng, lane);
                wave_sync();
                prof_mark(sh, lane, 3);
                if (st == kStOk) {  // this read's node per position: the next read's anchors resolve through it
                    const Slot s = slot_of(sh);
                    hbm_fence();
                    for (int t = lane; t < qlen; t += kWave) s.tnode[t] = s.qtgt[t];
                }
            }
            if (lane == 0) {
                lead_of(sh).pending = 0;
                lead_of(sh).st = st;
                lead_of(sh).n = n;
                lead_of(sh).ng = ng;
                lead_of(sh).cells += cells;
                lead_of(sh).rd = rd + 1;
            }
            wave_sync();
        }
        if (bcast0(lead_of(sh).active)) {  // the group's next read, or its end
            int st = bcast0(lead_of(sh).st);
            int64_t rd = uni64(lead_of(sh).rd);
            const int64_t r1 = uni64(lead_of(sh).r1);
            if (st == kStOk) {
                const uint8_t *q = nullptr;
                int64_t L = 0;
                while (rd < r1 && (L = read_len(sh, rd, q)) <= 0) ++rd;
                if (rd < r1) {
                    int np = 0, item = -1;
                    if (L > args_of(sh).caps.QC) {
                        st = kStCap;
                    } else {
                        item = seeded_item(sh, rd, np);
                        if (np < 0 || np >= (1 << 20) - 1) st = kStInternal;
                    }
                    if (st == kStOk) {  // publish the read as the team's next job
                        const int n = bcast0(lead_of(sh).n);
                        prof_mark(sh, lane, -1);
                        build_desc(sh, n, lane, kRing);
                        wave_sync();
                        prof_mark(sh, lane, 0);
                        const uint64_t job = lead_of(sh).job % 0xfffffeull + 1;
                        if (lane == 0) {  // every earlier job is done: nobody else writes the box now
                            __hip_atomic_store(&box->rd, rd, MANDO_RLX_AGENT);
                            __hip_atomic_store(&box->qlen, (int)L, MANDO_RLX_AGENT);
                            __hip_atomic_store(&box->item, item, MANDO_RLX_AGENT);
                            __hip_atomic_store(&box->cells, (int64_t)0, MANDO_RLX_AGENT);
                            __hip_atomic_store(&box->status, 0, MANDO_RLX_AGENT);
                            __hip_atomic_store(&box->done, 0u, MANDO_RLX_AGENT);
                        }
                        team_release();  // the descriptors, tnode and the job's words, then the claim word
                        if (lane == 0) {
                            __hip_atomic_store(&box->claim, (job << 40) | ((uint64_t)np << 20), MANDO_RLX_AGENT);
                            lead_of(sh).job = job;
                            lead_of(sh).pending = 1;
                            lead_of(sh).np = np;
                            lead_of(sh).item = item;
                            lead_of(sh).qlen = (int)L;
                            lead_of(sh).rd = rd;
                        }
                        wave_sync();
                        return 1;
                    }
                }
            }
            // the group is done (every read aligned, or a failure)
            int clen = 0;
            const int g = bcast0(lead_of(sh).g);
            if (st == kStOk) {
                const PoaRunArgs a = args_of(sh);
                int64_t *prof = a.prof ? a.prof + (int64_t)blockIdx.x * kProfPhases : nullptr;
                const uint64_t t6 = prof ? clock64() : 0;
                const int n = bcast0(lead_of(sh).n);
                int len = 0;
                const int64_t cap = uni64(a.cons_off[g + 1]) - uni64(a.cons_off[g]);
                st = consensus(sh, n, a.cons + uni64(a.cons_off[g]), cap, len, lane);
                clen = bcast0(len);
                if (prof && lane == 0) prof[4] += (int64_t)(clock64() - t6);
            }
            if (lane == 0) {
                const PoaRunArgs a = args_of(sh);
                a.status[g] = st;
                a.cons_len[g] = clen;
                a.cells[g] = lead_of(sh).cells;
                lead_of(sh).active = 0;
            }
            wave_sync();
            continue;
        }
        // the next group from the launch's queue
        int gi = 0;
        {
            const PoaRunArgs a = args_of(sh);
            if (lane == 0) gi = atomicAdd(a.counter, 1);
            gi = bcast0(gi);
            if (gi >= a.n_groups) {
                if (lane == 0) __hip_atomic_store(&box->claim, kJobExit << 40, MANDO_RLX_AGENT);
                return 0;
            }
        }
        int g;
        int64_t r0, r1;
        {
            const PoaRunArgs a = args_of(sh);
            g = a.gorder ? bcast0(a.gorder[gi]) : gi;
            r0 = uni64(a.grp_off[g]);
            r1 = uni64(a.grp_off[g + 1]);
        }
        if (lane == 0) {
            sh.slot.order = sh.order0;
            sh.slot.order2 = sh.order1;
        }
        wave_sync();
        int64_t first = r0;
        const uint8_t *q0 = nullptr;
        int64_t L0 = 0;
        while (first < r1 && (L0 = read_len(sh, first, q0)) <= 0) ++first;
        int st = kStOk, n = 0;
        if (first < r1) {
            st = init_chain(sh, q0, (int)L0, lane, n);
            if (st == kStOk) {  // the chain's node of every position (init_chain: 2 + t)
                const Slot s = slot_of(sh);
                for (int t = lane; t < (int)L0; t += kWave) s.tnode[t] = 2 + t;
            }
            wave_sync();
        }
        if (lane == 0) {
            if (first < r1) {
                lead_of(sh).r1 = r1;
                lead_of(sh).rd = first + 1;
                lead_of(sh).cells = 0;
                lead_of(sh).g = g;
                lead_of(sh).n = n;
                lead_of(sh).ng = 0;
                lead_of(sh).st = st;
                lead_of(sh).pending = 0;
                lead_of(sh).active = 1;
            } else {  // no read: an empty consensus
                const PoaRunArgs a = args_of(sh);
                a.status[g] = kStOk;
                a.cons_len[g] = 0;
                a.cells[g] = 0;
            }
        }
        wave_sync();
    }
}

template <class SC>
__device__ __forceinline__ void seeded_main(SharedState &sh, TeamBox *box, int member, int lane) {
    SC sc;
    if constexpr (!std::is_same<SC, DefaultScores>::value) {
        const PoaRunArgs a = args_of(sh);
        sc = SC{a.match, a.mismatch, a.o1, a.e1, a.o2, a.e2};
    }
    if (lane == 0) {
        lead_of(sh).job = 0;
        lead_of(sh).pending = 0;
        lead_of(sh).active = 0;
    }
    wave_sync();
    uint64_t last = 0;
    for (;;) {
        uint64_t job = 0;
        int64_t rd = 0;
        int qlen = 0, item = 0, np = 0;
        if (member == 0) {
            if (!leader_advance<SC>(sh, box, lane)) return;
            job = (uint64_t)uni64((int64_t)lead_of(sh).job);
            rd = uni64(lead_of(sh).rd);
            qlen = bcast0(lead_of(sh).qlen);
            item = bcast0(lead_of(sh).item);
            np = bcast0(lead_of(sh).np);
        } else {
            uint64_t c = 0;
            {
                const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
                for (;;) {
                    c = box_load64(&box->claim);
                    const uint64_t j = c >> 40;
                    if (j == kJobExit || (j != 0 && j != last && (c & 0xfffff) <= ((c >> 20) & 0xfffff))) break;
                    __builtin_amdgcn_s_sleep(4);
                    if (__builtin_amdgcn_s_memrealtime() - t0 > kTeamWaitTicks) {
                        c = kJobExit << 40;  // the leader is gone: stop
                        break;
                    }
                }
            }
            job = c >> 40;
            if (job == kJobExit) return;
            np = (int)((c >> 20) & 0xfffff);
            team_acquire();
            if (lane == 0) {
                rd = __hip_atomic_load(&box->rd, MANDO_RLX_AGENT);
                qlen = __hip_atomic_load(&box->qlen, MANDO_RLX_AGENT);
                item = __hip_atomic_load(&box->item, MANDO_RLX_AGENT);
            }
            rd = uni64((int64_t)readlane64((uint64_t)rd, 0));
            qlen = bcast0(qlen);
            item = bcast0(item);
        }
        const uint8_t *q;
        {
            const PoaRunArgs a = args_of(sh);
            q = a.seq + uni64(a.seq_off[rd]);
        }
        __builtin_amdgcn_s_setprio(0);
        team_windows(sh, sc, box, job, q, qlen, item, np, lane);
        last = job;
    }
}

#ifndef MANDO_WIDE_WPE
#define MANDO_WIDE_WPE 4  // waves per SIMD the one-wave wide instantiation is compiled for (register budget)
#endif
template <class SC, bool SEEDED, int RW, int NW = 1>
__global__ __launch_bounds__(kWave * NW, NW > 1 ? 2 : (RW == kWideRing ? MANDO_WIDE_WPE : 4)) void poa_kernel(PoaKArgs ka) {
    constexpr int kPrioDp = 0;                             // DP rows (see the unseeded read loop)
    constexpr int kPrioSerial = kPrioDp + kSerialPrio;     // descriptors, backtrack, update, consensus
    static_assert(RW == kChunk || (RW == kWideRing && !SEEDED), "wide rings: unseeded launches");
    static_assert(NW == 1 || (NW == 2 && RW == kWideRing), "two-wave workgroups: wide launches");
    __shared__ SharedState sh;
    const int lane = lane_id();
    if constexpr (NW > 1) {
        // wave 1 of a two-wave workgroup: upper halves of the wide rows (w2_helper), once wave 0 has set
        // up the workgroup's LDS state
        if (bcast0((int)(threadIdx.x >> 6)) != 0) {
            group_barrier();
            w2_helper<SC>(sh, lane);
            return;
        }
    }
    if (lane == 0) sh.args = ka;
    wave_sync();
    const PoaKArgs &a = ka;
    // -S teams: helpers (member > 0) read the graph from the team leader's slot and keep their own DP
    // scratch (window descriptors, row records, traceback, spills)
    int member = 0, team = 1;
    if constexpr (SEEDED) {
        team = a.team > 1 ? a.team : 1;
        member = (int)(blockIdx.x % (unsigned)team);
    }
    int sidx = (int)blockIdx.x;  // workspace slot
    if constexpr (!SEEDED) {
        if (a.one_group) {  // a free slot (at most n_slots workgroups hold one; wave-uniform loop)
            for (int k = 0;; ++k) {
                const int c = (int)((blockIdx.x + (unsigned)k) % (unsigned)a.n_slots);
                int got = 0;
                if (lane == 0) {
                    int z = 0;
                    got = __hip_atomic_compare_exchange_strong(a.slot_busy + c, &z, 1, __ATOMIC_RELAXED,
                                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                if (bcast0(got)) {
                    sidx = c;
                    break;
                }
                if ((k + 1) % a.n_slots == 0) __builtin_amdgcn_s_sleep(8);
            }
            // the slot's last user may have run on another CU: drop this CU's L1 copies of it
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    }
    char *ws = a.ws + (int64_t)sidx * a.slot_bytes;
    char *gw = ws - (int64_t)member * a.slot_bytes;
    Slot s;
    s.base = (gu8 *)(gw + a.lay.base);
    s.gid = (gint *)(gw + a.lay.gid);
    s.gtab = (gint *)(gw + a.lay.gtab);
    s.in_n = (gint *)(gw + a.lay.in_n);
    s.out_n = (gint *)(gw + a.lay.out_n);
    s.in_id = (gint *)(gw + a.lay.in_id);
    s.out_id = (gint *)(gw + a.lay.out_id);
    s.out_w = (gint *)(gw + a.lay.out_w);
    s.sink_in = (gint *)(gw + a.lay.sink_in);
    s.src_out = (gint *)(gw + a.lay.src_out);
    s.src_out_w = (gint *)(gw + a.lay.src_out_w);
    s.pos = (gint *)(gw + a.lay.pos);
    s.remrow = (gint *)(gw + a.lay.remrow);
    s.desc = (gint *)(gw + a.lay.desc);
    s.rinfo = (gint *)(ws + a.lay.rinfo);
    s.tb = (gu8 *)(ws + a.lay.tb);
    s.kp = (gu8 *)(ws + a.lay.kp);
    s.sv = (gint *)(ws + a.lay.sv);
    s.qnode = (gint *)(gw + a.lay.qnode);
    s.qtgt = (gint *)(ws + a.lay.qtgt);
    s.qflag = (gint *)(ws + a.lay.qflag);
    s.qnb = (gint *)(ws + a.lay.qnb);
    s.qoff = (gint *)(ws + a.lay.qoff);
    s.ins = (gint *)(ws + a.lay.ins);
    s.insmm = (gint *)(ws + a.lay.insmm);
    s.qmslot = (gint *)(ws + a.lay.qmslot);
    s.score = (gint *)(ws + a.lay.score);
    s.nxt = (gint *)(ws + a.lay.nxt);
    s.order = (gint *)(ws + a.lay.order0);
    s.order2 = (gint *)(ws + a.lay.order1);
    s.xpre = (gint *)(gw + a.lay.xpre);
    s.wdesc = (gint *)(ws + a.lay.wdesc);
    s.wxpre = (gint *)(ws + a.lay.wxpre);
    s.wmap = (gint *)(ws + a.lay.wmap);
    s.wlist = (gint *)(ws + a.lay.wlist);
    s.wf = (gint *)(ws + a.lay.wf);
    s.wb = (gint *)(ws + a.lay.wb);
    s.tnode = (gint *)(gw + a.lay.tnode);
    if (lane == 0) {
        sh.slot = s;
        sh.order0 = s.order;
        sh.order1 = s.order2;
        sh.win_on = 0;
        sh.win_sink = kSink;
        sh.win_pb = 0;
        sh.win_pe = 0;
        sh.desc_full = s.desc;
        sh.xpre_full = s.xpre;
        sh.qnode_full = s.qnode;
        sh.tmark = clock64();
        sh.slot_idx = sidx;
    }
    wave_sync();
    if constexpr (NW > 1) group_barrier();  // wave 1 may read the LDS state now

    if constexpr (SEEDED) {
        if (member > 0 && (a.dbg & 8)) return;  // MANDO_POA_DBG bit 3: helpers absent (leaders align alone)
        seeded_main<SC>(sh, a.boxes + blockIdx.x / (unsigned)team, member, lane);
        return;
    } else {

    // Nothing of the kernel arguments or the slot stays live across the loop: every phase re-reads
    // what it needs from LDS (args_of / slot_of), which keeps SGPRs free for the DP row loop.
    for (int it = 0;; ++it) {
        int gi = 0;
        {
            const PoaRunArgs a = args_of(sh);
            if (a.one_group) {
                if (it > 0) break;
                gi = (int)blockIdx.x;
            } else {
                if (lane == 0) gi = atomicAdd(a.counter, 1);
                gi = bcast0(gi);
            }
            if (gi >= a.n_groups) break;
        }
        int g;
        int64_t r0, r1;
        {
            const PoaRunArgs a = args_of(sh);
            g = a.gorder ? bcast0(a.gorder[gi]) : gi;
            r0 = uni64(a.grp_off[g]);
            r1 = uni64(a.grp_off[g + 1]);
        }
        if (lane == 0) {
            sh.slot.order = sh.order0;
            sh.slot.order2 = sh.order1;
        }
        wave_sync();
        auto prio_serial = [&] { __builtin_amdgcn_s_setprio(kPrioSerial); };
        auto prio_dp = [&] { __builtin_amdgcn_s_setprio(kPrioDp); };
        int st = kStOk;
        int n = 0, ng = 0;
        int64_t cells = 0;
        int64_t first = r0;
        {
            const PoaRunArgs a = args_of(sh);
            while (first < r1 && a.seq_off[first + 1] - a.seq_off[first] <= 0) ++first;
            first = uni64(first);
        }
        int clen = 0;
        if (first < r1) {
            {
                const PoaRunArgs a = args_of(sh);
                const int64_t o0 = uni64(a.seq_off[first]);
                const uint8_t *q0 = a.seq + o0;
                const int L0 = (int)(uni64(a.seq_off[first + 1]) - o0);
                st = init_chain(sh, q0, L0, lane, n);
            }
            wave_sync();
            for (int64_t rd = first + 1; rd < r1 && st == kStOk; ++rd) {
                int qlen;
                const uint8_t *q;
                int64_t *prof;
                {
                    const PoaRunArgs a = args_of(sh);
                    const int64_t o0 = uni64(a.seq_off[rd]);
                    qlen = (int)(uni64(a.seq_off[rd + 1]) - o0);
                    if (qlen <= 0) continue;
                    if (qlen > a.caps.QC) {
                        st = kStCap;
                        break;
                    }
                    q = a.seq + o0;
                    prof = a.prof ? a.prof + (int64_t)blockIdx.x * kProfPhases : nullptr;
                }
                SC sc;
                if constexpr (!std::is_same<SC, DefaultScores>::value) {
                    const PoaRunArgs aa = args_of(sh);
                    sc = SC{aa.match, aa.mismatch, aa.o1, aa.e1, aa.o2, aa.e2};
                }
                // The serial, latency-bound phases (descriptors, backtrack, graph update, consensus) issue
                // ahead of the co-resident waves' DP rows (s_setprio 3; the DP runs at 0, a fast row's head
                // at 2): those waves return to their DP sooner, the SIMD's issue slots stay busy (config-3
                // kernel -3.5 % at 1 over 0, r01).
                // (Running a wide launch's waves two levels higher changed neither the mean step nor
                // the slow steps: 10-step lines interleaved twice, r03 prio1.)
                prio_serial();
                uint64_t t0 = prof ? clock64() : 0;
                const bool try16 = r16_eligible<SC, RW>(sc, qlen) && !(args_of(sh).dbg & 1);
                build_desc(sh, n, lane, try16 ? kRing16 : kRing);
                uint64_t t1 = prof ? clock64() : 0;
                int bi = -1;
                prio_dp();
                // 16-bit mode when the read's score range allows it; a read that leaves the safe
                // range is re-aligned in 32-bit mode (the graph is untouched until update_graph)
                st = try16 ? run_dp<SC, true, RW, NW>(sh, sc, q, qlen, n, lane, cells, bi) : kStRetry32;
                if (st == kStRetry32) {
                    if (prof && lane == 0) prof[15] += 1;
                    if (try16) {  // descriptors of the 32-bit ring (far / fast flags depend on its depth)
                        wave_sync();
                        build_desc(sh, n, lane, kRing);
                    }
                    st = run_dp<SC, false, RW>(sh, sc, q, qlen, n, lane, cells, bi);
                }
                uint64_t t2 = prof ? clock64() : 0;
                if (prof && lane == 0) {
                    prof[0] += (int64_t)(t1 - t0);
                    prof[1] += (int64_t)(t2 - t1);
                    prof[5] += n;
                    prof[6] += 1;
                }
                if (st != kStOk) break;
                if (bi < 0) {
                    st = kStInternal;
                    break;
                }
                wave_sync();
                uint64_t t3 = prof ? clock64() : 0;
                prio_serial();
                st = backtrack<RW>(sh, bi, qlen, n, lane);
                if (st != kStOk) break;
                wave_sync();
                uint64_t t4 = prof ? clock64() : 0;
                st = update_graph(sh, q, qlen, n, ng, lane);
                wave_sync();
                uint64_t t5 = prof ? clock64() : 0;
                if (prof && lane == 0) {
                    prof[2] += (int64_t)(t4 - t3);
                    prof[3] += (int64_t)(t5 - t4);
                }
            }
            if (st == kStOk) {
                const PoaRunArgs a = args_of(sh);
                int64_t *prof = a.prof ? a.prof + (int64_t)blockIdx.x * kProfPhases : nullptr;
                uint64_t t6 = prof ? clock64() : 0;
                int len = 0;
                const int64_t cap = uni64(a.cons_off[g + 1]) - uni64(a.cons_off[g]);
                st = consensus(sh, n, a.cons + uni64(a.cons_off[g]), cap, len, lane);
                clen = bcast0(len);
                if (prof && lane == 0) prof[4] += (int64_t)(clock64() - t6);
            }
        }
        if (lane == 0) {
            const PoaRunArgs a = args_of(sh);
            a.status[g] = st;
            a.cons_len[g] = clen;
            a.cells[g] = cells;
        }
        wave_sync();
    }
    if constexpr (NW > 1) {  // wave 1 leaves its loop
        w2_post_op(kW2Exit, lane);
        group_barrier();
    }
    if (ka.one_group) {  // the slot is free again (this group's stores are done first)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) __hip_atomic_store(ka.slot_busy + sh.slot_idx, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    }  // unseeded launches
}

// ASCII -> 0..4, 16 bytes per thread (HBM-bound streaming map)
__global__ void encode_kernel(uint8_t *buf, int64_t n) {
    const int64_t i0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 16;
    if (i0 >= n) return;
    auto code = [](uint32_t c) -> uint32_t {
        c |= 0x20;  // lower case
        return c == 'a' ? 0u : c == 'c' ? 1u : c == 'g' ? 2u : c == 't' ? 3u : 4u;
    };
    if (i0 + 16 <= n && (((uintptr_t)(buf + i0)) & 15) == 0) {
        uint4 v = *reinterpret_cast<const uint4 *>(buf + i0);
        uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t x = w[k];
            w[k] = code(x & 0xff) | (code((x >> 8) & 0xff) << 8) | (code((x >> 16) & 0xff) << 16) |
                   (code(x >> 24) << 24);
        }
        *reinterpret_cast<uint4 *>(buf + i0) = make_uint4(w[0], w[1], w[2], w[3]);
    } else {
        for (int64_t i = i0; i < n && i < i0 + 16; ++i) buf[i] = (uint8_t)code(buf[i]);
    }
}

hipError_t launch_encode(uint8_t *buf, int64_t n, hipStream_t stream) {
    const int64_t threads = (n + 15) / 16;
    const int64_t blocks = (threads + 255) / 256;
    hipLaunchKernelGGL(encode_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, buf, n);
    return hipGetLastError();
}

static bool default_scores(const PoaKArgs &a) {
    return a.match == DefaultScores::match && a.mismatch == DefaultScores::mismatch && a.o1 == DefaultScores::o1 &&
           a.e1 == DefaultScores::e1 && a.o2 == DefaultScores::o2 && a.e2 == DefaultScores::e2;
}

// the six instantiations: scores (default / runtime) x kind (narrow, wide, seeded)
template <class F>
static auto by_kind(const PoaKArgs &a, F &&f) {
    const bool dflt = default_scores(a);
    if (a.caps.seeded) return dflt ? f(poa_kernel<DefaultScores, true, kChunk>) : f(poa_kernel<RuntimeScores, true, kChunk>);
    if (a.caps.wide && a.nw == 2)
        return dflt ? f(poa_kernel<DefaultScores, false, kWideRing, 2>) : f(poa_kernel<RuntimeScores, false, kWideRing, 2>);
    if (a.caps.wide)
        return dflt ? f(poa_kernel<DefaultScores, false, kWideRing>) : f(poa_kernel<RuntimeScores, false, kWideRing>);
    return dflt ? f(poa_kernel<DefaultScores, false, kChunk>) : f(poa_kernel<RuntimeScores, false, kChunk>);
}

int poa_blocks_per_cu(const PoaKArgs &a, int cap) {
    int nb = by_kind(a, [&](auto kern) {
        int v = 0;
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, kern, kWave * poa_waves(a), poa_dyn_lds(a)) == hipSuccess
                   ? v
                   : 0;
    });
    if (nb < 1) nb = 8;
    return nb < cap ? nb : cap;
}

hipError_t launch_poa(const PoaKArgs &a, int n_slots, hipStream_t stream) {
    by_kind(a, [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(n_slots), dim3(kWave * poa_waves(a)), poa_dyn_lds(a), stream, a);
        return 0;
    });
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
        // DPP forms used by the DP / graph update
        if (dpp_incl_max(v, -2147483647 - 1) != rmax) ++errs;
        if (dpp_incl_sum(v) != rsum) ++errs;
        const int prevv = lane == 0 ? 12345 : (int)(((lane - 1) * 2654435761u + trial * 40503u) % 1000u) - 500;
        if (dpp_shr1(v, 12345) != prevv) ++errs;
        // packed-pair helpers of the 16-bit rows: argmax keys (v_mad_i32_i16 with op_sel) and the
        // traceback bytes from sign bits (v_perm sign selectors)
        const uint32_t seed = (uint32_t)(lane * 2246822519u + trial * 3266489917u);
        uint32_t d[8];
        for (int k = 0; k < 8; ++k) d[k] = (seed * (2u * k + 1u)) ^ (seed >> (k + 3)) ^ (k & 1 ? 0x80000000u : 0x8000u);
        const uint32_t tb = tb_pack(d[0], d[1], d[2], d[3], d[4], d[5], d[6], d[7]);
        uint32_t want = 0;
        for (int k = 0; k < 8; ++k) want |= ((d[k] >> 15) & 1u) << k | ((d[k] >> 31) & 1u) << (8 + k);
        if ((tb & 0xffffu) != want) ++errs;
        const uint32_t hs = d[3];
        const int want_key = max((int)(short)(hs & 0xffff) * 128 + 127 - 2 * lane, (int)(short)(hs >> 16) * 128 + 126 - 2 * lane);
        if (pair_key(hs, 127 - 2 * lane, 126 - 2 * lane) != want_key) ++errs;
    }
    atomicAdd(bad, errs);
}

hipError_t run_wave_selftest(int *d_bad, hipStream_t stream) {
    hipLaunchKernelGGL(wave_selftest_kernel, dim3(1), dim3(kWave), 0, stream, d_bad);
    return hipGetLastError();
}

}  // namespace mando
