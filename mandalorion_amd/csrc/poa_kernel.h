// poa_kernel.h — internal interface between the C-ABI layer (capi.hip) and the POA kernel
// (poa_kernel.hip).  Not part of the public ABI (that is include/mando.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mando {

constexpr int kWave = 64;
constexpr int kCPL = 2;                  // DP cells per lane per chunk
constexpr int kChunk = kWave * kCPL;     // 128 band columns per chunk
constexpr int kRing = 4;                 // rows of H/E1/E2 kept in LDS (32-bit mode)
constexpr int kRing16 = 8;               // the same in 16-bit mode (same bytes)
constexpr int kRowRing = 32;             // rows of band info kept in LDS
// wide launches (groups whose band exceeds one chunk): the H/E1/E2 ring holds 2 chunks per row and
// lives at the start of the dynamic LDS, ahead of the read's nibbles
constexpr int kWideRing = 2 * kChunk;
constexpr int kWideRingBytes = kRing16 * 3 * kWideRing * 2;
static_assert(kWideRingBytes == kRing * 3 * kWideRing * 4, "the 16- and 32-bit rings share the bytes");
constexpr int kPreInline = 5;            // predecessor rows stored inline in a row descriptor
constexpr int kDescInts = 8;             // ints per row descriptor
constexpr int kRowInfoInts = 8;          // ints per row record in HBM
constexpr int kNegInf = -(1 << 28);      // "minus infinity" sentinel of the DP (never overflows)
constexpr int kSrc = 0, kSink = 1;
// aligned-node group table: [A C G T N] member per base, [5] head (first row of the group's
// contiguous block), [6] member count
constexpr int kGtabInts = 8;

// traceback byte layout (one byte per DP cell).  Raw "differs" bits rather than a resolved source
// type, so both the 32-bit and the packed 16-bit rows produce it with compares only; the backtrack
// resolves the source with abPOA's priority (M, then E1/E2 -- the lower predecessor index first on
// an E1/E2 tie --, then F1, then F2).  Gap bits are set for "extends" (open preferred on ties).
constexpr int kTbNM = 1 << 0;            // M[i][j] != H[i][j]
constexpr int kTbNX1 = 1 << 1;           // E1in[i][j] != H[i][j]
constexpr int kTbNX2 = 1 << 2;           // E2in[i][j] != H[i][j]
constexpr int kTbNF1 = 1 << 3;           // F1[i][j] != H[i][j]
constexpr int kTbE1Ext = 1 << 4;         // E1out[i][j] extends E1in (H[i][j]-oe1 < E1in-e1)
constexpr int kTbE2Ext = 1 << 5;
constexpr int kTbF1ExtNext = 1 << 6;     // F1[i][j+1] extends F1[i][j] (G1[j] < P1[j])
constexpr int kTbF2ExtNext = 1 << 7;

// phases timed when PoaKArgs::prof is set (MANDO_PROF=1)
constexpr int kProfPhases = 20;  // 0 desc, 1 dp, 2 backtrack, 3 update, 4 consensus, 5 rows, 6 reads, 16 diagonal runs,
                                 // 8.. in-row segments (MANDO_STAMPS builds only)

// per-group status codes written by the kernel (match include/mando.h)
constexpr int kStOk = 0, kStCap = -4, kStInternal = -6, kStUnsupported = -5;
constexpr int kStRetry32 = -100;  // kernel-internal: re-run the read's DP in 32-bit mode

struct PoaCaps {
    int32_t NC;      // node capacity per group
    int32_t DCAP;    // in/out edge capacity per ordinary node
    int32_t BIGCAP;  // in-edge capacity of the sink / out-edge capacity of the source
    int32_t QC;      // max read length
    int64_t TBC;     // traceback bytes per read
    int64_t KPC;     // predecessor-index bytes per read (multi-predecessor rows)
    int64_t SVC;     // spilled H/E1/E2 ints per read
    int32_t seeded;  // the launch has -S groups: window descriptors and maps, per-position read nodes
    int32_t wide;    // the launch keeps 256-column ring rows (kWideRing): bands up to 2 chunks take fast rows
};

struct SlotLayout {
    int64_t base, gid, gtab, in_n, out_n, in_id, out_id, out_w, sink_in, src_out, src_out_w;
    int64_t order0, order1, pos, remrow, desc, rinfo, tb, kp, sv, qnode, qtgt, qflag, qnb, qoff, qmslot,
        ins, insmm, score, nxt, xpre, wdesc, wxpre, wmap, wlist, wf, wb, tnode;
    int64_t total;
};

__host__ __device__ inline int64_t align256(int64_t x) { return (x + 255) & ~int64_t(255); }

__host__ __device__ inline SlotLayout make_layout(const PoaCaps &c) {
    SlotLayout L;
    int64_t o = 0;
    const int64_t nc = c.NC, dc = c.DCAP;
    L.base = o; o = align256(o + nc);
    L.gid = o; o = align256(o + 4 * nc);
    L.gtab = o; o = align256(o + 4 * kGtabInts * nc);
    L.in_n = o; o = align256(o + 4 * nc);
    L.out_n = o; o = align256(o + 4 * nc);
    L.in_id = o; o = align256(o + 4 * nc * dc);
    L.out_id = o; o = align256(o + 4 * nc * dc);
    L.out_w = o; o = align256(o + 4 * nc * dc);
    L.sink_in = o; o = align256(o + 4 * (int64_t)c.BIGCAP);
    L.src_out = o; o = align256(o + 4 * (int64_t)c.BIGCAP);
    L.src_out_w = o; o = align256(o + 4 * (int64_t)c.BIGCAP);
    L.order0 = o; o = align256(o + 4 * nc);
    L.order1 = o; o = align256(o + 4 * nc);
    L.pos = o; o = align256(o + 4 * nc);
    L.remrow = o; o = align256(o + 4 * nc);
    L.desc = o; o = align256(o + 4 * kDescInts * (nc + kWave));
    L.rinfo = o; o = align256(o + 4 * kRowInfoInts * nc);
    L.tb = o; o = align256(o + c.TBC);
    L.kp = o; o = align256(o + c.KPC);
    L.sv = o; o = align256(o + 4 * c.SVC);
    const int64_t qc = c.QC + kWave;
    L.qnode = o; o = align256(o + 4 * qc);
    L.qtgt = o; o = align256(o + 4 * qc);
    L.qflag = o; o = align256(o + 4 * qc);
    L.qnb = o; o = align256(o + 4 * qc);
    L.qoff = o; o = align256(o + 4 * qc);
    L.qmslot = o; o = align256(o + 4 * qc);
    L.ins = o; o = align256(o + 4 * nc);
    L.insmm = o; o = align256(o + 4 * nc);
    L.score = o; o = align256(o + 4 * nc);
    L.nxt = o; o = align256(o + 4 * nc);
    // predecessor rows past the kPreInline a descriptor holds (rows with more predecessors only)
    L.xpre = o; o = align256(o + 4 * nc * dc);
    // -S windows: window descriptors + their extra predecessors, topological row -> window row map,
    // window row -> topological row list, reachability flags, and the node each position of the
    // previous read was assigned to
    const int64_t sn = c.seeded ? nc : 0;
    L.wdesc = o; o = align256(o + 4 * kDescInts * (c.seeded ? nc + kWave : 0));
    L.wxpre = o; o = align256(o + 4 * sn * dc);
    L.wmap = o; o = align256(o + 4 * sn);
    L.wlist = o; o = align256(o + 4 * sn);
    L.wf = o; o = align256(o + 4 * sn);
    L.wb = o; o = align256(o + 4 * sn);
    L.tnode = o; o = align256(o + 4 * (c.seeded ? qc : 0));
    L.total = o;
    return L;
}

// The launch arguments the kernel reads while it runs (its LDS copy, see poa_kernel.hip args_of);
// PoaKArgs adds the workspace layout, which only the kernel's setup reads (from the argument segment).
struct PoaRunArgs {
    const uint8_t *seq;      // encoded bases 0..4
    const int64_t *seq_off;  // per read
    const int64_t *grp_off;  // per group, n_groups+1
    const int32_t *gorder;   // processing order (may be null: identity)
    int32_t n_groups;
    uint8_t *cons;           // encoded consensus output
    const int64_t *cons_off; // per group capacity offsets, n_groups+1
    int32_t *cons_len;
    int64_t *cells;
    int32_t *status;
    int32_t *counter;        // work-queue head (zeroed before launch)
    int64_t *prof;           // optional per-slot phase cycle counters (kProfPhases per slot) or null
    char *ws;
    int64_t slot_bytes;
    PoaCaps caps;
    int32_t match, mismatch, o1, e1, o2, e2, band_b;
    float band_f;
    int32_t qlds;            // dynamic LDS bytes for the read stream (see poa_qlds_bytes)
    // -S (a launch of seeded groups, caps.seeded): per read its seed item (-1: none), per item the
    // kept partition anchors from the seed kernel (k-mer starts in the previous read and in this read)
    const int32_t *par_item;
    const int32_t *par_n, *par_t, *par_q;
    int32_t pc, seed_k;
    int32_t dbg;             // MANDO_POA_DBG: bit 0 no 16-bit mode, bit 1 no 16-bit fast rows, bit 2 no 32-bit fast rows
    // -S teams (seeded launches): a.team consecutive one-wave workgroups share a group, member 0
    // leading; one TeamBox per team (zeroed before the launch; team 1: a leader without helpers)
    int32_t team;
    struct TeamBox *boxes;
    // unseeded launches, one_group: a grid of one workgroup per group (blockIdx -> gorder), each taking
    // a free workspace slot of n_slots (slot_busy, zeroed before the launch) for its group; workgroups
    // of other kernels get CUs as groups finish.  0: persistent slots pulling groups from `counter`.
    int32_t one_group, n_slots;
    int32_t *slot_busy;
};
struct PoaKArgs : PoaRunArgs {
    SlotLayout lay;
    int32_t nw = 1;  // waves per workgroup: 2 runs a wide launch's two-chunk rows over two waves
};
// waves per workgroup of a launch (two-wave workgroups for wide launches only)
inline int poa_waves(const PoaKArgs &a) { return a.caps.wide && !a.caps.seeded && a.nw == 2 ? 2 : 1; }

// A team's mailbox (see poa_kernel.hip, "-S teams").  claim = job << 40 | np << 20 | next window.
struct alignas(64) TeamBox {
    uint64_t claim;
    uint32_t done;     // windows of the current job completed (relaxed agent-scope adds)
    int32_t status;    // first failing window status of the job (0: none)
    int64_t cells;     // DP cells of the job's windows
    int64_t rd;        // the job's read
    int32_t qlen, item;
};
constexpr int kMaxTeam = 8;

// Columns a row can touch past the read: one 128-column chunk beyond `end` (<= qlen) plus slack.
constexpr int kQPad = 132;

// dynamic LDS the POA kernel needs for reads up to max_len: the read as 4-bit codes shifted by one
// (nibble j = base j-1, nibble 0 and everything past the read = 4), padded by kQPad columns
inline int poa_qlds_bytes(int64_t max_len) {
    const int64_t b = ((((max_len + kQPad + 2) / 2) + 15) & ~int64_t(15)) + 16;
    return (int)(b < 1040 ? 1040 : b);  // >= 1 KB: the backtrack's predecessor-byte window reuses it
}

// Resident workgroups per CU for these arguments (LDS / register limited), at most cap.
int poa_blocks_per_cu(const PoaKArgs &a, int cap);

constexpr int kLeadBytes = 80;  // -S launches: the team leader's state after the read (poa_kernel.hip LeadState)
// dynamic LDS of a launch: the read's nibbles, plus the wide ring in a wide launch, plus the leader's
// state in a -S launch
inline int poa_dyn_lds(const PoaKArgs &a) {
    if (a.caps.seeded) return ((a.qlds + 15) & ~15) + kLeadBytes;
    // a wide launch's backtrack windows use 16 KB of it (poa_kernel.hip bt_tb_win / bt_kp_win)
    return a.caps.wide ? (a.qlds + kWideRingBytes > 16384 ? a.qlds + kWideRingBytes : 16384) : a.qlds;
}

// Launch the persistent POA kernel on `stream` with `n_slots` one-wave workgroups.
hipError_t launch_poa(const PoaKArgs &a, int n_slots, hipStream_t stream);

// In-place ASCII -> base code (A C G T -> 0..3, either case; anything else -> 4) on the device.
hipError_t launch_encode(uint8_t *buf, int64_t n, hipStream_t stream);

// Device self-test of the wave primitives (scan/reduce); returns number of mismatches in *bad.
hipError_t run_wave_selftest(int *d_bad, hipStream_t stream);

}  // namespace mando
