// capi.hip — C-ABI of libmando (declared in include/mando.h): contexts, device buffers, batch
// planning for the POA kernel (capacity estimates, LPT work order, overflow re-runs).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <chrono>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <numeric>
#include <string>
#include <vector>

#include "../../include/mando.h"
#include "internal.h"
#include "orient_kernel.h"
#include "poa_kernel.h"
#include "seed_kernel.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

#define HIP_TRY(expr)                                                                       \
    do {                                                                                    \
        hipError_t _e = (expr);                                                             \
        if (_e != hipSuccess)                                                               \
            return fail(MANDO_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));   \
    } while (0)

struct DevBuf {
    void *p = nullptr;
    size_t bytes = 0;
    int ensure(size_t need) {
        if (need <= bytes && p) return MANDO_OK;
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
        size_t nb = std::max<size_t>(need, 256);
        const auto t0 = std::chrono::steady_clock::now();
        hipError_t e = hipMalloc(&p, nb);
        static const bool log = getenv("MANDO_WS_LOG") != nullptr;
        if (log && nb > ((size_t)1 << 30))
            fprintf(stderr, "[mando ws] hipMalloc %.2f GB: %.3f s\n", nb / 1e9,
                    std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
        if (e != hipSuccess) {
            p = nullptr;
            return fail(MANDO_E_NOMEM, std::string("hipMalloc(") + std::to_string(nb) +
                                           "): " + hipGetErrorString(e));
        }
        bytes = nb;
        return MANDO_OK;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    template <class T>
    T *as() const {
        return reinterpret_cast<T *>(p);
    }
};

// Segment gather for the device-resident inputs (mando_orient_segments / mando_poa_segments): read r is
// text[off[r] .. off[r] + len[r]), reverse-complemented like mappy.revcomp (revcomp.h) when rc[r];
// written ASCII at dst + dst_off[r].  One 256-thread block walks segments (grid-stride).
__device__ __forceinline__ uint8_t comp_base(uint8_t c) {
    switch (c | 0x20) {
        case 'a': return (uint8_t)(c ^ ('A' ^ 'T'));
        case 't': return (uint8_t)(c ^ ('A' ^ 'T'));
        case 'u': return (uint8_t)(c == 'U' ? 'A' : 'a');
        case 'c': return (uint8_t)(c ^ ('C' ^ 'G'));
        case 'g': return (uint8_t)(c ^ ('C' ^ 'G'));
        case 'r': return (uint8_t)(c ^ ('R' ^ 'Y'));
        case 'y': return (uint8_t)(c ^ ('R' ^ 'Y'));
        case 'k': return (uint8_t)(c ^ ('K' ^ 'M'));
        case 'm': return (uint8_t)(c ^ ('K' ^ 'M'));
        case 'b': return (uint8_t)(c ^ ('B' ^ 'V'));
        case 'v': return (uint8_t)(c ^ ('B' ^ 'V'));
        case 'd': return (uint8_t)(c ^ ('D' ^ 'H'));
        case 'h': return (uint8_t)(c ^ ('D' ^ 'H'));
        default: return c;  // S, W, N and anything else
    }
}

// base -> POA code 0..4 (A, C, G, T any case; anything else 4), as mando::encode_kernel
__device__ __forceinline__ uint8_t base_code(uint32_t c) {
    c |= 0x20;
    return c == 'a' ? 0 : c == 'c' ? 1 : c == 'g' ? 2 : c == 't' ? 3 : 4;
}

// segment r of the device text -> dst[dst_off[r] ..], reverse-complemented where rc[r]; encode: as POA
// codes (the complement of code c < 4 is 3 - c, of anything else 4: comp_base maps the IUPAC letters
// among themselves), which spares the POA batch its separate encoding pass over the gathered bytes
__global__ __launch_bounds__(256) void gather_kernel(const uint8_t *__restrict__ text, const int64_t *__restrict__ off,
                                                     const int32_t *__restrict__ len, const int8_t *__restrict__ rc,
                                                     const int64_t *__restrict__ dst_off, int64_t n,
                                                     uint8_t *__restrict__ dst, int encode) {
    for (int64_t r = blockIdx.x; r < n; r += gridDim.x) {
        const uint8_t *src = text + off[r];
        uint8_t *d = dst + dst_off[r];
        const int L = len[r];
        const bool rev = rc && rc[r];
        if (encode) {
            if (rev) {
                for (int k = threadIdx.x; k < L; k += 256) {
                    const uint8_t c = base_code(src[L - 1 - k]);
                    d[k] = c < 4 ? (uint8_t)(3 - c) : (uint8_t)4;
                }
            } else {
                for (int k = threadIdx.x; k < L; k += 256) d[k] = base_code(src[k]);
            }
        } else if (rev) {
            for (int k = threadIdx.x; k < L; k += 256) d[k] = comp_base(src[L - 1 - k]);
        } else {
            for (int k = threadIdx.x; k < L; k += 256) d[k] = src[k];
        }
    }
}

// consensus codes (0-4) of group g at cons[src_off[g] ..] -> ASCII at dst[dst_off[g] ..]
__global__ __launch_bounds__(256) void decode_cons_kernel(const uint8_t *__restrict__ cons,
                                                          const int64_t *__restrict__ src_off,
                                                          const int32_t *__restrict__ len,
                                                          const int64_t *__restrict__ dst_off, int64_t n,
                                                          uint8_t *__restrict__ dst) {
    for (int64_t g = blockIdx.x; g < n; g += gridDim.x) {
        const uint8_t *s = cons + src_off[g];
        uint8_t *d = dst + dst_off[g];
        for (int k = threadIdx.x; k < len[g]; k += 256) {
            const uint8_t c = s[k];
            d[k] = c == 0 ? 'A' : c == 1 ? 'C' : c == 2 ? 'G' : c == 3 ? 'T' : 'N';
        }
    }
}

uint8_t g_enc[256];
struct EncInit {
    EncInit() {
        for (int i = 0; i < 256; ++i) g_enc[i] = 4;
        g_enc['A'] = g_enc['a'] = 0;
        g_enc['C'] = g_enc['c'] = 1;
        g_enc['G'] = g_enc['g'] = 2;
        g_enc['T'] = g_enc['t'] = 3;
    }
} g_enc_init;

}  // namespace

struct mando_ctx {
    int device = 0;
    int n_cu = 256;
    int n_cu_act = 256;  // CUs the ctx's streams may use
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    int last_launches = 0;
    bool timed = false;
    int64_t total_mem = 0;    // device HBM (hipDeviceProp_t::totalGlobalMem)
    int64_t poa_budget = 0;   // mando_ctx_set_poa_budget: explicit cap on the POA workspaces (0: default policy)
    bool staged_encoded = false;       // the last POA stage wrote POA codes (gather_stage), not ASCII
    int64_t last_slots[3] = {0, 0, 0};  // slots of the last batch's launches by kind (narrow, wide, seeded)
    int64_t last_budget[3] = {0, 0, 0}; // the workspace budget each of them was sized with
    DevBuf ws, counter, prof, o_gidx;
    DevBuf seq, seq_off, grp_off, gorder, cons, cons_off, cons_len, cells, status;
    DevBuf o_hits, o_strand, o_status;
    DevBuf s_items, s_item_of, s_n, s_t, s_q, s_scratch, s_redo, gorder2;  // -S partition
    DevBuf gorder_w;                                                       // wide-launch groups
    DevBuf g_off, g_len, g_rc, g_dst;                                      // segment gather
    DevBuf cons_txt;                                                       // decoded consensi
    DevBuf o_scratch;                                                      // orientation slabs (per wave)
    // extra POA lanes: a batch's launches of different kinds (narrow, wide, seeded) run side by side,
    // each with its own stream and workspace
    hipStream_t lane_stream[2] = {nullptr, nullptr};
    hipEvent_t ev_fork = nullptr, ev_lane[2] = {nullptr, nullptr};
    DevBuf lane_ws[2], lane_counter[2], lane_prof[2];
    DevBuf boxes, lane_boxes[2];  // -S team mailboxes
    DevBuf busy, lane_busy[2];    // one-group launches: workspace slot flags
    ~mando_ctx() {
        for (DevBuf *b : {&ws, &counter, &prof, &seq, &seq_off, &grp_off, &gorder, &cons, &cons_off,
                          &cons_len, &cells, &status, &o_hits, &o_strand, &o_status, &o_gidx, &s_items,
                          &s_item_of, &s_n, &s_t, &s_q, &s_scratch, &s_redo, &gorder2, &g_off, &g_len, &g_rc,
                          &g_dst, &cons_txt, &o_scratch, &lane_ws[0], &lane_ws[1], &lane_counter[0],
                          &lane_counter[1], &lane_prof[0], &lane_prof[1], &gorder_w, &boxes, &lane_boxes[0],
                          &lane_boxes[1], &busy, &lane_busy[0], &lane_busy[1]})
            b->release();
        if (ev_fork) (void)hipEventDestroy(ev_fork);
        for (int k = 0; k < 2; ++k) {
            if (ev_lane[k]) (void)hipEventDestroy(ev_lane[k]);
            if (lane_stream[k]) (void)hipStreamDestroy(lane_stream[k]);
        }
        if (ev0) (void)hipEventDestroy(ev0);
        if (ev1) (void)hipEventDestroy(ev1);
        if (stream) (void)hipStreamDestroy(stream);
    }
};

namespace {

// the workspace of a POA launch kind (0 narrow, 1 wide, 2 -S)
DevBuf &kind_ws(mando_ctx *ctx, int kind) { return kind == 0 ? ctx->ws : ctx->lane_ws[kind - 1]; }

constexpr int kMaxWavesPerCu = 16;  // upper bound on resident POA waves per CU
// groups whose band 2w + 1 (at their mean read length) is wider than this run in the wide-ring
// launch: their rows mostly exceed one 128-column chunk (the band also drifts with the argmax).  Below
// it a group runs on one wave (16 per CU) with rows of one chunk; a row that drifts past the chunk
// takes the generic row.  Config 4 per step (profiles/r06k_ab_wide_band.txt): 96: 16.7 s, 104: 14.1,
// 108: 15.0, 112: 12.0-12.4, 114-118: 11.7-11.9, 120: 12.1, 124: 13.9, 140: 19.5 -- the bands 113 and
// 115 (mean reads of 4.6-4.8 kb) still fit a chunk often enough to be cheaper on one wave than on the
// two-wave wide kernel (8 waves per CU)
constexpr int64_t kWideBand = 116;
#ifndef MANDO_WS_SHARE
#define MANDO_WS_SHARE 0.8
#endif
// share of the free HBM the POA workspace may take (one slot per resident wave; deep, long groups
// need ~100 MB per slot, so the share decides how many waves run)
constexpr double kWsShare = MANDO_WS_SHARE;
// ... and at most this share of the device's HBM (the default policy, for callers that set no explicit
// budget).  0.45 was too tight for a config-3 chunk's narrow launch: half the slots it needs for the
// one-group grid (persistent grid, POA kernels +25 %, measured r03 abt3).  A many-chunk run (config 4 on
// one GPU) keeps its in-flight chunks' text and clustering scratch next to the workspaces: the D driver
// passes an explicit budget for it (mando_ctx_set_poa_budget).
constexpr double kWsTotalShare = 0.6;

struct GroupStat {
    int64_t nreads = 0, first_len = 0, sum = 0, maxlen = 0;
};

mando::PoaCaps plan_caps(const mando_poa_params &p, int64_t max_first, int64_t max_sum,
                         int64_t max_len, int64_t max_reads, int attempt) {
    mando::PoaCaps c{};
    const double grow = (double)(1 << attempt);
    int64_t rest = std::max<int64_t>(0, max_sum - max_first);
    int64_t nc = max_first + 2 + (int64_t)(0.06 * grow * (double)rest) + 256;
    nc = std::min<int64_t>(nc, max_sum + 2 + 64);
    nc = std::max<int64_t>(nc, max_first + 2 + 64);
    c.NC = (int32_t)nc;
    c.DCAP = attempt == 0 ? 16 : (attempt == 1 ? 64 : 255);
    c.BIGCAP = (int32_t)std::max<int64_t>(max_reads + 8, 16);
    c.QC = (int32_t)std::max<int64_t>(max_len, 1);
    const int64_t w = p.band_b + (int64_t)(p.band_f * (float)max_len);
    const int64_t rowb = ((2 * w + 1 + 96) + 3) & ~int64_t(3);
    c.TBC = nc * rowb * (int64_t)(attempt + 1);
    // predecessor bytes (multi-predecessor rows: one byte per cell for up to 4 predecessors) and spill
    // planes (3 x 128 ints per row whose successor is >= 8 rows later), per traceback byte: 0.75 byte
    // and 1.5 ints first; a group that needs more reports a capacity status and re-runs alone with
    // 1.5 / 1.5, then 3 / 3.  Measured on config 3 (profiles/r04_caps_sweep.txt): no group needs more than
    // 0.75 predecessor bytes, but 9 need more than 0.75 spill ints (73 more than 0.5): any re-run is a
    // second launch that pays its heaviest group's one-wave latency again (POA 1.26 -> 1.58 s), so the
    // spill planes keep their room.
    constexpr double kp0 = 0.75, sv0 = 1.5;
    c.KPC = attempt == 0 ? (int64_t)(kp0 * (double)c.TBC) : (attempt == 1 ? 3 * c.TBC / 2 : 3 * c.TBC);
    c.SVC = attempt == 0 ? (int64_t)(sv0 * (double)c.TBC) : (attempt == 1 ? 3 * c.TBC / 2 : 3 * c.TBC);
    // the kernel keeps its per-read usage counters in 32 bits
    const int64_t lim = int64_t(1) << 30;
    c.TBC = std::min(c.TBC, lim);
    c.KPC = std::min(c.KPC, lim);
    c.SVC = std::min(c.SVC, lim / 4);
    return c;
}

// device-side -S partition of a batch (mando_poa_batch; see seed_kernel.hip)
struct SeedPlan {
    const int32_t *par_item = nullptr, *par_n = nullptr, *par_t = nullptr, *par_q = nullptr;
    int32_t pc = 0, k = 0;
};

// waves per workgroup of wide launches: 2 (two-chunk rows split over two waves, poa_kernel.hip
// row16w_half); MANDO_POA_W2=0 keeps one wave per group.  Measured (r04): config 5 -6.5 %, lone 8.5 kb
// groups -7.5 % (of which -4 % is the 256-VGPR budget of the two-wave instantiation), configs 3 and 4 unchanged
int poa_wide_waves() {
    const char *ev = getenv("MANDO_POA_W2");
    return ev && ev[0] == '0' ? 1 : 2;
}

// The workspace bytes a launch kind wants: one slot per resident workgroup (a team of them per -S
// group when the groups are few), at most one per group -- what its one-group grid needs.
size_t kind_want(mando_ctx *ctx, const mando_poa_params &p, const mando::PoaCaps &caps, int64_t n_groups, bool seeded,
                 int max_per_cu) {
    mando::PoaKArgs a{};
    a.caps = caps;
    a.qlds = mando::poa_qlds_bytes(caps.QC);
    a.nw = caps.wide && !seeded ? poa_wide_waves() : 1;
    a.match = p.match;
    a.mismatch = p.mismatch;
    a.o1 = p.gap_open1;
    a.e1 = p.gap_ext1;
    a.o2 = p.gap_open2;
    a.e2 = p.gap_ext2;
    int cap = max_per_cu;
    if (const char *ev = getenv("MANDO_WAVES_PER_CU")) cap = std::max(1, atoi(ev));
    const int per_cu = mando::poa_blocks_per_cu(a, cap);
    const int64_t resident = (int64_t)ctx->n_cu_act * per_cu;
    int64_t team = 1;
    if (seeded) team = std::max<int64_t>(1, std::min<int64_t>(mando::kMaxTeam, resident / std::max<int64_t>(1, n_groups)));
    const int64_t teams = std::min<int64_t>(n_groups, std::max<int64_t>(1, resident / team));
    // 1/8 of headroom: the next batch's slots are a little larger or smaller, and reallocating a ~150 GB
    // workspace costs 3-4 s of hipMalloc (r04i)
    const size_t b = (size_t)(teams * team) * (size_t)mando::make_layout(caps).total;
    return b + b / 8;
}

// One POA launch over n_groups groups (d_gorder: their indices).  sp != null: the groups are -S
// groups (the seeded kernel instantiation).  ev_start / ev_end: record the ctx's timing events around
// this launch (a batch of several launches times from the first start to the last end).
int launch_batch(mando_ctx *ctx, const mando_poa_params &p, const mando::PoaCaps &caps,
                 const uint8_t *d_seq, const int64_t *d_seq_off, const int64_t *d_grp_off,
                 const int32_t *d_gorder, int64_t n_groups, uint8_t *d_cons,
                 const int64_t *d_cons_off, int32_t *d_cons_len, int64_t *d_cells,
                 int32_t *d_status, int max_per_cu, const SeedPlan *sp = nullptr, bool ev_start = true,
                 bool ev_end = true, int lane = 0, int kind = 0, size_t granted = 0) {
    // lane k > 0: the context's extra stream k - 1 (launches of other kinds alongside); the workspace
    // belongs to the launch kind (kind_ws), so a kind keeps its workspace from batch to batch
    hipStream_t stream = lane ? ctx->lane_stream[lane - 1] : ctx->stream;
    DevBuf &ws = kind_ws(ctx, kind);
    DevBuf &counter = lane ? ctx->lane_counter[lane - 1] : ctx->counter;
    DevBuf &profb = lane ? ctx->lane_prof[lane - 1] : ctx->prof;
    DevBuf &boxb = lane ? ctx->lane_boxes[lane - 1] : ctx->boxes;
    DevBuf &busyb = lane ? ctx->lane_busy[lane - 1] : ctx->busy;
    mando::PoaKArgs a{};
    if (sp) {
        a.par_item = sp->par_item;
        a.par_n = sp->par_n;
        a.par_t = sp->par_t;
        a.par_q = sp->par_q;
        a.pc = sp->pc;
        a.seed_k = sp->k;
    }
    a.seq = d_seq;
    a.seq_off = d_seq_off;
    a.grp_off = d_grp_off;
    a.gorder = d_gorder;
    a.n_groups = (int32_t)n_groups;
    a.cons = d_cons;
    a.cons_off = d_cons_off;
    a.cons_len = d_cons_len;
    a.cells = d_cells;
    a.status = d_status;
    a.caps = caps;
    a.lay = mando::make_layout(caps);
    a.slot_bytes = a.lay.total;
    a.match = p.match;
    a.mismatch = p.mismatch;
    a.o1 = p.gap_open1;
    a.e1 = p.gap_ext1;
    a.o2 = p.gap_open2;
    a.e2 = p.gap_ext2;
    a.band_b = p.band_b;
    a.band_f = p.band_f;
    a.qlds = mando::poa_qlds_bytes(caps.QC);
    a.dbg = 0;
    if (const char *ev = getenv("MANDO_POA_DBG")) a.dbg = atoi(ev);
    // wide launches: two-wave workgroups (the two-chunk rows split over both waves, poa_kernel.hip
    // row16w_half); MANDO_POA_W2=0 keeps one wave per group.  Measured (r04): config 5 -6.5 %, lone 8.5 kb
// groups -7.5 % (of which -4 % is the 256-VGPR budget of the two-wave instantiation), configs 3 and 4 unchanged
    a.nw = caps.wide && !sp ? poa_wide_waves() : 1;
    // slots: enough one-wave workgroups to fill every CU several times, bounded by HBM budget.  With an
    // explicit budget (mando_ctx_set_poa_budget: the D driver's per-call plan, which knows the chunks in
    // flight) the launch takes what the other lanes' workspaces leave of it -- no free-memory query, which
    // would race with the clustering thread's allocations; otherwise a share of the free HBM.
    size_t free_b = 0, total_b = (size_t)ctx->total_mem;
    size_t budget;
    if (granted > 0) {
        budget = granted;  // this kind's share of the explicit budget (poa_batch_impl grant_budgets)
    } else {
        HIP_TRY(hipMemGetInfo(&free_b, &total_b));
        budget = std::max<size_t>((size_t)1 << 30, std::min<size_t>((size_t)(kWsShare * (double)free_b) + ws.bytes,
                                                                    (size_t)(kWsTotalShare * (double)total_b)));
    }
    // resident one-wave workgroups per CU at this batch's LDS footprint (occupancy API)
    int cap = max_per_cu;
    if (const char *ev = getenv("MANDO_WAVES_PER_CU")) cap = std::max(1, atoi(ev));
    const int per_cu = mando::poa_blocks_per_cu(a, cap);
    // -S teams: when the seeded groups are too few to fill the resident waves, each gets a team of
    // up to kMaxTeam one-wave workgroups that align a read's windows side by side
    int team = 1;
    if (sp) {
        const int64_t resident = (int64_t)ctx->n_cu_act * per_cu;
        team = (int)std::max<int64_t>(1, std::min<int64_t>(mando::kMaxTeam, resident / std::max<int64_t>(1, n_groups)));
        if (const char *ev = getenv("MANDO_TEAM")) team = std::max(1, std::min(mando::kMaxTeam, atoi(ev)));
    }
    int64_t teams = std::min<int64_t>(n_groups, std::max<int64_t>(1, (int64_t)ctx->n_cu_act * per_cu / team));
    if (granted > 0) {
        teams = std::max<int64_t>(1, std::min<int64_t>(teams, (int64_t)(budget / ((size_t)team * a.slot_bytes))));
        // a workspace that must grow gets 1/8 of headroom within the grant, so the next chunk's slightly
        // larger slots do not reallocate it
        const size_t need = (size_t)(teams * team * a.slot_bytes);
        if (ws.bytes < need && ws.bytes >= need - need / 4) {
            // a workspace a little too small for this batch's (larger) slots: fewer slots rather than a
            // reallocation (a hipMalloc of ~150 GB costs 3-4 s; a few per cent fewer slots at most turn a
            // one-group grid into the persistent one, +25 % of the kernel)
            teams = std::max<int64_t>(1, (int64_t)(ws.bytes / ((size_t)team * a.slot_bytes)));
        } else if (ws.bytes < need) {
            ws.release();
            const int rc0 = ws.ensure(std::min(budget, need + need / 8));
            if (rc0 == MANDO_E_NOMEM) {
                // HBM held outside this grant (another context or process on the device): the halving
                // retry below finds the slots that fit, as the free-memory path does
                (void)hipGetLastError();
            } else if (rc0) {
                return rc0;
            }
        }
    } else {
        while (teams > 1 && (size_t)(teams * team * a.slot_bytes) > budget) teams /= 2;
    }
    if (getenv("MANDO_PROF") || getenv("MANDO_WS_LOG"))
        fprintf(stderr, "[mando prof] slot workspace %.1f MB, %lld slots, team %d, %d waves per CU (longest read %d, %d B of LDS) (free %.1f GB, budget %.1f GB)\n",
                a.slot_bytes / 1e6, (long long)(teams * team), team, per_cu, (int)a.caps.QC, mando::poa_dyn_lds(a),
                free_b / 1e9, budget / 1e9);
    if (teams < 1) teams = 1;
    int rc = ws.ensure((size_t)(teams * team * a.slot_bytes));
    while (rc == MANDO_E_NOMEM && teams > 1) {  // memory taken by others since hipMemGetInfo: fewer slots
        (void)hipGetLastError();                 // clear the failed allocation's error state
        teams /= 2;
        rc = ws.ensure((size_t)(teams * team * a.slot_bytes));
    }
    if (rc) return rc;
    const int64_t slots = teams * team;
    ctx->last_slots[kind] = slots;
    ctx->last_budget[kind] = (int64_t)budget;
    a.team = team;
    a.boxes = nullptr;
    if (sp) {  // seeded launches run as teams (of one, when the groups fill the chip)
        if ((rc = boxb.ensure((size_t)teams * sizeof(mando::TeamBox)))) return rc;
        HIP_TRY(hipMemsetAsync(boxb.p, 0, (size_t)teams * sizeof(mando::TeamBox), stream));
        a.boxes = boxb.as<mando::TeamBox>();
    }
    // unseeded launches run one workgroup per group when the slots cover the resident waves (else the
    // persistent grid over the slots): as groups finish, the CUs are shared with the other kernels in
    // flight (clustering and orientation of later chunks, other POA launches) instead of being held to
    // the launch's end
    int64_t grid = slots;
    a.one_group = 0;
    if (!sp) {
        // every resident workgroup must find a slot (a waiting one would hold its CU): one-group grids
        // only when the workspace covers the resident waves, or the groups
        const bool enough = slots >= std::min<int64_t>(n_groups, (int64_t)ctx->n_cu_act * per_cu);
        if (enough) {
            a.one_group = 1;
            a.n_slots = (int32_t)slots;
            grid = n_groups;
            if ((rc = busyb.ensure((size_t)slots * 4))) return rc;
            HIP_TRY(hipMemsetAsync(busyb.p, 0, (size_t)slots * 4, stream));
            a.slot_busy = busyb.as<int32_t>();
        }
    }
    rc = counter.ensure(256);
    if (rc) return rc;
    a.ws = ws.as<char>();
    a.counter = counter.as<int32_t>();
    HIP_TRY(hipMemsetAsync(a.counter, 0, sizeof(int32_t), stream));
    const char *pe = getenv("MANDO_PROF");
    const bool prof = pe && pe[0] == '1';
    if (prof) {
        rc = profb.ensure((size_t)grid * mando::kProfPhases * 8);
        if (rc) return rc;
        HIP_TRY(hipMemsetAsync(profb.p, 0, (size_t)grid * mando::kProfPhases * 8, stream));
        a.prof = profb.as<int64_t>();
    }
    if (ev_start) HIP_TRY(hipEventRecord(ctx->ev0, stream));
    HIP_TRY(mando::launch_poa(a, (int)grid, stream));
    if (ev_end) HIP_TRY(hipEventRecord(ctx->ev1, stream));
    ctx->timed = true;
    if (prof) {
        std::vector<int64_t> h((size_t)grid * mando::kProfPhases);
        HIP_TRY(hipMemcpyAsync(h.data(), profb.p, h.size() * 8, hipMemcpyDeviceToHost, stream));
        HIP_TRY(hipStreamSynchronize(stream));
        double tot[mando::kProfPhases] = {0};
        for (int64_t s = 0; s < grid; ++s)
            for (int k = 0; k < mando::kProfPhases; ++k) tot[k] += (double)h[(size_t)(s * mando::kProfPhases + k)];
        const double reads = std::max(1.0, tot[6]), rows = std::max(1.0, tot[5]);
        fprintf(stderr, "[mando prof] fast rows %.1f%%, reads re-aligned in 32-bit mode %.0f\n", 100.0 * tot[7] / rows,
                tot[15]);
        fprintf(stderr, "[mando prof] slots=%lld reads=%.0f rows/read=%.0f | cycles per read: desc %.0f dp %.0f (%.1f/row) backtrack %.0f update %.0f | consensus/slot %.0f\n",
                (long long)slots, reads, rows / reads, tot[0] / reads, tot[1] / reads, tot[1] / rows,
                tot[2] / reads, tot[3] / reads, tot[4] / (double)slots);
        fprintf(stderr, "[mando prof] total Gcycles: desc %.3f dp %.3f backtrack %.3f update %.3f consensus %.3f\n",
                tot[0] * 1e-9, tot[1] * 1e-9, tot[2] * 1e-9, tot[3] * 1e-9, tot[4] * 1e-9);
        if (a.dbg & 16) {
            for (int64_t s = 0; s < slots; ++s) {
                const int64_t *f = &h[(size_t)(s * mando::kProfPhases)];
                if (f[8] == 0) continue;
                fprintf(stderr, "[mando dbg] slot %lld row %lld lane %lld beg %lld end %lld am %lld | tb fast %04llx gen %04llx | H %08llx %08llx | E1 %08llx %08llx | E2 %08llx %08llx | am2 %lld qlen %lld n %lld\n",
                        (long long)s, (long long)f[8] - 1, (long long)(f[9] & 0xff), (long long)((f[9] >> 8) & 0xffff),
                        (long long)((f[9] >> 24) & 0xffff), (long long)(f[9] >> 40), (long long)(f[10] >> 16),
                        (long long)(f[10] & 0xffff), (long long)((uint64_t)f[11] >> 32), (long long)(f[11] & 0xffffffff),
                        (long long)((uint64_t)f[12] >> 32), (long long)(f[12] & 0xffffffff), (long long)((uint64_t)f[13] >> 32),
                        (long long)(f[13] & 0xffffffff), (long long)f[14], (long long)(f[15] & 0xfffff), (long long)(f[15] >> 20));
            }
        }
        if (tot[12] > 0)
            fprintf(stderr, "[mando prof] backtrack per read: refills %.1f (%.0f cyc each) diagonal runs %.1f serial blocks %.1f "
                            "walk %.0f cyc per run or block\n",
                    tot[13] / reads, tot[12] / std::max(1.0, tot[13]), tot[16] / reads, tot[14] / reads,
                    (tot[2] - tot[12]) / std::max(1.0, tot[14] + tot[16]));
        if (getenv("MANDO_BT_STATS"))
            fprintf(stderr, "[mando prof] run stops per read: window %.1f multi %.1f non-adjacent %.1f not-M %.1f\n",
                    tot[8] / reads, tot[9] / reads, tot[10] / reads, tot[11] / reads);
        if (tot[8] + tot[9] + tot[10] + tot[11] > 0)
            fprintf(stderr, "[mando prof] per DP row: seg0 %.3f  seg1 %.4f  seg2 %.4f  seg3 %.4f\n",
                    tot[8] / rows, tot[9] / rows, tot[10] / rows, tot[11] / rows);
    }
    return MANDO_OK;
}

// -S partitions of every seeded group (seed_kernel.hip): items pair each non-empty read after a group's
// first with the previous non-empty read; the reads are already encoded on the device (ctx->seq).
// Items over the launch's LDS capacity are re-run at twice the capacity.
template <class IsSeeded>
int plan_seeds(mando_ctx *ctx, const mando_poa_params &p, const std::vector<int64_t> &soff, const int64_t *grp_off,
               int64_t n_groups, IsSeeded seeded_group, SeedPlan &sp) {
    if (p.k < 1 || p.k > 19 || p.w < 1 || p.min_w < p.k)
        return fail(MANDO_E_UNSUPPORTED, "-S needs 1 <= k <= 19, w >= 1, min_w >= k on this build");
    const int64_t n_reads = (int64_t)soff.size() - 1;
    std::vector<int32_t> items, item_of((size_t)std::max<int64_t>(n_reads, 1), -1);
    int64_t max_len = 1, pc = 1;
    for (int64_t g = 0; g < n_groups; ++g) {
        if (!seeded_group(g)) continue;
        int64_t prev = -1;
        for (int64_t r = grp_off[g]; r < grp_off[g + 1]; ++r) {
            const int64_t L = soff[(size_t)r + 1] - soff[(size_t)r];
            if (L <= 0) continue;
            max_len = std::max(max_len, L);
            if (prev >= 0) {
                item_of[(size_t)r] = (int32_t)(items.size() / 2);
                items.push_back((int32_t)prev);
                items.push_back((int32_t)r);
                pc = std::max<int64_t>(pc, L / p.min_w + 2);
            }
            prev = r;
        }
    }
    if (max_len >= (1 << 25)) return fail(MANDO_E_UNSUPPORTED, "-S: read longer than 2^25 bases");
    const int64_t n_items = (int64_t)items.size() / 2;
    int rc;
    if ((rc = ctx->s_items.ensure(std::max<size_t>(items.size(), 1) * 4)) ||
        (rc = ctx->s_item_of.ensure(item_of.size() * 4)) ||
        (rc = ctx->s_n.ensure((size_t)std::max<int64_t>(n_items, 1) * 4)) ||
        (rc = ctx->s_t.ensure((size_t)std::max<int64_t>(n_items, 1) * (size_t)pc * 4)) ||
        (rc = ctx->s_q.ensure((size_t)std::max<int64_t>(n_items, 1) * (size_t)pc * 4)) ||
        (rc = ctx->counter.ensure(256)))
        return rc;
    if (!items.empty())
        HIP_TRY(hipMemcpyAsync(ctx->s_items.p, items.data(), items.size() * 4, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(hipMemcpyAsync(ctx->s_item_of.p, item_of.data(), item_of.size() * 4, hipMemcpyHostToDevice, ctx->stream));
    sp.par_item = ctx->s_item_of.as<int32_t>();
    sp.par_n = ctx->s_n.as<int32_t>();
    sp.par_t = ctx->s_t.as<int32_t>();
    sp.par_q = ctx->s_q.as<int32_t>();
    sp.pc = (int32_t)pc;
    sp.k = p.k;
    if (n_items == 0) {
        HIP_TRY(hipStreamSynchronize(ctx->stream));
        return MANDO_OK;
    }
    // minimizer capacity: ~2 per w+1 positions, with room for ties
    int cap = 1024;
    while (cap < mando::kSeedCapMax && cap < 3 * max_len / (p.w + 1)) cap *= 2;
    mando::SeedArgs a{};
    a.seq = ctx->seq.as<uint8_t>();
    a.seq_off = ctx->seq_off.as<int64_t>();
    a.items = ctx->s_items.as<int32_t>();
    a.k = p.k;
    a.w = p.w;
    a.min_w = p.min_w;
    a.max_occ = mando::kSeedMaxOcc;
    a.pc = (int32_t)pc;
    a.par_n = ctx->s_n.as<int32_t>();
    a.par_t = ctx->s_t.as<int32_t>();
    a.par_q = ctx->s_q.as<int32_t>();
    a.max_len = (int32_t)max_len;
    a.counter = ctx->counter.as<int32_t>();
    std::vector<int32_t> redo, nres((size_t)n_items);
    for (;;) {
        a.cap = cap;
        a.redo = redo.empty() ? nullptr : ctx->s_redo.as<int32_t>();
        a.n_items = (int32_t)(redo.empty() ? n_items : (int64_t)redo.size());
        const int blocks = (int)std::min<int64_t>(a.n_items, (int64_t)ctx->n_cu * 4);
        a.scratch_words = mando::seed_scratch_words((int)max_len, cap);
        if ((rc = ctx->s_scratch.ensure((size_t)blocks * (size_t)a.scratch_words * 8))) return rc;
        a.scratch = ctx->s_scratch.as<uint64_t>();
        HIP_TRY(hipMemsetAsync(a.counter, 0, 4, ctx->stream));
        HIP_TRY(mando::launch_seed(a, blocks, ctx->stream));
        HIP_TRY(hipMemcpyAsync(nres.data(), ctx->s_n.p, nres.size() * 4, hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(hipStreamSynchronize(ctx->stream));
        std::vector<int32_t> again;
        for (int64_t i = 0; i < n_items; ++i) {
            if (nres[(size_t)i] == -2) return fail(MANDO_E_INTERNAL, "-S: more kept anchors than the read allows");
            if (nres[(size_t)i] == -1) again.push_back((int32_t)i);
        }
        if (again.empty()) break;
        if (cap >= mando::kSeedCapMax)
            return fail(MANDO_E_UNSUPPORTED, "-S: a read has more than " + std::to_string(mando::kSeedCapMax) +
                                                 " minimizers or anchors");
        cap *= 2;
        redo.swap(again);
        if ((rc = ctx->s_redo.ensure(redo.size() * 4))) return rc;
        HIP_TRY(hipMemcpyAsync(ctx->s_redo.p, redo.data(), redo.size() * 4, hipMemcpyHostToDevice, ctx->stream));
    }
    return MANDO_OK;
}

}  // namespace

namespace mando {
int set_error(int code, const std::string &msg) { return fail(code, msg); }
int ctx_device(const mando_ctx *ctx) { return ctx->device; }
hipStream_t ctx_stream(const mando_ctx *ctx) { return ctx->stream; }

// Every stream of the library gets a hardware queue of its own.  HIP maps plain streams onto at most
// GPU_MAX_HW_QUEUES (4) hardware queues per process and, past that, puts a new stream on an existing
// queue, where its work waits behind everything queued before it whatever the streams' dependencies:
// one D call creates six (POA context, POA lanes x2, orientation context, clustering context and copy
// stream; a multi-rank run adds the communicator's), and the config-4 trace showed the orientation
// context sharing the narrow POA lane's queue -- each chunk's orientation started only when the previous
// chunk's narrow POA grid ended, 64 ms on the path between POA launches (profiles/r08a_trace_*,
// r08h_queue_probe_*).  A stream created with a CU mask always gets a new queue; the mask here enables
// every CU, so it changes nothing else.  MANDO_SHARED_QUEUES=1 goes back to plain streams (A/B).
hipError_t create_stream(hipStream_t *out) {
    static const bool shared = [] {
        const char *e = std::getenv("MANDO_SHARED_QUEUES");
        return e && std::atoi(e) != 0;
    }();
    if (shared) return hipStreamCreateWithFlags(out, hipStreamNonBlocking);
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    int n_cu = 0;
    e = hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return e;
    std::vector<uint32_t> mask((size_t)(n_cu + 31) / 32, 0xffffffffu);
    if (n_cu % 32) mask.back() = (1u << (n_cu % 32)) - 1u;
    return hipExtStreamCreateWithCUMask(out, (uint32_t)mask.size(), mask.data());
}
}  // namespace mando

extern "C" {

const char *mando_last_error(void) { return g_err.c_str(); }

int mando_abi_version(void) { return MANDO_ABI_VERSION; }

void mando_poa_default_params(mando_poa_params *p) {
    if (!p) return;
    p->match = 5;
    p->mismatch = 4;
    p->gap_open1 = 4;
    p->gap_ext1 = 2;
    p->gap_open2 = 24;
    p->gap_ext2 = 1;
    p->band_b = 10;
    p->band_f = 0.01f;
    p->seeding = 0;
    p->k = 19;
    p->w = 10;
    p->min_w = 500;
}

int mando_device_count(int *out) {
    if (!out) return fail(MANDO_E_ARG, "null out");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *out = n;
    return MANDO_OK;
}

int mando_ctx_create(int device_ordinal, mando_ctx **out) {
    if (!out) return fail(MANDO_E_ARG, "null out");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
        return fail(MANDO_E_NODEV, "no HIP device visible (libmando requires an MI355X / gfx950)");
    if (device_ordinal < 0 || device_ordinal >= n)
        return fail(MANDO_E_ARG, "device ordinal out of range");
    HIP_TRY(hipSetDevice(device_ordinal));
    // host threads waiting on the device sleep on the completion signal instead of spinning: one GPU's
    // waits took ~20 s of CPU per config-4 step (1.6 cores) for no gain in time
    // (profiles/r05q_ab_blocking_sync.txt), cores the other ranks of a node need (2 per rank at N = 8).
    // hipEventBlockingSync events on the library's own waits instead of this device flag were measured
    // in round 6: 56 s of host CPU per config-4 step and 12.29 s per step (profiles/r08a_*), i.e. the
    // waits still spin.  The flag is the device's (process-wide): include/mando.h says so, and
    // mando_ctx_blocking_sync() reports whether it took effect (refused when the application initialised
    // the device first with other flags).
    (void)hipSetDeviceFlags(hipDeviceScheduleBlockingSync);
    (void)hipGetLastError();
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device_ordinal));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(MANDO_E_NODEV, std::string("device is ") + prop.gcnArchName + ", libmando is built for gfx950");
    mando_ctx *c = new mando_ctx();
    c->device = device_ordinal;
    c->n_cu = prop.multiProcessorCount;
    c->n_cu_act = c->n_cu;
    c->total_mem = (int64_t)prop.totalGlobalMem;
    if (mando::create_stream(&c->stream) != hipSuccess ||
        hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess) {
        delete c;
        return fail(MANDO_E_HIP, "stream/event creation failed");
    }
    *out = c;
    return MANDO_OK;
}

void mando_ctx_destroy(mando_ctx *ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    delete ctx;
}

int mando_ctx_blocking_sync(mando_ctx *ctx) {
    if (!ctx) return fail(MANDO_E_ARG, "null ctx");
    HIP_TRY(hipSetDevice(ctx->device));
    unsigned int f = 0;
    HIP_TRY(hipGetDeviceFlags(&f));
    return (f & hipDeviceScheduleMask) == hipDeviceScheduleBlockingSync ? 1 : 0;
}

int mando_ctx_sync(mando_ctx *ctx) {
    if (!ctx) return fail(MANDO_E_ARG, "null ctx");
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return MANDO_OK;
}

float mando_last_kernel_ms(mando_ctx *ctx) {
    if (!ctx || !ctx->timed) return -1.0f;
    float ms = -1.0f;
    if (hipEventSynchronize(ctx->ev1) != hipSuccess) return -1.0f;
    if (hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1) != hipSuccess) return -1.0f;
    return ms;
}

int mando_last_kernel_launches(mando_ctx *ctx) { return ctx ? ctx->last_launches : 0; }

int mando_ctx_set_poa_budget(mando_ctx *ctx, int64_t bytes) {
    if (!ctx || bytes < 0) return fail(MANDO_E_ARG, "mando_ctx_set_poa_budget: bad argument");
    ctx->poa_budget = bytes;
    return MANDO_OK;
}

int mando_ctx_memory(mando_ctx *ctx, int64_t *total_bytes, int64_t *poa_ws_bytes) {
    if (!ctx) return fail(MANDO_E_ARG, "null ctx");
    if (total_bytes) *total_bytes = ctx->total_mem;
    if (poa_ws_bytes) *poa_ws_bytes = (int64_t)(ctx->ws.bytes + ctx->lane_ws[0].bytes + ctx->lane_ws[1].bytes);
    return MANDO_OK;
}

int mando_device_memory(int device_ordinal, int64_t *free_bytes, int64_t *total_bytes) {
    int n = 0;
    HIP_TRY(hipGetDeviceCount(&n));
    if (device_ordinal < 0 || device_ordinal >= n) return fail(MANDO_E_ARG, "mando_device_memory: bad device");
    HIP_TRY(hipSetDevice(device_ordinal));
    size_t f = 0, t = 0;
    HIP_TRY(hipMemGetInfo(&f, &t));
    if (free_bytes) *free_bytes = (int64_t)f;
    if (total_bytes) *total_bytes = (int64_t)t;
    return MANDO_OK;
}

int mando_poa_last_slots(mando_ctx *ctx, int64_t *slots, int64_t *budgets) {
    if (!ctx) return fail(MANDO_E_ARG, "null ctx");
    for (int k = 0; k < 3; ++k) {
        if (slots) slots[k] = ctx->last_slots[k];
        if (budgets) budgets[k] = ctx->last_budget[k];
    }
    return MANDO_OK;
}

int mando_poa_batch_device(mando_ctx *ctx, const mando_poa_params *params, const uint8_t *d_seqs,
                           const int64_t *d_seq_off, const int64_t *d_grp_off, int64_t n_groups,
                           int64_t max_read_len, int64_t max_group_bases, uint8_t *d_cons,
                           const int64_t *d_cons_off, int32_t *d_cons_len, int64_t *d_cells,
                           int32_t *d_status) {
    if (!ctx || !params || !d_seqs || !d_seq_off || !d_grp_off || !d_cons || !d_cons_off ||
        !d_cons_len || !d_cells || !d_status || n_groups < 0 || max_read_len < 0)
        return fail(MANDO_E_ARG, "mando_poa_batch_device: bad argument");
    if (n_groups == 0) return MANDO_OK;
    HIP_TRY(hipSetDevice(ctx->device));
    mando::PoaCaps caps = plan_caps(*params, max_read_len, max_group_bases, max_read_len,
                                    std::max<int64_t>(1, max_group_bases / std::max<int64_t>(1, max_read_len / 4)), 0);
    const int64_t w = params->band_b + (int64_t)(params->band_f * (float)max_read_len);
    caps.wide = 2 * w + 1 > kWideBand;
    ctx->last_launches = 1;
    return launch_batch(ctx, *params, caps, d_seqs, d_seq_off, d_grp_off, nullptr, n_groups,
                        d_cons, d_cons_off, d_cons_len, d_cells, d_status, kMaxWavesPerCu);
}

}  // extern "C"

namespace {

// Stages the reads of a batch as ASCII into ctx->seq (soff: their offsets there); returns a status.
using StageFn = std::function<int(mando_ctx *)>;

// The POA batch once its reads' layout (soff) is known: stage + encode, plan, launch, collect.
int poa_batch_impl(mando_ctx *ctx, const mando_poa_params *params, const std::vector<int64_t> &soff,
                   const int64_t *grp_off, int64_t n_groups, const uint8_t *seeding_per_group, uint8_t *cons_out,
                   int64_t cons_cap, int64_t *cons_off, int64_t *cells_out, const StageFn &stage) {
    // -S for a group: seeding_per_group[g], or params->seeding for every group
    auto seeded_group = [&](int64_t g) {
        return seeding_per_group ? seeding_per_group[g] != 0 : params->seeding != 0;
    };
    const int64_t n_reads = grp_off[n_groups];
    const int64_t total = soff[(size_t)n_reads];
    HIP_TRY(hipSetDevice(ctx->device));

    // per-group statistics (the bases are staged as ASCII and encoded on the device)
    std::vector<GroupStat> gs((size_t)n_groups);
    int64_t max_first = 0, max_sum = 0, max_len = 0, max_nreads = 0;
    std::vector<int64_t> ccap((size_t)n_groups + 1, 0);
    for (int64_t g = 0; g < n_groups; ++g) {
        GroupStat &s = gs[(size_t)g];
        s.nreads = grp_off[g + 1] - grp_off[g];
        for (int64_t r = grp_off[g]; r < grp_off[g + 1]; ++r) {
            const int64_t L = soff[(size_t)r + 1] - soff[(size_t)r];
            if (L > 0 && s.first_len == 0) s.first_len = L;
            s.sum += L;
            s.maxlen = std::max(s.maxlen, L);
        }
        max_first = std::max(max_first, s.first_len);
        max_sum = std::max(max_sum, s.sum);
        max_len = std::max(max_len, s.maxlen);
        max_nreads = std::max(max_nreads, s.nreads);
        ccap[(size_t)g + 1] = ccap[(size_t)g] + 2 * s.maxlen + 256;
    }
    // LPT order: most DP work first
    std::vector<int32_t> order((size_t)n_groups);
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(), [&](int32_t x, int32_t y) {
        const GroupStat &a = gs[(size_t)x], &b = gs[(size_t)y];
        return (double)(a.sum - a.first_len) * (double)a.first_len >
               (double)(b.sum - b.first_len) * (double)b.first_len;
    });

    int rc;
    if ((rc = ctx->seq.ensure((size_t)std::max<int64_t>(total, 1))) || (rc = ctx->seq_off.ensure(soff.size() * 8)) ||
        (rc = ctx->grp_off.ensure(((size_t)n_groups + 1) * 8)) ||
        (rc = ctx->gorder.ensure((size_t)n_groups * 4)) ||
        (rc = ctx->cons_off.ensure(((size_t)n_groups + 1) * 8)) ||
        (rc = ctx->cons.ensure((size_t)ccap[(size_t)n_groups])) ||
        (rc = ctx->cons_len.ensure((size_t)n_groups * 4)) ||
        (rc = ctx->cells.ensure((size_t)n_groups * 8)) ||
        (rc = ctx->status.ensure((size_t)n_groups * 4)))
        return rc;
    if (getenv("MANDO_WS_LOG"))
        fprintf(stderr, "[mando ws] poa: groups %lld bases %.3f GB (seq buffer %.3f GB, consensus %.3f GB)\n",
                (long long)n_groups, total / 1e9, ctx->seq.bytes / 1e9, ctx->cons.bytes / 1e9);
    std::vector<int64_t> goff((size_t)n_groups + 1);
    for (int64_t g = 0; g <= n_groups; ++g) goff[(size_t)g] = grp_off[g];
    if (total > 0) {
        ctx->staged_encoded = false;
        if ((rc = stage(ctx))) return rc;
        if (!ctx->staged_encoded) HIP_TRY(mando::launch_encode(ctx->seq.as<uint8_t>(), total, ctx->stream));
    }
    HIP_TRY(hipMemcpyAsync(ctx->seq_off.p, soff.data(), soff.size() * 8, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(hipMemcpyAsync(ctx->grp_off.p, goff.data(), goff.size() * 8, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(hipMemcpyAsync(ctx->cons_off.p, ccap.data(), ccap.size() * 8, hipMemcpyHostToDevice, ctx->stream));

    // -S groups: their window partitions first (seed kernel over every read of a seeded group paired
    // with the group's previous non-empty read)
    SeedPlan sp;
    bool any_seeded = false;
    for (int64_t g = 0; g < n_groups && !any_seeded; ++g) any_seeded = seeded_group(g);
    if (any_seeded) {
        rc = plan_seeds(ctx, *params, soff, grp_off, n_groups, seeded_group, sp);
        if (rc) return rc;
    }

    std::vector<int32_t> st((size_t)n_groups), clen((size_t)n_groups);
    std::vector<int64_t> cells((size_t)n_groups);
    std::vector<int32_t> todo = order;
    ctx->last_launches = 0;
    for (int k = 0; k < 3; ++k) ctx->last_slots[k] = ctx->last_budget[k] = 0;
    for (int attempt = 0; attempt < 4 && !todo.empty(); ++attempt) {
        // unseeded and seeded groups run as two launches of the two kernel instantiations
        // three kinds of launch: unseeded groups with bands of one chunk, unseeded groups whose band
        // (2w + 1 at their mean read length) exceeds one chunk (the wide-ring instantiation), -S groups
        std::vector<int32_t> lists[3];
        for (int32_t g : todo) {
            const GroupStat &q = gs[(size_t)g];
            const int64_t mean = q.sum / std::max<int64_t>(1, q.nreads);
            const int64_t w = params->band_b + (int64_t)(params->band_f * (float)mean);
            lists[seeded_group(g) ? 2 : (2 * w + 1 > kWideBand ? 1 : 0)].push_back(g);
        }
        // several kinds: each runs on its own lane (stream + workspace), concurrently, after everything
        // staged so far on the first stream
        int nk = 0;
        for (int kind = 0; kind < 3; ++kind) nk += !lists[kind].empty();
        if (nk > 1) {
            if (!ctx->ev_fork) {
                HIP_TRY(hipEventCreateWithFlags(&ctx->ev_fork, hipEventDisableTiming));
                for (int k = 0; k < 2; ++k) {
                    HIP_TRY(mando::create_stream(&ctx->lane_stream[k]));
                    HIP_TRY(hipEventCreateWithFlags(&ctx->ev_lane[k], hipEventDisableTiming));
                }
            }
            HIP_TRY(hipEventRecord(ctx->ev_fork, ctx->stream));
            for (int k = 0; k < nk - 1; ++k) HIP_TRY(hipStreamWaitEvent(ctx->lane_stream[k], ctx->ev_fork, 0));
        }
        // the kind holding the heaviest group is enqueued first (its slots take the CUs first: a
        // persistent launch holds them until its queue drains)
        int korder[3] = {0, 1, 2};
        double kcost[3] = {0, 0, 0};
        for (int kind = 0; kind < 3; ++kind)
            for (int32_t g : lists[kind]) {
                const GroupStat &q = gs[(size_t)g];
                kcost[kind] = std::max(kcost[kind], (double)(q.sum - q.first_len) * (double)q.first_len);
            }
        std::stable_sort(korder, korder + 3, [&](int x, int y) { return kcost[x] > kcost[y]; });
        mando::PoaCaps kcaps[3];
        for (int kind = 0; kind < 3; ++kind) {
            int64_t mf = 0, ms = 0, ml = 0, mr = 0;
            for (int32_t g : lists[kind]) {
                mf = std::max(mf, gs[(size_t)g].first_len);
                ms = std::max(ms, gs[(size_t)g].sum);
                ml = std::max(ml, gs[(size_t)g].maxlen);
                mr = std::max(mr, gs[(size_t)g].nreads);
            }
            kcaps[kind] = plan_caps(*params, mf, ms, ml, mr, attempt);
            kcaps[kind].seeded = kind == 2;
            kcaps[kind].wide = kind == 1;
        }
        // an explicit budget (mando_ctx_set_poa_budget) is shared by the batch's kinds: each kind wants the
        // workspace of its resident waves (one-group grids need that many slots); every kind first gets
        // up to an eighth of the budget, then the rest goes to the kinds in launch order (heaviest group
        // first) up to what they want.  Workspaces of kinds absent from the batch, and the excess of
        // larger ones, are released before any launch.
        size_t grant[3] = {0, 0, 0};
        if (ctx->poa_budget > 0) {
            const size_t B = (size_t)ctx->poa_budget;
            size_t want[3] = {0, 0, 0}, rem = B;
            for (int kind = 0; kind < 3; ++kind)
                if (!lists[kind].empty())
                    want[kind] = kind_want(ctx, *params, kcaps[kind], (int64_t)lists[kind].size(), kind == 2,
                                           kMaxWavesPerCu);
            for (int kind = 0; kind < 3; ++kind) {
                grant[kind] = std::min(want[kind], B / 8);
                rem -= std::min(rem, grant[kind]);
            }
            for (int ki = 0; ki < 3; ++ki) {
                const int kind = korder[ki];
                const size_t more = std::min(rem, want[kind] - grant[kind]);
                grant[kind] += more;
                rem -= more;
            }
            // a kind keeps a workspace larger than its grant while everything held fits the budget (a
            // hipFree synchronises the device and a fresh hipMalloc of ~100 GB costs seconds): absent
            // kinds' workspaces go first, then the excess of the others
            auto held = [&] {
                size_t t = 0;
                for (int kind = 0; kind < 3; ++kind) t += std::max(kind_ws(ctx, kind).bytes, grant[kind]);
                return t;
            };
            for (int kind = 0; kind < 3 && held() > B; ++kind)
                if (lists[kind].empty()) kind_ws(ctx, kind).release();
            for (int kind = 0; kind < 3 && held() > B; ++kind)
                if (kind_ws(ctx, kind).bytes > grant[kind]) kind_ws(ctx, kind).release();
        }
        int lane = 0;
        for (int ki = 0; ki < 3; ++ki) {
            const int kind = korder[ki];
            const std::vector<int32_t> &L = lists[kind];
            if (L.empty()) continue;
            hipStream_t lst = lane ? ctx->lane_stream[lane - 1] : ctx->stream;
            const mando::PoaCaps &caps = kcaps[kind];
            DevBuf &gb = kind == 0 ? ctx->gorder : (kind == 1 ? ctx->gorder_w : ctx->gorder2);
            if ((rc = gb.ensure(L.size() * 4))) return rc;
            HIP_TRY(hipMemcpyAsync(gb.p, L.data(), L.size() * 4, hipMemcpyHostToDevice, lst));
            rc = launch_batch(ctx, *params, caps, ctx->seq.as<uint8_t>(), ctx->seq_off.as<int64_t>(),
                              ctx->grp_off.as<int64_t>(), gb.as<int32_t>(), (int64_t)L.size(),
                              ctx->cons.as<uint8_t>(), ctx->cons_off.as<int64_t>(),
                              ctx->cons_len.as<int32_t>(), ctx->cells.as<int64_t>(),
                              ctx->status.as<int32_t>(), kMaxWavesPerCu, kind == 2 ? &sp : nullptr,
                              lane == 0 && attempt == 0,  // the batch's time runs from the first attempt
                              nk == 1, lane, kind, grant[kind]);
            if (rc) return rc;
            ctx->last_launches += 1;
            ++lane;
        }
        if (nk > 1) {  // join the extra lanes; the batch's timing ends when every launch has
            for (int k = 0; k < nk - 1; ++k) {
                HIP_TRY(hipEventRecord(ctx->ev_lane[k], ctx->lane_stream[k]));
                HIP_TRY(hipStreamWaitEvent(ctx->stream, ctx->ev_lane[k], 0));
            }
            HIP_TRY(hipEventRecord(ctx->ev1, ctx->stream));
        }
        HIP_TRY(hipMemcpyAsync(st.data(), ctx->status.p, st.size() * 4, hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(hipMemcpyAsync(clen.data(), ctx->cons_len.p, clen.size() * 4, hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(hipMemcpyAsync(cells.data(), ctx->cells.p, cells.size() * 8, hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(hipStreamSynchronize(ctx->stream));
        std::vector<int32_t> again;
        for (int32_t g : todo) {
            if (st[(size_t)g] == mando::kStCap) again.push_back(g);
            else if (st[(size_t)g] != mando::kStOk)
                return fail(MANDO_E_INTERNAL, "POA kernel reported status " + std::to_string(st[(size_t)g]) +
                                                  " for group " + std::to_string(g));
        }
        if (!again.empty() && getenv("MANDO_WS_LOG"))
            fprintf(stderr, "[mando ws] poa: %zu of %zu groups re-run with larger capacities (attempt %d)\n",
                    again.size(), todo.size(), attempt + 1);
        todo.swap(again);
    }
    if (!todo.empty())
        return fail(MANDO_E_INTERNAL, "POA workspace capacity still exceeded after retries");

    // consensi: decoded to ASCII and packed back to back on the device, then one copy of the used bytes
    int64_t used = 0;
    cons_off[0] = 0;
    for (int64_t g = 0; g < n_groups; ++g) {
        used += clen[(size_t)g];
        cons_off[g + 1] = used;
        if (cells_out) cells_out[g] = cells[(size_t)g];
    }
    if (cons_out && used > 0 && used <= cons_cap) {
        if ((rc = ctx->g_dst.ensure(((size_t)n_groups + 1) * 8)) || (rc = ctx->g_len.ensure((size_t)n_groups * 4)) ||
            (rc = ctx->g_off.ensure((size_t)(n_groups + 1) * 8)) || (rc = ctx->cons_txt.ensure((size_t)used + 16)))
            return rc;
        HIP_TRY(hipMemcpyAsync(ctx->g_dst.p, cons_off, ((size_t)n_groups + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
        HIP_TRY(hipMemcpyAsync(ctx->g_len.p, clen.data(), (size_t)n_groups * 4, hipMemcpyHostToDevice, ctx->stream));
        HIP_TRY(hipMemcpyAsync(ctx->g_off.p, ccap.data(), ((size_t)n_groups + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
        const int blocks = (int)std::min<int64_t>(n_groups, (int64_t)ctx->n_cu * 32);
        hipLaunchKernelGGL(decode_cons_kernel, dim3(blocks), dim3(256), 0, ctx->stream, ctx->cons.as<uint8_t>(),
                           ctx->g_off.as<int64_t>(), ctx->g_len.as<int32_t>(), ctx->g_dst.as<int64_t>(), n_groups,
                           ctx->cons_txt.as<uint8_t>());
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpyAsync(cons_out, ctx->cons_txt.p, (size_t)used, hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(hipStreamSynchronize(ctx->stream));
    }
    if (used > cons_cap || (!cons_out && used > 0)) return fail(MANDO_E_CAP, "cons_out too small");
    return MANDO_OK;
}

int check_groups(const int64_t *grp_off, int64_t n_groups) {
    if (grp_off[0] != 0) return fail(MANDO_E_ARG, "grp_off must start at 0");
    for (int64_t g = 0; g < n_groups; ++g)
        if (grp_off[g + 1] < grp_off[g]) return fail(MANDO_E_ARG, "grp_off not monotone");
    return MANDO_OK;
}

// segments of a device-resident text: layout (exclusive prefix of len) and the gather stage
int segment_layout(const int64_t *off, const int32_t *len, int64_t n, int64_t text_len, std::vector<int64_t> &soff) {
    soff.assign((size_t)n + 1, 0);
    for (int64_t r = 0; r < n; ++r) {
        if (len[r] < 0 || off[r] < 0 || off[r] + len[r] > text_len)
            return fail(MANDO_E_ARG, "segment " + std::to_string(r) + " outside the device text");
        soff[(size_t)r + 1] = soff[(size_t)r] + len[r];
    }
    return MANDO_OK;
}

int gather_stage(mando_ctx *ctx, const uint8_t *d_text, const int64_t *off, const int32_t *len, const int8_t *rc,
                 const std::vector<int64_t> &soff, bool encode = false) {
    const int64_t n = (int64_t)soff.size() - 1;
    if (n <= 0) return MANDO_OK;
    int e;
    if ((e = ctx->g_off.ensure((size_t)n * 8)) || (e = ctx->g_len.ensure((size_t)n * 4)) ||
        (e = ctx->g_dst.ensure((size_t)n * 8)) || (rc && (e = ctx->g_rc.ensure((size_t)n))))
        return e;
    HIP_TRY(hipMemcpyAsync(ctx->g_off.p, off, (size_t)n * 8, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(hipMemcpyAsync(ctx->g_len.p, len, (size_t)n * 4, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(hipMemcpyAsync(ctx->g_dst.p, soff.data(), (size_t)n * 8, hipMemcpyHostToDevice, ctx->stream));
    if (rc) HIP_TRY(hipMemcpyAsync(ctx->g_rc.p, rc, (size_t)n, hipMemcpyHostToDevice, ctx->stream));
    const int blocks = (int)std::min<int64_t>(n, (int64_t)ctx->n_cu * 32);
    hipLaunchKernelGGL(gather_kernel, dim3(blocks), dim3(256), 0, ctx->stream, d_text, ctx->g_off.as<int64_t>(),
                       ctx->g_len.as<int32_t>(), rc ? ctx->g_rc.as<int8_t>() : nullptr, ctx->g_dst.as<int64_t>(), n,
                       ctx->seq.as<uint8_t>(), encode ? 1 : 0);
    HIP_TRY(hipGetLastError());
    ctx->staged_encoded = encode;
    return MANDO_OK;
}

}  // namespace

extern "C" {

int mando_poa_batch(mando_ctx *ctx, const mando_poa_params *params, const uint8_t *seqs,
                    const int64_t *seq_off, const int64_t *grp_off, int64_t n_groups,
                    const uint8_t *seeding_per_group, uint8_t *cons_out, int64_t cons_cap,
                    int64_t *cons_off, int64_t *cells_out) {
    if (!ctx || !params || !seq_off || !grp_off || !cons_off || n_groups < 0 || cons_cap < 0)
        return fail(MANDO_E_ARG, "mando_poa_batch: bad argument");
    if (n_groups == 0) {
        cons_off[0] = 0;
        return MANDO_OK;
    }
    int rc = check_groups(grp_off, n_groups);
    if (rc) return rc;
    const int64_t n_reads = grp_off[n_groups];
    for (int64_t r = 0; r < n_reads; ++r)
        if (seq_off[r + 1] < seq_off[r]) return fail(MANDO_E_ARG, "seq_off not monotone");
    const int64_t total = seq_off[n_reads] - seq_off[0];
    if (total > 0 && !seqs) return fail(MANDO_E_ARG, "null seqs");
    std::vector<int64_t> soff((size_t)n_reads + 1);
    for (int64_t r = 0; r <= n_reads; ++r) soff[(size_t)r] = seq_off[r] - seq_off[0];
    return poa_batch_impl(ctx, params, soff, grp_off, n_groups, seeding_per_group, cons_out, cons_cap, cons_off,
                          cells_out, [&](mando_ctx *c) -> int {
                              HIP_TRY(hipMemcpyAsync(c->seq.p, seqs + seq_off[0], (size_t)total, hipMemcpyHostToDevice,
                                                     c->stream));
                              return MANDO_OK;
                          });
}

int mando_poa_segments(mando_ctx *ctx, const mando_poa_params *params, const uint8_t *d_text, int64_t text_len,
                       const int64_t *off, const int32_t *len, const int8_t *rc, const int64_t *grp_off,
                       int64_t n_groups, const uint8_t *seeding_per_group, uint8_t *cons_out, int64_t cons_cap,
                       int64_t *cons_off, int64_t *cells_out) {
    if (!ctx || !params || !grp_off || !cons_off || n_groups < 0 || cons_cap < 0)
        return fail(MANDO_E_ARG, "mando_poa_segments: bad argument");
    if (n_groups == 0) {
        cons_off[0] = 0;
        return MANDO_OK;
    }
    int e = check_groups(grp_off, n_groups);
    if (e) return e;
    const int64_t n_reads = grp_off[n_groups];
    if (n_reads > 0 && (!d_text || !off || !len)) return fail(MANDO_E_ARG, "mando_poa_segments: null segments");
    std::vector<int64_t> soff;
    if ((e = segment_layout(off, len, n_reads, text_len, soff))) return e;
    return poa_batch_impl(ctx, params, soff, grp_off, n_groups, seeding_per_group, cons_out, cons_cap, cons_off,
                          cells_out, [&](mando_ctx *c) { return gather_stage(c, d_text, off, len, rc, soff, true); });
}

int mando_selftest(mando_ctx *ctx, int *bad) {
    if (!ctx || !bad) return fail(MANDO_E_ARG, "bad argument");
    HIP_TRY(hipSetDevice(ctx->device));
    int rc = ctx->counter.ensure(256);
    if (rc) return rc;
    HIP_TRY(hipMemsetAsync(ctx->counter.p, 0, 4, ctx->stream));
    HIP_TRY(mando::run_wave_selftest(ctx->counter.as<int>(), ctx->stream));
    HIP_TRY(hipMemcpyAsync(bad, ctx->counter.p, 4, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return MANDO_OK;
}

}  // extern "C"

namespace {

int orient_impl(mando_ctx *ctx, const std::vector<int64_t> &soff, const int64_t *grp_off, int64_t n_groups,
                int8_t *hit_strands, int32_t max_hits, int32_t *n_hits, const StageFn &stage) {
    const int64_t n_reads = grp_off[n_groups];
    const int64_t total = soff[(size_t)n_reads];
    if (n_reads > 0 && (!hit_strands || !n_hits)) return fail(MANDO_E_ARG, "null outputs");
    if (n_groups > INT32_MAX) return fail(MANDO_E_ARG, "too many groups");
    HIP_TRY(hipSetDevice(ctx->device));
    int rc;
    if ((rc = ctx->seq.ensure((size_t)std::max<int64_t>(total, 1) + 16)) != MANDO_OK) return rc;
    if (getenv("MANDO_WS_LOG"))
        fprintf(stderr, "[mando ws] orient: reads %lld bases %.3f GB (seq buffer %.3f GB)\n", (long long)n_reads,
                total / 1e9, ctx->seq.bytes / 1e9);
    if ((rc = ctx->seq_off.ensure(sizeof(int64_t) * (size_t)(n_reads + 1))) != MANDO_OK) return rc;
    if ((rc = ctx->grp_off.ensure(sizeof(int64_t) * (size_t)(n_groups + 1))) != MANDO_OK) return rc;
    if ((rc = ctx->o_strand.ensure((size_t)std::max<int64_t>(n_reads, 1) * (size_t)max_hits)) != MANDO_OK) return rc;
    if ((rc = ctx->o_hits.ensure(sizeof(int32_t) * (size_t)std::max<int64_t>(n_reads, 1))) != MANDO_OK) return rc;
    if ((rc = ctx->o_status.ensure(sizeof(int32_t) * (size_t)n_groups)) != MANDO_OK) return rc;
    if ((rc = ctx->counter.ensure(sizeof(int32_t))) != MANDO_OK) return rc;
    if (total > 0 && (rc = stage(ctx))) return rc;
    HIP_TRY(hipMemcpyAsync(ctx->seq_off.p, soff.data(), soff.size() * sizeof(int64_t), hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(hipMemcpyAsync(ctx->grp_off.p, grp_off, sizeof(int64_t) * (size_t)(n_groups + 1), hipMemcpyHostToDevice,
                           ctx->stream));
    HIP_TRY(hipMemsetAsync(ctx->o_hits.p, 0, sizeof(int32_t) * (size_t)std::max<int64_t>(n_reads, 1), ctx->stream));
    HIP_TRY(hipMemsetAsync(ctx->counter.p, 0, sizeof(int32_t), ctx->stream));
    const int64_t *seq_off = soff.data();
    // per-read capacity (~2 minimizers per W+1 positions, with margin) sized for the 95th percentile of
    // the groups' longest reads, not the batch maximum: the capacity sets the LDS per wave and so the
    // waves per CU (1024: 5, 2048: 2), and one 6 kb read must not halve the occupancy of 40k groups of
    // 3 kb reads; groups that overflow are re-run at the next capacity
    std::vector<int64_t> gmax((size_t)n_groups, 0);
    for (int64_t g = 0; g < n_groups; ++g)
        for (int64_t r = grp_off[g]; r < grp_off[g + 1]; ++r)
            gmax[(size_t)g] = std::max<int64_t>(gmax[(size_t)g], seq_off[r + 1] - seq_off[r]);
    const size_t q95 = (size_t)((double)(n_groups - 1) * 0.95);
    std::nth_element(gmax.begin(), gmax.begin() + (ptrdiff_t)q95, gmax.end());
    const int64_t maxlen = gmax[q95];
    int cap = 1024;
    while (cap < mando::kOrientCap && maxlen * 26 / 110 > cap) cap *= 2;
    mando::OrientArgs a;
    a.seq = ctx->seq.as<uint8_t>();
    a.seq_off = ctx->seq_off.as<int64_t>();
    a.grp_off = ctx->grp_off.as<int64_t>();
    a.n_groups = (int32_t)n_groups;
    a.hits = ctx->o_strand.as<int8_t>();
    a.n_hits = ctx->o_hits.as<int32_t>();
    a.max_hits = max_hits;
    a.status = ctx->o_status.as<int32_t>();
    a.counter = ctx->counter.as<int32_t>();
    a.gidx = nullptr;
    a.cap = cap;
    a.gscratch = nullptr;
    a.cap_fb = cap < mando::kOrientCap ? mando::kOrientCap : 0;
    std::vector<int32_t> st((size_t)n_groups);
    std::vector<int32_t> redo;
    // the first launch takes the groups largest first (bases of the group's reads): the waves pull
    // groups from a queue, so the launch then ends on small groups instead of a late large one
    bool first = true;
    if (n_groups > 1) {
        std::vector<int64_t> key((size_t)n_groups);
        for (int64_t g = 0; g < n_groups; ++g)
            key[(size_t)g] = (int64_t)(seq_off[grp_off[g + 1]] - seq_off[grp_off[g]]) << 24 | (int64_t)(n_groups - 1 - g);
        std::vector<int32_t> order((size_t)n_groups);
        for (int64_t g = 0; g < n_groups; ++g) order[(size_t)g] = (int32_t)g;
        std::sort(order.begin(), order.end(), [&](int32_t x, int32_t y) { return key[(size_t)x] > key[(size_t)y]; });
        if ((rc = ctx->o_gidx.ensure(sizeof(int32_t) * order.size())) != MANDO_OK) return rc;
        HIP_TRY(hipMemcpyAsync(ctx->o_gidx.p, order.data(), sizeof(int32_t) * order.size(), hipMemcpyHostToDevice,
                               ctx->stream));
        a.gidx = ctx->o_gidx.as<int32_t>();
    }
    HIP_TRY(hipEventRecord(ctx->ev0, ctx->stream));
    ctx->last_launches = 0;
    for (;;) {
        const int64_t ng = first ? n_groups : (int64_t)redo.size();
        a.n_groups = (int32_t)ng;
        const int slots = (int)std::min<int64_t>(ng, (int64_t)ctx->n_cu * mando::orient_blocks_per_cu(a.cap));
        // one HBM slab per launched wave: the reference keys and chain table, or (past the LDS capacity)
        // every per-read array
        if ((rc = ctx->o_scratch.ensure((size_t)slots * mando::orient_slab_words(a.cap, a.cap_fb) * 8)) != MANDO_OK)
            return rc;
        a.gscratch = ctx->o_scratch.as<uint64_t>();
        HIP_TRY(hipMemsetAsync(ctx->counter.p, 0, sizeof(int32_t), ctx->stream));
        HIP_TRY(mando::launch_orient(a, slots, ctx->stream));
        ++ctx->last_launches;
        HIP_TRY(hipMemcpyAsync(st.data(), ctx->o_status.p, sizeof(int32_t) * (size_t)n_groups, hipMemcpyDeviceToHost,
                               ctx->stream));
        HIP_TRY(hipStreamSynchronize(ctx->stream));
        const std::vector<int32_t> prev = redo;
        redo.clear();
        if (!first) {
            for (int32_t g : prev)
                if (st[(size_t)g] != 0) redo.push_back(g);
        } else {
            for (int64_t g = 0; g < n_groups; ++g)
                if (st[(size_t)g] != 0) redo.push_back((int32_t)g);
        }
        first = false;
        if (redo.empty()) break;
        // (over the in-kernel fallback's capacity too: the re-run starts past it)
        if (a.cap_fb > a.cap) a.cap = a.cap_fb;
        a.cap_fb = 0;
        if (a.cap >= mando::kOrientCapMax)
            return fail(MANDO_E_UNSUPPORTED, "orientation: group " + std::to_string(redo[0]) + " has a read with more than " +
                                                 std::to_string(mando::kOrientCapMax) + " minimizers or anchors");
        // overflowed groups again, at the next capacity (their outputs are rewritten in full); past the
        // LDS capacity the arrays move to per-wave HBM slabs, sized for the longest read of those groups
        if ((rc = ctx->o_gidx.ensure(sizeof(int32_t) * redo.size())) != MANDO_OK) return rc;
        HIP_TRY(hipMemcpyAsync(ctx->o_gidx.p, redo.data(), sizeof(int32_t) * redo.size(), hipMemcpyHostToDevice,
                               ctx->stream));
        a.gidx = ctx->o_gidx.as<int32_t>();
        if (a.cap < mando::kOrientCap) {
            a.cap *= 2;
        } else {
            int64_t ml = 0;
            for (int32_t g : redo)
                for (int64_t r = grp_off[g]; r < grp_off[g + 1]; ++r) ml = std::max<int64_t>(ml, seq_off[r + 1] - seq_off[r]);
            int cap2 = a.cap * 2;
            while (cap2 < mando::kOrientCapMax && ml * 26 / 110 > cap2) cap2 *= 2;
            a.cap = cap2;
        }
    }
    HIP_TRY(hipEventRecord(ctx->ev1, ctx->stream));
    ctx->timed = true;
    if (n_reads > 0) {
        HIP_TRY(hipMemcpyAsync(hit_strands, ctx->o_strand.p, (size_t)n_reads * (size_t)max_hits, hipMemcpyDeviceToHost,
                               ctx->stream));
        HIP_TRY(hipMemcpyAsync(n_hits, ctx->o_hits.p, sizeof(int32_t) * (size_t)n_reads, hipMemcpyDeviceToHost,
                               ctx->stream));
    }
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return MANDO_OK;
}

}  // namespace

extern "C" {

int mando_orient_batch(mando_ctx *ctx, const uint8_t *seqs, const int64_t *seq_off, const int64_t *grp_off,
                       int64_t n_groups, int8_t *hit_strands, int32_t max_hits, int32_t *n_hits) {
    if (!ctx || n_groups < 0 || max_hits < 1 || max_hits > 8 || (n_groups > 0 && (!seq_off || !grp_off)))
        return fail(MANDO_E_ARG, "mando_orient_batch: bad argument (max_hits must be 1..8)");
    if (n_groups == 0) return MANDO_OK;
    int rc = check_groups(grp_off, n_groups);
    if (rc) return rc;
    const int64_t n_reads = grp_off[n_groups];
    for (int64_t r = 0; r < n_reads; ++r)
        if (seq_off[r + 1] < seq_off[r]) return fail(MANDO_E_ARG, "seq_off not monotone");
    const int64_t total = seq_off[n_reads] - seq_off[0];
    if (total > 0 && !seqs) return fail(MANDO_E_ARG, "null seqs");
    std::vector<int64_t> so((size_t)n_reads + 1);
    for (int64_t r = 0; r <= n_reads; ++r) so[(size_t)r] = seq_off[r] - seq_off[0];
    return orient_impl(ctx, so, grp_off, n_groups, hit_strands, max_hits, n_hits, [&](mando_ctx *c) -> int {
        HIP_TRY(hipMemcpyAsync(c->seq.p, seqs + seq_off[0], (size_t)total, hipMemcpyHostToDevice, c->stream));
        return MANDO_OK;
    });
}

int mando_orient_segments(mando_ctx *ctx, const uint8_t *d_text, int64_t text_len, const int64_t *off,
                          const int32_t *len, const int64_t *grp_off, int64_t n_groups, int8_t *hit_strands,
                          int32_t max_hits, int32_t *n_hits) {
    if (!ctx || n_groups < 0 || max_hits < 1 || max_hits > 8 || (n_groups > 0 && !grp_off))
        return fail(MANDO_E_ARG, "mando_orient_segments: bad argument (max_hits must be 1..8)");
    if (n_groups == 0) return MANDO_OK;
    int e = check_groups(grp_off, n_groups);
    if (e) return e;
    const int64_t n_reads = grp_off[n_groups];
    if (n_reads > 0 && (!d_text || !off || !len)) return fail(MANDO_E_ARG, "mando_orient_segments: null segments");
    std::vector<int64_t> soff;
    if ((e = segment_layout(off, len, n_reads, text_len, soff))) return e;
    return orient_impl(ctx, soff, grp_off, n_groups, hit_strands, max_hits, n_hits,
                       [&](mando_ctx *c) { return gather_stage(c, d_text, off, len, nullptr, soff); });
}

}  // extern "C"
