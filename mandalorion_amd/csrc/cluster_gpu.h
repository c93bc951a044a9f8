// cluster_gpu.h — layout shared by the per-locus clustering kernels (cluster_kernel.hip) and their
// host launcher (cluster.cpp).  Not part of the public ABI.
//
// Two kernels, one 64-lane wave (one workgroup) per locus:
//   K1 `cluster_parse`   locus PSL text in HBM -> records, blocks, tokenised cs runs (scratch A)
//   K2 `cluster_locus`   records -> coverage sets, splice-site histograms, peaks, splice identities,
//                        TSS/TES windows, isoform groups and the subsample draw (scratch B, outputs)
// The host sizes scratch B from K1's per-locus statistics.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/mando.h"

#if defined(__HIP__)
#define CL_HD __host__ __device__
#else
#define CL_HD
#endif

namespace mando {
namespace cl {

// locus status codes (mando_cluster_view::locus_status); the same values as the host restatement
constexpr int kOk = 0;
constexpr int kZeroDivision = -10;  // characterize_splicing_event: leftCS['Total'] == 0
constexpr int kKeyError = -11;      // scan_for_best_bin: strand column not '+' / '-'
constexpr int kParse = -12;         // malformed PSL line / cs string
constexpr int kIO = -13;            // file unreadable
constexpr int kValueError = -15;    // max() of an empty sequence in find_ends
constexpr int kCapacity = -16;      // internal: scratch capacity exceeded, the host re-runs the locus
constexpr int kRange = -17;         // a genome position beyond the kernel's position range

struct Locus {
    int64_t text_off;  // locus text in the device text buffer
    int64_t text_len;
    int64_t a_off;     // scratch A (bytes, 256-aligned)
    int64_t b_off;     // scratch B (bytes, 256-aligned)
    int64_t b_len;
    int64_t o_off;     // output region (bytes, 256-aligned)
    int64_t rec_base;  // first global record index (K2 writes the per-record text offsets there)
    int64_t map_lo;    // dense position maps cover [map_lo, map_lo + map_n)
    int64_t map_n;
    int32_t line_cap, op_cap, blk_cap;
    int32_t chrom_off, chrom_len;  // the locus chromosome in the chrom byte buffer
    int32_t ann_off[5];            // annotated bounds: ann_pos[ann_off[s] .. ann_off[s+1]), s = l5 l3 r5 r3
    int32_t pad;
};

struct Stats {  // written by K1 (and K2's status)
    int32_t status;
    int32_t n_rec;
    int32_t n_ops, n_blk;     // true totals, also when a capacity was exceeded
    int32_t n_hist_l, n_hist_r;
    int32_t max_nblk;
    int32_t cs_err;            // a record without the cs / seq columns (set by the cs-count waves)
    int64_t span_lo, span_hi;  // tStart / tEnd range of the records on the locus chromosome
    int64_t cov_cap;           // coverage-bin slots (sum over records of sum over blocks ceil(sz/10) + 11)
    int64_t ident_cap;         // bytes of rendered splice identities
    int32_t n_iso, n_mem, n_sub, n_peaks;  // K2 outputs
};

struct Rec {
    int64_t qsize, qstart, qend, tstart, tend;
    int32_t line_lo, line_hi;  // the stripped line
    int32_t name_off, name_len;
    int32_t chrom_off, chrom_len;
    int32_t cs_off, cs_len;
    int32_t seq_off, seq_len;
    int32_t blk_off, nblk;
    int32_t op_off, nop;
    int32_t run_off, nrun;
    int32_t adv_off, nadv;
    int32_t nrec_cs;
    int32_t cov_off, cov_n;
    int32_t cs_of;
    int8_t dirn;        // 0 '+', 1 '-', 2 anything else
    int8_t same_chrom;  // chrom column == the locus chromosome
    int8_t acc_lt;      // accuracy < 0.9
    int8_t cs_bad;      // build_cs of this cs string raises (checked only when a query needs it)
    int32_t pad;
};

// one cs operation, run-length form of getCSaroundSS's record list (cluster.cpp CsRun)
struct Run {
    int64_t g0;
    int32_t rec0, n;
    int32_t step;
    char st;
    char motif[4];
    char pad[3];
};

struct Peak {
    int64_t start, end;
    double prop;  // -1 for annotated bins
    char type, side;
    char pad[6];
};

struct Params {
    double cutoff;
    int32_t w, min_count, up, down, sub_k;
    int32_t n_junc;
    char junc[16][4];  // junction motifs (4 characters each); longer / shorter ones never match
    int8_t junc_len4[16];
    uint32_t mt_init[624];  // MT19937 state after init_genrand(seed)
};

struct Args {
    const uint8_t *text;
    const uint8_t *chroms;
    const int64_t *ann_pos;
    const Locus *loci;
    const int32_t *order;  // block b runs locus order[b]
    const int32_t *work;   // cs waves: block b takes locus work[2b], member work[2b+1] & 0xffff of work[2b+1] >> 16
    Stats *stats;
    uint8_t *scratch_a;
    uint8_t *scratch_b;
    uint8_t *out;
    int64_t *rec_text;  // per global record: name_off, name_len, seq_off, seq_len (text-absolute)
    const Params *prm;
    int64_t sort_tile;  // K2: keys of the launch's dynamic LDS (the sort tile; a power of two)
};

// host side (cluster_kernel.hip): both kernels over a batch of loci whose text is in host memory
struct ClusterIn {
    int64_t n_loci;
    const char *text;
    int64_t text_len;
    void *d_text;             // the same text already on (or being copied to) the device, stream-ordered
    const int64_t *foff;      // n_loci + 1 offsets of each locus file in text
    const int32_t *fstatus;   // kOk, or kIO for a file that could not be read
    const char *const *chroms;
    const int64_t *ann_pos, *ann_off;  // may be null
    double cutoff;
    int32_t w, min_count, up, down, sub_k;
    std::vector<std::string> junctions;
    uint32_t seed;
    hipEvent_t ready = nullptr;  // the text of these loci is on the device once this event completes
};
struct ClusterOut {
    std::vector<int32_t> status, n_rec;
    std::vector<int64_t> rec_base;  // n_loci + 1
    std::vector<int64_t> rec_text;  // per record: name_off, name_len, seq_off, seq_len (text-absolute)
    std::vector<std::vector<Peak>> peaks;
    std::vector<std::vector<int32_t>> iso_nmem, mem, iso_nsub, sub;  // locus-local record indices
};

// sizes of the K1 scratch for caps (bytes), 256-aligned pieces
CL_HD inline int64_t align256(int64_t x) { return (x + 255) & ~int64_t(255); }
CL_HD inline int64_t scratch_a_bytes(int64_t line_cap, int64_t op_cap, int64_t blk_cap) {
    return align256(line_cap * 4) + align256(line_cap * (int64_t)sizeof(Rec)) + align256(blk_cap * 16) +
           align256(op_cap * 4) + align256(op_cap * (int64_t)sizeof(Run)) + align256(op_cap * 4) +
           align256(op_cap * 8);
}

int cluster_gpu(mando_ctx *ctx, const ClusterIn &in, ClusterOut &out);
// the stream the clustering of ctx runs on (its kernels and the copies they wait for)
hipStream_t cluster_stream(mando_ctx *ctx);
// the device copy of the locus text (cached whole buffers; the result keeps one until it is freed)
void *acquire_text(mando_ctx *ctx, size_t need, size_t &cap);
void release_text(mando_ctx *ctx, void *d_text, size_t cap);

}  // namespace cl
}  // namespace mando
