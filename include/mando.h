/*
 * mando.h — C-ABI of libmando, the MI355X-native consensus core for Mandalorion's D module.
 *
 * Every entry point is extern "C", takes plain pointers and sizes, returns int (0 = ok, < 0 = error
 * code) and never throws.  mando_last_error() returns a thread-local message for the last failure.
 * Device memory lives inside an opaque mando_ctx (one per GPU, not re-entrant; several ctxs may run
 * concurrently).  The Python host binds these with ctypes (mandalorion_amd/_lib.py); the bindings a
 * reference maintainer would add are shown in INTEGRATION.md.
 *
 * Reference interfaces replaced (paths relative to the upstream Mandalorion tree):
 *   mando_poa_batch / mando_poa_batch_device
 *       replaces the abPOA CLI call `abpoa -M 5 -r 0 [-S] root.fasta > root.consensus.fasta`
 *       and the read-back of its FASTA  — utils/SpliceDefineConsensus.py:911-926
 *       (abPOA v1.4.1, pinned by setup.sh:17-20).
 *   mando_orient_batch
 *       replaces `mp.Aligner(seq=first, preset='map-ont')` + the per-read `map()` primary-hit /
 *       strand loop — utils/SpliceDefineConsensus.py:895-907.
 *   mando_mt_permutation
 *       replaces `np.random.choice(np.arange(n), min(n, k), replace=False)` on the process-global
 *       legacy RandomState — utils/SpliceDefineConsensus.py:505, :818, :884.
 */
#ifndef MANDO_H
#define MANDO_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MANDO_ABI_VERSION 1

enum mando_status {
    MANDO_OK = 0,
    MANDO_E_ARG = -1,         /* bad argument (null pointer, negative size, inconsistent offsets) */
    MANDO_E_HIP = -2,         /* HIP runtime error (message in mando_last_error) */
    MANDO_E_NOMEM = -3,       /* device or host allocation failed */
    MANDO_E_CAP = -4,         /* caller-provided output buffer too small */
    MANDO_E_UNSUPPORTED = -5, /* requested mode not implemented on this build */
    MANDO_E_INTERNAL = -6,    /* kernel reported an inconsistent state */
    MANDO_E_NODEV = -7        /* no HIP device visible */
};

typedef struct mando_ctx mando_ctx;

/* abPOA-equivalent parameters.  Defaults (mando_poa_default_params) are the reference's
 * `abpoa -M 5 -r 0`: match 5, mismatch 4, convex gaps (4,2) and (24,1), adaptive band
 * w = band_b + (int)(band_f * qlen) with band_b 10, band_f 0.01; seeding (-S) off, k 19, w 10,
 * min_w 500. */
typedef struct {
    int32_t match, mismatch;
    int32_t gap_open1, gap_ext1, gap_open2, gap_ext2;
    int32_t band_b;
    float band_f;
    int32_t seeding, k, w, min_w;
} mando_poa_params;

const char *mando_last_error(void);
int mando_abi_version(void);
void mando_poa_default_params(mando_poa_params *p);

/* Number of visible HIP devices (0 on a machine without a GPU; never fails for that reason). */
int mando_device_count(int *out);

/* A context: one device, its streams, cached device buffers and POA workspaces.  Creating one sets
 * the device's schedule flag to hipDeviceScheduleBlockingSync (host threads waiting on the device
 * sleep on its completion signal instead of spinning; spinning cost ~1.6 cores per GPU on config 4).
 * That flag is process-wide for the device: it also applies to the host application's own waits on
 * that device, and HIP refuses it when the application has already initialised the device with other
 * flags (the application's flags are then kept); mando_ctx_blocking_sync() reports which.
 * Each context's stream (and each internal stream: POA lanes, the clustering's copy stream) runs on a
 * hardware queue of its own -- a CU-masked stream with every CU enabled -- so two contexts' work
 * overlaps however many streams the process holds (HIP shares 4 hardware queues among plain streams).
 * Such streams are blocking with respect to the legacy null stream: an application's null-stream
 * commands on the same device wait for the library's queued work.  MANDO_SHARED_QUEUES=1 makes them
 * plain non-blocking streams. */
int mando_ctx_create(int device_ordinal, mando_ctx **out);
void mando_ctx_destroy(mando_ctx *ctx);
/* 1 when the ctx's device waits with blocking sync, 0 when it spins (flags set before the ctx), <0 on
 * error. */
int mando_ctx_blocking_sync(mando_ctx *ctx);

/* Batched POA consensus, host buffers.
 *   n_groups groups; group g = reads [grp_off[g], grp_off[g+1]) in FINAL abPOA input order
 *   (post-subsample, post-orientation, duplicates kept).  Read r = seqs[seq_off[r] .. seq_off[r+1])
 *   as ASCII (ACGTN, any case; other bytes are treated as N).
 *   seeding_per_group may be NULL (all 0); a nonzero entry requests the -S path.
 *   On success cons_off[0..n_groups] holds offsets into cons_out (ASCII ACGTN, no separators) and,
 *   when cells_out is non-NULL, cells_out[g] the number of banded DP cells evaluated for group g.
 *   Returns MANDO_E_CAP (and the required size in cons_off[n_groups]) when cons_cap is too small. */
int mando_poa_batch(mando_ctx *ctx, const mando_poa_params *params, const uint8_t *seqs,
                    const int64_t *seq_off, const int64_t *grp_off, int64_t n_groups,
                    const uint8_t *seeding_per_group, uint8_t *cons_out, int64_t cons_cap,
                    int64_t *cons_off, int64_t *cells_out);

/* Same computation with every input already resident in device memory (HBM) — the form the
 * benchmark times.  d_seqs holds 2-bit-free encoded bases (0..4 = ACGTN), d_seq_off/d_grp_off are
 * device int64 arrays as above, outputs are device arrays: d_cons (capacity cons_cap bytes, encoded
 * 0..4), d_cons_len[n_groups] (int32), d_cells[n_groups] (int64), d_status[n_groups] (int32).
 * Asynchronous on the ctx's stream; mando_ctx_sync() waits. */
int mando_poa_batch_device(mando_ctx *ctx, const mando_poa_params *params, const uint8_t *d_seqs,
                           const int64_t *d_seq_off, const int64_t *d_grp_off, int64_t n_groups,
                           int64_t max_read_len, int64_t max_group_bases, uint8_t *d_cons,
                           const int64_t *d_cons_off, int32_t *d_cons_len, int64_t *d_cells,
                           int32_t *d_status);
int mando_ctx_sync(mando_ctx *ctx);

/* Device-time of the most recent POA / orientation launch on the ctx stream, from HIP events
 * recorded around the kernel on that stream (milliseconds). */
float mando_last_kernel_ms(mando_ctx *ctx);
/* Number of kernel launches issued by the most recent batch call (the roofline divides by it). */
int mando_last_kernel_launches(mando_ctx *ctx);

/* Caps the POA workspaces of this ctx (every launch kind together) at `bytes` of HBM for the calls
 * that follow; 0 restores the default policy (a share of the free HBM at launch time).  The D driver
 * (defineIsoforms.py:130-166's per-locus Pool, here one call per chunk) sets it per call from its chunk
 * plan: the locus text, clustering scratch and gathered reads of the chunks in flight are reserved
 * first, so no free-memory query races with the clustering thread's allocations. */
int mando_ctx_set_poa_budget(mando_ctx *ctx, int64_t bytes);
/* The device's HBM and the bytes this ctx's POA workspaces hold now (either may be NULL). */
int mando_ctx_memory(mando_ctx *ctx, int64_t *total_bytes, int64_t *poa_ws_bytes);
/* Free and total HBM of a device now (hipMemGetInfo; either may be NULL). */
int mando_device_memory(int device_ordinal, int64_t *free_bytes, int64_t *total_bytes);
/* The clustering's cached device buffers on a device (the idle locus-text buffers and the per-context
 * scratch, kept between calls for reuse): frees idle text buffers larger than text_cap_max bytes and,
 * when the scratch of the device's contexts holds more than scratch_max bytes, all of that scratch
 * (negative limits: keep).  held_bytes (may be NULL) receives what the caches hold afterwards.  The D
 * driver calls it at the start of a call whose chunk plan is smaller than an earlier call's, so that
 * its HBM plan (mando_ctx_set_poa_budget) is not undercut by buffers a larger plan left behind. */
int mando_cache_trim(int device_ordinal, int64_t text_cap_max, int64_t scratch_max, int64_t *held_bytes);
/* Workspace slots and budget of the most recent batch's launches by kind [narrow, wide, -S] (0: that
 * kind did not run); either array may be NULL, else holds 3 entries. */
int mando_poa_last_slots(mando_ctx *ctx, int64_t *slots, int64_t *budgets);

/* Read orientation (mappy map-ont strand / primary-hit replacement).  For each group the
 * reference sequence is the group's first read.  For every read r, n_hits[r] is the number of primary
 * hits (0 = unmapped; the reference then drops the read) and hit_strands[r*max_hits + h] (+1 / -1) the
 * strand of hit h, in mappy's hit order; the reference writes the read once per primary hit, re-bound
 * by the hits before it (SpliceDefineConsensus.py:902-907).  Counting stops at max_hits + 1:
 * n_hits[r] == max_hits + 1 means "more than max_hits primaries" (only max_hits strands written), and
 * the caller re-runs with a larger max_hits (1..8). */
int mando_orient_batch(mando_ctx *ctx, const uint8_t *seqs, const int64_t *seq_off,
                       const int64_t *grp_off, int64_t n_groups, int8_t *hit_strands,
                       int32_t max_hits, int32_t *n_hits);

/* Device self-test of the wave-level primitives the kernels use (scan / reduce); *bad = number of
 * mismatching lanes (0 = pass). */
int mando_selftest(mando_ctx *ctx, int *bad);

/* numpy legacy RandomState(seed).permutation(n)[:k] replayed `n_draws` times in sequence from one
 * fresh MT19937 state: draw d uses n = ns[d], k = ks[d]; outputs concatenated in out (int64). */
int mando_mt_permutation(uint32_t seed, const int64_t *ns, const int64_t *ks, int64_t n_draws,
                         int64_t *out, int64_t out_cap);

/* ------------------------------------------------------------------------------------------------
 * Per-locus read clustering on the GPU: host threads read the locus files, then two HIP kernels run one
 * locus per 64-lane wave (parse + cs tokenisation; peaks, identities, isoform groups).  Replaces the
 * clustering half of process_locus (/root/reference/defineIsoforms.py:55-91 -> SpliceDefineConsensus.py
 * :107-868) and the subsample draw of determine_consensus (SpliceDefineConsensus.py:884-888), i.e. the
 * reference's per-locus Pool worker minus mappy/abPOA.  ctx: the device (its stream runs the kernels;
 * the call blocks until the results are on the host).  Every locus replays the
 * numpy legacy RNG stream of RandomState(seed), which is what each forked locus worker of the
 * reference sees when its parent seeded numpy (defineIsoforms.py:130).
 * ---------------------------------------------------------------------------------------------- */
typedef struct {
    double cutoff;              /* -c, find_peaks proportion cutoff (0.1) */
    int32_t splice_site_width;  /* -w (1) */
    int32_t minimum_read_count; /* -m (2) */
    int32_t upstream_buffer;    /* -u (10) */
    int32_t downstream_buffer;  /* -d (50) */
    const char *junctions;      /* -j, comma separated ("gtag,gcag,atac,ctac,ctgc,gtat") */
    uint32_t seed;              /* numpy global RNG seed every locus starts from */
    int32_t threads;            /* host threads reading the locus files (0 = all hardware threads) */
    int32_t poa_subsample;      /* determine_consensus subsample size (100) */
    mando_ctx *orient_ctx;      /* NULL (default), or a context of the same device: every isoform's
                                   subsample is oriented on it (mando_orient_segments, SDC:895-907) as
                                   its loci are clustered, and the view carries the hit strands */
    int32_t orient_max_hits;    /* first attempt's hit capacity per read (4); reads with more re-run at 8 */
} mando_cluster_params;

typedef struct mando_cluster_result mando_cluster_result;

/* Flat, read-only view of a clustering result (arrays owned by the result). */
typedef struct {
    int64_t n_loci;
    const int32_t *locus_status;   /* 0 ok; -10 ZeroDivisionError, -11 KeyError (strand), -12 parse,
                                      -13 I/O, -15 ValueError -- the reference's locus exceptions */
    const char *text;              /* all locus files, concatenated */
    int64_t text_len;
    int64_t n_records;             /* PSL lines, locus by locus in file order */
    const int64_t *name_off;       /* qName (col 9) of each record: text + name_off[r], name_len[r] */
    const int32_t *name_len;
    const int64_t *seq_off;        /* sequence (col 23) */
    const int32_t *seq_len;
    const int64_t *rec_locus;
    int64_t n_isoforms;            /* locus by locus, IsoDict order inside a locus */
    const int64_t *iso_locus;
    const int64_t *mem_off;        /* n_isoforms+1: member records (IsoDict read order) */
    const int64_t *mem;
    const int64_t *sub_off;        /* n_isoforms+1: determine_consensus subsample, draw order */
    const int64_t *sub;
    int64_t n_peaks;               /* accepted splice-site bins (make_genome_bins + find_peaks rows) */
    const int64_t *peak_locus;
    const int64_t *peak_start;
    const int64_t *peak_end;
    const char *peak_type;         /* '5' / '3' */
    const char *peak_side;         /* 'l' / 'r' */
    const double *peak_prop;       /* round(prop, 3), -1 for annotated ('A') bins */
    int32_t orient_max_hits;       /* 0: not oriented (no orient_ctx, or a read with more than 8 primary
                                      hits: the caller orients and reports it); else H: */
    const int8_t *orient_hits;     /* sub[] x H hit strands (+1 / -1), as mando_orient_segments writes them */
    const int32_t *orient_n_hits;  /* primary hits per subsampled read */
} mando_cluster_view;

void mando_cluster_default_params(mando_cluster_params *p);
/* psl_paths[i]: locus file tmp_SS/<chrom~start~end>.psl; chroms[i]: its chrom.  Annotated splice
 * bounds inside the locus (defineIsoforms.py:140-150) as 4 lists per locus (left '5', left '3',
 * right '5', right '3'): ann_pos[ann_off[4i+s] .. ann_off[4i+s+1]); both may be NULL. */
int mando_cluster_loci(mando_ctx *ctx, const mando_cluster_params *params, const char *const *psl_paths,
                       const char *const *chroms, int64_t n_loci, const int64_t *ann_pos,
                       const int64_t *ann_off, mando_cluster_result **out);
int mando_cluster_view_get(const mando_cluster_result *res, mando_cluster_view *view);
void mando_cluster_free(mando_cluster_result *res);
/* The same locus text on the device the clustering ran on (valid until mando_cluster_free): the
 * orientation and POA inputs are gathered from it (mando_orient_segments / mando_poa_segments) instead
 * of being packed on the host and copied again. */
int mando_cluster_device_text(const mando_cluster_result *res, const uint8_t **d_text, int64_t *len);

/* Device-resident inputs: read r of a batch is d_text[off[r] .. off[r] + len[r]) (a device pointer of
 * ctx's device, text_len bytes; off / len / rc are host arrays), reverse-complemented like
 * mappy.revcomp when rc && rc[r].  Otherwise identical to mando_orient_batch / mando_poa_batch: the
 * reads are gathered on the device into the batch layout, so only the (off, len, rc) arrays cross
 * PCIe. */
int mando_orient_segments(mando_ctx *ctx, const uint8_t *d_text, int64_t text_len, const int64_t *off,
                          const int32_t *len, const int64_t *grp_off, int64_t n_groups, int8_t *hit_strands,
                          int32_t max_hits, int32_t *n_hits);
int mando_poa_segments(mando_ctx *ctx, const mando_poa_params *params, const uint8_t *d_text, int64_t text_len,
                       const int64_t *off, const int32_t *len, const int8_t *rc, const int64_t *grp_off,
                       int64_t n_groups, const uint8_t *seeding_per_group, uint8_t *cons_out, int64_t cons_cap,
                       int64_t *cons_off, int64_t *cells_out);

/* ------------------------------------------------------------------------------------------------
 * Reassembly of the sharded D module: loci are split over ranks (one process per
 * GPU); the only exchange is one all-gather of each rank's results to the ordered writer on rank 0
 * (the reference's Pool writer, /root/reference/defineIsoforms.py:130-166).
 * Rendezvous is a TCP star (rank 0 listens on addr:port; the others connect, retrying for up to
 * timeout_s seconds).  With a device ctx the ranks then form an RCCL communicator on that device
 * (rank 0 draws the ncclUniqueId and ships it over the star) and mando_allgather_bytes runs over RCCL
 * / xGMI; with ctx == NULL the star carries the bytes (CPU-only runs).  nranks == 1 needs no peers.
 * ---------------------------------------------------------------------------------------------- */
typedef struct mando_comm mando_comm;

int mando_comm_init(mando_ctx *ctx, int nranks, int rank, const char *addr, int port, double timeout_s,
                    mando_comm **out);
/* 1 = RCCL, 0 = host sockets */
int mando_comm_backend(const mando_comm *comm);
/* counts[r] = rank r's n (every rank gets all nranks counts) */
int mando_allgather_counts(mando_comm *comm, int64_t n, int64_t *counts);
/* recv = every rank's send bytes concatenated in rank order; recv_counts from mando_allgather_counts */
int mando_allgather_bytes(mando_comm *comm, const uint8_t *send, int64_t n, uint8_t *recv,
                          const int64_t *recv_counts);
/* Every rank's bytes on rank 0 only, in rank order (recv_counts from mando_allgather_counts; recv may be
 * NULL on the other ranks): RCCL point-to-point sends to rank 0 between GPUs (xGMI), the TCP star without
 * a device.  The D driver's reassembly (defineIsoforms.py:155-166's writer is rank 0). */
int mando_gather_bytes(mando_comm *comm, const uint8_t *send, int64_t n, uint8_t *recv, const int64_t *recv_counts);
/* Personalised exchange: send holds the parts for ranks 0..nranks-1 back to back (send_counts[r] bytes
 * for rank r), recv receives the parts from ranks 0..nranks-1 back to back (recv_counts[r] bytes from
 * rank r; every rank must know what it receives, e.g. from an all-gather of the send counts).  RCCL
 * point-to-point sends / receives in one group; the host transport returns MANDO_E_UNSUPPORTED (callers
 * all-gather instead).  The D driver's range placement of the output files (defineIsoforms.py:155-166). */
int mando_alltoallv_bytes(mando_comm *comm, const uint8_t *send, const int64_t *send_counts, uint8_t *recv,
                          const int64_t *recv_counts);
/* *v = max over ranks of *v (the benchmark's max-over-ranks wall time) */
int mando_allreduce_max_f64(mando_comm *comm, double *v);
int mando_comm_barrier(mando_comm *comm);
void mando_comm_destroy(mando_comm *comm);
/* The RCCL paths' argument marshalling, exposed so a CPU run can replay it (no device needed).
 * All-gather: RCCL has no allgatherv, so every rank sends *maxc bytes (the largest count, >= 1) to one
 * ncclAllGather; rank r's bytes land at dev_off[r] = r * maxc of the padded receive buffer and are
 * compacted to host_off[r] (the prefix sum of recv_counts).
 * Gather to rank 0: on rank 0, peer p's bytes are received at peer_off[p] (their offset in the
 * concatenation), peer_len[p] = recv_counts[p] for p > 0, and the device range [d2h_off, d2h_off +
 * d2h_len) is copied back (rank 0's own bytes stay on the host); on rank r > 0, peer_len[0] =
 * recv_counts[r] (its send to rank 0) and every other entry is 0. */
int mando_rccl_allgather_plan(int nranks, const int64_t *recv_counts, int64_t *maxc, int64_t *dev_off,
                              int64_t *host_off);
int mando_rccl_gather_plan(int nranks, int rank, const int64_t *recv_counts, int64_t *peer_off, int64_t *peer_len,
                           int64_t *d2h_off, int64_t *d2h_len);
/* mando_alltoallv_bytes: the offsets of each rank's part in send and in recv (prefix sums). */
int mando_rccl_alltoallv_plan(int nranks, const int64_t *send_counts, const int64_t *recv_counts, int64_t *send_off,
                              int64_t *recv_off);

/* Host helper of the D driver (FASTA / read-group assembly without per-read interpreter work):
 * segment i = src[sel[i]] + starts[i], lens[i] bytes (sel may be NULL: src[0]), reverse-complemented
 * like mappy.revcomp when rc && rc[i], written at out + out_off[i]. */
int mando_pack_segments(const uint8_t *const *src, const int8_t *sel, const int64_t *starts,
                        const int64_t *lens, const int8_t *rc, int64_t n, uint8_t *out,
                        const int64_t *out_off, int32_t threads);

/* The D module's two output files for n_iso isoforms (replaces the per-isoform write loop of
 * defineIsoforms.py:155-166):
 *   fasta: ">Isoform{k}_{m}\n{consensus}\n"        r2i: "{name}\tIsoform{k}_{m}\n" per member
 * isoform i of the output is payload isoform g = order[i], numbered k = iso_k[i] (iso_k NULL: counter0+1+i);
 * its members are mem_off[g]..mem_off[g+1]-1 (m of them).  consensus g = cons_src[cons_sel[g]] +
 * cons_start[g], cons_len[g] bytes, reverse-complemented when cons_rc && cons_rc[g]; name j =
 * name_src[name_sel[j]] + name_start[j], name_len[j] bytes (a NULL selector means source 0).  fasta or
 * r2i NULL: that file is skipped.  Sets *fasta_len / *r2i_len and, when non-NULL, fasta_off / r2i_off
 * (n_iso + 1 entries: where output isoform i starts); MANDO_E_CAP (sizes and offsets still set, nothing
 * written) when a capacity is too small. */
int mando_format_outputs(int64_t n_iso, int64_t counter0, const int64_t *iso_k, const int64_t *order,
                         const int64_t *mem_off, const uint8_t *const *cons_src, const int16_t *cons_sel,
                         const int64_t *cons_start, const int64_t *cons_len, const int8_t *cons_rc,
                         const uint8_t *const *name_src, const int16_t *name_sel, const int64_t *name_start,
                         const int64_t *name_len, uint8_t *fasta, int64_t fasta_cap, int64_t *fasta_len,
                         uint8_t *r2i, int64_t r2i_cap, int64_t *r2i_len, int64_t *fasta_off, int64_t *r2i_off,
                         int32_t threads);

/* Block i of buf (src_off[i], len[i] bytes) written at file offset dst_off[i] of the open descriptor fd
 * with pwrite (the per-root blocks a rank places into the shared output files; neighbouring blocks
 * contiguous on both sides go out as one call).  threads <= 0: up to 8. */
int mando_write_blocks(int32_t fd, const uint8_t *buf, const int64_t *src_off, const int64_t *dst_off,
                       const int64_t *len, int64_t n, int32_t threads);

/* PSL ingest + locus split: `sort -k 14,14 -k 16,17n` (C locale) of the clean
 * PSL (Mando.py:343-349) when sort_lines != 0, optional write of the sorted file, then
 * get_chromosomes (SpliceDefineConsensus.py:442-495): one <out_dir>/<chrom>~<start>~<end>.psl per locus. */
int mando_split_loci(const char *psl_path, const char *out_dir, int32_t sort_lines, const char *sorted_out,
                     int64_t *n_records, int64_t *n_loci);
/* The same with the parse and the sort on the ctx's GPU (psl_kernel.hip: a wave per line, a chain of
 * stable radix sorts over the line order; the file writes stay on the host), byte-identical to
 * mando_split_loci; MANDO_E_UNSUPPORTED for a chromosome name over 32 bytes. */
int mando_split_loci_device(mando_ctx *ctx, const char *psl_path, const char *out_dir, int32_t sort_lines,
                            const char *sorted_out, int64_t *n_records, int64_t *n_loci);

/* The D module's locus roots (defineIsoforms.py:130-139, `roots` of main): every entry of `dir` that is a
 * regular file whose name holds ".psl", cut at the first ".psl", deduplicated, sorted by
 * (chromosome bytes, int(start)) (ties by the whole root); sizes[k] = size of <root k>.psl, -1 when no
 * entry is exactly that name.  Writes the roots NUL-terminated into names (capacity names_cap bytes)
 * and *n_roots / *names_bytes.  MANDO_E_CAP when names_cap or sizes_cap is too small (both required sizes
 * are still returned); MANDO_E_ARG when a root's second '~' field is not a plain decimal integer (the
 * caller then applies Python's int() itself).  threads <= 0: up to 16 threads for the stat calls. */
int mando_list_roots(const char *dir, int32_t threads, char *names, int64_t names_cap, int64_t *sizes,
                     int64_t sizes_cap, int64_t *n_roots, int64_t *names_bytes);

/* The same roots without their sizes: readdir's entry type decides where it can (only symlinks and
 * entries of unknown type are stat'ed), so listing 200,000 loci costs one directory read.  The
 * multi-rank driver lists on rank 0 and has every rank stat a slice (mando_root_sizes), replacing rank
 * 0's 200,000 stat calls (defineIsoforms.py:130-139 as in mando_list_roots; same return codes). */
int mando_list_root_names(const char *dir, char *names, int64_t names_cap, int64_t *n_roots, int64_t *names_bytes);

/* sizes[i] = size of <dir>/<root i>.psl if that is a regular file (symlinks followed), else -1, for n
 * NUL-terminated roots stored back to back in names (a slice of mando_list_root_names' output).
 * threads <= 0: up to 16 threads. */
int mando_root_sizes(const char *dir, const char *names, int64_t n, int32_t threads, int64_t *sizes);

/* SAM -> PSL, replacing `python3 emtrey.py -i sam -o psl -m -t T`
 * (emtrey.py:31-193, called at Mando.py:336-341): one PSL line per mapped SAM record, input order, with
 * the accuracy / cs / read-sequence columns when mando_mode != 0.  threads <= 0: all cores. */
int mando_sam_to_psl(const char *sam_path, const char *psl_path, int32_t mando_mode, int32_t threads,
                     int64_t *n_records);
/* The same conversion on the ctx's GPU (sam_kernel.hip: one wave per record, two launches), byte-identical
 * to mando_sam_to_psl; MANDO_E_ARG where emtrey raises, MANDO_E_UNSUPPORTED for a record of more than
 * 1,024 columns or an accuracy outside [1e-8, 1e9]. */
int mando_sam_to_psl_device(mando_ctx *ctx, const char *sam_path, const char *psl_path, int32_t mando_mode,
                            int64_t *n_records);

/* clean_psl (SpliceDefineConsensus.py:14-92, called at Mando.py:343): target gaps < 10 nt merged into
 * their blocks; primary != 0 keeps only the first line per read name. */
int mando_clean_psl(const char *in_path, const char *out_path, int32_t primary, int64_t *n_records);

/* Module F, filterIsoforms.py arguments (:19-47) */
typedef struct {
    double minimum_ratio;          /* -r */
    double minimum_reads;          /* -R */
    double internal_ratio;         /* -n */
    double Acutoff;                /* -A */
    int32_t overhangs[4];          /* -O "a,b,c,d" */
    int32_t splice_window;         /* -s */
    int32_t downstream_buffer;     /* -d */
    int32_t minimum_isoform_length; /* -I */
    int32_t multi_exon_only;       /* -M */
    int32_t threads;               /* -t (chromosomes in parallel; <= 0: all cores) */
} mando_filter_params;

void mando_filter_default_params(mando_filter_params *p);

/* filter_sam (filterIsoforms.py:280-296): drops secondary (256) and supplementary (2048) records. */
int mando_filter_sam(const char *sam_path, const char *out_path, int64_t *n_kept);

/* Per-chromosome isoform filters of module F (filterIsoforms.py:81-278, :310-410, :456-510) on the
 * clean PSL of the consensi's alignments: absolute filters, relative expression, polyA extension and
 * containment.  Writes the kept consensi (FASTA), their PSL lines and, if reasons_path, the filter
 * reasons (what the reference writes to stderr).  whitelist_bed: polyAWhiteList.bed (or NULL). */
int mando_filter_isoforms(const mando_filter_params *p, const char *isoform_fasta, const char *genome_fasta,
                          const char *clean_psl, const char *whitelist_bed, const char *out_fasta,
                          const char *out_psl, const char *reasons_path, int64_t *n_kept);
/* mando_filter_isoforms with look_for_contained_isoforms' candidate search (filterIsoforms.py:125-278) on the
 * GPU of ctx (modf_kernel.hip: one thread per isoform, all chromosomes in one launch); the parse, the
 * counts, the polyA test and the reason texts are the host path's, and so are the outputs, byte for byte. */
int mando_filter_isoforms_device(mando_ctx *ctx, const mando_filter_params *P, const char *isoform_fasta,
                                 const char *genome_fasta, const char *clean_psl, const char *whitelist_bed,
                                 const char *out_fasta, const char *out_psl, const char *reasons_path,
                                 int64_t *n_kept);

/* psl_to_gtf (filterIsoforms.py:413-433). */
int mando_psl_to_gtf(const char *psl_path, const char *gtf_path);

/* Module Q, assignReadsToIsoforms.py:27-105: per-sample read counts and TPM of
 * every isoform of the filtered PSL, from reads2isoforms.txt and the read files (FASTA/FASTQ, gz). */
int mando_quantify(const char *const *fasta_paths, int32_t n_fasta, const char *r2i_path,
                   const char *filtered_psl, const char *out_quant, const char *out_tpm);
/* mando_quantify with its two joins on the GPU of ctx (quant_kernel.hip): read name -> read file for every
 * reads2isoforms.txt line and isoform -> its lines' files for every filtered isoform, as radix sorts and
 * binary searches over 64-bit name hashes with every hit confirmed byte for byte.  The host reads the
 * files and writes the tables exactly as mando_quantify does (same outputs, same errors). */
int mando_quantify_device(mando_ctx *ctx, const char *const *fasta_paths, int32_t n_fasta, const char *r2i_path,
                          const char *filtered_psl, const char *out_quant, const char *out_tpm);

#ifdef __cplusplus
}
#endif

#endif /* MANDO_H */
