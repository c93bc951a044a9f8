// cluster.cpp — host side of the D module's per-locus read clustering: reads the locus PSL files
// (tmp_SS/*.psl) into one buffer, hands them to the GPU kernels (cluster_kernel.hip: one wave per
// locus for collect_reads, find_peaks, characterize_splicing_event, sort_reads_into_splice_junctions,
// define_start_end_sites and the determine_consensus subsample, SpliceDefineConsensus.py:107-931),
// and flattens their per-locus results into the mando_cluster_view arrays.  There is no CPU
// clustering path: the restatement in oracle/cluster_ref.cpp is the tests' checker only.
//
// Also mando_pack_segments, the byte gather the D driver uses to build the orientation / POA inputs
// and the output files.
#include "threads.h"
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <cerrno>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <sys/mman.h>
#include <thread>
#include <vector>

#include <hip/hip_runtime.h>

#include "../../include/mando.h"
#include "cluster_gpu.h"
#include "internal.h"
#include "revcomp.h"

using std::string;
using std::vector;

namespace {

// one copy stream per device for the locus text (sub-batched calls: the clustering kernels of the
// first loci run on the context's stream while the rest of the text is still being copied)
// Orientation of one batch of clustered loci (their isoforms' subsamples, in the order the result lists
// them: loci, isoforms, draw order; the first read of each group is its reference), as the D driver
// would run it after the whole call (SDC:895-907): H hits per read, re-run at 8 when a read has more;
// H = 0 when even 8 do not hold them (the caller then orients and reports it).
struct OrientPart {
    vector<int8_t> hits;
    vector<int32_t> nh;
    int H = 0;
};
int orient_part(mando_ctx *octx, const void *d_text, int64_t text_len, const mando::cl::ClusterOut &q, int h0,
                OrientPart &op) {
    vector<int64_t> off, grp{0};
    vector<int32_t> len;
    for (size_t i = 0; i < q.status.size(); ++i) {
        if (q.status[i] != mando::cl::kOk) continue;
        const int64_t base = q.rec_base[i];
        const auto &ns = q.iso_nsub[i];
        const auto &ss = q.sub[i];
        size_t ps = 0;
        for (size_t k = 0; k < ns.size(); ++k) {
            for (int32_t t = 0; t < ns[k]; ++t) {
                const int64_t r = base + ss[ps++];
                off.push_back(q.rec_text[(size_t)(4 * r + 2)]);
                len.push_back((int32_t)q.rec_text[(size_t)(4 * r + 3)]);
            }
            grp.push_back((int64_t)off.size());
        }
    }
    const int64_t n = (int64_t)off.size(), ng = (int64_t)grp.size() - 1;
    for (int H = std::max(1, std::min(8, h0));; H = 8) {
        op.hits.assign((size_t)std::max<int64_t>(n, 1) * (size_t)H, 0);
        op.nh.assign((size_t)std::max<int64_t>(n, 1), 0);
        const int rc = mando_orient_segments(octx, static_cast<const uint8_t *>(d_text), text_len, off.data(),
                                             len.data(), grp.data(), ng, op.hits.data(), H, op.nh.data());
        if (rc != MANDO_OK) return rc;
        int32_t mx = 0;
        for (int64_t r = 0; r < n; ++r) mx = std::max(mx, op.nh[(size_t)r]);
        op.hits.resize((size_t)n * (size_t)H);
        op.nh.resize((size_t)n);
        if (mx <= H) {
            op.H = H;
            return MANDO_OK;
        }
        if (H >= 8) {
            op.H = 0;
            return MANDO_OK;
        }
    }
}

// the copy streams live until the library is unloaded (each owns a hardware queue: handed back then)
struct CopyStreams {
    std::vector<hipStream_t> s;
    ~CopyStreams() {
        for (hipStream_t x : s)
            if (x) (void)hipStreamDestroy(x);
    }
};

hipStream_t copy_stream(int device) {
    static std::mutex mu;
    static CopyStreams holder;
    std::vector<hipStream_t> &streams = holder.s;
    std::lock_guard<std::mutex> g(mu);
    if ((int)streams.size() <= device) streams.resize((size_t)device + 1, nullptr);
    if (!streams[(size_t)device]) {
        int cur = 0;
        (void)hipGetDevice(&cur);
        (void)hipSetDevice(device);
        if (mando::create_stream(&streams[(size_t)device]) != hipSuccess)
            streams[(size_t)device] = nullptr;
        (void)hipSetDevice(cur);
    }
    return streams[(size_t)device];
}

// Host buffers for the locus text, kept for reuse: page-locked (hipHostMalloc, pinned once, reused
// by later calls), so the readers fread straight into DMA-able memory and the piecewise copies to the
// device run on the copy engine, asynchronously, instead of a host staging copy plus a blit kernel
// that competes with the POA grids for CU slots (2 MB-aligned pageable buffers with transparent huge
// pages only when page-locking fails).  Round 2 recorded stale bytes with
// reused page-locked buffers; that change was made together with moving the device text off the
// stream-ordered pool, whose recycled buffers are the measured cause (cluster_kernel.hip,
// tools/stale_probe.hip): a reused pinned source (scenario A) and a reused pinned D2H target (G, the
// K2 output path) gave no stale byte in 15 refills each; tests/test_cluster_gpu.py
// test_repeated_calls_reuse_buffers stays the regression test.
struct HostBuf {
    char *p = nullptr;
    size_t cap = 0;
    bool pinned = false;  // hipHostMalloc (else posix_memalign + THP: the fallback)
};
struct PinnedPool {
    // page-locked bytes the pool keeps between calls: the four largest buffers of a config-4 run
    // (8 GiB chunks) fit, more is returned to the system
    static constexpr size_t kKeepPinned = size_t(40) << 30;
    std::mutex mu;
    std::vector<HostBuf> free_list;
    HostBuf acquire(size_t need) {
        {
            std::lock_guard<std::mutex> g(mu);
            size_t best = (size_t)-1;
            for (size_t i = 0; i < free_list.size(); ++i)
                if (free_list[i].cap >= need && (best == (size_t)-1 || free_list[i].cap < free_list[best].cap))
                    best = i;
            if (best != (size_t)-1) {
                const HostBuf e = free_list[best];
                free_list.erase(free_list.begin() + (ptrdiff_t)best);
                return e;
            }
        }
        constexpr size_t kStep = size_t(256) << 20;
        HostBuf b;
        b.cap = (std::max<size_t>(need, 1) + kStep - 1) / kStep * kStep;
        void *p = nullptr;
        if (hipHostMalloc(&p, b.cap, hipHostMallocDefault) == hipSuccess) {
            b.p = static_cast<char *>(p);
            b.pinned = true;
            return b;
        }
        (void)hipGetLastError();  // page-locking failed (host memory limits): a pageable buffer instead
        p = nullptr;
        if (posix_memalign(&p, size_t(2) << 20, b.cap) != 0) return HostBuf{};
        (void)madvise(p, b.cap, MADV_HUGEPAGE);
        b.p = static_cast<char *>(p);
        return b;
    }
    static void free_buf(const HostBuf &b) {
        if (b.pinned) (void)hipHostFree(b.p);
        else free(b.p);
    }
    void release(const HostBuf &b) {
        if (!b.p) return;
        std::lock_guard<std::mutex> g(mu);
        free_list.push_back(b);
        // keep the four largest buffers (two chunks in flight, plus the previous call's two when their
        // release -- a background thread in the D driver -- comes late: a free() while the next call's
        // chunks are being read would otherwise recur), and at most kKeepPinned page-locked bytes
        auto pinned_bytes = [&] {
            size_t t = 0;
            for (const HostBuf &x : free_list) t += x.pinned ? x.cap : 0;
            return t;
        };
        while (free_list.size() > 4 || pinned_bytes() > kKeepPinned) {
            auto it = std::min_element(free_list.begin(), free_list.end(),
                                       [](const HostBuf &a, const HostBuf &b) { return a.cap < b.cap; });
            if (free_list.size() <= 4) {  // over the pinned cap: drop the smallest page-locked one
                it = free_list.end();
                for (auto j = free_list.begin(); j != free_list.end(); ++j)
                    if (j->pinned && (it == free_list.end() || j->cap < it->cap)) it = j;
            }
            free_buf(*it);
            free_list.erase(it);
        }
    }
};
PinnedPool &pool() {
    static PinnedPool *p = new PinnedPool();  // never destroyed: buffers live until process exit
    return *p;
}

}  // namespace

struct mando_cluster_result {
    // all locus files, in a buffer from the pool (returned to it on destruction)
    char *text_p = nullptr;
    HostBuf text_buf;
    size_t text_len = 0;
    vector<int64_t> name_off, seq_off, rec_locus;
    vector<int32_t> name_len, seq_len;
    vector<int64_t> iso_locus, mem_off, mem, sub_off, sub;
    vector<int64_t> peak_locus, peak_start, peak_end;
    vector<char> peak_type, peak_side;
    vector<double> peak_prop;
    vector<int32_t> locus_status;
    // orientation of the subsampled reads (orient_ctx): sub.size() x o_H strands, hits per read
    int32_t o_H = 0;
    vector<int8_t> o_hits;
    vector<int32_t> o_nh;
    // the same text on the device (freed stream-ordered on the clustering context's stream)
    mando_ctx *ctx = nullptr;
    void *d_text = nullptr;
    size_t d_cap = 0;
    ~mando_cluster_result() {
        mando::cl::release_text(ctx, d_text, d_cap);
        pool().release(text_buf);
    }
};

extern "C" {

void mando_cluster_default_params(mando_cluster_params *p) {
    if (!p) return;
    p->cutoff = 0.1;
    p->splice_site_width = 1;
    p->minimum_read_count = 2;
    p->upstream_buffer = 10;
    p->downstream_buffer = 50;
    p->junctions = "gtag,gcag,atac,ctac,ctgc,gtat";
    p->seed = 0;
    p->threads = 0;
    p->poa_subsample = 100;
    p->orient_ctx = nullptr;
    p->orient_max_hits = 4;
}

int mando_cluster_loci(mando_ctx *ctx, const mando_cluster_params *prm, const char *const *psl_paths,
                       const char *const *chroms, int64_t n_loci, const int64_t *ann_pos, const int64_t *ann_off,
                       mando_cluster_result **out) {
    if (!ctx || !prm || !out || n_loci < 0 || (n_loci > 0 && (!psl_paths || !chroms))) return MANDO_E_ARG;
    *out = nullptr;
    namespace cl = mando::cl;
    cl::ClusterIn in;
    in.n_loci = n_loci;
    in.cutoff = prm->cutoff;
    in.w = prm->splice_site_width;
    in.min_count = prm->minimum_read_count;
    in.up = prm->upstream_buffer;
    in.down = prm->downstream_buffer;
    in.sub_k = prm->poa_subsample > 0 ? prm->poa_subsample : 100;
    in.seed = prm->seed;
    if (in.w < 0 || in.up < 0 || in.down < 0)
        return mando::set_error(MANDO_E_ARG, "cluster: negative window parameter");
    if (prm->junctions) {
        string j(prm->junctions);
        size_t a = 0;
        while (true) {
            const size_t c = j.find(',', a);
            in.junctions.push_back(j.substr(a, c == string::npos ? string::npos : c - a));
            if (c == string::npos) break;
            a = c + 1;
        }
    }
    if (in.junctions.size() > 16) return mando::set_error(MANDO_E_ARG, "cluster: more than 16 junction motifs");
    auto res = std::make_unique<mando_cluster_result>();
    const bool timing = getenv("MANDO_CL_TIME") != nullptr;
    const auto t_0 = std::chrono::steady_clock::now();
    auto secs = [&]() { return std::chrono::duration<double>(std::chrono::steady_clock::now() - t_0).count(); };
    const int nth_all = prm->threads > 0 ? prm->threads : mando::usable_threads();
    int nth = (int)std::min<int64_t>(nth_all, std::max<int64_t>(1, n_loci));
    // read every locus file into one buffer: sizes first (stat, on the reader threads), then reads
    vector<int64_t> fsize((size_t)n_loci, 0), foff((size_t)n_loci + 1, 0);
    vector<int32_t> fstatus((size_t)n_loci, cl::kOk);
    {
        std::atomic<int64_t> nx{0};
        auto sizer = [&]() {
            for (int64_t i; (i = nx.fetch_add(256)) < n_loci;)
                for (int64_t k = i; k < std::min<int64_t>(n_loci, i + 256); ++k) {
                    struct stat sb;
                    fsize[(size_t)k] = (stat(psl_paths[k], &sb) == 0 && S_ISREG(sb.st_mode)) ? (int64_t)sb.st_size : -1;
                }
        };
        vector<std::thread> th;
        for (int t = 1; t < nth; ++t) th.emplace_back(sizer);
        sizer();
        for (auto &t : th) t.join();
    }
    const double t_size = secs();
    for (int64_t i = 0; i < n_loci; ++i) foff[(size_t)i + 1] = foff[(size_t)i] + std::max<int64_t>(0, fsize[(size_t)i]);
    res->text_len = (size_t)foff[(size_t)n_loci];
    const double t_acq0 = secs();
    res->text_buf = pool().acquire(res->text_len + 64);
    const double t_acq = secs() - t_acq0;
    res->text_p = res->text_buf.p;
    if (!res->text_p) return mando::set_error(MANDO_E_NOMEM, "cluster: host text buffer");
    // device copy of the text, filled piecewise while later files are still being read
    hipStream_t stream = cl::cluster_stream(ctx);
    size_t d_cap = 0;
    void *d_text = hipSetDevice(mando::ctx_device(ctx)) == hipSuccess
                       ? mando::cl::acquire_text(ctx, res->text_len + 64, d_cap) : nullptr;
    if (!d_text) return mando::set_error(MANDO_E_NOMEM, "cluster: device text buffer");
    const double t_dacq = secs() - t_acq0 - t_acq;
    res->ctx = ctx;
    res->d_text = d_text;
    res->d_cap = d_cap;
    // Files are read in pieces of at most kReadPiece bytes, pieces dealt to the reader threads in file
    // order: a few large loci (config 2: seven ~22 MB files) keep every reader busy instead of one
    // thread per file.  The thread that finishes a locus's last piece marks it done.
    constexpr int64_t kReadPiece = int64_t(4) << 20;
    vector<int64_t> pfirst((size_t)n_loci + 1, 0);
    for (int64_t i = 0; i < n_loci; ++i)
        pfirst[(size_t)i + 1] = pfirst[(size_t)i] + std::max<int64_t>(1, (fsize[(size_t)i] + kReadPiece - 1) / kReadPiece);
    const int64_t n_pieces = pfirst[(size_t)n_loci];
    nth = (int)std::min<int64_t>(nth_all, std::max<int64_t>(1, n_pieces));
    std::atomic<int64_t> next{0};
    vector<std::atomic<uint8_t>> done((size_t)n_loci), ioerr((size_t)n_loci);
    vector<std::atomic<int32_t>> left((size_t)n_loci);
    for (int64_t i = 0; i < n_loci; ++i) {
        done[(size_t)i].store(0);
        ioerr[(size_t)i].store(0);
        left[(size_t)i].store((int32_t)(pfirst[(size_t)i + 1] - pfirst[(size_t)i]));
    }
    std::mutex mu;
    std::condition_variable cv;
    std::atomic<int64_t> reader_ns{0};
    auto reader = [&]() {
        const auto r0 = std::chrono::steady_clock::now();
        struct Busy {  // this reader's time, added at its end
            std::atomic<int64_t> &sum;
            std::chrono::steady_clock::time_point t0;
            ~Busy() {
                sum.fetch_add(std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count());
            }
        } busy{reader_ns, r0};
        while (true) {
            const int64_t p = next.fetch_add(1);
            if (p >= n_pieces) break;
            const size_t i = (size_t)(std::upper_bound(pfirst.begin(), pfirst.end(), p) - pfirst.begin() - 1);
            bool ok = fsize[i] >= 0;
            if (ok) {
                const int64_t a = (p - pfirst[i]) * kReadPiece, len = std::min(kReadPiece, fsize[i] - a);
                const int fd = open(psl_paths[i], O_RDONLY | O_CLOEXEC);
                ok = fd >= 0;
                for (int64_t got = 0; ok && got < len;) {
                    const ssize_t r = pread(fd, res->text_p + foff[i] + a + got, (size_t)(len - got), (off_t)(a + got));
                    if (r < 0 && errno == EINTR) continue;
                    ok = r > 0;
                    got += r > 0 ? r : 0;
                }
                if (fd >= 0) close(fd);
            }
            if (!ok) ioerr[i].store(1, std::memory_order_relaxed);
            // acq_rel: the last piece's thread sees every other piece's bytes and error flag
            if (left[i].fetch_sub(1, std::memory_order_acq_rel) == 1) {
                if (ioerr[i].load(std::memory_order_relaxed)) fstatus[i] = cl::kIO;
                done[i].store(1, std::memory_order_release);
                cv.notify_one();
            }
        }
    };
    in.text = res->text_p;
    in.d_text = d_text;
    in.text_len = (int64_t)res->text_len;
    in.foff = foff.data();
    in.fstatus = fstatus.data();
    in.chroms = chroms;
    in.ann_pos = ann_pos;
    in.ann_off = ann_off;
    // Sub-batches: the loci split into up to four byte-balanced ranges, each clustered (K1, K2) on the
    // context's stream by a worker thread as soon as its text is on the device, while the readers and the
    // copy stream bring in the rest -- the kernels of the first ranges run under the reading and the
    // copy instead of after them.  Results are the same: every locus replays its own RNG state.
    hipStream_t cstream = stream;
    int nsub = (n_loci >= 1024 && res->text_len >= (size_t(256) << 20)) ? 4 : 1;
    if (const char *ev = getenv("MANDO_CL_SUB")) nsub = std::max(1, std::min(16, atoi(ev)));
    if (nsub > 1 && !(cstream = copy_stream(mando::ctx_device(ctx)))) {
        cstream = stream;
        nsub = 1;
    }
    vector<int64_t> bounds((size_t)nsub + 1, n_loci);
    bounds[0] = 0;
    for (int k = 1; k < nsub; ++k)
        bounds[(size_t)k] = (int64_t)(std::lower_bound(foff.begin(), foff.begin() + n_loci,
                                                       (int64_t)((double)res->text_len * k / nsub)) - foff.begin());
    for (int k = 1; k <= nsub; ++k) bounds[(size_t)k] = std::max(bounds[(size_t)k], bounds[(size_t)k - 1]);
    vector<cl::ClusterOut> parts((size_t)nsub);
    vector<hipEvent_t> ready((size_t)nsub, nullptr);
    vector<int> part_rc((size_t)nsub, MANDO_OK);
    int copied = 0;  // sub-batches whose text has been copied (events recorded)
    std::mutex pmu;
    std::condition_variable pcv;
    bool copy_failed = false;
    int clustered = 0;  // sub-batches clustered (the orientation worker follows)
    bool cluster_failed = false;
    auto worker = [&]() {
        for (int k = 0; k < nsub; ++k) {
            {
                std::unique_lock<std::mutex> lk(pmu);
                pcv.wait(lk, [&] { return copied > k || copy_failed; });
                if (copied <= k) return;
            }
            cl::ClusterIn ik = in;
            const int64_t a = bounds[(size_t)k], b = bounds[(size_t)k + 1];
            ik.n_loci = b - a;
            ik.foff = in.foff + a;
            ik.fstatus = in.fstatus + a;
            ik.chroms = in.chroms + a;
            if (in.ann_off) ik.ann_off = in.ann_off + 4 * a;
            ik.ready = ready[(size_t)k];
            part_rc[(size_t)k] = cl::cluster_gpu(ctx, ik, parts[(size_t)k]);
            std::lock_guard<std::mutex> g(pmu);
            if (part_rc[(size_t)k] != MANDO_OK) {
                cluster_failed = true;
                pcv.notify_all();
                return;
            }
            ++clustered;
            pcv.notify_all();
        }
    };
    // orientation of each sub-batch on prm->orient_ctx as soon as it is clustered, beside the
    // clustering of the next one
    mando_ctx *octx = prm->orient_ctx;
    vector<OrientPart> oparts((size_t)nsub);
    vector<int> orient_rc((size_t)nsub, MANDO_OK);
    auto orienter = [&]() {
        for (int k = 0; k < nsub; ++k) {
            {
                std::unique_lock<std::mutex> lk(pmu);
                pcv.wait(lk, [&] { return clustered > k || cluster_failed; });
                if (clustered <= k) return;
            }
            orient_rc[(size_t)k] = orient_part(octx, d_text, (int64_t)res->text_len, parts[(size_t)k],
                                               prm->orient_max_hits, oparts[(size_t)k]);
            if (orient_rc[(size_t)k] != MANDO_OK) return;
        }
    };
    int copy_rc = MANDO_OK;
    double copy_call_s = 0;  // (MANDO_CL_TIME: time inside the copy calls)
    {
        vector<std::thread> th;
        for (int t = 0; t < nth; ++t) th.emplace_back(reader);
        std::thread wk, ow;
        if (nsub > 1) wk = std::thread(worker);
        if (nsub > 1 && octx) ow = std::thread(orienter);
        // copy the completed prefix in >= 64 MB pieces as the readers advance
        constexpr int64_t kPiece = int64_t(64) << 20;
        int64_t upto = 0, sent = 0;
        while (upto < n_loci) {
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait_for(lk, std::chrono::microseconds(200),
                            [&] { return done[(size_t)upto].load(std::memory_order_acquire) != 0; });
            }
            while (upto < n_loci && done[(size_t)upto].load(std::memory_order_acquire)) ++upto;
            const int64_t avail = foff[(size_t)upto];
            // a sub-batch's last file read: its text goes out now, whatever the piece size
            const bool edge = nsub > 1 && copied < nsub && upto >= bounds[(size_t)copied + 1];
            if (avail - sent >= kPiece || (edge && avail > sent) || (upto == n_loci && avail > sent)) {
                const auto tc0 = std::chrono::steady_clock::now();
                const hipError_t ce = hipMemcpyAsync((char *)d_text + sent, res->text_p + sent, (size_t)(avail - sent),
                                                     hipMemcpyHostToDevice, cstream);
                copy_call_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - tc0).count();
                if (ce != hipSuccess) {
                    copy_rc = mando::set_error(MANDO_E_HIP, "cluster: text copy to the device");
                    break;
                }
                sent = avail;
            }
            while (nsub > 1 && copied < nsub && upto >= bounds[(size_t)copied + 1] && sent >= foff[(size_t)bounds[(size_t)copied + 1]]) {
                hipEvent_t e = nullptr;
                if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess ||
                    hipEventRecord(e, cstream) != hipSuccess) {
                    copy_rc = mando::set_error(MANDO_E_HIP, "cluster: copy event");
                    break;
                }
                ready[(size_t)copied] = e;
                std::lock_guard<std::mutex> g(pmu);
                ++copied;
                pcv.notify_all();
            }
            if (copy_rc != MANDO_OK) break;
        }
        if (copy_rc != MANDO_OK) {
            next.store(n_pieces);  // stop the readers
            std::lock_guard<std::mutex> g(pmu);
            copy_failed = true;
            pcv.notify_all();
        }
        for (auto &t : th) t.join();
        if (wk.joinable()) wk.join();
        if (ow.joinable()) {  // a clustering worker that stopped early releases the orientation worker
            {
                std::lock_guard<std::mutex> g(pmu);
                if (clustered < nsub) cluster_failed = true;
                pcv.notify_all();
            }
            ow.join();
        }
    }
    for (hipEvent_t e : ready)
        if (e) (void)hipEventDestroy(e);
    if (copy_rc != MANDO_OK) return copy_rc;
    const double t_read = secs();
    cl::ClusterOut o;
    if (nsub == 1) {
        const int rc = cl::cluster_gpu(ctx, in, o);
        if (rc != MANDO_OK) return rc;
        if (octx) {
            const int orc = orient_part(octx, d_text, (int64_t)res->text_len, o, prm->orient_max_hits, oparts[0]);
            if (orc != MANDO_OK) return orc;
        }
    } else {
        for (int k = 0; k < nsub; ++k)
            if (part_rc[(size_t)k] != MANDO_OK) return part_rc[(size_t)k];
        for (int k = 0; k < nsub && octx; ++k)
            if (orient_rc[(size_t)k] != MANDO_OK) return orient_rc[(size_t)k];
        // the sub-batches' outputs, concatenated in locus order (record bases shifted)
        o.rec_base.assign(1, 0);
        for (int k = 0; k < nsub; ++k) {
            cl::ClusterOut &q = parts[(size_t)k];
            const int64_t base = o.rec_base.back();
            o.status.insert(o.status.end(), q.status.begin(), q.status.end());
            o.n_rec.insert(o.n_rec.end(), q.n_rec.begin(), q.n_rec.end());
            for (size_t i = 1; i < q.rec_base.size(); ++i) o.rec_base.push_back(base + q.rec_base[i]);
            o.rec_text.insert(o.rec_text.end(), q.rec_text.begin(), q.rec_text.end());
            auto mv = [](auto &dst, auto &src) {
                for (auto &x : src) dst.push_back(std::move(x));
            };
            mv(o.peaks, q.peaks);
            mv(o.iso_nmem, q.iso_nmem);
            mv(o.mem, q.mem);
            mv(o.iso_nsub, q.iso_nsub);
            mv(o.sub, q.sub);
        }
    }
    const double t_gpu = secs();
    // flatten: records in locus order, isoforms in locus then IsoDict order
    const int64_t nr = o.rec_base[(size_t)n_loci];
    res->name_off.resize((size_t)nr);
    res->name_len.resize((size_t)nr);
    res->seq_off.resize((size_t)nr);
    res->seq_len.resize((size_t)nr);
    res->rec_locus.resize((size_t)nr);
    for (int64_t i = 0; i < n_loci; ++i)
        for (int64_t r = o.rec_base[(size_t)i]; r < o.rec_base[(size_t)i + 1]; ++r) {
            const int64_t *t = o.rec_text.data() + 4 * r;
            res->name_off[(size_t)r] = t[0];
            res->name_len[(size_t)r] = (int32_t)t[1];
            res->seq_off[(size_t)r] = t[2];
            res->seq_len[(size_t)r] = (int32_t)t[3];
            res->rec_locus[(size_t)r] = i;
        }
    // exact sizes first: the per-locus appends below then never reallocate
    size_t n_iso = 0, n_mem = 0, n_sub = 0, n_pk = 0;
    for (int64_t i = 0; i < n_loci; ++i) {
        if (o.status[(size_t)i] != cl::kOk) continue;
        n_iso += o.iso_nmem[(size_t)i].size();
        n_mem += o.mem[(size_t)i].size();
        n_sub += o.sub[(size_t)i].size();
        n_pk += o.peaks[(size_t)i].size();
    }
    res->iso_locus.reserve(n_iso);
    res->mem_off.reserve(n_iso + 1);
    res->sub_off.reserve(n_iso + 1);
    res->mem.reserve(n_mem);
    res->sub.reserve(n_sub);
    res->peak_locus.reserve(n_pk);
    res->peak_start.reserve(n_pk);
    res->peak_end.reserve(n_pk);
    res->peak_type.reserve(n_pk);
    res->peak_side.reserve(n_pk);
    res->peak_prop.reserve(n_pk);
    res->mem_off.push_back(0);
    res->sub_off.push_back(0);
    res->locus_status = o.status;
    for (int64_t i = 0; i < n_loci; ++i) {
        if (o.status[(size_t)i] != cl::kOk) continue;
        const int64_t base = o.rec_base[(size_t)i];
        const auto &nm = o.iso_nmem[(size_t)i], &ns = o.iso_nsub[(size_t)i];
        const auto &mm = o.mem[(size_t)i], &ss = o.sub[(size_t)i];
        size_t pm = 0, ps = 0;
        for (size_t k = 0; k < nm.size(); ++k) {
            res->iso_locus.push_back(i);
            for (int32_t q = 0; q < nm[k]; ++q) res->mem.push_back(base + mm[pm++]);
            res->mem_off.push_back((int64_t)res->mem.size());
            for (int32_t q = 0; q < ns[k]; ++q) res->sub.push_back(base + ss[ps++]);
            res->sub_off.push_back((int64_t)res->sub.size());
        }
        for (const cl::Peak &pk : o.peaks[(size_t)i]) {
            res->peak_locus.push_back(i);
            res->peak_start.push_back(pk.start);
            res->peak_end.push_back(pk.end);
            res->peak_type.push_back(pk.type);
            res->peak_side.push_back(pk.side);
            res->peak_prop.push_back(pk.prop);
        }
    }
    if (octx) {  // the sub-batches' hit strands, in the result's subsample order, at one width
        int H = 0;
        size_t rows = 0;
        for (const OrientPart &q : oparts) {
            H = (q.H == 0 || H < 0) ? -1 : std::max(H, q.H);
            rows += q.nh.size();
        }
        if (H > 0 && rows == res->sub.size()) {
            res->o_H = H;
            res->o_hits.assign(rows * (size_t)H, 0);
            res->o_nh.resize(rows);
            size_t r0 = 0;
            for (const OrientPart &q : oparts) {
                for (size_t r = 0; r < q.nh.size(); ++r) {
                    res->o_nh[r0 + r] = q.nh[r];
                    memcpy(&res->o_hits[(r0 + r) * (size_t)H], &q.hits[r * (size_t)q.H], (size_t)q.H);
                }
                r0 += q.nh.size();
            }
        }
    }
    if (timing)
        fprintf(stderr, "[cluster] %lld loci, %.1f MB: sizes %.3f s, read + copy %.3f s (buffers %.3f + %.3f s, "
                        "readers %.3f s each on %d threads, copy calls %.3f s), kernels %.3f s, flatten %.3f s\n",
                (long long)n_loci, res->text_len / 1e6, t_size, t_read - t_size, t_acq, t_dacq,
                reader_ns.load() * 1e-9 / std::max(1, nth), nth, copy_call_s, t_gpu - t_read, secs() - t_gpu);
    *out = res.release();
    return MANDO_OK;
}

int mando_cluster_view_get(const mando_cluster_result *r, mando_cluster_view *v) {
    if (!r || !v) return MANDO_E_ARG;
    v->n_loci = (int64_t)r->locus_status.size();
    v->locus_status = r->locus_status.data();
    v->text = r->text_p;
    v->text_len = (int64_t)r->text_len;
    v->n_records = (int64_t)r->name_off.size();
    v->name_off = r->name_off.data();
    v->name_len = r->name_len.data();
    v->seq_off = r->seq_off.data();
    v->seq_len = r->seq_len.data();
    v->rec_locus = r->rec_locus.data();
    v->n_isoforms = (int64_t)r->iso_locus.size();
    v->iso_locus = r->iso_locus.data();
    v->mem_off = r->mem_off.data();
    v->mem = r->mem.data();
    v->sub_off = r->sub_off.data();
    v->sub = r->sub.data();
    v->n_peaks = (int64_t)r->peak_locus.size();
    v->peak_locus = r->peak_locus.data();
    v->peak_start = r->peak_start.data();
    v->peak_end = r->peak_end.data();
    v->peak_type = r->peak_type.data();
    v->peak_side = r->peak_side.data();
    v->peak_prop = r->peak_prop.data();
    v->orient_max_hits = r->o_H;
    v->orient_hits = r->o_hits.data();
    v->orient_n_hits = r->o_nh.data();
    return MANDO_OK;
}

void mando_cluster_free(mando_cluster_result *r) { delete r; }

int mando_cluster_device_text(const mando_cluster_result *r, const uint8_t **d_text, int64_t *len) {
    if (!r || !d_text || !len) return MANDO_E_ARG;
    *d_text = static_cast<const uint8_t *>(r->d_text);
    *len = (int64_t)r->text_len;
    return MANDO_OK;
}

// Host helper of the D driver: concatenates n byte segments into out (at out_off[i], caller-computed
// exclusive prefix sums of lens).  Segment i is src[sel[i]] + starts[i], lens[i] bytes, reverse-
// complemented like mappy.revcomp (revcomp.h) when rc && rc[i].  Threaded.
int mando_pack_segments(const uint8_t *const *src, const int8_t *sel, const int64_t *starts, const int64_t *lens,
                        const int8_t *rc, int64_t n, uint8_t *out, const int64_t *out_off, int32_t threads) {
    if (n < 0 || (n > 0 && (!src || !starts || !lens || !out || !out_off))) return MANDO_E_ARG;
    const mando::CompTable &comp = mando::comp_table();
    int nth = threads > 0 ? threads : mando::usable_threads();
    nth = (int)std::min<int64_t>(nth, std::max<int64_t>(1, n / 256));
    auto work = [&](int64_t a, int64_t b) {
        for (int64_t i = a; i < b; ++i) {
            const uint8_t *s = src[sel ? sel[i] : 0] + starts[i];
            uint8_t *d = out + out_off[i];
            const int64_t L = lens[i];
            if (rc && rc[i]) {
                for (int64_t k = 0; k < L; ++k) d[k] = comp.t[s[L - 1 - k]];
            } else {
                memcpy(d, s, (size_t)L);
            }
        }
    };
    if (nth <= 1) {
        work(0, n);
    } else {
        vector<std::thread> th;
        const int64_t chunk = (n + nth - 1) / nth;
        for (int t = 0; t < nth; ++t) {
            const int64_t a = t * chunk, b = std::min<int64_t>(n, a + chunk);
            if (a < b) th.emplace_back(work, a, b);
        }
        for (auto &x : th) x.join();
    }
    return MANDO_OK;
}

}  // extern "C"
