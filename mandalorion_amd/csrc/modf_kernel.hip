// modf_kernel.hip — module F's containment search on the GPU:
// look_for_contained_isoforms (filterIsoforms.py:125-278) for every isoform that passed the absolute and
// relative-expression filters, all chromosomes in one launch.  The parse, the counts, the polyA test and the
// reason texts stay the host path's (module_f.cpp, modf.h: the same chr_stage1 / chr_stage3 run on both
// sides), so the outputs are the host path's byte for byte (tests/test_modf_gpu.py).
//
// One thread per isoform k.  Its candidates are the same-direction isoforms whose merged blocks (± the
// splice window) overlap k's span: a binary search over the chromosome's candidates sorted by their first
// merged start, bounded by the longest merged span, as on the host.  For each candidate: does it reach 10
// bases into k's putative polyA window (extend), and does one merged interval cover each of k's trimmed
// blocks (status).  For every status member other than k, in any order, the junction test of the
// reference's `dd` table -- for a base1 position, the window of the member's LAST junction whose base1
// window holds it -- and the member's verdict (zero abundance, internal ratio, near-identical ends); the
// member with the smallest name among those with a verdict is the one the reference's name-ordered loop
// stops at.  Without any non-empty trimmed block the reference's status is every parsed isoform of the
// chromosome, and so it is here.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <numeric>
#include <string>
#include <vector>

#include "internal.h"
#include "modf.h"

namespace mando {
namespace modfk {

__device__ __forceinline__ int64_t imin(int64_t a, int64_t b) { return a < b ? a : b; }
__device__ __forceinline__ int64_t imax(int64_t a, int64_t b) { return a > b ? a : b; }
__device__ __forceinline__ int64_t iabs(int64_t a) { return a < 0 ? -a : a; }

struct Args {
    // per isoform (global index over all chromosomes)
    const int64_t *co;    // block coordinates, flat
    const int64_t *coff;  // first coordinate
    const int32_t *clen;  // coordinates (2 x blocks)
    const int64_t *elo, *ehi;  // merged intervals, flat
    const int64_t *eoff;
    const int32_t *elen;
    const int8_t *dir;  // 0 '+', 1 '-'
    const int64_t *ab;
    const int32_t *rank;  // name order within the chromosome
    // per chromosome and direction (2c + d): candidates by first merged start, and their longest span
    const int32_t *cand;
    const int64_t *cand_off;
    const int32_t *cand_len;
    const int64_t *maxspan;
    // per chromosome: every parsed isoform
    const int32_t *listed;
    const int64_t *listed_off;
    const int32_t *listed_len;
    // work: isoform and chromosome of each kept1 entry
    const int32_t *work_g, *work_c;
    int64_t n_work;
    int32_t sw;
    int64_t dbuf;
    double internal_ratio;
    // outputs
    int64_t *n_status, *n_extend;
    int32_t *ext_first, *trig, *kind;
};

__device__ __forceinline__ int64_t ivs_count(const Args &A, int32_t x, int64_t s, int64_t e) {
    int64_t n = 0;
    const int64_t o = A.eoff[x];
    for (int32_t k = 0; k < A.elen[x]; ++k) n += imax(0, imin(e, A.ehi[o + k]) - imax(s, A.elo[o + k]));
    return n;
}

// [s, e) inside the merged interval with the largest start <= s
__device__ __forceinline__ bool ivs_cover(const Args &A, int32_t x, int64_t s, int64_t e) {
    const int64_t o = A.eoff[x];
    int32_t lo = 0, hi = A.elen[x];
    while (lo < hi) {
        const int32_t m = (lo + hi) >> 1;
        if (A.elo[o + m] <= s) lo = m + 1;
        else hi = m;
    }
    if (lo == 0) return false;
    return A.elo[o + lo - 1] <= s && e <= A.ehi[o + lo - 1];
}

__global__ void contain_kernel(Args A) {
    const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= A.n_work) return;
    const int32_t g = A.work_g[w], c = A.work_c[w];
    const int64_t *co = A.co + A.coff[g];
    const int32_t n = A.clen[g];
    const int d = A.dir[g];
    const int sw = A.sw;
    // trimmed coordinates: the first start +20 (clamped by its end), the last end -20 (clamped by its
    // start, for one block the trimmed start)
    const int64_t c0 = imin(co[0] + 20, co[1]);
    const int64_t cl = imax(co[n - 1] - 20, n == 2 ? c0 : co[n - 2]);
    auto cc = [&](int32_t q) -> int64_t { return q == 0 ? c0 : (q == n - 1 ? cl : co[q]); };
    const int64_t start = co[0], end = co[n - 1];
    const int64_t pa0 = d == 0 ? end + 3 : start - 23;
    const int64_t lo = imin(cc(0), pa0), hi = imax(cc(n - 1), pa0 + 20);
    bool any_base = false;
    for (int32_t q = 0; q + 1 < n; q += 2)
        if (cc(q) < cc(q + 1)) any_base = true;

    int64_t n_status = 0, n_extend = 0;
    int32_t ext_first = -1, ext_rank = 0x7fffffff, best = -1, best_rank = 0x7fffffff, best_kind = 0;
    // the verdict of a status member mk (0: the reference's loop goes on past it)
    auto verdict = [&](int32_t mk) {
        if (mk == g || A.rank[mk] >= best_rank) return;
        const int64_t *mc = A.co + A.coff[mk];
        const int32_t mn = A.clen[mk];
        for (int32_t jn = 1; jn + 1 < n; jn += 2) {
            bool hit = false;
            const int64_t a2lo = cc(jn + 1) - sw, a2hi = cc(jn + 1) + sw;
            for (int64_t b1 = cc(jn) - sw; b1 < cc(jn) + sw && !hit; ++b1) {
                int32_t found = -1;
                for (int32_t jm = 1; jm + 1 < mn; jm += 2)
                    if (mc[jm] - sw <= b1 && b1 < mc[jm] + sw) found = jm;
                if (found < 0) continue;
                const int64_t b2lo = mc[found + 1] - sw, b2hi = mc[found + 1] + sw;
                if (imax(a2lo, b2lo) < imin(a2hi, b2hi)) hit = true;
            }
            if (!hit) return;
        }
        int kd = 0;
        if (A.ab[mk] == 0)
            kd = 3;
        else if ((double)A.ab[g] / (double)A.ab[mk] < A.internal_ratio)
            kd = 1;
        else if (iabs(start - mc[0]) < A.dbuf && iabs(end - mc[mn - 1]) < A.dbuf && A.ab[g] < A.ab[mk])
            kd = 2;
        if (kd) {
            best = mk;
            best_rank = A.rank[mk];
            best_kind = kd;
        }
    };
    // candidates of k's direction overlapping [lo, hi)
    const int64_t co2 = A.cand_off[2 * c + d];
    const int32_t cn = A.cand_len[2 * c + d];
    const int64_t bound = lo - A.maxspan[2 * c + d] - 1;
    int32_t a = 0, b = cn;
    while (a < b) {
        const int32_t m = (a + b) >> 1;
        if (A.elo[A.eoff[A.cand[co2 + m]]] < bound) a = m + 1;
        else b = m;
    }
    for (int32_t t = a; t < cn; ++t) {
        const int32_t x = A.cand[co2 + t];
        const int64_t front = A.elo[A.eoff[x]], back = A.ehi[A.eoff[x] + A.elen[x] - 1];
        if (front >= hi) break;
        if (back <= lo) continue;
        if (ivs_count(A, x, pa0, pa0 + 20) >= 10) {
            ++n_extend;
            if (A.rank[x] < ext_rank) {
                ext_rank = A.rank[x];
                ext_first = x;
            }
        }
        if (any_base) {
            bool all = true;
            for (int32_t q = 0; q + 1 < n && all; q += 2)
                if (cc(q) < cc(q + 1) && !ivs_cover(A, x, cc(q), cc(q + 1))) all = false;
            if (all) {
                ++n_status;
                verdict(x);
            }
        }
    }
    if (!any_base) {
        const int64_t lo2 = A.listed_off[c];
        n_status = A.listed_len[c];
        for (int32_t t = 0; t < A.listed_len[c]; ++t) verdict(A.listed[lo2 + t]);
    }
    A.n_status[w] = n_status;
    A.n_extend[w] = n_extend;
    A.ext_first[w] = ext_first;
    A.trig[w] = best;
    A.kind[w] = best_kind;
}

struct Dev {
    void *p = nullptr;
    ~Dev() {
        if (p) (void)hipFree(p);
    }
    template <class T>
    int put(const std::vector<T> &v, hipStream_t s) {
        if (hipMalloc(&p, std::max<size_t>(1, v.size() * sizeof(T))) != hipSuccess) return MANDO_E_NOMEM;
        if (!v.empty() && hipMemcpyAsync(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s) != hipSuccess)
            return MANDO_E_HIP;
        return MANDO_OK;
    }
    int alloc(size_t n) { return hipMalloc(&p, n ? n : 1) == hipSuccess ? MANDO_OK : MANDO_E_NOMEM; }
    template <class T>
    T *as() const {
        return static_cast<T *>(p);
    }
};

// the ContainStage of modf.h on the GPU of ctx
int contain_device(mando_ctx *ctx, const mando_filter_params &P, const std::vector<std::vector<modf::Iso>> &isos,
                   const std::vector<modf::ChrState> &S, std::vector<std::vector<modf::Contain>> &dec) {
    const size_t nc = isos.size();
    std::vector<int64_t> gbase(nc + 1, 0);
    for (size_t c = 0; c < nc; ++c) gbase[c + 1] = gbase[c] + (int64_t)isos[c].size();
    const int64_t ng = gbase[nc];
    if (ng > INT32_MAX) return set_error(MANDO_E_UNSUPPORTED, "filter: more than 2^31 isoforms");
    std::vector<int64_t> co, coff((size_t)ng), elo, ehi, eoff((size_t)ng), ab((size_t)ng), cand_off(2 * nc),
        maxspan(2 * nc), listed_off(nc);
    std::vector<int32_t> clen((size_t)ng), elen((size_t)ng), rank((size_t)ng), cand, cand_len(2 * nc), listed,
        listed_len(nc), work_g, work_c;
    std::vector<int8_t> dir((size_t)ng);
    for (size_t c = 0; c < nc; ++c) {
        const auto &I = isos[c];
        std::vector<int32_t> ord(I.size());
        std::iota(ord.begin(), ord.end(), 0);
        std::sort(ord.begin(), ord.end(), [&](int32_t x, int32_t y) { return I[(size_t)x].name < I[(size_t)y].name; });
        for (size_t r = 0; r < ord.size(); ++r) rank[(size_t)(gbase[c] + ord[r])] = (int32_t)r;
        for (size_t i = 0; i < I.size(); ++i) {
            const size_t g = (size_t)(gbase[c] + (int64_t)i);
            if (I[i].coords.size() < 2) return set_error(MANDO_E_ARG, "filter: an isoform without blocks");
            coff[g] = (int64_t)co.size();
            clen[g] = (int32_t)I[i].coords.size();
            co.insert(co.end(), I[i].coords.begin(), I[i].coords.end());
            eoff[g] = (int64_t)elo.size();
            elen[g] = (int32_t)S[c].ext[i].size();
            for (auto &x : S[c].ext[i]) {
                elo.push_back(x.first);
                ehi.push_back(x.second);
            }
            dir[g] = I[i].dir == '-';
            ab[g] = I[i].abundance;
        }
        for (int d = 0; d < 2; ++d) {
            cand_off[2 * c + d] = (int64_t)cand.size();
            cand_len[2 * c + d] = (int32_t)S[c].bydir[d].size();
            maxspan[2 * c + d] = S[c].maxspan[d];
            for (int k : S[c].bydir[d]) cand.push_back((int32_t)(gbase[c] + k));
        }
        listed_off[c] = (int64_t)listed.size();
        listed_len[c] = (int32_t)S[c].listed.size();
        for (int k : S[c].listed) listed.push_back((int32_t)(gbase[c] + k));
        for (int k : S[c].kept1) {
            work_g.push_back((int32_t)(gbase[c] + k));
            work_c.push_back((int32_t)c);
        }
    }
    const int64_t nw = (int64_t)work_g.size();
    for (size_t c = 0; c < nc; ++c) dec[c].assign(S[c].kept1.size(), modf::Contain());
    if (nw == 0) return MANDO_OK;
    if (hipSetDevice(ctx_device(ctx)) != hipSuccess) return set_error(MANDO_E_HIP, "filter: hipSetDevice");
    hipStream_t s = ctx_stream(ctx);
    Dev d_co, d_coff, d_clen, d_elo, d_ehi, d_eoff, d_elen, d_dir, d_ab, d_rank, d_cand, d_cand_off, d_cand_len,
        d_maxspan, d_listed, d_listed_off, d_listed_len, d_wg, d_wc, d_ns, d_ne, d_ef, d_tr, d_kd;
    int rc;
    if ((rc = d_co.put(co, s)) || (rc = d_coff.put(coff, s)) || (rc = d_clen.put(clen, s)) || (rc = d_elo.put(elo, s)) ||
        (rc = d_ehi.put(ehi, s)) || (rc = d_eoff.put(eoff, s)) || (rc = d_elen.put(elen, s)) || (rc = d_dir.put(dir, s)) ||
        (rc = d_ab.put(ab, s)) || (rc = d_rank.put(rank, s)) || (rc = d_cand.put(cand, s)) ||
        (rc = d_cand_off.put(cand_off, s)) || (rc = d_cand_len.put(cand_len, s)) || (rc = d_maxspan.put(maxspan, s)) ||
        (rc = d_listed.put(listed, s)) || (rc = d_listed_off.put(listed_off, s)) ||
        (rc = d_listed_len.put(listed_len, s)) || (rc = d_wg.put(work_g, s)) || (rc = d_wc.put(work_c, s)) ||
        (rc = d_ns.alloc((size_t)nw * 8)) || (rc = d_ne.alloc((size_t)nw * 8)) || (rc = d_ef.alloc((size_t)nw * 4)) ||
        (rc = d_tr.alloc((size_t)nw * 4)) || (rc = d_kd.alloc((size_t)nw * 4)))
        return set_error(rc, "filter: device buffers");
    Args A{d_co.as<int64_t>(), d_coff.as<int64_t>(), d_clen.as<int32_t>(), d_elo.as<int64_t>(), d_ehi.as<int64_t>(),
           d_eoff.as<int64_t>(), d_elen.as<int32_t>(), d_dir.as<int8_t>(), d_ab.as<int64_t>(), d_rank.as<int32_t>(),
           d_cand.as<int32_t>(), d_cand_off.as<int64_t>(), d_cand_len.as<int32_t>(), d_maxspan.as<int64_t>(),
           d_listed.as<int32_t>(), d_listed_off.as<int64_t>(), d_listed_len.as<int32_t>(), d_wg.as<int32_t>(),
           d_wc.as<int32_t>(), nw, P.splice_window, (int64_t)P.downstream_buffer, P.internal_ratio,
           d_ns.as<int64_t>(), d_ne.as<int64_t>(), d_ef.as<int32_t>(), d_tr.as<int32_t>(), d_kd.as<int32_t>()};
    const int tpb = 256;
    hipLaunchKernelGGL(contain_kernel, dim3((unsigned)((nw + tpb - 1) / tpb)), dim3(tpb), 0, s, A);
    if (hipGetLastError() != hipSuccess) return set_error(MANDO_E_HIP, "filter: contain_kernel launch");
    std::vector<int64_t> ns((size_t)nw), ne((size_t)nw);
    std::vector<int32_t> ef((size_t)nw), tr((size_t)nw), kd((size_t)nw);
    if (hipMemcpyAsync(ns.data(), d_ns.p, (size_t)nw * 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(ne.data(), d_ne.p, (size_t)nw * 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(ef.data(), d_ef.p, (size_t)nw * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(tr.data(), d_tr.p, (size_t)nw * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(kd.data(), d_kd.p, (size_t)nw * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return set_error(MANDO_E_HIP, "filter: contain_kernel results");
    int64_t w = 0;
    for (size_t c = 0; c < nc; ++c)
        for (size_t t = 0; t < S[c].kept1.size(); ++t, ++w) {
            modf::Contain &r = dec[c][t];
            r.n_status = ns[(size_t)w];
            r.n_extend = ne[(size_t)w];
            r.ext_first = ef[(size_t)w] >= 0 ? (int)(ef[(size_t)w] - gbase[c]) : -1;
            r.trig = tr[(size_t)w] >= 0 ? (int)(tr[(size_t)w] - gbase[c]) : -1;
            r.kind = kd[(size_t)w];
        }
    return MANDO_OK;
}

}  // namespace modfk
}  // namespace mando

extern "C" int mando_filter_isoforms_device(mando_ctx *ctx, const mando_filter_params *P, const char *isoform_fasta,
                                            const char *genome_fasta, const char *clean_psl, const char *whitelist_bed,
                                            const char *out_fasta, const char *out_psl, const char *reasons_path,
                                            int64_t *n_kept) {
    if (!ctx) return mando::set_error(MANDO_E_ARG, "mando_filter_isoforms_device: null ctx");
    const mando::modf::ContainStage stage = [ctx](const mando_filter_params &p,
                                                  const std::vector<std::vector<mando::modf::Iso>> &isos,
                                                  const std::vector<mando::modf::ChrState> &S,
                                                  std::vector<std::vector<mando::modf::Contain>> &dec) {
        return mando::modfk::contain_device(ctx, p, isos, S, dec);
    };
    return mando::modf::filter_isoforms_impl(P, isoform_fasta, genome_fasta, clean_psl, whitelist_bed, out_fasta,
                                             out_psl, reasons_path, n_kept, &stage);
}
