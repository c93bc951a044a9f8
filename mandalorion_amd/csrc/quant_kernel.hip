// quant_kernel.hip — module Q (assignReadsToIsoforms.py:27-105) with its two joins on the GPU (SURVEY.md
// §8(f) row 4): read name -> sample file (readMapDict, :56-66) for every reads2isoforms line (:72-85), and
// isoform -> its lines' samples (r2i_dict, :27-47) for every filtered isoform, as sorts and binary searches
// over 64-bit name hashes in HBM with every hit confirmed byte for byte (a hash collision costs a compare,
// never a wrong count).  The host reads the files (zlib for the read files, like mappy.fastx_read), delimits
// records and lines, and writes the two tables through the same code as the host path (quant.h), whose
// output this equals byte for byte (tests/test_quant_gpu.py).
//
//  1. name_hash: one thread per read-file record name;
//  2. r2i_parse: one thread per reads2isoforms line: Python's strip() + split('\t') -> (read, isoform), both
//     hashed;
//  3. the read-name hashes sorted with their record indices (hipCUB DeviceRadixSort, stable: equal hashes
//     keep file order);
//  4. r2i_lookup: per line, the equal-hash run of its read name, scanned from its end: the last record
//     with the same bytes is the one the dict kept (readMapDict[name] = location, later files and records
//     overwrite) -> the line's sample; none: the reference's KeyError;
//  5. the lines' isoform hashes sorted with their line indices;
//  6. iso_count: one thread per filtered-PSL line: the equal-hash run of its isoform, every line with the
//     same bytes counted for its sample; none: KeyError.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cctype>
#include <cstdint>
#include <cstdio>
#include <string>
#include <string_view>
#include <vector>

#include "internal.h"
#include "quant.h"

namespace mando {
namespace quantk {

enum : int32_t { kOk = 0, kErrFields = 1, kErrMissing = 2 };

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

// FNV-1a over the bytes, then a finaliser so that the radix sort's digits are spread
__device__ uint64_t hash_bytes(const uint8_t *t, int64_t a, int32_t n) {
    uint64_t h = 0xcbf29ce484222325ull;
    for (int32_t k = 0; k < n; ++k) h = (h ^ t[a + k]) * 0x100000001b3ull;
    return mix64(h ^ (uint64_t)n);
}

__device__ bool same_bytes(const uint8_t *ta, int64_t a, int32_t na, const uint8_t *tb, int64_t b, int32_t nb) {
    if (na != nb) return false;
    for (int32_t k = 0; k < na; ++k)
        if (ta[a + k] != tb[b + k]) return false;
    return true;
}

// the C locale's isspace (the host path's strip)
__device__ __forceinline__ bool is_space(uint8_t c) { return c == ' ' || (c >= '\t' && c <= '\r'); }

__global__ void name_hash(const uint8_t *text, const int64_t *off, const int32_t *len, int64_t n, uint64_t *h,
                          int64_t *idx) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    h[i] = hash_bytes(text, off[i], len[i]);
    idx[i] = i;
}

// a = line.strip().split('\t'): a[0] the read, a[1] the isoform (the next tab or the stripped end)
__global__ void r2i_parse(const uint8_t *text, const int64_t *loff, const int32_t *llen, int64_t n, int64_t *roff,
                          int32_t *rlen, int64_t *ioff, int32_t *ilen, uint64_t *rh, uint64_t *ih, int64_t *idx,
                          int32_t *status) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int64_t a = loff[i], b = a + llen[i];
    while (a < b && is_space(text[a])) ++a;
    while (b > a && is_space(text[b - 1])) --b;
    int64_t t1 = a;
    while (t1 < b && text[t1] != '\t') ++t1;
    int32_t st = kOk;
    int64_t t2 = t1;
    if (t1 >= b) {
        st = kErrFields;  // fewer than two fields: IndexError in the reference
    } else {
        t2 = t1 + 1;
        while (t2 < b && text[t2] != '\t') ++t2;
    }
    roff[i] = a;
    rlen[i] = (int32_t)(t1 - a);
    ioff[i] = t1 + 1;
    ilen[i] = st == kOk ? (int32_t)(t2 - t1 - 1) : 0;
    rh[i] = hash_bytes(text, a, (int32_t)(t1 - a));
    ih[i] = st == kOk ? hash_bytes(text, t1 + 1, (int32_t)(t2 - t1 - 1)) : 0;
    idx[i] = i;
    status[i] = st;
}

// first k in [0, n) with keys[k] >= x
__device__ int64_t lower(const uint64_t *keys, int64_t n, uint64_t x) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t m = (lo + hi) >> 1;
        if (keys[m] < x) lo = m + 1;
        else hi = m;
    }
    return lo;
}

__global__ void r2i_lookup(const uint8_t *r2i_text, const int64_t *roff, const int32_t *rlen, const uint64_t *rh,
                           int64_t n_lines, const uint8_t *names, const int64_t *noff, const int32_t *nlen,
                           const uint64_t *sorted_h, const int64_t *sorted_idx, int64_t n_names,
                           const int32_t *rec_sample, int32_t *line_sample, int32_t *status) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_lines || status[i] != kOk) return;
    const uint64_t h = rh[i];
    int64_t k = lower(sorted_h, n_names, h);
    int64_t e = k;
    while (e < n_names && sorted_h[e] == h) ++e;
    int32_t s = -1;
    for (int64_t j = e - 1; j >= k; --j) {
        const int64_t r = sorted_idx[j];
        if (same_bytes(r2i_text, roff[i], rlen[i], names, noff[r], nlen[r])) {
            s = rec_sample[r];
            break;
        }
    }
    line_sample[i] = s;
    if (s < 0) status[i] = kErrMissing;
}

__global__ void iso_count(const uint8_t *psl_text, const int64_t *poff, const int32_t *plen, int64_t n_iso,
                          const uint8_t *r2i_text, const int64_t *ioff, const int32_t *ilen, const uint64_t *sorted_ih,
                          const int64_t *sorted_line, int64_t n_lines, const int32_t *line_sample, int32_t n_samples,
                          int64_t *counts, int32_t *iso_status) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n_iso) return;
    const uint64_t h = hash_bytes(psl_text, poff[k], plen[k]);
    int64_t j = lower(sorted_ih, n_lines, h);
    int64_t hits = 0;
    for (; j < n_lines && sorted_ih[j] == h; ++j) {
        const int64_t l = sorted_line[j];
        if (!same_bytes(psl_text, poff[k], plen[k], r2i_text, ioff[l], ilen[l])) continue;
        counts[k * n_samples + line_sample[l]] += 1;
        ++hits;
    }
    iso_status[k] = hits ? kOk : kErrMissing;
}

struct Dev {
    void *p = nullptr;
    ~Dev() {
        if (p) (void)hipFree(p);
    }
    int alloc(size_t n) { return hipMalloc(&p, n ? n : 1) == hipSuccess ? MANDO_OK : MANDO_E_NOMEM; }
    template <class T>
    T *as() const {
        return static_cast<T *>(p);
    }
};

bool read_file(const char *path, std::string &out) {
    FILE *fh = fopen(path, "rb");
    if (!fh) return false;
    fseek(fh, 0, SEEK_END);
    const long sz = ftell(fh);
    fseek(fh, 0, SEEK_SET);
    out.resize((size_t)std::max(0L, sz));
    const size_t got = sz > 0 ? fread(&out[0], 1, (size_t)sz, fh) : 0;
    fclose(fh);
    return (long)got == sz;
}

unsigned blocks_for(int64_t n, int tpb) { return (unsigned)std::max<int64_t>(1, (n + tpb - 1) / tpb); }

}  // namespace quantk
}  // namespace mando

#define QK_TRY(x)                                                                                                  \
    do {                                                                                                           \
        const hipError_t e_ = (x);                                                                                 \
        if (e_ != hipSuccess) return mando::set_error(MANDO_E_HIP, std::string("quantify: ") + hipGetErrorString(e_)); \
    } while (0)
#define QK_ALLOC(d, bytes)                                                                                         \
    do {                                                                                                           \
        if ((d).alloc(bytes)) return mando::set_error(MANDO_E_NOMEM, "quantify: device allocation failed");       \
    } while (0)

extern "C" int mando_quantify_device(mando_ctx *ctx, const char *const *fasta_paths, int32_t n_fasta,
                                     const char *r2i_path, const char *filtered_psl, const char *out_quant,
                                     const char *out_tpm) {
    using namespace mando::quantk;
    if (!ctx || !fasta_paths || n_fasta < 0 || !r2i_path || !filtered_psl || !out_quant || !out_tpm)
        return mando::set_error(MANDO_E_ARG, "mando_quantify_device: bad argument");
    // the read files' record names, all files' names in one blob (file order), each with its sample
    std::vector<std::string> samples;
    std::vector<int64_t> total;
    std::string names;
    std::vector<int64_t> noff;
    std::vector<int32_t> nlen, rec_sample;
    {
        std::string buf;
        std::vector<std::pair<int64_t, int32_t>> recs;
        for (int32_t f = 0; f < n_fasta; ++f) {
            std::string_view loc(fasta_paths[f]);
            while (!loc.empty() && isspace((unsigned char)loc.front())) loc.remove_prefix(1);
            while (!loc.empty() && isspace((unsigned char)loc.back())) loc.remove_suffix(1);
            samples.emplace_back(loc);
            if (!mando::modq::fastx_names(samples.back().c_str(), buf, recs))
                return mando::set_error(MANDO_E_ARG, "cannot read " + samples.back());
            total.push_back((int64_t)recs.size());
            for (auto &r : recs) {
                noff.push_back((int64_t)names.size());
                nlen.push_back(r.second);
                rec_sample.push_back(f);
                names.append(buf, (size_t)r.first, (size_t)r.second);
            }
        }
    }
    std::string r2i;
    if (!read_file(r2i_path, r2i)) return mando::set_error(MANDO_E_ARG, std::string("cannot read ") + r2i_path);
    std::vector<int64_t> loff;
    std::vector<int32_t> llen;
    for (size_t p = 0; p < r2i.size();) {
        size_t e = r2i.find('\n', p);
        if (e == std::string::npos) e = r2i.size();
        loff.push_back((int64_t)p);
        llen.push_back((int32_t)(e - p));
        p = e + 1;
    }
    std::string pbuf;
    std::vector<std::string_view> isos;
    if (!read_file(filtered_psl, pbuf)) return mando::set_error(MANDO_E_ARG, std::string("cannot read ") + filtered_psl);
    if (!mando::modq::psl_isoforms(pbuf, isos))
        return mando::set_error(MANDO_E_ARG, "filtered PSL: a line with fewer than 10 fields");
    std::vector<int64_t> poff(isos.size());
    std::vector<int32_t> plen(isos.size());
    for (size_t k = 0; k < isos.size(); ++k) {
        poff[k] = (int64_t)(isos[k].data() - pbuf.data());
        plen[k] = (int32_t)isos[k].size();
    }
    const int64_t nn = (int64_t)noff.size(), nl = (int64_t)loff.size(), ni = (int64_t)isos.size();
    const int32_t ns = n_fasta;
    std::vector<int64_t> counts((size_t)(ni * ns), 0);
    QK_TRY(hipSetDevice(mando::ctx_device(ctx)));
    hipStream_t s = mando::ctx_stream(ctx);
    const int tpb = 256;
    Dev d_names, d_noff, d_nlen, d_rs, d_nh, d_nidx, d_nh2, d_nidx2;
    Dev d_r2i, d_loff, d_llen, d_roff, d_rlen, d_ioff, d_ilen, d_rh, d_ih, d_lidx, d_st, d_ih2, d_lidx2, d_lsam;
    Dev d_psl, d_poff, d_plen, d_counts, d_ist, d_tmp;
    QK_ALLOC(d_names, names.size());
    QK_ALLOC(d_noff, (size_t)nn * 8);
    QK_ALLOC(d_nlen, (size_t)nn * 4);
    QK_ALLOC(d_rs, (size_t)nn * 4);
    QK_ALLOC(d_nh, (size_t)nn * 8);
    QK_ALLOC(d_nidx, (size_t)nn * 8);
    QK_ALLOC(d_nh2, (size_t)nn * 8);
    QK_ALLOC(d_nidx2, (size_t)nn * 8);
    QK_ALLOC(d_r2i, r2i.size());
    QK_ALLOC(d_loff, (size_t)nl * 8);
    QK_ALLOC(d_llen, (size_t)nl * 4);
    QK_ALLOC(d_roff, (size_t)nl * 8);
    QK_ALLOC(d_rlen, (size_t)nl * 4);
    QK_ALLOC(d_ioff, (size_t)nl * 8);
    QK_ALLOC(d_ilen, (size_t)nl * 4);
    QK_ALLOC(d_rh, (size_t)nl * 8);
    QK_ALLOC(d_ih, (size_t)nl * 8);
    QK_ALLOC(d_lidx, (size_t)nl * 8);
    QK_ALLOC(d_st, (size_t)nl * 4);
    QK_ALLOC(d_ih2, (size_t)nl * 8);
    QK_ALLOC(d_lidx2, (size_t)nl * 8);
    QK_ALLOC(d_lsam, (size_t)nl * 4);
    QK_ALLOC(d_psl, pbuf.size());
    QK_ALLOC(d_poff, (size_t)ni * 8);
    QK_ALLOC(d_plen, (size_t)ni * 4);
    QK_ALLOC(d_counts, (size_t)(ni * ns) * 8);
    QK_ALLOC(d_ist, (size_t)ni * 4);
    if (!names.empty()) QK_TRY(hipMemcpyAsync(d_names.p, names.data(), names.size(), hipMemcpyHostToDevice, s));
    if (nn) {
        QK_TRY(hipMemcpyAsync(d_noff.p, noff.data(), (size_t)nn * 8, hipMemcpyHostToDevice, s));
        QK_TRY(hipMemcpyAsync(d_nlen.p, nlen.data(), (size_t)nn * 4, hipMemcpyHostToDevice, s));
        QK_TRY(hipMemcpyAsync(d_rs.p, rec_sample.data(), (size_t)nn * 4, hipMemcpyHostToDevice, s));
    }
    if (!r2i.empty()) QK_TRY(hipMemcpyAsync(d_r2i.p, r2i.data(), r2i.size(), hipMemcpyHostToDevice, s));
    if (nl) {
        QK_TRY(hipMemcpyAsync(d_loff.p, loff.data(), (size_t)nl * 8, hipMemcpyHostToDevice, s));
        QK_TRY(hipMemcpyAsync(d_llen.p, llen.data(), (size_t)nl * 4, hipMemcpyHostToDevice, s));
    }
    if (!pbuf.empty()) QK_TRY(hipMemcpyAsync(d_psl.p, pbuf.data(), pbuf.size(), hipMemcpyHostToDevice, s));
    if (ni) {
        QK_TRY(hipMemcpyAsync(d_poff.p, poff.data(), (size_t)ni * 8, hipMemcpyHostToDevice, s));
        QK_TRY(hipMemcpyAsync(d_plen.p, plen.data(), (size_t)ni * 4, hipMemcpyHostToDevice, s));
        QK_TRY(hipMemsetAsync(d_counts.p, 0, (size_t)(ni * ns) * 8, s));
    }
    // 1-2: hashes of the record names and of the lines' two fields
    if (nn)
        hipLaunchKernelGGL(name_hash, dim3(blocks_for(nn, tpb)), dim3(tpb), 0, s, d_names.as<uint8_t>(),
                           d_noff.as<int64_t>(), d_nlen.as<int32_t>(), nn, d_nh.as<uint64_t>(), d_nidx.as<int64_t>());
    if (nl)
        hipLaunchKernelGGL(r2i_parse, dim3(blocks_for(nl, tpb)), dim3(tpb), 0, s, d_r2i.as<uint8_t>(),
                           d_loff.as<int64_t>(), d_llen.as<int32_t>(), nl, d_roff.as<int64_t>(), d_rlen.as<int32_t>(),
                           d_ioff.as<int64_t>(), d_ilen.as<int32_t>(), d_rh.as<uint64_t>(), d_ih.as<uint64_t>(),
                           d_lidx.as<int64_t>(), d_st.as<int32_t>());
    QK_TRY(hipGetLastError());
    // 3, 5: stable radix sorts (hash -> index)
    size_t tmp_a = 0, tmp_b = 0;
    if (nn > INT32_MAX || nl > INT32_MAX)
        return mando::set_error(MANDO_E_UNSUPPORTED, "quantify: more than 2^31 records or lines");
    QK_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_a, d_nh.as<uint64_t>(), d_nh2.as<uint64_t>(),
                                              d_nidx.as<int64_t>(), d_nidx2.as<int64_t>(), (int)nn, 0, 64, s));
    QK_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_b, d_ih.as<uint64_t>(), d_ih2.as<uint64_t>(),
                                              d_lidx.as<int64_t>(), d_lidx2.as<int64_t>(), (int)nl, 0, 64, s));
    QK_ALLOC(d_tmp, std::max(tmp_a, tmp_b));
    if (nn)
        QK_TRY(hipcub::DeviceRadixSort::SortPairs(d_tmp.p, tmp_a, d_nh.as<uint64_t>(), d_nh2.as<uint64_t>(),
                                                  d_nidx.as<int64_t>(), d_nidx2.as<int64_t>(), (int)nn, 0, 64, s));
    // 4: every line's sample
    if (nl)
        hipLaunchKernelGGL(r2i_lookup, dim3(blocks_for(nl, tpb)), dim3(tpb), 0, s, d_r2i.as<uint8_t>(),
                           d_roff.as<int64_t>(), d_rlen.as<int32_t>(), d_rh.as<uint64_t>(), nl, d_names.as<uint8_t>(),
                           d_noff.as<int64_t>(), d_nlen.as<int32_t>(), d_nh2.as<uint64_t>(), d_nidx2.as<int64_t>(), nn,
                           d_rs.as<int32_t>(), d_lsam.as<int32_t>(), d_st.as<int32_t>());
    QK_TRY(hipGetLastError());
    if (nl)
        QK_TRY(hipcub::DeviceRadixSort::SortPairs(d_tmp.p, tmp_b, d_ih.as<uint64_t>(), d_ih2.as<uint64_t>(),
                                                  d_lidx.as<int64_t>(), d_lidx2.as<int64_t>(), (int)nl, 0, 64, s));
    // 6: every filtered isoform's counts
    if (ni)
        hipLaunchKernelGGL(iso_count, dim3(blocks_for(ni, tpb)), dim3(tpb), 0, s, d_psl.as<uint8_t>(),
                           d_poff.as<int64_t>(), d_plen.as<int32_t>(), ni, d_r2i.as<uint8_t>(), d_ioff.as<int64_t>(),
                           d_ilen.as<int32_t>(), d_ih2.as<uint64_t>(), d_lidx2.as<int64_t>(), nl, d_lsam.as<int32_t>(),
                           ns, d_counts.as<int64_t>(), d_ist.as<int32_t>());
    QK_TRY(hipGetLastError());
    std::vector<int32_t> st((size_t)nl), ist((size_t)ni);
    if (nl) QK_TRY(hipMemcpyAsync(st.data(), d_st.p, (size_t)nl * 4, hipMemcpyDeviceToHost, s));
    if (ni) {
        QK_TRY(hipMemcpyAsync(ist.data(), d_ist.p, (size_t)ni * 4, hipMemcpyDeviceToHost, s));
        QK_TRY(hipMemcpyAsync(counts.data(), d_counts.p, (size_t)(ni * ns) * 8, hipMemcpyDeviceToHost, s));
    }
    QK_TRY(hipStreamSynchronize(s));
    // the reference fails at the first bad line of reads2isoforms.txt, before any isoform is counted
    for (int64_t i = 0; i < nl; ++i) {
        if (st[(size_t)i] == kErrFields)
            return mando::set_error(MANDO_E_ARG, "reads2isoforms.txt line " + std::to_string(i + 1) + ": fewer than 2 fields");
        if (st[(size_t)i] == kErrMissing)
            return mando::set_error(MANDO_E_ARG, "reads2isoforms.txt line " + std::to_string(i + 1) +
                                                     ": read in none of the read files (KeyError)");
    }
    for (int64_t k = 0; k < ni; ++k)
        if (ist[(size_t)k] != kOk)
            return mando::set_error(MANDO_E_ARG, "filtered isoform " + std::string(isos[(size_t)k]) +
                                                     " has no reads2isoforms line (KeyError)");
    const int rc = mando::modq::write_tables(samples, total, isos, counts, out_quant, out_tpm);
    return rc ? mando::set_error(rc, "quantify: a read file without records, or an output not writable") : MANDO_OK;
}
