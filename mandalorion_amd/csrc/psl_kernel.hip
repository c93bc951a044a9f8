// psl_kernel.hip — PSL ingest + locus split on the GPU: the parse and the
// `sort -k 14,14 -k 16,17n` (C locale) of the clean PSL (Mando.py:343-349) on the device, then
// get_chromosomes' cut (SpliceDefineConsensus.py:442-495) and the file writes on the host
// (psl_split.h, shared with the host path psl.cpp, whose output this equals byte for byte:
// tests/test_split_gpu.py).
//
// The file goes to HBM once.  One 64-lane wave per line finds the first 16 tabs by ballots over 64-byte
// chunks and takes fields 14 / 16 / 17 (the chromosome, and the numbers `sort -n` and get_chromosomes
// read from start and end).  The order is a least-significant-key-first chain of stable radix sorts over
// a line permutation (hipCUB's DeviceRadixSort): the start (sign-flipped 64-bit key), then the
// chromosome as big-endian 8-byte words from the last to the first (names up to 32 bytes; byte order
// is the C locale's).  Lines tied on (chromosome, start) keep their input order there; GNU sort breaks
// such ties by the whole line, which the host does run by run (tie runs are short) before the cut.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <string>
#include <string_view>
#include <vector>

#include "internal.h"
#include "psl_split.h"

namespace mando {
namespace pslk {

constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;
constexpr int kMaxChrom = 32;
enum : int32_t { kOk = 0, kErrFields = 1, kErrNumber = 2, kErrChrom = 3 };

struct Parsed {
    int64_t *start, *end, *coff;
    int32_t *clen, *status;
    uint64_t *kw[4];  // chromosome bytes [8w, 8w + 8), big-endian, zero-padded
};

// `sort -n`'s leading number of a field in the C locale (psl.cpp sort_num): blanks skipped, an optional
// '-', the digits that follow; ok when there is at least one digit
__device__ int64_t sort_num(const uint8_t *t, int64_t a, int64_t b, bool &ok) {
    while (a < b && (t[a] == ' ' || t[a] == '\t')) ++a;
    bool neg = false;
    if (a < b && t[a] == '-') {
        neg = true;
        ++a;
    }
    int64_t v = 0;
    ok = false;
    while (a < b && t[a] >= '0' && t[a] <= '9') {
        v = v * 10 + (t[a] - '0');
        ++a;
        ok = true;
    }
    return neg ? -v : v;
}

__global__ __launch_bounds__(kWave * kWavesPerBlock) void parse_kernel(const uint8_t *text, const int64_t *off,
                                                                       const int32_t *len, int64_t n, Parsed P) {
    __shared__ int64_t tabs[kWavesPerBlock][17];
    const int w = threadIdx.x / kWave, lane = threadIdx.x % kWave;
    const int64_t nw = (int64_t)gridDim.x * kWavesPerBlock;
    for (int64_t r = (int64_t)blockIdx.x * kWavesPerBlock + w; r < n; r += nw) {
        const int64_t a = off[r], b = a + len[r];
        int ntab = 0;
        for (int64_t base = a; base < b && ntab < 17; base += kWave) {
            const int64_t p = base + lane;
            const bool tab = p < b && text[p] == '\t';
            const uint64_t m = __ballot(tab);
            const int k = ntab + __popcll(m & (lane ? (~0ull >> (64 - lane)) : 0ull));
            if (tab && k < 17) tabs[w][k] = p;
            ntab += __popcll(m);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0) {
            int st = kOk;
            // 17 fields need 16 tabs; field 16 ends at the 17th tab or at the line end
            if (ntab < 16) st = kErrFields;
            int64_t s = 0, e = 0, c0 = 0;
            int cl = 0;
            if (st == kOk) {
                c0 = tabs[w][12] + 1;
                cl = (int)(tabs[w][13] - c0);
                const int64_t e16 = ntab >= 17 ? tabs[w][16] : b;
                bool ok1, ok2;
                s = sort_num(text, tabs[w][14] + 1, tabs[w][15], ok1);
                e = sort_num(text, tabs[w][15] + 1, e16, ok2);
                if (!(ok1 && ok2)) st = kErrNumber;
                if (cl > kMaxChrom) st = kErrChrom;
            }
            P.start[r] = s;
            P.end[r] = e;
            P.coff[r] = c0;
            P.clen[r] = cl;
            P.status[r] = st;
            for (int q = 0; q < 4; ++q) {
                uint64_t word = 0;
                for (int k = 0; k < 8; ++k) {
                    const int x = 8 * q + k;
                    word = (word << 8) | (st == kOk && x < cl ? (uint64_t)text[c0 + x] : 0u);
                }
                P.kw[q][r] = word;
            }
        }
    }
}

__global__ void iota_kernel(int64_t *perm, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) perm[i] = i;
}

// keys in the current order: key[i] = src[perm[i]] (flip: the sign bit, for signed starts)
__global__ void gather_key_kernel(const uint64_t *src, const int64_t *perm, int64_t n, uint64_t flip, uint64_t *key) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) key[i] = src[perm[i]] ^ flip;
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

}  // namespace pslk
}  // namespace mando

#define PSLK_TRY(x)                                                                                                \
    do {                                                                                                           \
        const hipError_t e_ = (x);                                                                                 \
        if (e_ != hipSuccess) return mando::set_error(MANDO_E_HIP, std::string("split: ") + hipGetErrorString(e_)); \
    } while (0)

extern "C" int mando_split_loci_device(mando_ctx *ctx, const char *psl_path, const char *out_dir, int32_t sort_lines,
                                       const char *sorted_out, int64_t *n_records, int64_t *n_loci) {
    using namespace mando::pslk;
    using mando::psl::Line;
    if (!ctx || !psl_path || !out_dir) return mando::set_error(MANDO_E_ARG, "mando_split_loci_device: bad argument");
    std::string buf;
    {
        FILE *fh = fopen(psl_path, "rb");
        if (!fh) return mando::set_error(MANDO_E_ARG, std::string("cannot read ") + psl_path);
        fseek(fh, 0, SEEK_END);
        const long sz = ftell(fh);
        fseek(fh, 0, SEEK_SET);
        buf.resize((size_t)std::max(0L, sz));
        const size_t got = sz > 0 ? fread(&buf[0], 1, (size_t)sz, fh) : 0;
        fclose(fh);
        if ((long)got != sz) return mando::set_error(MANDO_E_ARG, std::string("short read of ") + psl_path);
    }
    std::vector<int64_t> off;
    std::vector<int32_t> len;
    for (size_t p = 0; p < buf.size();) {
        size_t e = buf.find('\n', p);
        if (e == std::string::npos) e = buf.size();
        if (e > p) {
            off.push_back((int64_t)p);
            len.push_back((int32_t)(e - p));
        }
        p = e + 1;
    }
    const int64_t n = (int64_t)off.size();
    std::vector<Line> lines((size_t)n);
    if (n > 0) {
        PSLK_TRY(hipSetDevice(mando::ctx_device(ctx)));
        hipStream_t s = mando::ctx_stream(ctx);
        Dev d_text, d_off, d_len, d_start, d_end, d_coff, d_clen, d_st, d_kw[4], d_perm, d_perm2, d_key, d_key2, d_tmp;
        int rc;
        if ((rc = d_text.alloc(buf.size())) || (rc = d_off.alloc((size_t)n * 8)) || (rc = d_len.alloc((size_t)n * 4)) ||
            (rc = d_start.alloc((size_t)n * 8)) || (rc = d_end.alloc((size_t)n * 8)) || (rc = d_coff.alloc((size_t)n * 8)) ||
            (rc = d_clen.alloc((size_t)n * 4)) || (rc = d_st.alloc((size_t)n * 4)) || (rc = d_perm.alloc((size_t)n * 8)) ||
            (rc = d_perm2.alloc((size_t)n * 8)) || (rc = d_key.alloc((size_t)n * 8)) || (rc = d_key2.alloc((size_t)n * 8)))
            return mando::set_error(rc, "split: device allocation failed");
        for (int q = 0; q < 4; ++q)
            if ((rc = d_kw[q].alloc((size_t)n * 8))) return mando::set_error(rc, "split: device allocation failed");
        PSLK_TRY(hipMemcpyAsync(d_text.p, buf.data(), buf.size(), hipMemcpyHostToDevice, s));
        PSLK_TRY(hipMemcpyAsync(d_off.p, off.data(), (size_t)n * 8, hipMemcpyHostToDevice, s));
        PSLK_TRY(hipMemcpyAsync(d_len.p, len.data(), (size_t)n * 4, hipMemcpyHostToDevice, s));
        Parsed P{d_start.as<int64_t>(), d_end.as<int64_t>(), d_coff.as<int64_t>(), d_clen.as<int32_t>(),
                 d_st.as<int32_t>(), {d_kw[0].as<uint64_t>(), d_kw[1].as<uint64_t>(), d_kw[2].as<uint64_t>(),
                                      d_kw[3].as<uint64_t>()}};
        const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((n + kWavesPerBlock - 1) / kWavesPerBlock, 8192));
        hipLaunchKernelGGL(parse_kernel, dim3(blocks), dim3(kWave * kWavesPerBlock), 0, s, d_text.as<uint8_t>(),
                           d_off.as<int64_t>(), d_len.as<int32_t>(), n, P);
        PSLK_TRY(hipGetLastError());
        std::vector<int64_t> start((size_t)n), end((size_t)n), coff((size_t)n);
        std::vector<int32_t> clen((size_t)n), st((size_t)n);
        PSLK_TRY(hipMemcpyAsync(st.data(), d_st.p, (size_t)n * 4, hipMemcpyDeviceToHost, s));
        PSLK_TRY(hipMemcpyAsync(clen.data(), d_clen.p, (size_t)n * 4, hipMemcpyDeviceToHost, s));
        PSLK_TRY(hipMemcpyAsync(start.data(), d_start.p, (size_t)n * 8, hipMemcpyDeviceToHost, s));
        PSLK_TRY(hipMemcpyAsync(end.data(), d_end.p, (size_t)n * 8, hipMemcpyDeviceToHost, s));
        PSLK_TRY(hipMemcpyAsync(coff.data(), d_coff.p, (size_t)n * 8, hipMemcpyDeviceToHost, s));
        PSLK_TRY(hipStreamSynchronize(s));
        int maxc = 0;
        for (int64_t r = 0; r < n; ++r) {
            if (st[(size_t)r] == kErrChrom)
                return mando::set_error(MANDO_E_UNSUPPORTED, "PSL line " + std::to_string(r) +
                                                                 ": chromosome name over 32 bytes (the host split takes it)");
            if (st[(size_t)r] != kOk)
                return mando::set_error(MANDO_E_ARG, "PSL line " + std::to_string(r) +
                                                         ": fewer than 17 fields, or a start / end get_chromosomes cannot read");
            maxc = std::max(maxc, clen[(size_t)r]);
        }
        std::vector<int64_t> perm((size_t)n);
        if (sort_lines) {
            // stable LSD chain: start, then the chromosome's words from the last that any name reaches
            const int tpb = 256;
            const unsigned g = (unsigned)((n + tpb - 1) / tpb);
            hipLaunchKernelGGL(iota_kernel, dim3(g), dim3(tpb), 0, s, d_perm.as<int64_t>(), n);
            size_t tmp_bytes = 0;
            PSLK_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, d_key.as<uint64_t>(), d_key2.as<uint64_t>(),
                                                        d_perm.as<int64_t>(), d_perm2.as<int64_t>(), (int)n, 0, 64, s));
            if ((rc = d_tmp.alloc(tmp_bytes))) return mando::set_error(rc, "split: device allocation failed");
            const int nwords = (maxc + 7) / 8;
            for (int pass = 0; pass <= nwords; ++pass) {
                const uint64_t *src = pass == 0 ? reinterpret_cast<const uint64_t *>(d_start.p) : d_kw[nwords - pass].as<uint64_t>();
                const uint64_t flip = pass == 0 ? (1ull << 63) : 0ull;
                hipLaunchKernelGGL(gather_key_kernel, dim3(g), dim3(tpb), 0, s, src, d_perm.as<int64_t>(), n, flip,
                                   d_key.as<uint64_t>());
                PSLK_TRY(hipGetLastError());
                size_t tb = tmp_bytes;
                PSLK_TRY(hipcub::DeviceRadixSort::SortPairs(d_tmp.p, tb, d_key.as<uint64_t>(), d_key2.as<uint64_t>(),
                                                            d_perm.as<int64_t>(), d_perm2.as<int64_t>(), (int)n, 0, 64, s));
                std::swap(d_perm.p, d_perm2.p);
            }
            PSLK_TRY(hipMemcpyAsync(perm.data(), d_perm.p, (size_t)n * 8, hipMemcpyDeviceToHost, s));
            PSLK_TRY(hipStreamSynchronize(s));
        } else {
            for (int64_t r = 0; r < n; ++r) perm[(size_t)r] = r;
        }
        for (int64_t k = 0; k < n; ++k) {
            const int64_t r = perm[(size_t)k];
            Line &L = lines[(size_t)k];
            L.text = std::string_view(buf.data() + off[(size_t)r], (size_t)len[(size_t)r]);
            L.chrom = std::string_view(buf.data() + coff[(size_t)r], (size_t)clen[(size_t)r]);
            L.start = start[(size_t)r];
            L.end = end[(size_t)r];
            L.start_ok = true;
        }
        if (sort_lines) {
            // GNU sort's last-resort key: lines tied on (chromosome, start) ordered by their bytes
            for (int64_t a = 0; a < n;) {
                int64_t b = a + 1;
                while (b < n && lines[(size_t)b].start == lines[(size_t)a].start &&
                       lines[(size_t)b].chrom == lines[(size_t)a].chrom)
                    ++b;
                if (b - a > 1)
                    std::stable_sort(lines.begin() + a, lines.begin() + b,
                                     [](const Line &x, const Line &y) { return x.text < y.text; });
                a = b;
            }
        }
    }
    return mando::psl::split_write_ordered(lines, out_dir, sorted_out, n_records, n_loci);
}
