// writer.cpp — the bytes of the D module's two output files (defineIsoforms.py:155-166), formatted on host
// threads straight from the payload arrays: one pass over the isoforms in output order, no per-member
// intermediate arrays (the numpy form built ~20 segments-arrays of 10M entries for config 4's 10M records
// and took ~0.5 s of the writer's critical path on rank 0).
//   FASTA:            ">Isoform{k}_{m}\n" + consensus (reverse-complemented when rc) + "\n"
//   reads2isoforms:   "{name}\tIsoform{k}_{m}\n" per member
// with k = counter0 + 1 + (position in output order), or iso_k[position], and m = the isoform's member
// count.
#include <sys/mman.h>
#include <sys/vfs.h>
#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "internal.h"
#include "revcomp.h"
#include "threads.h"

namespace {

int dec_len(int64_t x) {
    int d = 1;
    while (x >= 10) {
        x /= 10;
        ++d;
    }
    return d;
}

uint8_t *put_dec(uint8_t *p, int64_t x, int d) {
    for (int i = d - 1; i >= 0; --i) {
        p[i] = (uint8_t)('0' + x % 10);
        x /= 10;
    }
    return p + d;
}

// "Isoform{k}_{m}"
int label_len(int64_t k, int64_t m) { return 7 + dec_len(k) + 1 + dec_len(m); }
uint8_t *put_label(uint8_t *p, int64_t k, int64_t m) {
    memcpy(p, "Isoform", 7);
    p = put_dec(p + 7, k, dec_len(k));
    *p++ = '_';
    return put_dec(p, m, dec_len(m));
}

template <class F>
void parallel(int64_t n, int threads, F &&f) {
    int nt = threads > 0 ? threads : mando::usable_threads();
    nt = (int)std::max<int64_t>(1, std::min<int64_t>(nt, n / 4096 + 1));
    if (nt <= 1) {
        f(0, n);
        return;
    }
    std::vector<std::thread> th;
    const int64_t chunk = (n + nt - 1) / nt;
    for (int t = 0; t < nt; ++t) {
        const int64_t a = t * chunk, b = std::min<int64_t>(n, a + chunk);
        if (a < b) th.emplace_back(f, a, b);
    }
    for (auto &x : th) x.join();
}

}  // namespace

extern "C" int mando_format_outputs(int64_t n_iso, int64_t counter0, const int64_t *iso_k, const int64_t *order,
                                    const int64_t *mem_off,
                                    const uint8_t *const *cons_src, const int16_t *cons_sel, const int64_t *cons_start,
                                    const int64_t *cons_len, const int8_t *cons_rc, const uint8_t *const *name_src,
                                    const int16_t *name_sel, const int64_t *name_start, const int64_t *name_len,
                                    uint8_t *fasta, int64_t fasta_cap, int64_t *fasta_len, uint8_t *r2i,
                                    int64_t r2i_cap, int64_t *r2i_len, int64_t *fasta_off, int64_t *r2i_off,
                                    int32_t threads) {
    if (n_iso < 0 || !order || !mem_off || (fasta && (!fasta_len || !cons_src || !cons_start || !cons_len)) ||
        (r2i && (!r2i_len || !name_src || !name_start || !name_len)))
        return MANDO_E_ARG;
    // pass 1: each isoform's bytes in both files (per output position), then offsets by a prefix sum
    std::vector<int64_t> fo_own, ro_own;
    if (!fasta_off) fo_own.resize((size_t)n_iso + 1);
    if (!r2i_off) ro_own.resize((size_t)n_iso + 1);
    int64_t *fo = fasta_off ? fasta_off : fo_own.data(), *ro = r2i_off ? r2i_off : ro_own.data();
    fo[0] = ro[0] = 0;
    auto num = [&](int64_t i) { return iso_k ? iso_k[i] : counter0 + 1 + i; };
    parallel(n_iso, threads, [&](int64_t a, int64_t b) {
        for (int64_t i = a; i < b; ++i) {
            const int64_t g = order[i], m = mem_off[g + 1] - mem_off[g];
            const int L = label_len(num(i), m);
            fo[(size_t)i + 1] = fasta ? L + 2 + cons_len[g] + 1 : 0;
            ro[(size_t)i + 1] = 0;
            if (r2i) {
                int64_t s = 0;
                for (int64_t j = mem_off[g]; j < mem_off[g + 1]; ++j) s += name_len[j];
                ro[(size_t)i + 1] = s + m * (L + 2);
            }
        }
    });
    for (int64_t i = 0; i < n_iso; ++i) {
        fo[(size_t)i + 1] += fo[(size_t)i];
        ro[(size_t)i + 1] += ro[(size_t)i];
    }
    if (fasta) *fasta_len = fo[(size_t)n_iso];
    if (r2i) *r2i_len = ro[(size_t)n_iso];
    if ((fasta && fo[(size_t)n_iso] > fasta_cap) || (r2i && ro[(size_t)n_iso] > r2i_cap)) return MANDO_E_CAP;
    const mando::CompTable &comp = mando::comp_table();
    // pass 2: fill, isoform ranges on threads
    parallel(n_iso, threads, [&](int64_t a, int64_t b) {
        uint8_t lab[64];
        for (int64_t i = a; i < b; ++i) {
            const int64_t g = order[i], m = mem_off[g + 1] - mem_off[g];
            const int L = (int)(put_label(lab, num(i), m) - lab);
            if (fasta) {
                uint8_t *p = fasta + fo[(size_t)i];
                *p++ = '>';
                memcpy(p, lab, (size_t)L);
                p += L;
                *p++ = '\n';
                const uint8_t *s = cons_src[cons_sel ? cons_sel[g] : 0] + cons_start[g];
                const int64_t n = cons_len[g];
                if (cons_rc && cons_rc[g]) {
                    for (int64_t k = 0; k < n; ++k) p[k] = comp.t[s[n - 1 - k]];
                } else {
                    memcpy(p, s, (size_t)n);
                }
                p[n] = '\n';
            }
            if (r2i) {
                uint8_t *p = r2i + ro[(size_t)i];
                for (int64_t j = mem_off[g]; j < mem_off[g + 1]; ++j) {
                    const int64_t n = name_len[j];
                    memcpy(p, name_src[name_sel ? name_sel[j] : 0] + name_start[j], (size_t)n);
                    p += n;
                    *p++ = '\t';
                    memcpy(p, lab, (size_t)L);
                    p += L;
                    *p++ = '\n';
                }
            }
        }
    });
    return MANDO_OK;
}

namespace {
// true for a file on a local file system (the shared-mapping path of mando_write_blocks); network and
// cluster file systems (NFS, SMB, Lustre, GPFS, Ceph, BeeGFS, FUSE mounts) take pwrite()
bool local_fs(int fd) {
    struct statfs sf;
    if (fstatfs(fd, &sf) != 0) return false;
    switch ((unsigned long)sf.f_type) {
        case 0x6969UL:      // NFS
        case 0xFF534D42UL:  // CIFS
        case 0xFE534D42UL:  // SMB2
        case 0x517BUL:      // SMB
        case 0x0BD00BD0UL:  // Lustre
        case 0x47504653UL:  // GPFS
        case 0x00C36400UL:  // Ceph
        case 0x19830326UL:  // BeeGFS
        case 0x65735546UL:  // FUSE
        case 0x01021997UL:  // 9p
            return false;
        default:
            return true;
    }
}
}  // namespace

extern "C" int mando_write_blocks(int32_t fd, const uint8_t *buf, const int64_t *src_off, const int64_t *dst_off,
                                  const int64_t *len, int64_t n, int32_t threads) {
    if (fd < 0 || n < 0 || (n && (!buf || !src_off || !dst_off || !len))) return MANDO_E_ARG;
    // neighbouring blocks that are contiguous on both sides become one pwrite
    struct Piece {
        int64_t src, dst, n;
    };
    std::vector<Piece> pc;
    int64_t total = 0;
    for (int64_t i = 0; i < n; ++i) {
        if (len[i] < 0) return MANDO_E_ARG;
        if (len[i] == 0) continue;
        total += len[i];
        if (!pc.empty() && pc.back().src + pc.back().n == src_off[i] && pc.back().dst + pc.back().n == dst_off[i])
            pc.back().n += len[i];
        else
            pc.push_back({src_off[i], dst_off[i], len[i]});
    }
    // threads take runs of pieces of about equal bytes (the page-cache copy is the cost)
    int nt = threads > 0 ? threads : std::min(8, mando::usable_threads());
    nt = (int)std::max<int64_t>(1, std::min<int64_t>(nt, total >> 22));
    std::vector<size_t> cut{0};
    for (size_t q = 0, acc = 0; q < pc.size(); ++q) {
        acc += (size_t)pc[q].n;
        if (acc * nt >= (size_t)total * cut.size() && cut.size() < (size_t)nt) cut.push_back(q + 1);
    }
    cut.push_back(pc.size());
    if (pc.empty()) return MANDO_OK;
    // Through a shared mapping of the file range the blocks span (the caller has sized the file): page
    // faults on one file scale over processes, while buffered pwrite()s into one file serialise on its
    // inode lock (8 ranks placing 1 GB into one file: 0.35-0.44 s mapped, 0.9-1.4 s with pwrite).  A
    // descriptor that cannot be mapped (not opened for reading and writing, a pipe) takes pwrite().
    int64_t lo = INT64_MAX, hi = 0;
    for (const Piece &q : pc) {
        lo = std::min(lo, q.dst);
        hi = std::max(hi, q.dst + q.n);
    }
    // The mapping only on a local file system, and only over blocks allocated first: a store into a hole
    // that the disk cannot back would raise SIGBUS (and leave the other ranks waiting in their barrier),
    // where fallocate() reports ENOSPC as an error; and on a network file system two nodes' dirty pages
    // of one page would overwrite each other's bytes, where pwrite() writes only its own.
    const int64_t pg = (int64_t)sysconf(_SC_PAGESIZE);
    const int64_t base = lo / pg * pg;
    void *map = MAP_FAILED;
    if (local_fs(fd)) {
        if (fallocate(fd, 0, (off_t)lo, (off_t)(hi - lo)) == 0)
            map = mmap(nullptr, (size_t)(hi - base), PROT_WRITE, MAP_SHARED, fd, (off_t)base);
        else if (errno != EOPNOTSUPP && errno != ENOSYS && errno != EINVAL)
            return mando::set_error(MANDO_E_INTERNAL, std::string("fallocate: ") + strerror(errno));
    }
    std::atomic<int> err{0};
    auto work = [&](size_t a, size_t b) {
        for (size_t q = a; q < b && !err.load(std::memory_order_relaxed); ++q) {
            if (map != MAP_FAILED) {
                memcpy(static_cast<uint8_t *>(map) + (pc[q].dst - base), buf + pc[q].src, (size_t)pc[q].n);
                continue;
            }
            int64_t done = 0;
            while (done < pc[q].n) {
                const ssize_t w = pwrite(fd, buf + pc[q].src + done, (size_t)(pc[q].n - done), pc[q].dst + done);
                if (w < 0) {
                    if (errno == EINTR) continue;
                    err.store(errno);
                    return;
                }
                done += w;
            }
        }
    };
    std::vector<std::thread> th;
    for (size_t t = 0; t + 1 < cut.size(); ++t)
        if (cut[t] < cut[t + 1]) th.emplace_back(work, cut[t], cut[t + 1]);
    for (auto &x : th) x.join();
    if (map != MAP_FAILED) munmap(map, (size_t)(hi - base));
    if (err.load()) return mando::set_error(MANDO_E_INTERNAL, std::string("pwrite: ") + strerror(err.load()));
    return MANDO_OK;
}
