// psl.cpp — PSL ingest + locus split (the part of module P that feeds the D
// module).  Restates
//   `sort -T tmp -k 14,14 -k 16,17n clean.psl > clean.sorted.psl`     Mando.py:343-349
//   get_chromosomes(clean.sorted.psl, tmp_SS, ...)                     SpliceDefineConsensus.py:442-495
// as one native pass: lines are read once, ordered like GNU sort in the C locale (key 1 = field 14
// compared as bytes, key 2 = the number at the start of field 16, ties by the whole line as bytes),
// and cut into loci exactly like get_chromosomes (a new locus when the chromosome changes or a read
// starts after the running locus end; the first read of a locus sets start/end, later reads only
// extend end), one `<chrom>~<start>~<end>.psl` file per locus.
// Fields are separated by tabs (PSL); GNU sort's blank-separated fields coincide because PSL fields
// hold no blanks.  The sort's locale is assumed to be C (Mando.py does not set one; under a UTF-8
// collation the chromosome order could differ).
#include "threads.h"
#include <fcntl.h>
#include <unistd.h>
#include <dirent.h>
#include <sys/stat.h>

#include <algorithm>
#include <thread>
#include <unordered_map>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <string_view>
#include <vector>

#include "../../include/mando.h"

#include "psl_split.h"

namespace {

using mando::psl::Line;

// leading number of a field the way `sort -n` reads it in the C locale (no thousands separator)
int64_t sort_num(std::string_view s, bool &ok) {
    size_t i = 0;
    while (i < s.size() && (s[i] == ' ' || s[i] == '\t')) ++i;
    bool neg = false;
    if (i < s.size() && s[i] == '-') {
        neg = true;
        ++i;
    }
    int64_t v = 0;
    ok = false;
    while (i < s.size() && s[i] >= '0' && s[i] <= '9') {
        v = v * 10 + (s[i] - '0');
        ++i;
        ok = true;
    }
    return neg ? -v : v;
}

bool parse_line(std::string_view t, Line &L) {
    L.text = t;
    size_t f = 0, a = 0;
    std::string_view fld[17];
    for (size_t i = 0; i <= t.size() && f < 17; ++i) {
        if (i == t.size() || t[i] == '\t') {
            fld[f++] = t.substr(a, i - a);
            a = i + 1;
        }
    }
    if (f < 17) return false;
    L.chrom = fld[13];
    bool ok1 = false, ok2 = false;
    L.start = sort_num(fld[15], ok1);
    L.end = sort_num(fld[16], ok2);
    L.start_ok = ok1;
    return ok1 && ok2;
}

}  // namespace

extern "C" int mando_split_loci(const char *psl_path, const char *out_dir, int32_t sort_lines,
                                const char *sorted_out, int64_t *n_records, int64_t *n_loci) {
    if (!psl_path || !out_dir) return MANDO_E_ARG;
    FILE *fh = fopen(psl_path, "rb");
    if (!fh) return MANDO_E_ARG;
    fseek(fh, 0, SEEK_END);
    const long sz = ftell(fh);
    fseek(fh, 0, SEEK_SET);
    std::string buf((size_t)std::max(0L, sz), '\0');
    const size_t got = sz > 0 ? fread(&buf[0], 1, (size_t)sz, fh) : 0;
    fclose(fh);
    if ((long)got != sz) return MANDO_E_ARG;
    std::vector<Line> lines;
    size_t p = 0;
    while (p < buf.size()) {
        size_t e = buf.find('\n', p);
        if (e == std::string::npos) e = buf.size();
        if (e > p) {
            Line L;
            if (!parse_line(std::string_view(buf.data() + p, e - p), L)) return MANDO_E_ARG;
            lines.push_back(L);
        }
        p = e + 1;
    }
    if (sort_lines) {
        std::stable_sort(lines.begin(), lines.end(), [](const Line &a, const Line &b) {
            const int c = a.chrom.compare(b.chrom);
            if (c != 0) return c < 0;
            if (a.start != b.start) return a.start < b.start;
            return a.text < b.text;  // GNU sort's last-resort comparison (whole line, bytes)
        });
    }
    return mando::psl::split_write_ordered(lines, out_dir, sorted_out, n_records, n_loci);
}

namespace mando {
namespace psl {

int split_write_ordered(const std::vector<Line> &lines, const char *out_dir, const char *sorted_out,
                        int64_t *n_records, int64_t *n_loci) {
    if (sorted_out) {  // clean.sorted.psl, as the reference's sort writes it
        FILE *o = fopen(sorted_out, "wb");
        if (!o) return MANDO_E_ARG;
        for (const Line &L : lines) {
            fwrite(L.text.data(), 1, L.text.size(), o);
            fputc('\n', o);
        }
        fclose(o);
    }
    int64_t nrec = 0, nloc = 0;
    std::string prev_chrom;
    bool have_prev = false;
    int64_t prev_start = 0, prev_end = 0;
    std::vector<const Line *> cur;
    auto flush = [&]() -> int {
        if (cur.empty()) return MANDO_OK;
        const std::string path = std::string(out_dir) + "/" + prev_chrom + "~" + std::to_string(prev_start) + "~" +
                                 std::to_string(prev_end) + ".psl";
        FILE *o = fopen(path.c_str(), "wb");
        if (!o) return MANDO_E_ARG;
        for (const Line *L : cur) {
            fwrite(L->text.data(), 1, L->text.size(), o);
            fputc('\n', o);
        }
        fclose(o);
        nrec += (int64_t)cur.size();
        ++nloc;
        cur.clear();
        return MANDO_OK;
    };
    for (const Line &L : lines) {
        const bool fresh = !have_prev || L.chrom != std::string_view(prev_chrom) || L.start > prev_end;
        if (!fresh) {
            prev_end = std::max(prev_end, L.end);
            cur.push_back(&L);
        } else {
            const int rc = flush();
            if (rc) return rc;
            cur.push_back(&L);
            prev_chrom.assign(L.chrom.data(), L.chrom.size());
            prev_end = L.end;
            prev_start = L.start;
            have_prev = true;
        }
    }
    const int rc = flush();
    if (rc) return rc;
    if (n_records) *n_records = nrec;
    if (n_loci) *n_loci = nloc;
    return MANDO_OK;
}

}  // namespace psl
}  // namespace mando

// The directory scan of defineIsoforms.py:130-139 (+ the file sizes the D driver plans its chunks
// with) without a Python stat per file.  with_sizes == false (mando_list_root_names): the entry type
// comes from readdir's d_type where it answers (DT_REG: a regular file, DT_DIR etc.: not one), and only
// symlinks and DT_UNKNOWN entries are stat'ed (is_file() follows symlinks, as stat does).
namespace {
int list_roots(const char *dir, int32_t threads, bool with_sizes, char *names, int64_t names_cap, int64_t *sizes,
               int64_t sizes_cap, int64_t *n_roots, int64_t *names_bytes) {
    if (!dir || !n_roots || !names_bytes || names_cap < 0 || sizes_cap < 0) return MANDO_E_ARG;
    DIR *d = opendir(dir);
    if (!d) return MANDO_E_ARG;
    std::vector<std::string> ents;
    std::vector<int64_t> fsize;  // -2: not a regular file, -3: to be stat'ed
    while (struct dirent *e = readdir(d)) {
        if (!strstr(e->d_name, ".psl")) continue;
        ents.emplace_back(e->d_name);
        fsize.push_back(with_sizes || e->d_type == DT_LNK || e->d_type == DT_UNKNOWN ? -3
                        : e->d_type == DT_REG                                     ? 0
                                                                                   : -2);
    }
    closedir(d);
    const std::string base = std::string(dir) + "/";
    // regular files only, sizes from the same stat
    std::vector<size_t> todo;
    for (size_t i = 0; i < ents.size(); ++i)
        if (fsize[i] == -3) todo.push_back(i);
    int nt = threads > 0 ? threads : mando::usable_threads();
    nt = (int)std::max<size_t>(1, std::min<size_t>((size_t)nt, todo.size() / 256 + 1));
    const int dfd = open(dir, O_RDONLY | O_DIRECTORY);
    auto work = [&](int t) {
        struct stat st;
        for (size_t k = (size_t)t; k < todo.size(); k += (size_t)nt) {
            const size_t i = todo[k];
            const int r = dfd >= 0 ? fstatat(dfd, ents[i].c_str(), &st, 0) : stat((base + ents[i]).c_str(), &st);
            fsize[i] = (r == 0 && S_ISREG(st.st_mode)) ? (int64_t)st.st_size : -2;
        }
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < nt; ++t) pool.emplace_back(work, t);
    work(0);
    for (auto &th : pool) th.join();
    if (dfd >= 0) close(dfd);
    struct Root {
        std::string name;
        size_t clen;  // the chromosome is name[0, clen) (a length: short names move with their string)
        int64_t start;
        int64_t size;
    };
    std::vector<Root> roots;
    roots.reserve(ents.size());
    for (size_t i = 0; i < ents.size(); ++i) {
        if (fsize[i] == -2) continue;
        const std::string &n = ents[i];
        const size_t cut = n.find(".psl");
        roots.push_back(Root{n.substr(0, cut), 0, 0, cut + 4 == n.size() ? fsize[i] : -1});
    }
    // one root per name; the exact <root>.psl entry carries the size (only an entry with more after
    // ".psl" -- a.psl.bak -- can repeat a root: the usual directory needs no de-duplication pass)
    bool extra = false;
    for (const Root &r : roots) extra |= r.size < 0;
    if (extra) {
        std::sort(roots.begin(), roots.end(), [](const Root &a, const Root &b) {
            return a.name != b.name ? a.name < b.name : a.size > b.size;
        });
        roots.erase(std::unique(roots.begin(), roots.end(), [](const Root &a, const Root &b) { return a.name == b.name; }),
                    roots.end());
    }
    for (Root &r : roots) {
        const size_t t1 = r.name.find('~');
        if (t1 == std::string::npos) return MANDO_E_ARG;  // the reference's split('~')[1] raises
        const size_t t2 = r.name.find('~', t1 + 1);
        const std::string_view f(r.name.data() + t1 + 1, (t2 == std::string::npos ? r.name.size() : t2) - t1 - 1);
        if (f.empty() || f.size() > 18) return MANDO_E_ARG;
        int64_t v = 0;
        for (char c : f) {
            if (c < '0' || c > '9') return MANDO_E_ARG;
            v = v * 10 + (c - '0');
        }
        r.clen = t1;
        r.start = v;
    }
    // order by (chromosome bytes, start, root): chromosomes ranked once (a few dozen distinct names), then
    // an index sort on (rank, start) -- string compares only on the rare (chromosome, start) ties
    std::unordered_map<std::string_view, int32_t> chrom_rank;
    for (const Root &r : roots) chrom_rank.try_emplace(std::string_view(r.name.data(), r.clen), 0);
    {
        std::vector<std::string_view> ch;
        ch.reserve(chrom_rank.size());
        for (const auto &kv : chrom_rank) ch.push_back(kv.first);
        std::sort(ch.begin(), ch.end());  // bytes (UTF-8 keeps code point order)
        for (size_t k = 0; k < ch.size(); ++k) chrom_rank[ch[k]] = (int32_t)k;
    }
    struct Key {
        int32_t chrom;
        int32_t idx;
        int64_t start;
    };
    std::vector<Key> key(roots.size());
    for (size_t i = 0; i < roots.size(); ++i)
        key[i] = Key{chrom_rank[std::string_view(roots[i].name.data(), roots[i].clen)], (int32_t)i, roots[i].start};
    std::sort(key.begin(), key.end(), [&](const Key &a, const Key &b) {
        if (a.chrom != b.chrom) return a.chrom < b.chrom;
        if (a.start != b.start) return a.start < b.start;
        return roots[(size_t)a.idx].name < roots[(size_t)b.idx].name;
    });
    int64_t need = 0;
    for (const Root &r : roots) need += (int64_t)r.name.size() + 1;
    *n_roots = (int64_t)roots.size();
    *names_bytes = need;
    if (need > names_cap || (int64_t)roots.size() > sizes_cap || (!names && need) || (with_sizes && !sizes && !roots.empty()))
        return MANDO_E_CAP;
    int64_t o = 0;
    for (size_t k = 0; k < roots.size(); ++k) {
        const Root &r = roots[(size_t)key[k].idx];
        memcpy(names + o, r.name.c_str(), r.name.size() + 1);
        o += (int64_t)r.name.size() + 1;
        if (with_sizes) sizes[k] = r.size;
    }
    return MANDO_OK;
}
}  // namespace

extern "C" int mando_list_roots(const char *dir, int32_t threads, char *names, int64_t names_cap, int64_t *sizes,
                                int64_t sizes_cap, int64_t *n_roots, int64_t *names_bytes) {
    return list_roots(dir, threads, true, names, names_cap, sizes, sizes_cap, n_roots, names_bytes);
}

extern "C" int mando_list_root_names(const char *dir, char *names, int64_t names_cap, int64_t *n_roots,
                                     int64_t *names_bytes) {
    return list_roots(dir, 0, false, names, names_cap, nullptr, INT64_MAX, n_roots, names_bytes);
}

// sizes[i] = size of <dir>/<root i>.psl when that is a regular file (symlinks followed), else -1; the
// roots are n NUL-terminated names back to back (a slice of mando_list_root_names' output)
extern "C" int mando_root_sizes(const char *dir, const char *names, int64_t n, int32_t threads, int64_t *sizes) {
    if (!dir || n < 0 || (n && (!names || !sizes))) return MANDO_E_ARG;
    std::vector<const char *> nm((size_t)n);
    for (int64_t i = 0, o = 0; i < n; ++i) {
        nm[(size_t)i] = names + o;
        o += (int64_t)strlen(names + o) + 1;
    }
    int nt = threads > 0 ? threads : mando::usable_threads();
    nt = (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)nt, n / 256 + 1));
    const int dfd = open(dir, O_RDONLY | O_DIRECTORY);
    if (dfd < 0) return MANDO_E_ARG;
    auto work = [&](int t) {
        struct stat st;
        std::string f;
        for (int64_t i = t; i < n; i += nt) {
            f.assign(nm[(size_t)i]);
            f += ".psl";
            sizes[i] = (fstatat(dfd, f.c_str(), &st, 0) == 0 && S_ISREG(st.st_mode)) ? (int64_t)st.st_size : -1;
        }
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < nt; ++t) pool.emplace_back(work, t);
    work(0);
    for (auto &th : pool) th.join();
    close(dfd);
    return MANDO_OK;
}
