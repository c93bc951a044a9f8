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
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <string_view>
#include <vector>

#include "../../include/mando.h"

namespace {

struct Line {
    std::string_view text;  // without the trailing newline
    std::string_view chrom; // field 14 (index 13)
    int64_t start = 0, end = 0;
    bool start_ok = false;
};

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
