// module_f.cpp — modules F (isoform filtering) and Q (quantification) natively (SURVEY.md §8(f) rows
// 3 and 4), the consumers of the D module's consensi.  Restates
//   filterIsoforms.py:280-296 filter_sam, :310-385 parse_clean_psl, :81-123 get_count / filter_isoforms,
//   :125-278 look_for_contained_isoforms, :388-410 collect_chromosomes / readWhiteList /
//   write_isoforms, :413-433 psl_to_gtf, :456-510 process_chr / main (minus the minimap2 call, which
//   stays an external aligner, and emtrey / clean_psl, which are sam.cpp)
//   assignReadsToIsoforms.py:27-105 (quant + TPM tables)
// with the reference's Python semantics: half-even `round(x, -1)`, float division and `repr` in the
// reason texts, Python slicing for the genomic A content, the junction-table quirk of the containment
// test (a later junction's window resets an earlier one's base1 rows) and input-order outputs.
// Chromosomes are processed in parallel (independent, like the reference's Pool) and written in
// sorted order.  Where the reference picks "the first element of a set" (reason texts only) this
// picks the smallest name.
#include "threads.h"
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <charconv>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/mando.h"
#include "modf.h"
#include "quant.h"

namespace {

using std::string;
using std::string_view;
using std::vector;

bool read_file(const char *path, string &out) {
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

// whole file through zlib (plain or gzip, like mappy.fastx_read)
bool read_any(const char *path, string &out) {
    gzFile g = gzopen(path, "rb");
    if (!g) return false;
    out.clear();
    char buf[1 << 16];
    int n;
    while ((n = gzread(g, buf, sizeof buf)) > 0) out.append(buf, (size_t)n);
    const bool ok = n == 0;
    gzclose(g);
    return ok;
}

// mappy.fastx_read: FASTA or FASTQ records, name = header up to the first blank
template <bool kSeq = true, class F>
bool fastx_each_in(const string &buf, F &&fn) {
    size_t p = 0;
    const size_t n = buf.size();
    auto line_end = [&](size_t a) {
        const size_t e = buf.find('\n', a);
        return e == string::npos ? n : e;
    };
    while (p < n && buf[p] != '>' && buf[p] != '@') p = line_end(p) + 1;
    while (p < n) {
        const bool fq = buf[p] == '@';
        size_t e = line_end(p);
        string_view head(buf.data() + p + 1, e - p - 1);
        if (!head.empty() && head.back() == '\r') head.remove_suffix(1);
        size_t sp = 0;
        while (sp < head.size() && head[sp] != ' ' && head[sp] != '\t') ++sp;
        const string_view name = head.substr(0, sp);
        p = e + 1;
        string seq;
        size_t seqlen = 0;
        while (p < n && buf[p] != '>' && buf[p] != '@' && !(fq && buf[p] == '+')) {
            e = line_end(p);
            string_view l(buf.data() + p, e - p);
            if (!l.empty() && l.back() == '\r') l.remove_suffix(1);
            if (kSeq) seq.append(l.data(), l.size());
            seqlen += l.size();
            p = e + 1;
        }
        if (fq && p < n && buf[p] == '+') {
            p = line_end(p) + 1;  // '+' line
            size_t q = 0;
            while (p < n && q < seqlen) {
                e = line_end(p);
                q += e - p;
                p = e + 1;
            }
        }
        fn(name, std::move(seq));
    }
    return true;
}
template <class F>
bool fastx_each(const char *path, F &&fn) {
    string buf;
    if (!read_any(path, buf)) return false;
    return fastx_each_in(buf, std::forward<F>(fn));
}

void split(string_view s, char sep, vector<string_view> &out) {
    out.clear();
    size_t a = 0;
    while (true) {
        const size_t c = s.find(sep, a);
        if (c == string_view::npos) {
            out.push_back(s.substr(a));
            return;
        }
        out.push_back(s.substr(a, c - a));
        a = c + 1;
    }
}

string_view strip(string_view s) {
    size_t a = 0, b = s.size();
    while (a < b && isspace((unsigned char)s[a])) ++a;
    while (b > a && isspace((unsigned char)s[b - 1])) --b;
    return s.substr(a, b - a);
}

bool to_i64(string_view s, int64_t &v) {
    s = strip(s);
    if (s.empty()) return false;
    bool neg = false;
    size_t i = 0;
    if (s[0] == '-' || s[0] == '+') {
        neg = s[0] == '-';
        i = 1;
    }
    if (i == s.size()) return false;
    v = 0;
    for (; i < s.size(); ++i) {
        if (s[i] < '0' || s[i] > '9') return false;
        v = v * 10 + (s[i] - '0');
    }
    if (neg) v = -v;
    return true;
}

// Python repr(float)
string py_repr(double x) {
    if (x == 0) return std::signbit(x) ? "-0.0" : "0.0";
    if (std::isinf(x)) return x > 0 ? "inf" : "-inf";
    char buf[64];
    auto r = std::to_chars(buf, buf + sizeof buf, x, std::chars_format::scientific);
    string sci(buf, r.ptr);
    const size_t e = sci.find('e');
    string mant = sci.substr(0, e);
    const int exp = atoi(sci.c_str() + e + 1);
    bool neg = false;
    if (mant[0] == '-') {
        neg = true;
        mant.erase(0, 1);
    }
    string digits;
    for (char c : mant)
        if (c != '.') digits += c;
    string out;
    if (exp < -4 || exp >= 16) {
        out = digits.substr(0, 1);
        if (digits.size() > 1) out += "." + digits.substr(1);
        char eb[16];
        snprintf(eb, sizeof eb, "e%c%02d", exp < 0 ? '-' : '+', exp < 0 ? -exp : exp);
        out += eb;
    } else if (exp >= 0) {
        if ((int)digits.size() <= exp + 1)
            out = digits + string((size_t)(exp + 1 - (int)digits.size()), '0') + ".0";
        else
            out = digits.substr(0, (size_t)exp + 1) + "." + digits.substr((size_t)exp + 1);
    } else {
        out = "0." + string((size_t)(-exp - 1), '0') + digits;
    }
    return neg ? "-" + out : out;
}

// Python round(x, 3): the exact binary value rounded half-even to 3 decimals, back to the nearest double
double py_round3(double x) {
    char buf[64];
    snprintf(buf, sizeof buf, "%.3f", x);
    return strtod(buf, nullptr);
}

// Python round(int, -1): half-even to a multiple of 10
int64_t round10(int64_t x) {
    int64_t q = x / 10, r = x % 10;
    if (r < 0) {
        r += 10;
        --q;
    }
    if (r > 5 || (r == 5 && (q & 1))) ++q;
    return q * 10;
}

int64_t abundance_of(string_view name, bool &ok) {
    const size_t u = name.rfind('_');
    int64_t v = 0;
    ok = to_i64(u == string_view::npos ? name : name.substr(u + 1), v);
    return v;
}

using mando::modf::ChrState;
using mando::modf::Contain;
using mando::modf::Iso;
using mando::modf::Ivs;

struct ChrOut {
    vector<int> kept;  // indices into isos, output order
    string reasons;
    int err = 0;
};

Ivs merged_extended(const vector<int64_t> &c, int sw) {
    Ivs v;
    for (size_t k = 0; k + 1 < c.size(); k += 2) v.push_back({c[k] - sw, c[k + 1] + sw});
    std::sort(v.begin(), v.end());
    Ivs m;
    for (auto &x : v) {
        if (x.first >= x.second) continue;
        if (!m.empty() && x.first <= m.back().second)
            m.back().second = std::max(m.back().second, x.second);
        else
            m.push_back(x);
    }
    return m;
}
bool ivs_cover(const Ivs &m, int64_t s, int64_t e) {  // [s, e) inside one merged interval
    auto it = std::upper_bound(m.begin(), m.end(), std::make_pair(s, INT64_MAX));
    if (it == m.begin()) return false;
    --it;
    return it->first <= s && e <= it->second;
}
int64_t ivs_count(const Ivs &m, int64_t s, int64_t e) {  // bases of [s, e) covered
    int64_t n = 0;
    for (auto &x : m) n += std::max<int64_t>(0, std::min(e, x.second) - std::max(s, x.first));
    return n;
}

// filterIsoforms.process_chr for one chromosome, part 1: parse_clean_psl (absolute filters), get_count and
// filter_isoforms (relative expression), and the candidate index of look_for_contained_isoforms
void chr_stage1(const mando_filter_params &P, const string &chrom, vector<Iso> &isos,
                const vector<std::pair<string_view, string_view>> &lines_raw, ChrState &S, ChrOut &out) {
    string &R = out.reasons;
    R += chrom + "\n";
    // parse_clean_psl (absolute filters), input order
    std::unordered_set<string> done;
    vector<int> &listed = S.listed;  // names passing parse, in line order (psl_dict)
    vector<string_view> a, bs, bt;
    for (auto &lr : lines_raw) {
        split(strip(lr.second), '\t', a);
        if (a.size() < 21) {
            out.err = MANDO_E_ARG;
            return;
        }
        int64_t qs, qe, qsize;
        if (!to_i64(a[11], qs) || !to_i64(a[12], qe) || !to_i64(a[10], qsize)) {
            out.err = MANDO_E_ARG;
            return;
        }
        const int64_t readlength = qe - qs;
        const string_view dir = a[8];
        split(a[18], ',', bs);
        const int64_t exon_number = (int64_t)bs.size() - 1;
        int64_t o5 = 0, o3 = 0;
        if (dir == "+") {
            o5 = qs;
            o3 = qsize - qe;
        } else if (dir == "-") {
            o3 = qs;
            o5 = qsize - qe;
        } else {
            out.err = MANDO_E_ARG;
            return;
        }
        const string name(a[9]);
        if (done.count(name)) continue;  // (the reference prints the line to stdout)
        done.insert(name);
        bool ok;
        const int64_t ab = abundance_of(name, ok);
        if (!ok) {
            out.err = MANDO_E_ARG;
            return;
        }
        if (readlength >= P.minimum_isoform_length) {
            if ((double)ab >= P.minimum_reads) {
                if (P.overhangs[0] <= o5 && o5 <= P.overhangs[1] && P.overhangs[2] <= o3 && o3 <= P.overhangs[3]) {
                    if (P.multi_exon_only == 0 || exon_number > 1) {
                        Iso I;
                        I.name = name;
                        for (auto f : a) I.fields.emplace_back(f);
                        I.dir = dir[0];
                        I.abundance = ab;
                        split(a[20], ',', bt);
                        for (int64_t k = 0; k < exon_number; ++k) {
                            int64_t s0, sz;
                            if ((size_t)k >= bt.size() || !to_i64(bt[(size_t)k], s0) || !to_i64(bs[(size_t)k], sz)) {
                                out.err = MANDO_E_ARG;
                                return;
                            }
                            I.coords.push_back(s0);
                            I.coords.push_back(s0 + sz);
                        }
                        listed.push_back((int)isos.size());
                        isos.push_back(std::move(I));
                    } else {
                        R += name + " filtered because it only had a single exon and the multi_exon_only flag was set \n";
                    }
                } else {
                    R += name + " filtered because at " + std::to_string(o5) + " and " + std::to_string(o3) +
                         " its number of overhanging bases did not fall within the predefined bins of " +
                         std::to_string(P.overhangs[0]) + "-" + std::to_string(P.overhangs[1]) + " and " +
                         std::to_string(P.overhangs[2]) + "-" + std::to_string(P.overhangs[3]) + "\n";
                }
            } else {
                R += name + " filtered because it at " + std::to_string(ab) +
                     " reads it did not match the minimum absolute read requirement of " + py_repr(P.minimum_reads) +
                     "\n";
            }
        } else {
            R += name + " filtered because at " + std::to_string(readlength) +
                 "nt it did not match the minimum isoform length requirement of " +
                 std::to_string(P.minimum_isoform_length) + "\n";
        }
    }
    // get_count: per direction, 10-nt bins of round(start,-1)..round(end,-1) summed over isoforms
    std::unordered_map<int64_t, int64_t> count[2];
    for (int k : listed) {
        const Iso &I = isos[(size_t)k];
        if (I.coords.empty()) {  // IndexError in the reference
            out.err = MANDO_E_ARG;
            return;
        }
        auto &cm = count[I.dir == '-'];
        for (int64_t b = round10(I.coords.front()); b < round10(I.coords.back()); b += 10) cm[b] += I.abundance;
    }
    // filter_isoforms: sorted names, relative expression
    vector<int> order = listed;
    std::sort(order.begin(), order.end(), [&](int x, int y) { return isos[(size_t)x].name < isos[(size_t)y].name; });
    vector<int> &kept1 = S.kept1;
    for (int k : order) {
        const Iso &I = isos[(size_t)k];
        int64_t s0, e0;
        if (!to_i64(I.fields[15], s0) || !to_i64(I.fields[16], e0)) {
            out.err = MANDO_E_ARG;
            return;
        }
        auto &cm = count[I.dir == '-'];
        int64_t mx = 0;
        bool any = false;
        for (int64_t b = round10(s0); b < round10(e0); b += 10) {
            auto it = cm.find(b);
            if (it == cm.end()) {  // KeyError in the reference
                out.err = MANDO_E_ARG;
                return;
            }
            mx = any ? std::max(mx, it->second) : it->second;
            any = true;
        }
        if (!any || mx == 0) {  // max([]) / ZeroDivisionError in the reference
            out.err = MANDO_E_ARG;
            return;
        }
        const double ratio = (double)I.abundance / (double)mx;
        if (ratio >= P.minimum_ratio) {
            kept1.push_back(k);
        } else {
            R += I.name + " filtered because it at " + std::to_string(I.abundance) + " reads it only reached a " +
                 py_repr(ratio) + " ratio of expression in its locus which is below the minimum ratio of " +
                 py_repr(P.minimum_ratio) + "\n";
        }
    }
    // look_for_contained_isoforms
    const int sw = P.splice_window;
    vector<Ivs> &ext = S.ext;
    ext.assign(isos.size(), Ivs());
    for (int k : kept1) ext[(size_t)k] = merged_extended(isos[(size_t)k].coords, sw);
    // candidates by direction, sorted by span start for the overlap search
    auto &bydir = S.bydir;
    for (int k : kept1) bydir[isos[(size_t)k].dir == '-'].push_back(k);
    for (auto &v : bydir)
        std::sort(v.begin(), v.end(), [&](int x, int y) {
            return ext[(size_t)x].front().first < ext[(size_t)y].front().first;
        });
    auto &maxspan = S.maxspan;
    for (int d = 0; d < 2; ++d)
        for (int k : bydir[d])
            maxspan[d] = std::max(maxspan[d], ext[(size_t)k].back().second - ext[(size_t)k].front().first);
}

// trimmed block coordinates of look_for_contained_isoforms (the first start +20, the last end -20,
// each clamped by its block's other end; for one block the end clamps against the trimmed start)
void trimmed(const vector<int64_t> &co, vector<int64_t> &c) {
    c = co;
    c[0] = std::min(c[0] + 20, c[1]);
    c[c.size() - 1] = std::max(c[c.size() - 1] - 20, c[c.size() - 2]);
}

// every junction of c (trimmed, isoform A) matches one of mc (isoform B): the reference's dd table keeps,
// for a base1 position, the window of B's LAST junction whose base1 window holds it
bool junctions_contained(const vector<int64_t> &c, const vector<int64_t> &mc, int sw) {
    std::unordered_map<int64_t, std::pair<int64_t, int64_t>> dd;  // base1 -> [b2lo, b2hi)
    for (size_t jn = 1; jn + 1 < mc.size(); jn += 2)
        for (int64_t b1 = mc[jn] - sw; b1 < mc[jn] + sw; ++b1) dd[b1] = {mc[jn + 1] - sw, mc[jn + 1] + sw};
    for (size_t jn = 1; jn + 1 < c.size(); jn += 2) {
        bool hit = false;
        for (int64_t b1 = c[jn] - sw; b1 < c[jn] + sw && !hit; ++b1) {
            auto it = dd.find(b1);
            if (it == dd.end()) continue;
            const int64_t a2lo = c[jn + 1] - sw, a2hi = c[jn + 1] + sw;
            if (std::max(a2lo, it->second.first) < std::min(a2hi, it->second.second)) hit = true;
        }
        if (!hit) return false;
    }
    return true;
}

// look_for_contained_isoforms' candidate search for isoform k on the host (modf.h Contain)
Contain contain_host(const mando_filter_params &P, const vector<Iso> &isos, const ChrState &S, int k) {
    const Iso &I = isos[(size_t)k];
    const int d = I.dir == '-';
    vector<int64_t> c;
    trimmed(I.coords, c);
    const int64_t start = I.coords.front(), end = I.coords.back();
    const int64_t pa0 = I.dir == '+' ? end + 3 : start - 23;
    const int64_t lo = std::min(c.front(), pa0), hi = std::max(c.back(), pa0 + 20);
    bool any_base = false;
    for (size_t q = 0; q + 1 < c.size(); q += 2)
        if (c[q] < c[q + 1]) any_base = true;
    Contain r;
    vector<int> status;
    const auto &cand = S.bydir[d];
    auto first = std::lower_bound(cand.begin(), cand.end(), lo - S.maxspan[d] - 1, [&](int x, int64_t v) {
        return S.ext[(size_t)x].front().first < v;
    });
    for (auto it = first; it != cand.end(); ++it) {
        const Ivs &m = S.ext[(size_t)*it];
        if (m.front().first >= hi) break;
        if (m.back().second <= lo) continue;
        if (ivs_count(m, pa0, pa0 + 20) >= 10) {
            ++r.n_extend;
            if (r.ext_first < 0 || isos[(size_t)*it].name < isos[(size_t)r.ext_first].name) r.ext_first = *it;
        }
        if (any_base) {
            bool all = true;
            for (size_t q = 0; q + 1 < c.size() && all; q += 2)
                if (c[q] < c[q + 1] && !ivs_cover(m, c[q], c[q + 1])) all = false;
            if (all) status.push_back(*it);
        }
    }
    if (!any_base) status = S.listed;  // no base to intersect over: every parsed isoform of the chromosome
    r.n_status = (int64_t)status.size();
    for (int mk : status) {
        if (mk == k) continue;
        const Iso &Mt = isos[(size_t)mk];
        if (r.trig >= 0 && !(Mt.name < isos[(size_t)r.trig].name)) continue;
        if (!junctions_contained(c, Mt.coords, P.splice_window)) continue;
        int kind = 0;
        if (Mt.abundance == 0)
            kind = 3;
        else if ((double)I.abundance / (double)Mt.abundance < P.internal_ratio)
            kind = 1;
        else if (std::llabs(I.coords.front() - Mt.coords.front()) < P.downstream_buffer &&
                 std::llabs(I.coords.back() - Mt.coords.back()) < P.downstream_buffer && I.abundance < Mt.abundance)
            kind = 2;
        if (kind) {
            r.trig = mk;
            r.kind = kind;
        }
    }
    return r;
}

// part 3: the polyA test and the containment decisions of kept1, in order, into the kept list and the
// reason texts (filterIsoforms.py:125-278)
void chr_stage3(const mando_filter_params &P, const vector<Iso> &isos, const ChrState &S, const vector<Contain> &dec,
                const string *chr_seq, const std::set<int64_t> *wl_plus, const std::set<int64_t> *wl_minus,
                ChrOut &out) {
    string &R = out.reasons;
    const int64_t L = chr_seq ? (int64_t)chr_seq->size() : 0;
    auto py_slice_count = [&](int64_t s, int64_t e, char ch) {
        // chr_sequence[s:e].upper().count(ch) with Python slice semantics
        if (s < 0) s = std::max<int64_t>(0, s + L);
        if (e < 0) e = std::max<int64_t>(0, e + L);
        s = std::min(s, L);
        e = std::min(e, L);
        int64_t n = 0;
        for (int64_t x = s; x < e; ++x) n += (toupper((unsigned char)(*chr_seq)[(size_t)x]) == ch);
        return n;
    };
    for (size_t t = 0; t < S.kept1.size(); ++t) {
        const int k = S.kept1[t];
        const Iso &I = isos[(size_t)k];
        const Contain &D = dec[t];
        if (!chr_seq) {
            out.err = MANDO_E_ARG;  // KeyError: chromosome not in the genome
            return;
        }
        const int64_t start = I.coords.front(), end = I.coords.back();
        double Acontent;
        int64_t polyApos;
        if (I.dir == '+') {
            Acontent = (double)py_slice_count(end, end + 15, 'A') / 15.0;
            polyApos = end;
        } else {
            Acontent = (double)py_slice_count(start - 15, start, 'T') / 15.0;
            polyApos = start;
        }
        if (D.n_status + D.n_extend == 1) {
            out.kept.push_back(k);
            continue;
        }
        bool decision = true;
        if (D.n_extend > 0 && Acontent > P.Acutoff) {
            const std::set<int64_t> *wl = I.dir == '+' ? wl_plus : wl_minus;
            const string &fname = isos[(size_t)D.ext_first].name;
            if (wl && wl->count(polyApos)) {
                R += I.name + " would have been filtered because at least one isoform (including " + fname +
                     ") is extending beyond its polyA site and the genomic A content at its putative polyA site is " +
                     py_repr(Acontent) + " which is higher than the cutoff set to " + py_repr(P.Acutoff) +
                     "but it was kept because its polyA site was part of the polyA site whitelist\n";
            } else {
                decision = false;
                R += I.name + " filtered because at least one isoform (including " + fname +
                     ") is extending beyond its polyA site and the genomic A content at its putative polyA site is " +
                     py_repr(Acontent) + " which is higher than the cutoff set to " + py_repr(P.Acutoff) + "\n";
            }
        }
        if (decision && D.trig >= 0) {
            const Iso &Mt = isos[(size_t)D.trig];
            if (D.kind == 3) {  // ZeroDivisionError in the reference
                out.err = MANDO_E_ARG;
                return;
            }
            if (D.kind == 1) {
                R += I.name + " filtered because it is internal to (all bases and splice junctions contained in) " +
                     Mt.name + " and expressed at " + std::to_string(I.abundance) + " reads compared to " +
                     std::to_string(Mt.abundance) +
                     " reads for the isoform containing it which is below that internal ratio of " +
                     py_repr(P.internal_ratio) + "\n";
            } else {
                R += I.name + " filtered because it is internal (all bases and splice junctions contained in) and almost identical to " +
                     Mt.name + "\n";
            }
            decision = false;
        }
        if (decision) out.kept.push_back(k);
    }
}

// filterIsoforms.process_chr for one chromosome on the host
void process_chr(const mando_filter_params &P, const string &chrom, vector<Iso> &isos,
                 const vector<std::pair<string_view, string_view>> &lines_raw, const string *chr_seq,
                 const std::set<int64_t> *wl_plus, const std::set<int64_t> *wl_minus, ChrOut &out) {
    ChrState S;
    chr_stage1(P, chrom, isos, lines_raw, S, out);
    if (out.err) return;
    vector<Contain> dec;
    dec.reserve(S.kept1.size());
    for (int k : S.kept1) dec.push_back(contain_host(P, isos, S, k));
    chr_stage3(P, isos, S, dec, chr_seq, wl_plus, wl_minus, out);
}

}  // namespace

namespace mando {
namespace modq {

bool fastx_names(const char *path, std::string &buf, std::vector<std::pair<int64_t, int32_t>> &names) {
    names.clear();
    if (!read_any(path, buf)) return false;
    const char *base = buf.data();
    return fastx_each_in<false>(buf, [&](string_view nm, string &&) {
        names.push_back({(int64_t)(nm.data() - base), (int32_t)nm.size()});
    });
}

bool psl_isoforms(const std::string &buf, std::vector<std::string_view> &isos) {
    vector<string_view> a;
    size_t p = 0;
    while (p < buf.size()) {
        size_t e = buf.find('\n', p);
        if (e == string::npos) e = buf.size();
        const string_view ln(buf.data() + p, e - p);
        p = e + 1;
        split(strip(ln), '\t', a);
        if (a.size() < 10) return false;
        isos.push_back(a[9]);
    }
    return true;
}

int write_tables(const std::vector<std::string> &samples, const std::vector<int64_t> &total,
                 const std::vector<std::string_view> &isos, const std::vector<int64_t> &counts, const char *out_quant,
                 const char *out_tpm) {
    string q = "Isoform\t", t = "Isoform\t";
    for (auto &s : samples) {
        q += s + "\t";
        t += s + "\t";
    }
    q += "\n";
    t += "\n";
    const size_t ns = samples.size();
    for (size_t k = 0; k < isos.size(); ++k) {
        q += string(isos[k]) + "\t";
        t += string(isos[k]) + "\t";
        for (size_t s = 0; s < ns; ++s) {
            if (total[s] == 0) return MANDO_E_ARG;  // ZeroDivisionError in the reference
            const int64_t c = counts[k * ns + s];
            q += std::to_string(c) + "\t";
            t += py_repr(py_round3((double)c / (double)total[s] * 1000000.0)) + "\t";
        }
        q += "\n";
        t += "\n";
    }
    FILE *fq = fopen(out_quant, "wb");
    FILE *ft = fopen(out_tpm, "wb");
    if (!fq || !ft) {
        if (fq) fclose(fq);
        if (ft) fclose(ft);
        return MANDO_E_ARG;
    }
    fwrite(q.data(), 1, q.size(), fq);
    fwrite(t.data(), 1, t.size(), ft);
    fclose(fq);
    fclose(ft);
    return MANDO_OK;
}

}  // namespace modq

namespace modf {

int filter_isoforms_impl(const mando_filter_params *P, const char *isoform_fasta, const char *genome_fasta,
                         const char *clean_psl, const char *whitelist_bed, const char *out_fasta, const char *out_psl,
                         const char *reasons_path, int64_t *n_kept, const ContainStage *stage) {
    if (!P || !isoform_fasta || !genome_fasta || !clean_psl || !out_fasta || !out_psl) return MANDO_E_ARG;
    std::unordered_map<string, string> isoforms, genome;
    if (!fastx_each(isoform_fasta, [&](string_view n, string &&s) { isoforms[string(n)] = std::move(s); }))
        return MANDO_E_ARG;
    if (!fastx_each(genome_fasta, [&](string_view n, string &&s) { genome[string(n)] = std::move(s); }))
        return MANDO_E_ARG;
    string pbuf;
    if (!read_file(clean_psl, pbuf)) return MANDO_E_ARG;
    // collect_chromosomes (sorted) and the per-chromosome line lists (file order)
    std::map<string, vector<std::pair<string_view, string_view>>> bychr;
    {
        size_t p = 0;
        vector<string_view> a;
        while (p < pbuf.size()) {
            size_t e = pbuf.find('\n', p);
            if (e == string::npos) e = pbuf.size();
            const string_view ln(pbuf.data() + p, e - p);
            p = e + 1;
            split(strip(ln), '\t', a);
            if (a.size() < 14) return MANDO_E_ARG;
            bychr[string(a[13])].push_back({a[13], ln});
        }
    }
    // readWhiteList: bed [start, end) positions per chromosome and strand (column 6)
    std::unordered_map<string, std::set<int64_t>> wlp, wlm;
    if (whitelist_bed) {
        string wbuf;
        if (read_file(whitelist_bed, wbuf)) {
            size_t p = 0;
            vector<string_view> a;
            while (p < wbuf.size()) {
                size_t e = wbuf.find('\n', p);
                if (e == string::npos) e = wbuf.size();
                const string_view ln(wbuf.data() + p, e - p);
                p = e + 1;
                split(strip(ln), '\t', a);
                if (a.size() < 6) continue;
                int64_t s0, e0;
                if (!to_i64(a[1], s0) || !to_i64(a[2], e0)) return MANDO_E_ARG;
                auto &st = a[5] == "+" ? wlp[string(a[0])] : wlm[string(a[0])];
                for (int64_t x = s0; x < e0; ++x) st.insert(x);
            }
        } else {
            return MANDO_E_ARG;  // open() fails in the reference
        }
    }
    vector<string> chroms;
    for (auto &kv : bychr) {
        chroms.push_back(kv.first);
        if (!genome.count(kv.first)) return MANDO_E_ARG;  // KeyError on genome_sequence[chromosome]
    }
    vector<vector<Iso>> isos(chroms.size());
    vector<ChrOut> outs(chroms.size());
    std::atomic<size_t> next{0};
    int nth = P->threads > 0 ? P->threads : mando::usable_threads();
    nth = (int)std::min<size_t>((size_t)nth, std::max<size_t>(1, chroms.size()));
    auto run = [&](auto &&fn) {
        next = 0;
        auto work = [&]() {
            for (size_t i; (i = next.fetch_add(1)) < chroms.size();) fn(i);
        };
        vector<std::thread> th;
        for (int t = 0; t < nth; ++t) th.emplace_back(work);
        for (auto &t : th) t.join();
    };
    auto seq_of = [&](size_t i) {
        auto g = genome.find(chroms[i]);
        return g == genome.end() ? nullptr : &g->second;
    };
    auto wl_of = [&](std::unordered_map<string, std::set<int64_t>> &w, size_t i) {
        auto it = w.find(chroms[i]);
        return it == w.end() ? nullptr : &it->second;
    };
    if (!stage) {
        run([&](size_t i) {
            process_chr(*P, chroms[i], isos[i], bychr[chroms[i]], seq_of(i), wl_of(wlp, i), wl_of(wlm, i), outs[i]);
        });
    } else {
        // the parse and the ratio filter per chromosome, then every chromosome's containment search at
        // once, then the decisions
        vector<ChrState> states(chroms.size());
        run([&](size_t i) { chr_stage1(*P, chroms[i], isos[i], bychr[chroms[i]], states[i], outs[i]); });
        for (auto &o : outs)
            if (o.err) return o.err;
        vector<vector<Contain>> dec(chroms.size());
        const int rc = (*stage)(*P, isos, states, dec);
        if (rc) return rc;
        run([&](size_t i) {
            chr_stage3(*P, isos[i], states[i], dec[i], seq_of(i), wl_of(wlp, i), wl_of(wlm, i), outs[i]);
        });
    }
    for (auto &o : outs)
        if (o.err) return o.err;
    FILE *fa = fopen(out_fasta, "wb");
    FILE *fp = fopen(out_psl, "wb");
    if (!fa || !fp) {
        if (fa) fclose(fa);
        if (fp) fclose(fp);
        return MANDO_E_ARG;
    }
    int64_t kept = 0;
    int rc = MANDO_OK;
    for (size_t i = 0; i < chroms.size() && rc == MANDO_OK; ++i) {
        for (int k : outs[i].kept) {
            const Iso &I = isos[i][(size_t)k];
            auto it = isoforms.find(I.name);
            if (it == isoforms.end()) {  // KeyError in the reference
                rc = MANDO_E_ARG;
                break;
            }
            fprintf(fa, ">%s\n%s\n", I.name.c_str(), it->second.c_str());
            string line;
            for (size_t f = 0; f < I.fields.size(); ++f) {
                if (f) line += '\t';
                line += I.fields[f];
            }
            line += '\n';
            fwrite(line.data(), 1, line.size(), fp);
            ++kept;
        }
    }
    fclose(fa);
    fclose(fp);
    if (rc) return rc;
    if (reasons_path) {
        FILE *fr = fopen(reasons_path, "wb");
        if (!fr) return MANDO_E_ARG;
        for (auto &o : outs) fwrite(o.reasons.data(), 1, o.reasons.size(), fr);
        fclose(fr);
    }
    if (n_kept) *n_kept = kept;
    return MANDO_OK;
}

}  // namespace modf
}  // namespace mando

extern "C" {

void mando_filter_default_params(mando_filter_params *p) {
    p->minimum_ratio = 0.01;
    p->minimum_reads = 3;
    p->internal_ratio = 1;
    p->Acutoff = 0.5;
    p->overhangs[0] = 0;
    p->overhangs[1] = 40;
    p->overhangs[2] = 0;
    p->overhangs[3] = 40;
    p->splice_window = 1;
    p->downstream_buffer = 50;
    p->minimum_isoform_length = 200;
    p->multi_exon_only = 0;
    p->threads = 0;
}

int mando_filter_sam(const char *sam_path, const char *out_path, int64_t *n_kept) {
    if (!sam_path || !out_path) return MANDO_E_ARG;
    string buf;
    if (!read_file(sam_path, buf)) return MANDO_E_ARG;
    FILE *o = fopen(out_path, "wb");
    if (!o) return MANDO_E_ARG;
    int64_t kept = 0;
    size_t p = 0;
    vector<string_view> a;
    int rc = MANDO_OK;
    while (p < buf.size()) {
        size_t e = buf.find('\n', p);
        const size_t ee = e == string::npos ? buf.size() : e + 1;
        const string_view ln(buf.data() + p, ee - p);
        p = ee;
        if (!ln.empty() && ln[0] == '@') {
            fwrite(ln.data(), 1, ln.size(), o);
            continue;
        }
        split(strip(ln), '\t', a);
        int64_t flag;
        if (a.size() < 2 || !to_i64(a[1], flag)) {
            rc = MANDO_E_ARG;
            break;
        }
        if ((flag >> 8) & 1 || (flag >> 11) & 1) continue;  // secondary / supplementary
        fwrite(ln.data(), 1, ln.size(), o);
        ++kept;
    }
    fclose(o);
    if (n_kept) *n_kept = kept;
    return rc;
}

int mando_psl_to_gtf(const char *psl_path, const char *gtf_path) {
    if (!psl_path || !gtf_path) return MANDO_E_ARG;
    string buf;
    if (!read_file(psl_path, buf)) return MANDO_E_ARG;
    string out;
    vector<string_view> a, bs, bt;
    size_t p = 0;
    while (p < buf.size()) {
        size_t e = buf.find('\n', p);
        if (e == string::npos) e = buf.size();
        const string_view ln(buf.data() + p, e - p);
        p = e + 1;
        split(strip(ln), '\t', a);
        int64_t start, end;
        if (a.size() < 21 || !to_i64(a[15], start) || !to_i64(a[16], end)) return MANDO_E_ARG;
        const string chrom(a[13]), dir(a[8]), name(a[9]);
        const string attr = "\t.\t" + dir + "\t.\ttranscript_id \"" + name + "\"; gene_id \"" + name + ".gene\"; gene_name \"" + name + "\"\n";
        out += chrom + "\tMandalorion\ttranscript\t" + std::to_string(start + 1) + "\t" + std::to_string(end) + attr;
        split(a[18], ',', bs);
        split(a[20], ',', bt);
        for (size_t k = 0; k + 1 < bs.size(); ++k) {
            int64_t s0, sz;
            if (k >= bt.size() || !to_i64(bt[k], s0) || !to_i64(bs[k], sz)) return MANDO_E_ARG;
            out += chrom + "\tMandalorion\texon\t" + std::to_string(s0 + 1) + "\t" + std::to_string(s0 + sz) + attr;
        }
    }
    FILE *o = fopen(gtf_path, "wb");
    if (!o) return MANDO_E_ARG;
    fwrite(out.data(), 1, out.size(), o);
    fclose(o);
    return MANDO_OK;
}

int mando_filter_isoforms(const mando_filter_params *P, const char *isoform_fasta, const char *genome_fasta,
                          const char *clean_psl, const char *whitelist_bed, const char *out_fasta, const char *out_psl,
                          const char *reasons_path, int64_t *n_kept) {
    return mando::modf::filter_isoforms_impl(P, isoform_fasta, genome_fasta, clean_psl, whitelist_bed, out_fasta,
                                             out_psl, reasons_path, n_kept, nullptr);
}

// assignReadsToIsoforms.py: per-sample read counts (.quant) and TPM (.tpm) of every filtered isoform
int mando_quantify(const char *const *fasta_paths, int32_t n_fasta, const char *r2i_path, const char *filtered_psl,
                   const char *out_quant, const char *out_tpm) {
    if (!fasta_paths || n_fasta < 0 || !r2i_path || !filtered_psl || !out_quant || !out_tpm) return MANDO_E_ARG;
    vector<string> samples;
    std::unordered_map<string, int> read_sample;
    vector<int64_t> total;
    for (int32_t i = 0; i < n_fasta; ++i) {
        const string loc(strip(string_view(fasta_paths[i])));
        samples.push_back(loc);
        total.push_back(0);
        const int si = (int)samples.size() - 1;
        string fbuf;
        if (!read_any(loc.c_str(), fbuf)) return MANDO_E_ARG;
        if (!fastx_each_in<false>(fbuf, [&](string_view nm, string &&) {
                read_sample[string(nm)] = si;
                ++total[(size_t)si];
            }))
            return MANDO_E_ARG;
    }
    std::unordered_map<string, vector<int>> r2i;  // isoform -> sample of each read
    string buf;
    if (!read_file(r2i_path, buf)) return MANDO_E_ARG;
    vector<string_view> a;
    size_t p = 0;
    while (p < buf.size()) {
        size_t e = buf.find('\n', p);
        if (e == string::npos) e = buf.size();
        const string_view ln(buf.data() + p, e - p);
        p = e + 1;
        split(strip(ln), '\t', a);
        if (a.size() < 2) return MANDO_E_ARG;
        auto it = read_sample.find(string(a[0]));
        if (it == read_sample.end()) return MANDO_E_ARG;  // KeyError in the reference
        r2i[string(a[1])].push_back(it->second);
    }
    string pbuf;
    vector<string_view> isos;
    if (!read_file(filtered_psl, pbuf) || !mando::modq::psl_isoforms(pbuf, isos)) return MANDO_E_ARG;
    vector<int64_t> counts(isos.size() * samples.size(), 0);
    for (size_t k = 0; k < isos.size(); ++k) {
        auto it = r2i.find(string(isos[k]));
        if (it == r2i.end()) return MANDO_E_ARG;  // KeyError in the reference
        for (int s : it->second) ++counts[k * samples.size() + (size_t)s];
    }
    return mando::modq::write_tables(samples, total, isos, counts, out_quant, out_tpm);
}

}  // extern "C"
