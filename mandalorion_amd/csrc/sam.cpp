// sam.cpp — SAM -> "Mando PSL" conversion and PSL cleaning (SURVEY.md §8(f) row 2 and the clean step
// of module P), native and threaded.  Restates
//   emtrey.py:31-152 (parseLine, `-m` mode) + :154-193 (batching, @SQ lengths, unmapped skipped)
//   clean_psl                      SpliceDefineConsensus.py:14-92 (gaps < 10 nt merged, primary only)
// including their output formatting: Python `repr` of the float accuracy, `','.join(...)+','` lists,
// the strand flip by the `ts:A:-` tag and mappy.revcomp of '-' strand sequences.  Lines keep input
// order.  Known reference crash cases (no cs tag in -m mode, zero-length alignment) return an error.
#include "threads.h"
#include <algorithm>
#include <atomic>
#include <charconv>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/mando.h"
#include "revcomp.h"

namespace {

using std::string;
using std::string_view;

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

void split(string_view s, char sep, std::vector<string_view> &out) {
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

// Python repr(float): shortest round-trip digits; scientific when the exponent is < -4 or >= 16
string py_repr(double x) {
    if (x == 0) return std::signbit(x) ? "-0.0" : "0.0";
    char buf[64];
    auto r = std::to_chars(buf, buf + sizeof buf, x, std::chars_format::scientific);
    string sci(buf, r.ptr);  // d.ddde[+-]XX
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
        if ((int)digits.size() <= exp + 1) {
            out = digits + string((size_t)(exp + 1 - (int)digits.size()), '0') + ".0";
        } else {
            out = digits.substr(0, (size_t)exp + 1) + "." + digits.substr((size_t)exp + 1);
        }
    } else {
        out = "0." + string((size_t)(-exp - 1), '0') + digits;
    }
    return neg ? "-" + out : out;
}

string revcomp(string_view s) {
    const mando::CompTable &ct = mando::comp_table();
    string o(s.rbegin(), s.rend());
    for (char &c : o) c = (char)ct.t[(uint8_t)c];
    return o;
}

string join_list(const std::vector<int64_t> &v) {
    string s;
    for (size_t i = 0; i < v.size(); ++i) {
        if (i) s += ',';
        s += std::to_string(v[i]);
    }
    return s + ",";
}

// emtrey.parseLine (mando mode when `mando`): returns false when the reference would raise
bool parse_sam_line(const std::vector<string_view> &a, int64_t qsize, bool mando, string &line) {
    if (a.size() < 11) return false;
    int64_t tstart, flag;
    if (!to_i64(a[3], tstart) || !to_i64(a[1], flag)) return false;
    tstart -= 1;
    char strand = (flag >> 4) & 1 ? '-' : '+';
    const string_view cstr = a[5];
    string sequence(a[9]);
    if (strand == '-') sequence = revcomp(sequence);
    // re.split('([MIDNSHP=X])'): numbers followed by an op letter
    struct Op {
        int64_t n;
        char op;
    };
    std::vector<Op> ops;
    {
        size_t i = 0;
        while (i < cstr.size()) {
            size_t j = i;
            while (j < cstr.size() && strchr("MIDNSHP=X", cstr[j]) == nullptr) ++j;
            if (j >= cstr.size()) break;  // trailing text without an op is dropped by the zip
            int64_t n;
            if (!to_i64(cstr.substr(i, j - i), n)) return false;
            ops.push_back({n, cstr[j]});
            i = j + 1;
        }
    }
    std::vector<int64_t> bs, qs, ts{tstart};
    int64_t qstart = 0, M = 0, I = 0, nI = 0, D = 0, nD = 0, N = 0, S = 0, H = 0, EQ = 0, X = 0, qend = 0;
    for (size_t i = 0; i < ops.size(); ++i) {
        const int64_t num = ops[i].n;
        const char op = ops[i].op;
        if (op == 'S' || op == 'H') {
            if (i == 0)
                qstart = num;
            else if (i == ops.size() - 1)
                qend = num;
        }
        if (i == 0) qs.push_back(qstart);
        switch (op) {
            case 'M':
                M += num;
                bs.push_back(num);
                qs.push_back(num + qs.back());
                ts.push_back(num + ts.back());
                break;
            case 'I':
                I += num;
                nI += 1;
                qs.back() += num;
                break;
            case 'D':
                D += num;
                nD += 1;
                ts.back() += num;
                break;
            case 'N':
                N += num;
                ts.back() += num;
                break;
            case 'S': S += num; break;
            case 'H': H += num; break;
            case '=': EQ += num; break;
            case 'X': X += num; break;
            default: break;
        }
    }
    const int64_t ID = I + D;
    const int64_t sLen = M + I + S + H + EQ + X;
    const int64_t tend = tstart + M + D + N + EQ + X;
    const int64_t end = qend == 0 ? sLen : sLen - qend;
    if (!qs.empty()) qs.pop_back();
    if (!ts.empty()) ts.pop_back();
    int64_t NM = 0, ambig = 0;
    string cs;
    bool have_cs = false;
    for (size_t k = 9; k < a.size(); ++k) {
        const string_view col = a[k];
        auto third = [&](string_view c) -> string_view {
            const size_t p1 = c.find(':');
            const size_t p2 = p1 == string_view::npos ? p1 : c.find(':', p1 + 1);
            if (p2 == string_view::npos) return string_view();
            const size_t p3 = c.find(':', p2 + 1);
            return c.substr(p2 + 1, p3 == string_view::npos ? string_view::npos : p3 - p2 - 1);
        };
        if (col.find("NM:i:") != string_view::npos) {
            if (!to_i64(third(col), NM)) return false;
        }
        if (col.find("nn:i:") != string_view::npos) {
            if (!to_i64(third(col), ambig)) return false;
        }
        if (col.find("ts:A:") != string_view::npos) {
            const string_view ns = third(col);
            if (ns == "-" && strand == '+')
                strand = '-';
            else if (ns == "-" && strand == '-')
                strand = '+';
        }
        if (col.find("cs:Z:") != string_view::npos) {
            cs = string(third(col));
            have_cs = true;
        }
    }
    int64_t mismatch = NM - ID - ambig;
    if (mismatch < 0) mismatch = 0;
    const int64_t matches = M - mismatch;
    const int64_t den = matches + mismatch + ID + ambig;
    if (den == 0) return false;  // ZeroDivisionError in the reference
    const double accuracy = (double)matches / (double)den;
    line = std::to_string(matches) + "\t" + std::to_string(mismatch) + "\t0\t" + std::to_string(N) + "\t" +
           std::to_string(nI) + "\t" + std::to_string(I) + "\t" + std::to_string(nD) + "\t" + std::to_string(D) + "\t" +
           strand + "\t" + string(a[0]) + "\t" + std::to_string(sLen) + "\t" + std::to_string(qstart) + "\t" +
           std::to_string(end) + "\t" + string(a[2]) + "\t" + std::to_string(qsize) + "\t" + std::to_string(tstart) +
           "\t" + std::to_string(tend) + "\t" + std::to_string(bs.size()) + "\t" + join_list(bs) + "\t" +
           join_list(qs) + "\t" + join_list(ts);
    if (mando) {
        if (!have_cs) return false;  // NameError in the reference
        line += "\t" + py_repr(accuracy) + "\t" + cs + "\t" + sequence;
    }
    line += "\n";
    return true;
}

}  // namespace

extern "C" {

int mando_sam_to_psl(const char *sam_path, const char *psl_path, int32_t mando_mode, int32_t threads,
                     int64_t *n_records) {
    if (!sam_path || !psl_path) return MANDO_E_ARG;
    string buf;
    if (!read_file(sam_path, buf)) return MANDO_E_ARG;
    std::unordered_map<string, int64_t> chroms;
    std::vector<string_view> lines;
    std::vector<string_view> f;
    size_t p = 0;
    while (p < buf.size()) {
        size_t e = buf.find('\n', p);
        if (e == string::npos) e = buf.size();
        const string_view ln(buf.data() + p, e - p);
        p = e + 1;
        if (ln.empty()) continue;
        if (ln[0] == '@') {
            if (ln.substr(0, 3) == "@SQ") {
                split(strip(ln), '\t', f);
                if (f.size() < 3) return MANDO_E_ARG;
                const size_t c1 = f[1].find(':'), c2 = f[2].find(':');
                int64_t len;
                if (c1 == string_view::npos || c2 == string_view::npos || !to_i64(f[2].substr(c2 + 1), len))
                    return MANDO_E_ARG;
                chroms[string(f[1].substr(c1 + 1))] = len;
            }
            continue;
        }
        lines.push_back(ln);
    }
    const int64_t n = (int64_t)lines.size();
    std::vector<string> out((size_t)n);
    std::vector<char> keep((size_t)n, 0);
    std::atomic<int> err{0};
    int nth = threads > 0 ? threads : mando::usable_threads();
    nth = (int)std::min<int64_t>(nth, std::max<int64_t>(1, n / 1024));
    auto work = [&](int64_t a0, int64_t a1) {
        std::vector<string_view> a;
        for (int64_t i = a0; i < a1 && !err.load(); ++i) {
            split(strip(lines[(size_t)i]), '\t', a);
            if (a.size() < 3) {
                err = MANDO_E_ARG;
                return;
            }
            if (a[2] == "*") continue;
            auto it = chroms.find(string(a[2]));
            if (it == chroms.end() || !parse_sam_line(a, it->second, mando_mode != 0, out[(size_t)i])) {
                err = MANDO_E_ARG;  // KeyError / ValueError / NameError / ZeroDivisionError in emtrey
                return;
            }
            keep[(size_t)i] = 1;
        }
    };
    std::vector<std::thread> th;
    const int64_t chunk = (n + nth - 1) / std::max(1, nth);
    for (int t = 0; t < nth; ++t) {
        const int64_t a0 = t * chunk, a1 = std::min<int64_t>(n, a0 + chunk);
        if (a0 < a1) th.emplace_back(work, a0, a1);
    }
    for (auto &x : th) x.join();
    if (err) return err;
    FILE *o = fopen(psl_path, "wb");
    if (!o) return MANDO_E_ARG;
    int64_t written = 0;
    for (int64_t i = 0; i < n; ++i)
        if (keep[(size_t)i]) {
            fwrite(out[(size_t)i].data(), 1, out[(size_t)i].size(), o);
            ++written;
        }
    fclose(o);
    if (n_records) *n_records = written;
    return MANDO_OK;
}

// clean_psl (SpliceDefineConsensus.py:14-92): blocks separated by target gaps < 10 nt are merged,
// query starts recomputed from qStart by cumulative sizes, and with `primary` only the first line of
// each read name is kept.
int mando_clean_psl(const char *in_path, const char *out_path, int32_t primary, int64_t *n_records) {
    if (!in_path || !out_path) return MANDO_E_ARG;
    string buf;
    if (!read_file(in_path, buf)) return MANDO_E_ARG;
    FILE *o = fopen(out_path, "wb");
    if (!o) return MANDO_E_ARG;
    std::unordered_set<string> used;
    std::vector<string_view> a, bsz, bst;
    int64_t written = 0;
    size_t p = 0;
    int rc = MANDO_OK;
    while (p < buf.size()) {
        size_t e = buf.find('\n', p);
        if (e == string::npos) e = buf.size();
        const string_view ln(buf.data() + p, e - p);
        p = e + 1;
        split(strip(ln), '\t', a);
        if (a.size() < 21) {
            rc = MANDO_E_ARG;
            break;
        }
        int64_t start, qs0;
        if (!to_i64(a[15], start) || !to_i64(a[11], qs0)) {
            rc = MANDO_E_ARG;
            break;
        }
        const string name(a[9]);
        if (primary && used.count(name)) continue;
        split(a[18], ',', bsz);
        split(a[20], ',', bst);
        bsz.pop_back();  // .split(',')[:-1]
        bst.pop_back();
        std::vector<int64_t> size_gap;
        bool bad = false;
        for (size_t x = 0; x < bsz.size(); ++x) {
            int64_t bstart, bsize;
            if (x >= bst.size() || !to_i64(bst[x], bstart) || !to_i64(bsz[x], bsize)) {
                bad = true;
                break;
            }
            size_gap.push_back(bsize);
            if (x + 1 < bst.size()) {
                int64_t nb;
                if (!to_i64(bst[x + 1], nb)) {
                    bad = true;
                    break;
                }
                size_gap.push_back(nb - (bstart + bsize));
            }
        }
        if (bad) {
            rc = MANDO_E_ARG;
            break;
        }
        std::vector<int64_t> ng;
        int64_t block = 0;
        for (size_t idx = 0; idx < size_gap.size(); ++idx) {
            if (idx % 2 == 0) block += size_gap[idx];
            if (idx % 2 == 1) {
                if (size_gap[idx] < 10) {
                    block += size_gap[idx];
                } else {
                    ng.push_back(block);
                    ng.push_back(size_gap[idx]);
                    block = 0;
                }
            }
        }
        ng.push_back(block);
        std::vector<int64_t> cst, csz, cqs;
        int64_t cur = start, curq = qs0;
        for (size_t idx = 0; idx < ng.size(); ++idx) {
            if (idx % 2 == 0) {
                cst.push_back(cur);
                csz.push_back(ng[idx]);
                cqs.push_back(curq);
                cur += ng[idx];
                curq += ng[idx];
            } else {
                cur += ng[idx];
            }
        }
        string line;
        for (size_t k = 0; k < a.size(); ++k) {
            if (k) line += '\t';
            if (k == 17)
                line += std::to_string(cst.size());
            else if (k == 18)
                line += join_list(csz);
            else if (k == 19)
                line += join_list(cqs);
            else if (k == 20)
                line += join_list(cst);
            else
                line += string(a[k]);
        }
        line += '\n';
        fwrite(line.data(), 1, line.size(), o);
        ++written;
        used.insert(name);
    }
    fclose(o);
    if (rc) return rc;
    if (n_records) *n_records = written;
    return MANDO_OK;
}

}  // extern "C"
