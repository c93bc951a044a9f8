// synth.cpp — fast synthetic read-group generator for the benchmark (libmando_synth.so).
// Not part of the product ABI: it only produces R2C2 / PacBio-shaped test data (SURVEY.md §8d error
// model: substitutions, insertions, deletions, indels twice as likely inside homopolymers).  Each
// group uses its own SplitMix64-seeded xoshiro256** stream, so output is independent of threads.
#include <omp.h>

#include <algorithm>
#include <cstdio>
#include <string>
#include <tuple>

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace {

struct Rng {
    uint64_t s[4];
    static uint64_t splitmix(uint64_t &x) {
        uint64_t z = (x += 0x9e3779b97f4a7c15ull);
        z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
        z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
        return z ^ (z >> 31);
    }
    Rng(uint64_t seed, uint64_t stream) {
        uint64_t x = seed ^ (stream * 0xd1b54a32d192ed03ull);
        for (int i = 0; i < 4; ++i) s[i] = splitmix(x);
    }
    static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
    uint64_t next() {
        const uint64_t r = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
        s[2] ^= s[0];
        s[3] ^= s[1];
        s[1] ^= s[2];
        s[0] ^= s[3];
        s[2] ^= t;
        s[3] = rotl(s[3], 45);
        return r;
    }
    double uni() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
    int below(int n) { return (int)((next() >> 33) % (uint64_t)n); }
};

const char kB[4] = {'A', 'C', 'G', 'T'};

int idx(char c) { return c == 'A' ? 0 : c == 'C' ? 1 : c == 'G' ? 2 : 3; }

}  // namespace

extern "C" {

// Generates n_groups groups.  Group g: template length uniform in [len_lo, len_hi], depth uniform in
// [depth_lo, depth_hi]; reads are noisy copies (sub/ins/dele per base).  Output: reads concatenated
// (ASCII) into *out (malloc'd, caller frees with mando_synth_free), seq_off/grp_off malloc'd too.
// templates (optional) receives the templates concatenated with tmpl_off.
int mando_synth_groups(uint64_t seed, int64_t n_groups, int32_t len_lo, int32_t len_hi,
                       int32_t depth_lo, int32_t depth_hi, double sub, double ins, double dele,
                       char **out, int64_t **seq_off, int64_t *n_reads, int64_t **grp_off,
                       char **templates, int64_t **tmpl_off, int threads) {
    if (n_groups < 0 || len_lo < 1 || len_hi < len_lo || depth_lo < 1 || depth_hi < depth_lo)
        return -1;
    std::vector<std::vector<char>> gseq((size_t)n_groups), gtmpl((size_t)n_groups);
    std::vector<std::vector<int64_t>> glen((size_t)n_groups);
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 16)
    for (int64_t g = 0; g < n_groups; ++g) {
        Rng r(seed, (uint64_t)g + 1);
        const int L = len_lo + r.below(len_hi - len_lo + 1);
        const int d = depth_lo + r.below(depth_hi - depth_lo + 1);
        std::vector<char> &t = gtmpl[(size_t)g];
        t.resize((size_t)L);
        for (int i = 0; i < L; ++i) t[(size_t)i] = kB[r.below(4)];
        std::vector<char> &o = gseq[(size_t)g];
        o.reserve((size_t)d * (size_t)(L + L / 20 + 16));
        for (int k = 0; k < d; ++k) {
            const size_t st = o.size();
            for (int i = 0; i < L; ++i) {
                const bool hp = (i > 0 && t[(size_t)i] == t[(size_t)i - 1]) ||
                                (i + 1 < L && t[(size_t)i] == t[(size_t)i + 1]);
                const double f = hp ? 2.0 : 1.0;
                const double u = r.uni();
                if (u < dele * f) {
                    // deleted
                } else if (u < dele * f + sub) {
                    o.push_back(kB[(idx(t[(size_t)i]) + 1 + r.below(3)) & 3]);
                } else {
                    o.push_back(t[(size_t)i]);
                }
                if (r.uni() < ins * f) o.push_back(r.uni() < 0.5 ? t[(size_t)i] : kB[r.below(4)]);
            }
            glen[(size_t)g].push_back((int64_t)(o.size() - st));
        }
    }
    int64_t nr = 0, total = 0, ttotal = 0;
    for (int64_t g = 0; g < n_groups; ++g) {
        nr += (int64_t)glen[(size_t)g].size();
        total += (int64_t)gseq[(size_t)g].size();
        ttotal += (int64_t)gtmpl[(size_t)g].size();
    }
    char *o = (char *)malloc((size_t)total + 1);
    int64_t *so = (int64_t *)malloc(sizeof(int64_t) * (size_t)(nr + 1));
    int64_t *go = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n_groups + 1));
    char *tp = templates ? (char *)malloc((size_t)ttotal + 1) : nullptr;
    int64_t *to = tmpl_off ? (int64_t *)malloc(sizeof(int64_t) * (size_t)(n_groups + 1)) : nullptr;
    if (!o || !so || !go) return -3;
    std::vector<int64_t> gbase((size_t)n_groups + 1, 0), rbase((size_t)n_groups + 1, 0),
        tbase((size_t)n_groups + 1, 0);
    for (int64_t g = 0; g < n_groups; ++g) {
        gbase[(size_t)g + 1] = gbase[(size_t)g] + (int64_t)gseq[(size_t)g].size();
        rbase[(size_t)g + 1] = rbase[(size_t)g] + (int64_t)glen[(size_t)g].size();
        tbase[(size_t)g + 1] = tbase[(size_t)g] + (int64_t)gtmpl[(size_t)g].size();
    }
#pragma omp parallel for schedule(dynamic, 64)
    for (int64_t g = 0; g < n_groups; ++g) {
        memcpy(o + gbase[(size_t)g], gseq[(size_t)g].data(), gseq[(size_t)g].size());
        int64_t off = gbase[(size_t)g];
        int64_t r0 = rbase[(size_t)g];
        for (size_t k = 0; k < glen[(size_t)g].size(); ++k) {
            so[r0 + (int64_t)k] = off;
            off += glen[(size_t)g][k];
        }
        go[g] = r0;
        if (tp) memcpy(tp + tbase[(size_t)g], gtmpl[(size_t)g].data(), gtmpl[(size_t)g].size());
        if (to) to[g] = tbase[(size_t)g];
        std::vector<char>().swap(gseq[(size_t)g]);
    }
    so[nr] = total;
    go[n_groups] = nr;
    if (to) to[n_groups] = ttotal;
    *out = o;
    *seq_off = so;
    *n_reads = nr;
    *grp_off = go;
    if (templates) *templates = tp;
    if (tmpl_off) *tmpl_off = to;
    return 0;
}

void mando_synth_free(void *p) { free(p); }

// ---------------------------------------------------------------------------------------------
// Spliced loci written as Mandalorion locus PSL files (<dir>/<chrom>~<start>~<end>.psl), the same
// format as mandalorion_amd/simdata.py (24 columns, cs=long, whole-exon blocks, lines in (tStart,
// tEnd) order), for benchmark-scale D-module inputs.  Locus i sits on chr(i % 24 + 1) at
// 10,000 + (i / 24) * 200,000.  Returns the number of PSL records written, or < 0 on error.
// ---------------------------------------------------------------------------------------------
int64_t mando_synth_loci(const char *dir, uint64_t seed, int64_t n_loci, int32_t reads_lo, int32_t reads_hi,
                         int32_t ex_lo, int32_t ex_hi, int32_t elen_lo, int32_t elen_hi, int32_t ilen_lo,
                         int32_t ilen_hi, int32_t iso_lo, int32_t iso_hi, double sub, double ins, double dele,
                         double pb_frac, double pb_sub, double pb_ins, double pb_dele, double rev_frac,
                         int threads) {
    if (n_loci < 0 || reads_lo < 1 || reads_hi < reads_lo || ex_lo < 1 || ex_hi < ex_lo || elen_lo < 20 ||
        elen_hi < elen_lo || ilen_lo < 60 || ilen_hi < ilen_lo || iso_lo < 1 || iso_hi < iso_lo)
        return -1;
    if (threads > 0) omp_set_num_threads(threads);
    int64_t total = 0;
    int err = 0;
#pragma omp parallel for schedule(dynamic, 4) reduction(+ : total)
    for (int64_t li = 0; li < n_loci; ++li) {
        Rng r(seed, (uint64_t)li + 0x51ed);
        const std::string chrom = "chr" + std::to_string(li % 24 + 1);
        const int64_t g0 = 10000 + (li / 24) * 200000;
        const int nex = ex_lo + r.below(ex_hi - ex_lo + 1);
        std::vector<int> el(nex), il(nex > 0 ? nex - 1 : 0);
        for (int k = 0; k < nex; ++k) el[k] = elen_lo + r.below(elen_hi - elen_lo + 1);
        for (int k = 0; k + 1 < nex; ++k) il[k] = ilen_lo + r.below(ilen_hi - ilen_lo + 1);
        const int pad = 50;
        int64_t span = 2 * pad;
        for (int v : el) span += v;
        for (int v : il) span += v;
        std::string g((size_t)span, 'A');
        for (auto &c : g) c = kB[r.below(4)];
        std::vector<std::pair<int64_t, int64_t>> ex;
        int64_t p = pad;
        for (int k = 0; k < nex; ++k) {
            ex.push_back({g0 + p, g0 + p + el[k]});
            p += el[k];
            if (k + 1 < nex) {
                const bool gc = r.uni() < 0.05;
                g[(size_t)p] = 'G';
                g[(size_t)p + 1] = gc ? 'C' : 'T';
                g[(size_t)(p + il[k] - 2)] = 'A';
                g[(size_t)(p + il[k] - 1)] = 'G';
                p += il[k];
            }
        }
        auto gs = [&](int64_t a, int64_t b) { return g.substr((size_t)(a - g0), (size_t)(b - a)); };
        const int niso = iso_lo + r.below(iso_hi - iso_lo + 1);
        std::vector<std::vector<int>> isos;
        {
            std::vector<int> all;
            for (int k = 0; k < nex; ++k) all.push_back(k);
            isos.push_back(all);
            std::vector<int> internal;
            for (int k = 1; k + 1 < nex; ++k) internal.push_back(k);
            for (int k = (int)internal.size() - 1; k > 0; --k) std::swap(internal[(size_t)k], internal[(size_t)r.below(k + 1)]);
            for (int t = 0; t < niso - 1 && t < (int)internal.size(); ++t) {
                std::vector<int> v;
                for (int k = 0; k < nex; ++k)
                    if (k != internal[(size_t)t]) v.push_back(k);
                isos.push_back(v);
            }
        }
        const int nreads = reads_lo + r.below(reads_hi - reads_lo + 1);
        std::vector<std::tuple<int64_t, int64_t, std::string>> lines;
        for (int rd = 0; rd < nreads; ++rd) {
            const auto &iso = isos[(size_t)r.below((int)isos.size())];
            // per read: PacBio-like rates for a pb_frac share of the reads (config 4's mix), and the
            // read's own orientation (a '-' strand record carries the reverse-complemented read, as
            // emtrey writes it); no extra draws when the shares are 0, so those streams are unchanged
            const bool pb = pb_frac > 0 && r.uni() < pb_frac;
            const bool rev = rev_frac > 0 && r.uni() < rev_frac;
            const double sub_r = pb ? pb_sub : sub, ins_r = pb ? pb_ins : ins, dele_r = pb ? pb_dele : dele;
            std::vector<std::pair<int64_t, int64_t>> e;
            for (int k : iso) e.push_back(ex[(size_t)k]);
            e.front().first += r.below(7) - 3;
            e.back().second += r.below(7) - 3;
            std::string q, cs;
            int64_t match = 0, mis = 0, qins = 0, qbase = 0, tins = 0, tbase = 0;
            char last = 0;
            for (size_t k = 0; k < e.size(); ++k) {
                const std::string ref = gs(e[k].first, e[k].second);
                const int n = (int)ref.size();
                for (int i = 0; i < n; ++i) {
                    const char c = ref[(size_t)i];
                    const bool hp = (i > 0 && ref[(size_t)i - 1] == c) || (i + 1 < n && ref[(size_t)i + 1] == c);
                    const double f = hp ? 2.0 : 1.0;
                    const bool edge = (k == 0 && i == 0) || (k + 1 == e.size() && i == n - 1);
                    const double u = r.uni();
                    if (!edge && u < dele_r * f) {
                        if (last != '-') { cs += '-'; ++tins; }
                        cs += (char)(c | 0x20);
                        last = '-';
                        ++tbase;
                    } else if (!edge && u < dele_r * f + sub_r) {
                        const char qb = kB[(idx(c) + 1 + r.below(3)) & 3];
                        cs += '*';
                        cs += (char)(c | 0x20);
                        cs += (char)(qb | 0x20);
                        q += qb;
                        last = '*';
                        ++mis;
                    } else {
                        if (last != '=') cs += '=';
                        cs += c;
                        q += c;
                        last = '=';
                        ++match;
                    }
                    if (!(k + 1 == e.size() && i == n - 1) && r.uni() < ins_r * f) {
                        const char b = r.uni() < 0.5 ? c : kB[r.below(4)];
                        if (last != '+') { cs += '+'; ++qins; }
                        cs += (char)(b | 0x20);
                        q += b;
                        last = '+';
                        ++qbase;
                    }
                }
                if (k + 1 < e.size()) {
                    const int64_t b = e[k].second, na = e[k + 1].first;
                    std::string d = gs(b, b + 2), a = gs(na - 2, na);
                    for (auto &ch : d) ch = (char)(ch | 0x20);
                    for (auto &ch : a) ch = (char)(ch | 0x20);
                    cs += '~' + d + std::to_string(na - b) + a;
                    last = '~';
                }
            }
            std::string bs, qs, ts;
            int64_t qq = 0, introns = 0;
            for (size_t k = 0; k < e.size(); ++k) {
                bs += std::to_string(e[k].second - e[k].first) + ",";
                qs += std::to_string(qq) + ",";
                ts += std::to_string(e[k].first) + ",";
                qq += e[k].second - e[k].first;
                if (k + 1 < e.size()) introns += e[k + 1].first - e[k].second;
            }
            if (rev) {
                std::reverse(q.begin(), q.end());
                for (auto &ch : q) ch = ch == 'A' ? 'T' : ch == 'C' ? 'G' : ch == 'G' ? 'C' : ch == 'T' ? 'A' : ch;
            }
            const int64_t alen = match + mis + qbase + tbase;
            char acc[32];
            snprintf(acc, sizeof acc, "%.4f", alen ? (double)match / (double)alen : 1.0);
            std::string line = std::to_string(match) + "\t" + std::to_string(mis) + "\t0\t" + std::to_string(introns) +
                               "\t" + std::to_string(qins) + "\t" + std::to_string(qbase) + "\t" + std::to_string(tins) +
                               "\t" + std::to_string(tbase) + (rev ? "\t-\tS" : "\t+\tS") + std::to_string(li) + "_r" + std::to_string(rd) +
                               "\t" + std::to_string(q.size()) + "\t0\t" + std::to_string(q.size()) + "\t" + chrom +
                               "\t250000000\t" + std::to_string(e.front().first) + "\t" + std::to_string(e.back().second) +
                               "\t" + std::to_string(e.size()) + "\t" + bs + "\t" + qs + "\t" + ts + "\t" + acc + "\t" +
                               cs + "\t" + q;
            lines.emplace_back(e.front().first, e.back().second, std::move(line));
        }
        std::sort(lines.begin(), lines.end());
        int64_t lo = std::get<0>(lines.front()), hi = 0;
        for (auto &t : lines) hi = std::max(hi, std::get<1>(t));
        const std::string path = std::string(dir) + "/" + chrom + "~" + std::to_string(lo) + "~" + std::to_string(hi) + ".psl";
        FILE *fh = fopen(path.c_str(), "w");
        if (!fh) {
#pragma omp atomic write
            err = 1;
            continue;
        }
        for (auto &t : lines) {
            fputs(std::get<2>(t).c_str(), fh);
            fputc('\n', fh);
        }
        fclose(fh);
        total += (int64_t)lines.size();
    }
    return err ? -2 : total;
}
}
