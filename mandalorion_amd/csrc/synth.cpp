// synth.cpp — fast synthetic read-group generator for the benchmark (libmando_synth.so).
// Not part of the product ABI: it only produces R2C2 / PacBio-shaped test data (SURVEY.md §8d error
// model: substitutions, insertions, deletions, indels twice as likely inside homopolymers).  Each
// group uses its own SplitMix64-seeded xoshiro256** stream, so output is independent of threads.
#include <omp.h>

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
}
