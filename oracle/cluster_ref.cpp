// oracle/cluster_ref.cpp — TEST INFRASTRUCTURE ONLY: the CPU restatement of the D module's per-locus
// read clustering, used as the checker of the HIP kernels (mandalorion_amd/csrc/cluster_kernel.hip) by
// tests/, and by bench.py's cpu_baseline leg.  Never linked into libmando.
//
// Restates, function by function, the clustering half of the reference's process_locus
// (/root/reference/defineIsoforms.py:55-91) so that a locus produces the same splice-site peaks, the
// same isoform groups in the same order, and the same RNG draws as the reference under a seeded
// parent:
//   collect_reads                      SpliceDefineConsensus.py:278-331
//   make_genome_bins                   :392-438
//   find_peaks / scan_for_best_bin     :232-275, :163-197
//   determine_cov / myround            :200-224, :227-229
//   characterize_splicing_event        :499-550   (RNG draw #1 per accepted candidate)
//   getCSaroundSS                      :107-161   (tokenised once per read, then O(log L) per query)
//   sort_reads_into_splice_junctions   :714-769
//   group_mono_exon_transcripts        :772-794
//   define_start_end_sites / find_ends :797-868, :554-711   (RNG draw #2 per identity)
//   determine_consensus subsample      :884-888   (RNG draw #3 per isoform)
// PINNED: tests/golden/cluster_vectors.json and define_vectors.json are outputs of the unmodified
// reference run here (seeded parent, stand-in mappy / abpoa); tests/test_cluster.py and
// tests/test_define_ref.py check this restatement against them byte for byte.
// Python semantics reproduced on purpose: dict insertion order, stable sorts,
// round-half-even myround, correctly rounded round(x, 3), negative-slice wrap in getCSaroundSS,
// the dead branch of make_genome_bins, `identity.split('_')[1]`, `previous_end = end`, tuple order of
// the mono-exon sort, and the ZeroDivisionError / KeyError cases (reported as a locus status).
#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include <emmintrin.h>
#include <sys/mman.h>

#include "../include/mando.h"
#include "mt19937_ref.h"

namespace {

using std::string;
using std::string_view;
using std::vector;

// locus status codes (mando_cluster_view::locus_status)
constexpr int kLocusOk = 0;
constexpr int kLocusZeroDivision = -10;  // characterize_splicing_event: leftCS['Total'] == 0
constexpr int kLocusKeyError = -11;      // scan_for_best_bin: strand column not '+' / '-'
constexpr int kLocusParse = -12;         // malformed PSL line / cs string
constexpr int kLocusIO = -13;            // file unreadable
[[maybe_unused]] constexpr int kLocusIndexError = -14;  // host side: zero reads orient (IndexError)
constexpr int kLocusValueError = -15;    // max() of an empty sequence in find_ends

struct LocusError {
    int code;
};

// optional phase timing (MANDO_CLUSTER_PROF=1): nanoseconds summed over loci / threads
std::atomic<int64_t> g_ph[8];
const char *kPhName[8] = {"parse", "collect", "peaks", "characterize", "sort_reads", "start_end", "subsample", "io"};
inline int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
struct PhTimer {
    int ph;
    int64_t t0;
    explicit PhTimer(int p) : ph(p), t0(now_ns()) {}
    ~PhTimer() { g_ph[ph] += now_ns() - t0; }
};

// ---------------------------------------------------------------------------------------------
// parsing helpers
// ---------------------------------------------------------------------------------------------
int64_t to_i64(string_view s) {
    // Python int(): optional surrounding whitespace, optional sign, decimal digits
    size_t a = 0, b = s.size();
    while (a < b && (s[a] == ' ' || s[a] == '\t' || s[a] == '\r' || s[a] == '\n')) ++a;
    while (b > a && (s[b - 1] == ' ' || s[b - 1] == '\t' || s[b - 1] == '\r' || s[b - 1] == '\n')) --b;
    if (a == b) throw LocusError{kLocusParse};
    bool neg = false;
    if (s[a] == '+' || s[a] == '-') {
        neg = s[a] == '-';
        ++a;
    }
    if (a == b) throw LocusError{kLocusParse};
    int64_t v = 0;
    for (size_t i = a; i < b; ++i) {
        const char c = s[i];
        if (c == '_' ) continue;
        if (c < '0' || c > '9') throw LocusError{kLocusParse};
        v = v * 10 + (c - '0');
    }
    return neg ? -v : v;
}

double to_f64(string_view s) {
    string t(s);
    char *end = nullptr;
    const double v = strtod(t.c_str(), &end);  // glibc strtod is correctly rounded, like float()
    if (end == t.c_str()) throw LocusError{kLocusParse};
    return v;
}

// str.split(',')[:-1] of a PSL list column
void split_list(string_view s, vector<int64_t> &out) {
    out.clear();
    size_t a = 0;
    vector<string_view> parts;
    while (true) {
        const size_t c = s.find(',', a);
        if (c == string_view::npos) {
            parts.push_back(s.substr(a));
            break;
        }
        parts.push_back(s.substr(a, c - a));
        a = c + 1;
    }
    for (size_t i = 0; i + 1 < parts.size(); ++i) out.push_back(to_i64(parts[i]));
}

// Python round(x) (half-even) of x / 10 for integer x, times 10 (myround, SDC:227-229)
inline int64_t myround(int64_t x) {
    // x / 10 is exact at the .5 ties (k + 0.5 is representable), so the float round is half-even on
    // the exact quotient.
    int64_t q = x >= 0 ? x / 10 : -((-x + 9) / 10);
    int64_t r = x - 10 * q;
    if (r > 5 || (r == 5 && (q & 1))) ++q;
    return 10 * q;
}

// Python round(x, 3): correctly rounded decimal, then back to double (glibc printf is exact)
inline double py_round3(double x) {
    char buf[64];
    snprintf(buf, sizeof buf, "%.3f", x);
    return strtod(buf, nullptr);
}

// ---------------------------------------------------------------------------------------------
// records
// ---------------------------------------------------------------------------------------------
struct Record {
    string_view name, dirn, chrom, cs, seq;
    int64_t qsize = 0, qstart = 0, qend = 0, tstart = 0, tend = 0;
    vector<int64_t> bsize, bstart;
    double accuracy = 0;
    int64_t global = 0;  // index in the batch
};

// line.strip().split('\t')
void split_tabs(string_view line, vector<string_view> &f) {
    f.clear();
    size_t a = 0, b = line.size();
    while (a < b && isspace((unsigned char)line[a])) ++a;
    while (b > a && isspace((unsigned char)line[b - 1])) --b;
    line = line.substr(a, b - a);
    size_t p = 0;
    while (true) {
        const size_t t = line.find('\t', p);
        if (t == string_view::npos) {
            f.push_back(line.substr(p));
            break;
        }
        f.push_back(line.substr(p, t - p));
        p = t + 1;
    }
}

// ---------------------------------------------------------------------------------------------
// getCSaroundSS: tokenised cs string
// ---------------------------------------------------------------------------------------------
// Run-length view of getCSaroundSS's `record` list: one run per cs operation.  Record t of the
// reference list is record (t - rec0) of the run containing it; run k covers records
// [rec0, rec0 + n) whose genome positions (after the per-record increment) are g0 + step * (i + 1).
struct CsRun {
    int32_t rec0, n;
    int64_t g0;
    int32_t step;  // 1 for '=', '-', '*'; 0 for '+'; the intron length for '~' (n == 1)
    char st;       // '=', '+', '-', '*', '|'
    std::array<char, 4> motif;
};
struct CsIndex {
    vector<CsRun> runs;
    vector<int32_t> adv;       // indices of advancing runs (step > 0), in order
    vector<int64_t> adv_first; // genome position of each advancing run's first record
    int32_t nrec = 0;
    bool built = false;
};

struct OpTable {
    bool t[256];
    OpTable() {
        for (auto &x : t) x = false;
        for (unsigned char c : {'\\', '=', '+', '-', '*', '~'}) t[c] = true;
    }
};
const OpTable kOps;
inline bool is_op(char c) { return kOps.t[(unsigned char)c]; }

// first cs operator at or after i ('=' runs carry the read bases, so the scan is 16 bytes a step)
inline size_t next_op(string_view cs, size_t i) {
    const char *p = cs.data();
    const size_t n = cs.size();
    const __m128i c0 = _mm_set1_epi8('='), c1 = _mm_set1_epi8('+'), c2 = _mm_set1_epi8('-'),
                  c3 = _mm_set1_epi8('*'), c4 = _mm_set1_epi8('~'), c5 = _mm_set1_epi8('\\');
    for (; i + 16 <= n; i += 16) {
        const __m128i v = _mm_loadu_si128((const __m128i *)(p + i));
        const __m128i m = _mm_or_si128(
            _mm_or_si128(_mm_or_si128(_mm_cmpeq_epi8(v, c0), _mm_cmpeq_epi8(v, c1)),
                         _mm_or_si128(_mm_cmpeq_epi8(v, c2), _mm_cmpeq_epi8(v, c3))),
            _mm_or_si128(_mm_cmpeq_epi8(v, c4), _mm_cmpeq_epi8(v, c5)));
        const int bits = _mm_movemask_epi8(m);
        if (bits) return i + (size_t)__builtin_ctz((unsigned)bits);
    }
    while (i < n && !is_op(p[i])) ++i;
    return i;
}

void build_cs(string_view cs, int64_t begin, CsIndex &ix) {
    ix.runs.clear();
    ix.adv.clear();
    ix.adv_first.clear();
    ix.runs.reserve(cs.size() / 8 + 8);
    ix.adv.reserve(cs.size() / 8 + 8);
    ix.adv_first.reserve(cs.size() / 8 + 8);
    int64_t g = begin;
    int32_t rec = 0;
    size_t i = 0;
    // re.split keeps text before the first operator as element 0, which the zip drops
    i = next_op(cs, i);
    while (i < cs.size()) {
        const char op = cs[i++];
        const size_t j = next_op(cs, i);
        const string_view e = cs.substr(i, j - i);
        i = j;
        CsRun r{rec, 0, g, 0, op, {0, 0, 0, 0}};
        switch (op) {
            case '=':
            case '-':
                r.n = (int32_t)e.size();
                r.step = 1;
                break;
            case '+':
                r.n = (int32_t)e.size();
                r.step = 0;
                break;
            case '*':
                r.n = (int32_t)((e.size() + 1) / 2);  // entry[::2]
                r.step = 1;
                r.st = '*';
                break;
            case '~': {
                if (e.size() < 4) throw LocusError{kLocusParse};
                r.n = 1;
                r.step = (int32_t)to_i64(e.substr(2, e.size() - 4));
                r.st = '|';
                r.motif = {e[0], e[1], e[e.size() - 2], e[e.size() - 1]};
                break;
            }
            default:  // '\\' never occurs in a cs string
                continue;
        }
        if (r.n == 0) continue;
        if (r.step > 0 || r.st == '|') {
            ix.adv.push_back((int32_t)ix.runs.size());
            ix.adv_first.push_back(g + r.step);
        }
        g += (int64_t)r.step * r.n;
        rec += r.n;
        ix.runs.push_back(r);
    }
    ix.nrec = rec;
    ix.built = true;
}

// run containing record t (0 <= t < nrec)
inline int run_of(const CsIndex &ix, int32_t t) {
    int lo = 0, hi = (int)ix.runs.size() - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (ix.runs[(size_t)mid].rec0 <= t)
            lo = mid;
        else
            hi = mid - 1;
    }
    return lo;
}

struct CsResult {
    string bases;        // 4 chars, "nnnn" when no intron in the window
    int cnt_l[6] = {0};  // '*','+','-','=','|' counts of `left` and Total
    int cnt_r[6] = {0};
    bool has_l = false, has_r = false;
};

inline int st_slot(char c) {
    switch (c) {
        case '*': return 0;
        case '+': return 1;
        case '-': return 2;
        case '=': return 3;
        default: return 4;  // '|'
    }
}

// count statuses of records [a, b) into cnt (and cnt[5] += b - a)
inline void count_range(const CsIndex &ix, int32_t a, int32_t b, int *cnt) {
    if (a >= b) return;
    int k = run_of(ix, a);
    while (a < b) {
        const CsRun &R = ix.runs[(size_t)k];
        const int32_t e = std::min(b, R.rec0 + R.n);
        cnt[st_slot(R.st)] += e - a;
        cnt[5] += e - a;
        a = e;
        ++k;
    }
}

void cs_around(const CsIndex &ix, int64_t start, int64_t end, CsResult &r) {
    r.bases = "nnnn";
    r.has_l = r.has_r = false;
    std::fill(r.cnt_l, r.cnt_l + 6, 0);
    std::fill(r.cnt_r, r.cnt_r + 6, 0);
    const int32_t n = ix.nrec;
    // last advancing record with start <= pos <= end ('+' records never set spliceIndex)
    const int64_t ka = (int64_t)(std::upper_bound(ix.adv_first.begin(), ix.adv_first.end(), end) - ix.adv_first.begin()) - 1;
    if (ka < 0) return;
    const CsRun &R = ix.runs[(size_t)ix.adv[(size_t)ka]];
    const int64_t i_in = R.n == 1 ? 0 : std::min<int64_t>(R.n - 1, (end - R.g0) / R.step - 1);
    const int64_t pos = R.g0 + (int64_t)R.step * (i_in + 1);
    if (pos < start) return;
    const int64_t si = R.rec0 + i_in + 1;  // len(record) after appending that record
    const int64_t lo = std::max<int64_t>(si - 10, 0), hi = std::min<int64_t>(si + 10, n);
    // last intron record in [lo, hi)
    int64_t idx = -1;
    const CsRun *IR = nullptr;
    if (lo < hi) {
        for (int k = run_of(ix, (int32_t)(hi - 1)); k >= 0 && ix.runs[(size_t)k].rec0 + ix.runs[(size_t)k].n > lo; --k)
            if (ix.runs[(size_t)k].st == '|') {
                idx = ix.runs[(size_t)k].rec0;
                IR = &ix.runs[(size_t)k];
                break;
            }
    }
    if (idx < 0) return;
    r.bases.assign(IR->motif.begin(), IR->motif.end());
    // left = record[idx-5:idx] with Python slice normalisation
    int64_t a = idx - 5, b = idx;
    if (a < 0) a += n;
    if (a < 0) a = 0;
    if (a < b) {
        count_range(ix, (int32_t)a, (int32_t)std::min<int64_t>(b, n), r.cnt_l);
        r.has_l = true;
    }
    // right = record[idx+1:idx+6]
    const int64_t ra = idx + 1, rb = std::min<int64_t>(idx + 6, n);
    if (ra < rb) {
        count_range(ix, (int32_t)ra, (int32_t)rb, r.cnt_r);
        r.has_r = true;
    }
}

// Position set (peak_areas): a byte map over the locus span, a hash set for anything outside it
struct PosSet {
    int64_t lo = 0;
    vector<uint8_t> bits;
    std::unordered_set<int64_t> extra;
    void init(int64_t a, int64_t b) {
        lo = a;
        bits.assign(b >= a ? (size_t)(b - a + 1) : 0, 0);
    }
    bool has(int64_t p) const {
        const uint64_t k = (uint64_t)(p - lo);
        return k < bits.size() ? bits[k] != 0 : extra.count(p) != 0;
    }
    void add(int64_t p) {
        const uint64_t k = (uint64_t)(p - lo);
        if (k < bits.size())
            bits[k] = 1;
        else
            extra.insert(p);
    }
};

// ---------------------------------------------------------------------------------------------
// ordered dict helper (Python dict: insertion order)
// ---------------------------------------------------------------------------------------------
template <class V>
struct OrderedMap {
    vector<int64_t> keys;
    vector<V> vals;
    std::unordered_map<int64_t, size_t> idx;
    V &at(int64_t k) {
        auto it = idx.find(k);
        if (it != idx.end()) return vals[it->second];
        idx.emplace(k, keys.size());
        keys.push_back(k);
        vals.emplace_back();
        return vals.back();
    }
    const V *find(int64_t k) const {
        auto it = idx.find(k);
        return it == idx.end() ? nullptr : &vals[it->second];
    }
};

struct HistEntry {
    int32_t rec;  // record index within the locus
};

struct Peak {
    int64_t start, end;
    char type, side;
    double prop;  // -1 for annotated ('A')
};

struct Params {
    double cutoff;
    int w, min_count, up, down, sub_k;
    vector<string> junctions;
    uint32_t seed;
};

// ---------------------------------------------------------------------------------------------
// one locus
// ---------------------------------------------------------------------------------------------
struct LocusOut {
    int status = kLocusOk;
    vector<Peak> peaks;
    vector<vector<int32_t>> iso_members;  // record indices (locus-local), IsoDict order
    vector<vector<int32_t>> iso_sub;      // subsample, in draw order
};

struct LocusIn {
    string_view text;
    string chrom;
    vector<int64_t> ann[4];  // left '5', left '3', right '5', right '3'
    int64_t rec_base = 0;
};

class LocusRunner {
  public:
    LocusRunner(const Params &p, const LocusIn &in, vector<Record> &recs, LocusOut &out)
        : P(p), in(in), recs(recs), out(out), mt(p.seed) {}

    void run() {
        {
            PhTimer t(1);
            collect_reads();
        }
        PosSet areas_l, areas_r;
        areas_l.init(span_lo - 64, span_hi + 64);
        areas_r.init(span_lo - 64, span_hi + 64);
        vector<Peak> a_l, a_r, n_l, n_r;
        make_genome_bins(in.ann[0], in.ann[1], 'l', areas_l, a_l);
        make_genome_bins(in.ann[2], in.ann[3], 'r', areas_r, a_r);
        {
            PhTimer t(2);
            find_peaks(hist_l, true, 'l', areas_l, n_l);
            find_peaks(hist_r, false, 'r', areas_r, n_r);
        }
        // spliceDict (defineIsoforms.py:71-83): per-side counters, later rows overwrite
        int counter[2] = {0, 0};
        for (auto *tw : {&a_l, &a_r, &n_l, &n_r}) {
            for (const Peak &pk : *tw) {
                const int s = pk.side == 'l' ? 0 : 1;
                counter[s] += 1;
                const int32_t lab = (int32_t)labels.size();
                labels.push_back(string(1, pk.type) + pk.side + std::to_string(counter[s]));
                for (int64_t b = pk.start; b <= pk.end; ++b) splice[b] = lab;
                out.peaks.push_back(pk);
            }
        }
        {
            PhTimer t(4);
            sort_reads();
        }
        {
            PhTimer t(5);
            define_start_end_sites();
        }
        // determine_consensus subsample draw per isoform (SDC:884-888)
        vector<int64_t> perm, pick;
        for (auto &mem : out.iso_members) {
            const int64_t n = (int64_t)mem.size();
            mando_ref::mt_choice(mt, n, std::min<int64_t>(n, P.sub_k), perm, pick);
            vector<int32_t> sub;
            sub.reserve(pick.size());
            for (int64_t t : pick) sub.push_back(mem[(size_t)t]);
            out.iso_sub.push_back(std::move(sub));
        }
    }

  private:
    const Params &P;
    const LocusIn &in;
    vector<Record> &recs;
    LocusOut &out;
    mando_ref::MT19937 mt;

    // collect_reads state
    int64_t bin_lo = INT64_MAX, bin_hi = INT64_MIN, nbins = 0;
    int64_t span_lo = 0, span_hi = -1;  // genome span of the locus' records  // rounded positions (multiples of 10)
    vector<int32_t> hcov;     // histo_cov, dense over [bin_lo, bin_hi] step 10
    OrderedMap<vector<HistEntry>> hist_l, hist_r;
    vector<vector<int64_t>> cov_sets;                    // per record (rounded, unique, sorted)
    std::unordered_map<string_view, int32_t> cs_dict;     // name -> last record
    vector<CsIndex> cs_ix;
    vector<int32_t> cs_of;  // record -> cs_dict[name] once the dict is complete (-1: other chrom)
    // spliceDict
    std::unordered_map<int64_t, int32_t> splice;
    vector<string> labels;
    // sort_reads output
    struct Pos {
        int64_t start, end;
        int32_t rec;
        int64_t lx, rx;
    };
    std::map<string, int> ident_index_unused;
    vector<string> ident_order;
    std::unordered_map<string, vector<Pos>> se_dict;
    vector<string> mono_order;
    std::unordered_map<string, vector<Pos>> se_mono;

    void collect_reads() {
        const size_t n = recs.size();
        cov_sets.resize(n);
        cs_ix.resize(n);
        vector<int64_t> v;
        for (size_t r = 0; r < n; ++r) {
            Record &R = recs[r];
            if (R.chrom != string_view(in.chrom)) continue;
            if (span_hi < span_lo) {
                span_lo = R.tstart;
                span_hi = R.tend;
            }
            span_lo = std::min(span_lo, R.tstart);
            span_hi = std::max(span_hi, R.tend);
            cs_dict[R.name] = (int32_t)r;
            v.clear();
            vector<int64_t> low, up;
            int64_t y = -1;
            bool y_set = false;
            for (size_t x = 0; x < R.bsize.size(); ++x) {
                const int64_t bs = R.bstart[x], sz = R.bsize[x], be = bs + sz;
                for (int64_t t = 0; t < sz; t += 10) {
                    v.push_back(myround(bs + t));
                    y = t;
                    y_set = true;
                }
                if (!y_set) throw LocusError{kLocusParse};  // NameError in the reference
                int64_t last = INT64_MIN;
                for (int64_t t = y; t < sz; ++t) {
                    const int64_t b = myround(bs + t);
                    if (b != last) v.push_back(b);
                    last = b;
                }
                if (bs != R.tstart) up.push_back(bs);
                if (be != R.tend) low.push_back(be);
            }
            std::sort(v.begin(), v.end());
            v.erase(std::unique(v.begin(), v.end()), v.end());
            if (!v.empty()) {
                bin_lo = std::min(bin_lo, v.front());
                bin_hi = std::max(bin_hi, v.back());
            }
            cov_sets[r] = v;
            if (R.accuracy < 0.9) continue;
            for (int64_t b : low) hist_l.at(b).push_back({(int32_t)r});
            for (int64_t b : up) hist_r.at(b).push_back({(int32_t)r});
        }
        cs_of.assign(n, -1);
        for (size_t r = 0; r < n; ++r)
            if (recs[r].chrom == string_view(in.chrom)) cs_of[r] = cs_dict.at(recs[r].name);
        // dense per-locus coverage histogram over 10-nt bins (histo_cov)
        if (bin_lo <= bin_hi) {
            nbins = (bin_hi - bin_lo) / 10 + 1;
            hcov.assign((size_t)nbins, 0);
            for (size_t r = 0; r < n; ++r)
                for (int64_t b : cov_sets[r]) hcov[(size_t)((b - bin_lo) / 10)] += 1;
        }
    }

    void make_genome_bins(const vector<int64_t> &b5, const vector<int64_t> &b3, char side,
                          PosSet &areas, vector<Peak> &tw) {
        for (int ti = 0; ti < 2; ++ti) {
            const char type = ti == 0 ? '5' : '3';
            vector<int64_t> pl = ti == 0 ? b5 : b3;
            std::stable_sort(pl.begin(), pl.end());
            std::unordered_set<size_t> covered;
            for (size_t i1 = 0; i1 < pl.size(); ++i1) {
                if (covered.count(i1)) continue;
                // sub_list starts with pl[i1] and the inner loop re-adds it (index2 = index1), so
                // min(splice_dists) == 0 and the multi-bin branch (SDC:412-426) never runs
                int64_t mx = pl[i1], mn = pl[i1];
                for (size_t i2 = i1; i2 < pl.size(); ++i2) {
                    if (pl[i2] - mx <= P.w) {
                        mx = std::max(mx, pl[i2]);
                        mn = std::min(mn, pl[i2]);
                        covered.insert(i2);
                    } else {
                        break;
                    }
                }
                Peak pk{mn - P.w, mx + P.w, type, side, -1.0};
                tw.push_back(pk);
                for (int64_t b = pk.start; b <= pk.end; ++b) areas.add(b);
            }
        }
    }

    bool characterize(int64_t left, int64_t right, const vector<int32_t> &names) {
        PhTimer tm(3);
        const int64_t n = (int64_t)names.size();
        vector<int64_t> perm, pick;
        mando_ref::mt_choice(mt, n, std::min<int64_t>(n, 500), perm, pick);
        int64_t allowed = 0, all = 0;
        int64_t lc[6] = {0}, rc[6] = {0};
        CsResult res;
        for (int64_t t : pick) {
            const int32_t ri = cs_of[(size_t)names[(size_t)t]];
            CsIndex &ix = cs_ix[(size_t)ri];
            if (!ix.built) build_cs(recs[(size_t)ri].cs, recs[(size_t)ri].tstart, ix);
            cs_around(ix, left, right, res);
            all += 1;
            for (const string &j : P.junctions)
                if (res.bases == j) {
                    allowed += 1;
                    break;
                }
            if (res.has_l)
                for (int s = 0; s < 6; ++s) lc[s] += res.cnt_l[s];
            if (res.has_r)
                for (int s = 0; s < 6; ++s) rc[s] += res.cnt_r[s];
        }
        if (all == 0) throw LocusError{kLocusZeroDivision};
        bool basepass = (double)allowed / (double)all > 0.85;
        if (!basepass) return false;
        if (lc[5] == 0 || rc[5] == 0) throw LocusError{kLocusZeroDivision};
        const double la = (double)lc[3] / (double)lc[5], ra = (double)rc[3] / (double)rc[5];
        return la > 0.85 && ra > 0.85;
    }

    // determine_cov (SDC:200-224): over the winners' coverage bins (a multiset: a read listed twice
    // counts twice), the first 4 bins with count > 1 strictly beyond the centre (downward for the
    // left side); max of histo_cov over them.  The winners' sorted coverage sets are merged from the
    // centre outwards, so a candidate touches only the bins up to the fourth hit instead of
    // scattering every winner's ~300 bins.
    int64_t determine_cov(const vector<int32_t> &names, int64_t center, bool reverse) {
        using Ent = std::pair<int64_t, int32_t>;  // (bin position, cursor)
        int64_t kstart;
        if (reverse) {
            const int64_t k = center - 1 - bin_lo;
            kstart = k < 0 ? -1 : std::min<int64_t>(k / 10, nbins - 1);
            if (kstart < 0) return 0;
        } else {
            const int64_t k = center + 1 - bin_lo;
            kstart = k <= 0 ? 0 : (k + 9) / 10;
            if (kstart >= nbins) return 0;
        }
        const int64_t bound = bin_lo + 10 * kstart;
        merge_pos.assign(names.size(), 0);
        merge_heap.clear();
        for (size_t c = 0; c < names.size(); ++c) {
            const vector<int64_t> &cs = cov_sets[(size_t)names[c]];
            if (reverse) {
                const size_t i = (size_t)(std::upper_bound(cs.begin(), cs.end(), bound) - cs.begin());
                if (i == 0) continue;
                merge_pos[c] = i - 1;
                merge_heap.push_back({cs[i - 1], (int32_t)c});
            } else {
                const size_t i = (size_t)(std::lower_bound(cs.begin(), cs.end(), bound) - cs.begin());
                if (i == cs.size()) continue;
                merge_pos[c] = i;
                merge_heap.push_back({-cs[i], (int32_t)c});  // max-heap on -position: smallest first
            }
        }
        auto cmp = [](const Ent &a, const Ent &b) { return a.first < b.first; };
        std::make_heap(merge_heap.begin(), merge_heap.end(), cmp);
        int64_t cov = 0;
        int counter = 0;
        while (!merge_heap.empty() && counter < 4) {
            const int64_t top = merge_heap.front().first;
            int64_t count = 0;
            while (!merge_heap.empty() && merge_heap.front().first == top) {
                std::pop_heap(merge_heap.begin(), merge_heap.end(), cmp);
                const int32_t c = merge_heap.back().second;
                merge_heap.pop_back();
                ++count;
                const vector<int64_t> &cs = cov_sets[(size_t)names[(size_t)c]];
                size_t &i = merge_pos[(size_t)c];
                if (reverse) {
                    if (i > 0) {
                        --i;
                        merge_heap.push_back({cs[i], c});
                        std::push_heap(merge_heap.begin(), merge_heap.end(), cmp);
                    }
                } else if (++i < cs.size()) {
                    merge_heap.push_back({-cs[i], c});
                    std::push_heap(merge_heap.begin(), merge_heap.end(), cmp);
                }
            }
            if (count > 1) {
                ++counter;
                const int64_t pos = reverse ? top : -top;
                cov = std::max<int64_t>(cov, hcov[(size_t)((pos - bin_lo) / 10)]);
            }
        }
        return cov;
    }
    vector<size_t> merge_pos;
    vector<std::pair<int64_t, int32_t>> merge_heap;
    vector<int64_t> win_cnt, win_p, win_m;  // find_peaks: per-position counts over entry +- 2w
    vector<uint8_t> win_flag;               // bit 0: called area, bit 1: record with a bad strand

    void find_peaks(OrderedMap<vector<HistEntry>> &dd, bool reverse, char side,
                    PosSet &areas, vector<Peak> &tw) {
        vector<int64_t> dist{0};
        for (int s = 1; s <= P.w; ++s) {
            dist.push_back(s);
            dist.push_back(-s);
        }
        vector<size_t> cand;
        for (size_t i = 0; i < dd.keys.size(); ++i)
            if ((int64_t)dd.vals[i].size() >= P.min_count) cand.push_back(i);
        std::stable_sort(cand.begin(), cand.end(),
                         [&](size_t a, size_t b) { return dd.vals[a].size() > dd.vals[b].size(); });
        for (size_t ci : cand) {
            const int64_t entry = dd.keys[ci];
            if (areas.has(entry)) continue;
            // scan_for_best_bin: the winning shift by read count (strict >, first wins); the
            // coverage counts are only needed for the winner.  Every window entry+x+y lies in
            // entry +- 2w, so the per-position read counts and called flags are gathered once and
            // the 2w+1 windows summed from them (a record with a strand other than +/- raises the
            // KeyError as soon as an uncalled window covers it, as the per-read loop did).
            const int64_t w = P.w, span = 4 * w + 1;
            win_cnt.assign((size_t)span, 0);
            win_p.assign((size_t)span, 0);
            win_m.assign((size_t)span, 0);
            win_flag.assign((size_t)span, 0);
            for (int64_t d = 0; d < span; ++d) {
                const int64_t pos = entry - 2 * w + d;
                if (areas.has(pos)) win_flag[(size_t)d] |= 1;
                const vector<HistEntry> *lst = dd.find(pos);
                if (!lst) continue;
                win_cnt[(size_t)d] = (int64_t)lst->size();
                for (const HistEntry &h : *lst) {
                    const string_view dn = recs[(size_t)h.rec].dirn;
                    if (dn == "+")
                        win_p[(size_t)d] += 1;
                    else if (dn == "-")
                        win_m[(size_t)d] += 1;
                    else
                        win_flag[(size_t)d] |= 2;
                }
            }
            int64_t best = 0, center = 0, bx = 0;
            int64_t bdir_p = 0, bdir_m = 0;
            for (int64_t x : dist) {
                const size_t d0 = (size_t)(x + w);  // index of entry+x-w
                uint8_t fl = 0;
                for (size_t d = d0; d < d0 + (size_t)(2 * w + 1); ++d) fl |= win_flag[d];
                if (fl & 1) continue;
                if (fl & 2) throw LocusError{kLocusKeyError};
                int64_t cnt = 0, dp = 0, dm = 0;
                for (size_t d = d0; d < d0 + (size_t)(2 * w + 1); ++d) {
                    cnt += win_cnt[d];
                    dp += win_p[d];
                    dm += win_m[d];
                }
                if (cnt > best) {
                    best = cnt;
                    center = entry + x;
                    bx = x;
                    bdir_p = dp;
                    bdir_m = dm;
                }
            }
            vector<int32_t> best_names;
            int64_t cov = 0;
            if (best > 0) {
                for (int64_t y : dist) {
                    const vector<HistEntry> *lst = dd.find(entry + bx + y);
                    if (!lst) continue;
                    for (const HistEntry &h : *lst) best_names.push_back(h.rec);
                }
                cov = determine_cov(best_names, center, reverse);
            }
            if (cov <= 0) continue;
            const double prop = py_round3((double)best / (double)cov);
            if (!(prop > P.cutoff)) continue;
            char type = 0;
            if (bdir_p < bdir_m)
                type = reverse ? '3' : '5';
            else if (bdir_p > bdir_m)
                type = reverse ? '5' : '3';
            if (!type) continue;
            if (characterize(center - P.w, center + P.w, best_names)) {
                Peak pk{center - P.w, center + P.w, type, side, prop};
                tw.push_back(pk);
                for (int64_t b = pk.start; b <= pk.end; ++b) areas.add(b);
            }
        }
    }

    void sort_reads() {
        for (size_t r = 0; r < recs.size(); ++r) {
            const Record &R = recs[r];
            const int64_t lx = R.qstart, rx = R.qsize - R.qend;  // direction forced '+'
            bool failed = false;
            string ident(R.chrom);
            ident += '_';
            const bool chrom_known = R.chrom == string_view(in.chrom);
            for (size_t x = 0; x + 1 < R.bsize.size(); ++x) {
                const int64_t ls = R.bstart[x] + R.bsize[x], rs = R.bstart[x + 1];
                if (rs - ls > 50) {
                    if (!chrom_known) {
                        failed = true;
                        break;
                    }
                    auto a = splice.find(ls), b = splice.find(rs);
                    if (a == splice.end() || b == splice.end()) {
                        failed = true;
                        break;
                    }
                    ident += labels[(size_t)a->second];
                    ident += '-';
                    ident += labels[(size_t)b->second];
                    ident += '~';
                }
            }
            if (failed) continue;
            // identity.split('_')[1] != ''
            const size_t u1 = ident.find('_');
            const size_t u2 = ident.find('_', u1 + 1);
            const bool spliced = (u2 == string::npos ? ident.size() : u2) > u1 + 1;
            Pos p{R.tstart, R.tend, (int32_t)r, lx, rx};
            if (spliced) {
                auto it = se_dict.find(ident);
                if (it == se_dict.end()) {
                    ident_order.push_back(ident);
                    se_dict[ident].push_back(p);
                } else {
                    it->second.push_back(p);
                }
            } else {
                auto it = se_mono.find(ident);
                if (it == se_mono.end()) {
                    mono_order.push_back(ident);
                    se_mono[ident].push_back(p);
                } else {
                    it->second.push_back(p);
                }
            }
        }
    }

    // position tuple order: (start, end, (name, seq), left_extra, right_extra, '+')
    bool pos_less(const Pos &a, const Pos &b) const {
        if (a.start != b.start) return a.start < b.start;
        if (a.end != b.end) return a.end < b.end;
        const Record &A = recs[(size_t)a.rec], &B = recs[(size_t)b.rec];
        if (A.name != B.name) return A.name < B.name;
        if (A.seq != B.seq) return A.seq < B.seq;
        if (a.lx != b.lx) return a.lx < b.lx;
        return a.rx < b.rx;
    }

    void group_mono() {
        for (const string &id : mono_order) {
            vector<Pos> ps = se_mono[id];
            std::stable_sort(ps.begin(), ps.end(), [&](const Pos &a, const Pos &b) { return pos_less(a, b); });
            int64_t prev_end = 0;
            int counter = 0;
            string nid = id + "M0";
            for (const Pos &p : ps) {
                if (p.start > prev_end) {
                    counter += 1;
                    nid = id + "M" + std::to_string(counter);
                    prev_end = std::max(p.end, prev_end);
                } else {
                    prev_end = p.end;
                }
                auto it = se_dict.find(nid);
                if (it == se_dict.end()) {
                    ident_order.push_back(nid);
                    se_dict[nid].push_back(p);
                } else {
                    it->second.push_back(p);
                }
            }
        }
    }

    // find_ends for one identity (SDC:554-711); peaks map position -> owning position
    void find_ends(const vector<int64_t> &starts, const vector<int64_t> &ends,
                   std::unordered_map<int64_t, int64_t> &sp, std::unordered_map<int64_t, int64_t> &ep) {
        const int64_t up = P.up, down = P.down, mc = P.min_count;
        std::unordered_map<int64_t, int64_t> sc, ec;
        for (int64_t p : starts) sc[p] += 1;
        for (int64_t p : ends) ec[p] += 1;
        auto cnt = [](const std::unordered_map<int64_t, int64_t> &m, int64_t k) -> int64_t {
            auto it = m.find(k);
            return it == m.end() ? 0 : it->second;
        };
        vector<int64_t> ss = starts;
        std::sort(ss.begin(), ss.end());
        for (int64_t position : ss) {
            if (sp.count(position - up)) continue;
            int64_t wc = 0;
            for (int64_t i = 0; i < 10; ++i) wc += cnt(sc, position + i);
            if (wc < mc) continue;
            int64_t ob_min = INT64_MAX, ob_max = INT64_MIN;
            for (int64_t s = -up; s < down; ++s) {
                sp[position + s] = position;
                ob_min = std::min(ob_min, position + s);
                ob_max = std::max(ob_max, position + s);
            }
            if (ob_min == INT64_MAX) throw LocusError{kLocusValueError};
            int64_t best_bin = INT64_MIN;
            for (int64_t i = ob_min; i < ob_max; ++i) {
                int64_t b = 0;
                for (int64_t s = 0; s < 10; ++s) b += cnt(sc, i + s);
                best_bin = std::max(best_bin, b);
            }
            if (best_bin == INT64_MIN) throw LocusError{kLocusValueError};
            extend(sp, sc, position, position - up, -1, best_bin, mc);
            extend(sp, sc, position, position + down - 1, +1, best_bin, mc);
        }
        vector<int64_t> es = ends;
        std::sort(es.begin(), es.end(), std::greater<int64_t>());
        for (int64_t position : es) {
            if (ep.count(position + up - 1)) continue;
            int64_t wc = 0;
            for (int64_t i = 0; i < 10; ++i) wc += cnt(ec, position - i);
            if (wc < mc) continue;
            int64_t ob_min = INT64_MAX, ob_max = INT64_MIN;
            for (int64_t s = -down; s < up; ++s) {
                ep[position + s] = position;
                ob_min = std::min(ob_min, position + s);
                ob_max = std::max(ob_max, position + s);
            }
            if (ob_min == INT64_MAX) throw LocusError{kLocusValueError};
            int64_t best_bin = INT64_MIN;
            for (int64_t i = ob_min; i < ob_max; ++i) {
                int64_t b = 0;
                for (int64_t s = 0; s < 10; ++s) b += cnt(ec, i + s);
                best_bin = std::max(best_bin, b);
            }
            if (best_bin == INT64_MIN) throw LocusError{kLocusValueError};
            extend(ep, ec, position, position - down, -1, best_bin, mc);
            extend(ep, ec, position, position + up - 1, +1, best_bin, mc);
        }
    }

    // one extension loop of find_ends (SDC:598-620 and mirrors): windows of 10 beyond `adjacent`
    static void extend(std::unordered_map<int64_t, int64_t> &peaks, const std::unordered_map<int64_t, int64_t> &cnt,
                       int64_t position, int64_t adjacent, int dir, int64_t best_bin, int64_t mc) {
        bool extended = true;
        while (extended) {
            int64_t wc = 0;
            int64_t adj[10];
            for (int i = 1; i <= 10; ++i) {
                adj[i - 1] = adjacent + dir * i;
                auto it = cnt.find(adj[i - 1]);
                if (it != cnt.end()) wc += it->second;
            }
            if (best_bin > wc && wc >= mc) {
                for (int i = 0; i < 10; ++i) {
                    if (!peaks.count(adj[i]))
                        peaks[adj[i]] = position;
                    else
                        extended = false;
                }
            } else {
                extended = false;
            }
            adjacent = adj[9];
        }
    }

    void define_start_end_sites() {
        group_mono();
        vector<string> ids = ident_order;
        std::sort(ids.begin(), ids.end());
        int isoform_counter = 0;
        std::map<std::tuple<string, int64_t, int64_t>, int> iso_of;
        vector<int64_t> perm, pick;
        for (const string &id : ids) {
            const vector<Pos> &ps = se_dict[id];
            const int64_t n = (int64_t)ps.size();
            mando_ref::mt_choice(mt, n, std::min<int64_t>(n, 10000), perm, pick);
            vector<int64_t> starts, ends;
            for (int64_t t : pick) {
                starts.push_back(ps[(size_t)t].start);
                ends.push_back(ps[(size_t)t].end);
            }
            std::unordered_map<int64_t, int64_t> sp, ep;
            find_ends(starts, ends, sp, ep);
            for (const Pos &p : ps) {
                auto a = sp.find(p.start), b = ep.find(p.end);
                if (a == sp.end() || b == ep.end()) continue;
                auto key = std::make_tuple(id, a->second, b->second);
                auto it = iso_of.find(key);
                int iso;
                if (it == iso_of.end()) {
                    iso = isoform_counter++;
                    iso_of.emplace(key, iso);
                    out.iso_members.emplace_back();
                } else {
                    iso = it->second;
                }
                out.iso_members[(size_t)iso].push_back(p.rec);
            }
        }
    }
};

// ---------------------------------------------------------------------------------------------
// batch
// ---------------------------------------------------------------------------------------------
void parse_locus(string_view text, int64_t base, vector<Record> &recs) {
    size_t p = 0;
    vector<string_view> f;
    while (p < text.size()) {
        size_t e = text.find('\n', p);
        if (e == string_view::npos) e = text.size();
        const string_view line = text.substr(p, e - p);
        p = e + 1;
        split_tabs(line, f);
        if (f.size() < 24) throw LocusError{kLocusParse};
        Record R;
        R.dirn = f[8];
        R.name = f[9];
        R.qsize = to_i64(f[10]);
        R.qstart = to_i64(f[11]);
        R.qend = to_i64(f[12]);
        R.chrom = f[13];
        R.tstart = to_i64(f[15]);
        R.tend = to_i64(f[16]);
        split_list(f[18], R.bsize);
        split_list(f[20], R.bstart);
        if (R.bsize.size() != R.bstart.size()) throw LocusError{kLocusParse};
        R.accuracy = to_f64(f[21]);
        R.cs = f[22];
        R.seq = f[23];
        R.global = base + (int64_t)recs.size();
        recs.push_back(std::move(R));
    }
}

}  // namespace

struct mando_cluster_result {
    // all locus files; left uninitialised (the parallel reads fault it in), 2 MB-aligned and advised
    // for transparent huge pages, so a chunk's ~1 GB costs a few hundred faults, not ~300k
    std::unique_ptr<char, void (*)(void *)> text{nullptr, free};
    size_t text_len = 0;
    vector<int64_t> name_off, seq_off, rec_locus;
    vector<int32_t> name_len, seq_len;
    vector<int64_t> iso_locus, mem_off, mem, sub_off, sub;
    vector<int64_t> peak_locus, peak_start, peak_end;
    vector<char> peak_type, peak_side;
    vector<double> peak_prop;
    vector<int32_t> locus_status;
};

namespace {
thread_local string g_cluster_err;
}

extern "C" {

void cluster_ref_default_params(mando_cluster_params *p) {
    if (!p) return;
    p->cutoff = 0.1;
    p->splice_site_width = 1;
    p->minimum_read_count = 2;
    p->upstream_buffer = 10;
    p->downstream_buffer = 50;
    p->junctions = "gtag,gcag,atac,ctac,ctgc,gtat";
    p->seed = 0;
    p->threads = 0;
    p->poa_subsample = 100;
}

int cluster_ref_loci(const mando_cluster_params *prm, const char *const *psl_paths, const char *const *chroms,
                       int64_t n_loci, const int64_t *ann_pos, const int64_t *ann_off,
                       mando_cluster_result **out) {
    if (!prm || !out || n_loci < 0 || (n_loci > 0 && (!psl_paths || !chroms))) return MANDO_E_ARG;
    *out = nullptr;
    Params P;
    P.cutoff = prm->cutoff;
    P.w = prm->splice_site_width;
    P.min_count = prm->minimum_read_count;
    P.up = prm->upstream_buffer;
    P.down = prm->downstream_buffer;
    P.sub_k = prm->poa_subsample > 0 ? prm->poa_subsample : 100;
    P.seed = prm->seed;
    if (prm->junctions) {
        string j(prm->junctions);
        size_t a = 0;
        while (true) {
            const size_t c = j.find(',', a);
            P.junctions.push_back(j.substr(a, c == string::npos ? string::npos : c - a));
            if (c == string::npos) break;
            a = c + 1;
        }
    }
    auto res = std::make_unique<mando_cluster_result>();
    // read every locus file into one buffer (sizes first, then parallel reads)
    vector<int64_t> fsize((size_t)n_loci, 0), foff((size_t)n_loci + 1, 0);
    for (int64_t i = 0; i < n_loci; ++i) {
        FILE *fh = fopen(psl_paths[i], "rb");
        if (!fh) {
            fsize[(size_t)i] = -1;
            continue;
        }
        fseek(fh, 0, SEEK_END);
        fsize[(size_t)i] = ftell(fh);
        fclose(fh);
    }
    for (int64_t i = 0; i < n_loci; ++i) foff[(size_t)i + 1] = foff[(size_t)i] + std::max<int64_t>(0, fsize[(size_t)i]);
    res->text_len = (size_t)foff[(size_t)n_loci];
    {
        constexpr size_t kHuge = size_t(2) << 20;
        const size_t bytes = (std::max<size_t>(res->text_len, 1) + kHuge - 1) / kHuge * kHuge;
        void *buf = nullptr;
        if (posix_memalign(&buf, kHuge, bytes) != 0) return MANDO_E_NOMEM;
        (void)madvise(buf, bytes, MADV_HUGEPAGE);
        res->text.reset(static_cast<char *>(buf));
    }
    int nth = prm->threads > 0 ? prm->threads : (int)std::max(1u, std::thread::hardware_concurrency());
    nth = (int)std::min<int64_t>(nth, std::max<int64_t>(1, n_loci));
    vector<LocusIn> ins((size_t)n_loci);
    vector<vector<Record>> recs((size_t)n_loci);
    vector<LocusOut> outs((size_t)n_loci);
    // heaviest loci first
    vector<int64_t> order((size_t)n_loci);
    for (int64_t i = 0; i < n_loci; ++i) order[(size_t)i] = i;
    std::stable_sort(order.begin(), order.end(), [&](int64_t a, int64_t b) { return fsize[(size_t)a] > fsize[(size_t)b]; });
    std::atomic<int64_t> next{0};
    auto worker = [&]() {
        while (true) {
            const int64_t k = next.fetch_add(1);
            if (k >= n_loci) break;
            const int64_t i = order[(size_t)k];
            LocusOut &lo = outs[(size_t)i];
            try {
                if (fsize[(size_t)i] < 0) throw LocusError{kLocusIO};
                char *dst = res->text.get() + foff[(size_t)i];
                FILE *fh = fopen(psl_paths[i], "rb");
                if (!fh) throw LocusError{kLocusIO};
                const size_t got = fread(dst, 1, (size_t)fsize[(size_t)i], fh);
                fclose(fh);
                if ((int64_t)got != fsize[(size_t)i]) throw LocusError{kLocusIO};
                LocusIn &li = ins[(size_t)i];
                li.text = string_view(dst, got);
                li.chrom = chroms[i];
                if (ann_pos && ann_off)
                    for (int s = 0; s < 4; ++s) {
                        const int64_t a = ann_off[4 * i + s], b = ann_off[4 * i + s + 1];
                        li.ann[s].assign(ann_pos + a, ann_pos + b);
                    }
                {
                    PhTimer t(0);
                    parse_locus(li.text, 0, recs[(size_t)i]);
                }
                LocusRunner run(P, li, recs[(size_t)i], lo);
                run.run();
            } catch (const LocusError &e) {
                lo = LocusOut();
                lo.status = e.code;
            } catch (const std::exception &) {
                lo = LocusOut();
                lo.status = kLocusParse;
            }
        }
    };
    const char *pe = getenv("MANDO_CLUSTER_PROF");
    const bool prof = pe && pe[0] == '1';
    for (auto &x : g_ph) x = 0;
    vector<std::thread> th;
    for (int t = 0; t < nth; ++t) th.emplace_back(worker);
    for (auto &t : th) t.join();
    if (prof) {
        fprintf(stderr, "[mando cluster] thread-seconds:");
        for (int k = 0; k < 8; ++k) fprintf(stderr, " %s %.3f", kPhName[k], (double)g_ph[k].load() * 1e-9);
        fprintf(stderr, "\n");
    }
    // flatten
    const char *base = res->text.get();
    vector<int64_t> rec_base((size_t)n_loci + 1, 0);
    for (int64_t i = 0; i < n_loci; ++i) rec_base[(size_t)i + 1] = rec_base[(size_t)i] + (int64_t)recs[(size_t)i].size();
    const int64_t nr = rec_base[(size_t)n_loci];
    res->name_off.resize((size_t)nr);
    res->name_len.resize((size_t)nr);
    res->seq_off.resize((size_t)nr);
    res->seq_len.resize((size_t)nr);
    res->rec_locus.resize((size_t)nr);
    for (int64_t i = 0; i < n_loci; ++i)
        for (size_t r = 0; r < recs[(size_t)i].size(); ++r) {
            const Record &R = recs[(size_t)i][r];
            const size_t g = (size_t)(rec_base[(size_t)i] + (int64_t)r);
            res->name_off[g] = R.name.data() - base;
            res->name_len[g] = (int32_t)R.name.size();
            res->seq_off[g] = R.seq.data() - base;
            res->seq_len[g] = (int32_t)R.seq.size();
            res->rec_locus[g] = i;
        }
    res->mem_off.push_back(0);
    res->sub_off.push_back(0);
    res->locus_status.resize((size_t)n_loci);
    for (int64_t i = 0; i < n_loci; ++i) {
        const LocusOut &lo = outs[(size_t)i];
        res->locus_status[(size_t)i] = lo.status;
        for (size_t k = 0; k < lo.iso_members.size(); ++k) {
            res->iso_locus.push_back(i);
            for (int32_t r : lo.iso_members[k]) res->mem.push_back(rec_base[(size_t)i] + r);
            res->mem_off.push_back((int64_t)res->mem.size());
            for (int32_t r : lo.iso_sub[k]) res->sub.push_back(rec_base[(size_t)i] + r);
            res->sub_off.push_back((int64_t)res->sub.size());
        }
        for (const Peak &pk : lo.peaks) {
            res->peak_locus.push_back(i);
            res->peak_start.push_back(pk.start);
            res->peak_end.push_back(pk.end);
            res->peak_type.push_back(pk.type);
            res->peak_side.push_back(pk.side);
            res->peak_prop.push_back(pk.prop);
        }
    }
    *out = res.release();
    return MANDO_OK;
}

int cluster_ref_view_get(const mando_cluster_result *r, mando_cluster_view *v) {
    if (!r || !v) return MANDO_E_ARG;
    v->n_loci = (int64_t)r->locus_status.size();
    v->locus_status = r->locus_status.data();
    v->text = r->text.get();
    v->text_len = (int64_t)r->text_len;
    v->n_records = (int64_t)r->name_off.size();
    v->name_off = r->name_off.data();
    v->name_len = r->name_len.data();
    v->seq_off = r->seq_off.data();
    v->seq_len = r->seq_len.data();
    v->rec_locus = r->rec_locus.data();
    v->n_isoforms = (int64_t)r->iso_locus.size();
    v->iso_locus = r->iso_locus.data();
    v->mem_off = r->mem_off.data();
    v->mem = r->mem.data();
    v->sub_off = r->sub_off.data();
    v->sub = r->sub.data();
    v->n_peaks = (int64_t)r->peak_locus.size();
    v->peak_locus = r->peak_locus.data();
    v->peak_start = r->peak_start.data();
    v->peak_end = r->peak_end.data();
    v->peak_type = r->peak_type.data();
    v->peak_side = r->peak_side.data();
    v->peak_prop = r->peak_prop.data();
    return MANDO_OK;
}

void cluster_ref_free(mando_cluster_result *r) { delete r; }

}  // extern "C"
