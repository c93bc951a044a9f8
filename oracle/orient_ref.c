/* oracle/orient_ref.c — CPU restatement of the orientation step.  TEST INFRASTRUCTURE ONLY: the
 * checker for the HIP kernel (mandalorion_amd/csrc/orient_kernel.hip); never shipped or measured.
 *
 * PARITY UNPINNED.  The reference orients each subsampled read with
 *     mappy.Aligner(seq=first, preset='map-ont').map(seq) -> hit.is_primary, hit.strand
 * (/root/reference/utils/SpliceDefineConsensus.py:895-907).  mappy / minimap2 are third-party,
 * unpinned (`pip install mappy --upgrade`, /root/reference/setup.sh:9), absent from the image, and
 * the reference has no test or fixture for this step.  This file restates the documented map-ont
 * behaviour the step depends on, as the build's own specification that GPU and CPU both follow:
 *   - (k=15, w=10) minimizers, canonical k-mers, minimap2's invertible 2k-bit hash, strand-ambiguous
 *     k-mers skipped; a k-mer end position is a minimizer when its hash is the minimum of some window
 *     of w consecutive k-mers (all ties kept);
 *   - one-sequence index of the reference (the group's first subsampled read); query minimizers whose
 *     hash occurs more than 10 times in the index are skipped (minimap2's min mid-occ);
 *   - anchors (rev, x = ref end pos, y = query end pos, on the reverse-complemented query for rev),
 *     sorted by (rev, x, y);
 *   - chaining DP as mm_chain_dp: f_i = max(k, max_j f_j + min(dq, dr, k) - gap(|dr - dq|)) over the 64
 *     previous anchors of the same strand with 0 < dq <= 5000, 0 < dr <= 5000, |dr-dq| <= 500,
 *     gap(d) = floor(0.15 d) + floor(log2 d) / 2; ties -> the nearest predecessor;
 *   - chains taken greedily from the highest f (ties: lowest index), walking back until an anchor
 *     already used, score = f_end - f_stop; kept when >= 3 anchors and score >= 40;
 *   - chains in decreasing score; a chain is primary unless it overlaps an earlier primary chain on
 *     the query by more than half of the shorter one (mask_level 0.5); primaries are reported in that
 *     order (strand +1 / -1).
 * Differences from minimap2 that can change a strand call: no base-level extension / DP score filter,
 * fixed 64-anchor chaining look-back instead of max_iter/max_skip.  Synthetic reads carry their true
 * strand, which the tests check.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define OK_ 0
#define E_ARG -1
#define E_NOMEM -3
#define E_UNSUP -5

enum { K = 15, W = 10, MAX_OCC = 10, MAX_GAP = 5000, BW = 500, LOOKBACK = 64, MIN_CNT = 3, MIN_SCORE = 40 };

static inline int enc(uint8_t c) {
    switch (c) {
        case 'A': case 'a': return 0;
        case 'C': case 'c': return 1;
        case 'G': case 'g': return 2;
        case 'T': case 't': return 3;
        default: return 4;
    }
}

static inline uint64_t hash64(uint64_t key, uint64_t mask) {
    key = (~key + (key << 21)) & mask;
    key = key ^ key >> 24;
    key = ((key + (key << 3)) + (key << 8)) & mask;
    key = key ^ key >> 14;
    key = ((key + (key << 2)) + (key << 4)) & mask;
    key = key ^ key >> 28;
    key = (key + (key << 31)) & mask;
    return key;
}

/* minimizer keys (h << 33 | pos << 1 | z) of s[0..L), in position order; returns count or -1 */
static int64_t minimizers(const uint8_t *s, int64_t L, uint64_t *out, int64_t cap) {
    if (L < K) return 0;
    const uint64_t mask = (1ull << (2 * K)) - 1;
    const int64_t np = L - K + 1;
    uint64_t *H = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)np);
    uint8_t *z = (uint8_t *)malloc((size_t)np);
    uint8_t *mark = (uint8_t *)calloc((size_t)np, 1);
    if (!H || !z || !mark) {
        free(H); free(z); free(mark);
        return -1;
    }
    for (int64_t p = 0; p < np; ++p) {
        uint64_t f = 0, r = 0;
        int bad = 0;
        for (int t = 0; t < K; ++t) {
            const int c = enc(s[p + t]);
            if (c > 3) { bad = 1; break; }
            f = (f << 2) | (uint64_t)c;
            r |= (uint64_t)(3 - c) << (2 * t);
        }
        if (bad || f == r) {
            H[p] = UINT64_MAX;
            z[p] = 0;
        } else {
            z[p] = f < r ? 0 : 1;
            H[p] = hash64(f < r ? f : r, mask);
        }
    }
    const int64_t nw = np <= W ? 1 : np - W + 1;
    const int64_t ww = np <= W ? np : W;
    for (int64_t w0 = 0; w0 < nw; ++w0) {
        uint64_t m = UINT64_MAX;
        for (int64_t t = 0; t < ww; ++t) if (H[w0 + t] < m) m = H[w0 + t];
        if (m == UINT64_MAX) continue;
        for (int64_t t = 0; t < ww; ++t) if (H[w0 + t] == m) mark[w0 + t] = 1;
    }
    int64_t n = 0;
    for (int64_t p = 0; p < np; ++p)
        if (mark[p]) {
            if (n >= cap) { n = -2; break; }
            out[n++] = (H[p] << 33) | ((uint64_t)(p + K - 1) << 1) | z[p];
        }
    free(H); free(z); free(mark);
    return n;
}

static int cmp_u64(const void *a, const void *b) {
    const uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
    return x < y ? -1 : x > y;
}

static inline int ilog2_u32(uint32_t v) {
    int r = 0;
    while (v >>= 1) ++r;
    return r;
}

typedef struct { int32_t score, rev, ys, ye, order; } chain_t;

static int cmp_chain(const void *a, const void *b) {
    const chain_t *x = (const chain_t *)a, *y = (const chain_t *)b;
    if (x->score != y->score) return x->score > y->score ? -1 : 1;
    return x->order - y->order;
}

/* one query against the sorted reference keys; writes up to max_hits strands */
static int orient_one(const uint64_t *ref, int64_t nref, const uint8_t *q, int64_t qlen, int8_t *hits,
                      int32_t max_hits, int32_t *n_hits) {
    /* no capacity limit (mappy has none): at most one minimizer per position, MAX_OCC anchors each */
    const size_t qcap = (size_t)(qlen > 0 ? qlen : 1), acap = qcap * MAX_OCC + 1;
    uint64_t *qm = (uint64_t *)malloc(sizeof(uint64_t) * qcap);
    uint64_t *an = (uint64_t *)malloc(sizeof(uint64_t) * acap);
    int32_t *f = (int32_t *)malloc(sizeof(int32_t) * acap);
    int32_t *p = (int32_t *)malloc(sizeof(int32_t) * acap);
    uint8_t *used = (uint8_t *)malloc(acap);
    chain_t *ch = (chain_t *)malloc(sizeof(chain_t) * acap);
    int rc = OK_;
    *n_hits = 0;
    if (!qm || !an || !f || !p || !used || !ch) { rc = E_NOMEM; goto done; }
    const int64_t nq = minimizers(q, qlen, qm, (int64_t)qcap);
    if (nq == -1) { rc = E_NOMEM; goto done; }
    if (nq == -2) { rc = E_UNSUP; goto done; }
    int64_t na = 0;
    for (int64_t i = 0; i < nq; ++i) {
        const uint64_t h = qm[i] >> 33;
        /* lower bound of h in ref */
        int64_t lo = 0, hi = nref;
        while (lo < hi) {
            const int64_t mid = (lo + hi) / 2;
            if ((ref[mid] >> 33) < h) lo = mid + 1; else hi = mid;
        }
        int64_t e = lo;
        while (e < nref && (ref[e] >> 33) == h) ++e;
        if (e - lo > MAX_OCC) continue;
        const int64_t qpos = (int64_t)((qm[i] >> 1) & 0xffffffffull);
        const int qz = (int)(qm[i] & 1);
        for (int64_t t = lo; t < e; ++t) {
            const int64_t rpos = (int64_t)((ref[t] >> 1) & 0xffffffffull);
            const int rev = qz ^ (int)(ref[t] & 1);
            const int64_t y = rev ? qlen - 1 - (qpos - K + 1) : qpos;
            if ((size_t)na >= acap) { rc = E_UNSUP; goto done; }
            an[na++] = ((uint64_t)rev << 62) | ((uint64_t)rpos << 31) | (uint64_t)y;
        }
    }
    qsort(an, (size_t)na, sizeof(uint64_t), cmp_u64);
    for (int64_t i = 0; i < na; ++i) {
        const int64_t ri = (int64_t)(an[i] >> 62), xi = (int64_t)((an[i] >> 31) & 0x7fffffff),
                      yi = (int64_t)(an[i] & 0x7fffffff);
        int32_t best = INT32_MIN, bj = -1;
        for (int64_t j = i - LOOKBACK < 0 ? 0 : i - LOOKBACK; j < i; ++j) {
            const int64_t rj = (int64_t)(an[j] >> 62), xj = (int64_t)((an[j] >> 31) & 0x7fffffff),
                          yj = (int64_t)(an[j] & 0x7fffffff);
            if (rj != ri) continue;
            const int64_t dr = xi - xj, dq = yi - yj;
            if (dr <= 0 || dq <= 0 || dr > MAX_GAP || dq > MAX_GAP) continue;
            const int64_t dd = dr > dq ? dr - dq : dq - dr;
            if (dd > BW) continue;
            int64_t sc = dq < dr ? dq : dr;
            if (sc > K) sc = K;
            sc -= dd ? (dd * 15) / 100 + (ilog2_u32((uint32_t)dd) >> 1) : 0;
            const int32_t cand = f[j] + (int32_t)sc;
            if (cand >= best) { best = cand; bj = (int32_t)j; }
        }
        if (bj >= 0 && best > K) { f[i] = best; p[i] = bj; } else { f[i] = K; p[i] = -1; }
    }
    memset(used, 0, (size_t)(na > 0 ? na : 1));
    int32_t nch = 0;
    for (;;) {
        int64_t bi = -1;
        for (int64_t i = 0; i < na; ++i)
            if (!used[i] && (bi < 0 || f[i] > f[bi])) bi = i;
        if (bi < 0 || f[bi] < MIN_SCORE) break;
        int64_t k = bi, first = bi;
        int32_t cnt = 0;
        while (k >= 0 && !used[k]) { used[k] = 1; ++cnt; first = k; k = p[k]; }
        const int32_t score = f[bi] - (k >= 0 ? f[k] : 0);
        if (cnt >= MIN_CNT && score >= MIN_SCORE) {
            chain_t c;
            c.score = score;
            c.rev = (int32_t)(an[bi] >> 62);
            c.ys = (int32_t)(an[first] & 0x7fffffff) - K + 1;
            c.ye = (int32_t)(an[bi] & 0x7fffffff) + 1;
            c.order = nch;
            ch[nch++] = c;
        }
    }
    qsort(ch, (size_t)nch, sizeof(chain_t), cmp_chain);
    int32_t np_ = 0;
    int32_t pqs[64], pqe[64];
    /* one primary past max_hits is still counted: *n_hits == max_hits + 1 reports the overflow */
    for (int32_t c = 0; c < nch && np_ <= max_hits && np_ < 64; ++c) {
        const int32_t qs = ch[c].rev ? (int32_t)qlen - ch[c].ye : ch[c].ys;
        const int32_t qe = ch[c].rev ? (int32_t)qlen - ch[c].ys : ch[c].ye;
        int prim = 1;
        for (int32_t t = 0; t < np_; ++t) {
            const int32_t ov = (qe < pqe[t] ? qe : pqe[t]) - (qs > pqs[t] ? qs : pqs[t]);
            const int32_t l0 = qe - qs, l1 = pqe[t] - pqs[t];
            if (2 * ov > (l0 < l1 ? l0 : l1)) { prim = 0; break; }
        }
        if (!prim) continue;
        pqs[np_] = qs;
        pqe[np_] = qe;
        if (np_ < max_hits) hits[np_] = ch[c].rev ? -1 : 1;
        ++np_;
    }
    *n_hits = np_;
done:
    free(qm); free(an); free(f); free(p); free(used); free(ch);
    return rc;
}

/* Mirrors mando_orient_batch: ASCII reads, groups by grp_off; reference = each group's first read. */
int orient_ref_batch(const uint8_t *seqs, const int64_t *seq_off, const int64_t *grp_off, int64_t n_groups,
                     int8_t *hit_strands, int32_t max_hits, int32_t *n_hits) {
    if (n_groups < 0 || max_hits < 1) return E_ARG;
    int rc = OK_;
    uint64_t *ref = NULL;
    for (int64_t g = 0; g < n_groups && rc == OK_; ++g) {
        const int64_t r0 = grp_off[g], r1 = grp_off[g + 1];
        if (r1 <= r0) continue;
        const int64_t L0 = seq_off[r0 + 1] - seq_off[r0];
        free(ref);
        ref = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)(L0 > 0 ? L0 : 1));
        if (!ref) return E_NOMEM;
        const int64_t nref = minimizers(seqs + seq_off[r0], L0, ref, L0 > 0 ? L0 : 1);
        if (nref == -1) { rc = E_NOMEM; break; }
        if (nref == -2) { rc = E_UNSUP; break; }
        qsort(ref, (size_t)nref, sizeof(uint64_t), cmp_u64);
        for (int64_t r = r0; r < r1; ++r) {
            rc = orient_one(ref, nref, seqs + seq_off[r], seq_off[r + 1] - seq_off[r], hit_strands + r * max_hits,
                            max_hits, n_hits + r);
            if (rc != OK_) break;
        }
    }
    free(ref);
    return rc;
}

/* exposed for tests: minimizer keys of one sequence */
int64_t orient_ref_minimizers(const uint8_t *s, int64_t L, uint64_t *out, int64_t cap) {
    return minimizers(s, L, out, cap);
}
