/*
 * oracle/poa_simd.c — TEST INFRASTRUCTURE ONLY: the CPU baseline of bench.py (cpu_baseline, kind
 * "simd-port") and the checker tests/test_poa_simd.py.  Never linked into or called by the product path.
 *
 * The same restatement of abPOA v1.4.1 as oracle/poa_ref.c (this file includes it), with the banded DP
 * rows of align_window vectorised the way abPOA vectorises them (SIMD over the band of one graph row,
 * 16-bit score lanes when the scores fit, abpoa_align_simd.c in abPOA's source tree; SURVEY.md
 * Appendix C): AVX2, 16 int16 cells per vector, the horizontal-gap states F1 / F2 by an in-register
 * prefix-max scan with a carry across vectors, the argmax by a vector max and a movemask search.  The
 * row records, the score-comparison backtrack, the graph update and the consensus are the scalar
 * restatement's.  Output is byte-identical to poa_ref.c (tests/test_poa_simd.py), which is what makes
 * it a CPU baseline of the same work: it is NOT abPOA (absent here), and it is timed, not trusted.
 *
 * 16-bit exactness.  Scores are held in int16 with saturating arithmetic; -inf is -32768.  Values
 * derived from -inf stay near it (a row adds at most one score or gap term to them before the band
 * masks them again), finite values of reads under ~5,600 nt at the default scores are far above it.
 * Every stored H / E1 / E2 value is checked to be either <= T_LO (the -inf class) or in
 * [T_HI, T_TOP] (finite, and exact because nothing near it saturates); H0 / F1 / F2 differ from those
 * by bounded terms within a row, and are not stored: the backtrack recomputes the rows it tests for a
 * horizontal gap with the same int16 operations.  When the check fails, or a read is too long for int16, or a row's
 * band lies outside the padded storage of a predecessor, the window is re-aligned by the scalar code
 * (align_window in poa_ref.c): abPOA's 32-bit fallback plays that role there.  Inside the two classes
 * every comparison the outputs depend on (row argmax, the backtrack's equality tests, the end cell)
 * orders and equates values exactly as the scalar code's ints do.
 */
#define _POSIX_C_SOURCE 200809L
#define POA_SIMD 1
#include "poa_ref.c"

#include <immintrin.h>

#define SPAD 32 /* -inf cells stored on each side of a row (>= 16: vector loads past a band edge) */
#define NEG16 ((int16_t)-32768)
#define T_LO (-30000)
#define T_HI (-16000)
#define T_TOP 30000

typedef struct {
    int beg, end, argmax;
    int64_t off; /* first stored cell (column beg - SPAD) in the plane pools */
} srow;

/* the six int16 planes, kept per host thread from window to window (abPOA keeps its DP matrix in the
 * abpoa_t object across reads the same way): a fresh allocation per window cost more in page faults
 * than the DP itself */
#include <pthread.h>
typedef struct {
    int16_t *pl[3];
    int64_t cap;
} sarena;
static pthread_key_t arena_key;
static pthread_once_t arena_once = PTHREAD_ONCE_INIT;
static void arena_free(void *x) {
    sarena *a = (sarena *)x;
    for (int k = 0; k < 3; ++k) free(a->pl[k]);
    free(a);
}
static void arena_key_init(void) { (void)pthread_key_create(&arena_key, arena_free); }
static sarena *arena_get(void) {
    (void)pthread_once(&arena_once, arena_key_init);
    sarena *a = (sarena *)pthread_getspecific(arena_key);
    if (!a) {
        a = (sarena *)calloc(1, sizeof(sarena));
        (void)pthread_setspecific(arena_key, a);
    }
    return a;
}

/* inclusive prefix max of the 16 int16 lanes of x (lane i gets max of lanes 0..i) */
static inline __m256i pmax16(__m256i x, __m256i negv) {
    x = _mm256_max_epi16(x, _mm256_alignr_epi8(x, negv, 14));
    x = _mm256_max_epi16(x, _mm256_alignr_epi8(x, negv, 12));
    x = _mm256_max_epi16(x, _mm256_alignr_epi8(x, negv, 8));
    /* lane 7 of the low half into every lane of the high half */
    const __m256i b7 = _mm256_shuffle_epi8(x, _mm256_set1_epi16(0x0f0e));
    return _mm256_max_epi16(x, _mm256_permute2x128_si256(b7, negv, 0x02));
}

/* lane 15 of x in every lane */
static inline __m256i last16(__m256i x) {
    const __m256i b = _mm256_shuffle_epi8(x, _mm256_set1_epi16(0x0f0e));
    return _mm256_permute2x128_si256(b, b, 0x11);
}

/* x shifted up by one lane across the whole vector, lane 0 taking lane 15 of carry */
static inline __m256i shift1(__m256i x, __m256i carry) {
    return _mm256_alignr_epi8(x, _mm256_permute2x128_si256(x, carry, 0x02), 14);
}

static inline int16_t sat16(int x) { return (int16_t)(x < -32768 ? -32768 : x > 32767 ? 32767 : x); }

/* H0, F1, F2 of window row (beg rb, width rw) as the vector row computes them (saturating int16, F by
 * the prefix form with its ramps), from the predecessors' stored H / E1 / E2 */
static void recompute_row(const graph_t *g, int v, const int *pos, int pB, int pE, const int *wrow, const srow *ri,
                          const int16_t *H, const int16_t *E1, const int16_t *E2, const int16_t *sp, int rb, int rw,
                          int e1, int e2, int oe1, int oe2, int16_t *rh0, int16_t *rf1, int16_t *rf2) {
    const ivec *in = &g->in[v];
    for (int x = 0; x < rw; ++x) {
        const int j = rb + x;
        int mv = -32768, a1 = -32768, a2 = -32768;
        for (int k = 0; k < in->n; ++k) {
            const int u = in->a[k];
            const int pr = (pos[u] >= pB && pos[u] <= pE) ? wrow[pos[u] - pB] : -1;
            if (pr < 0) continue;
            const int64_t b = ri[pr].off + SPAD + (j - ri[pr].beg);
            mv = imax(mv, H[b - 1]);
            a1 = imax(a1, E1[b]);
            a2 = imax(a2, E2[b]);
        }
        rh0[x] = (int16_t)imax(sat16(mv + sp[j]), imax(a1, a2));
    }
    int p1 = -32768, p2 = -32768; /* exclusive prefix maxima */
    for (int x = 0; x < rw; ++x) {
        rf1[x] = sat16(p1 - (int16_t)(e1 * x + oe1 - e1));
        rf2[x] = sat16(p2 - (int16_t)(e2 * x + oe2 - e2));
        p1 = imax(p1, sat16(rh0[x] + (int16_t)(e1 * x)));
        p2 = imax(p2, sat16(rh0[x] + (int16_t)(e2 * x)));
    }
}

static int64_t align_window_simd(const graph_t *g, const int *order, const int *pos, const int *remain, int B,
                                 int E, const uint8_t *q, int qlen, const scorer *sc, int *qnode) {
    const mando_poa_params *p = sc->p;
    const int e1 = p->gap_ext1, e2 = p->gap_ext2, o1 = p->gap_open1, o2 = p->gap_open2;
    const int oe1 = sc->oe1, oe2 = sc->oe2;
    /* int16 range: the largest finite score is match * qlen; small gap / score terms keep the per-row
     * offsets of the -inf class and of F's ramps bounded */
    if ((int64_t)p->match * qlen >= T_TOP - 512 || p->match > 64 || p->mismatch > 64 || oe1 > 128 || oe2 > 128 ||
        e1 > 8 || e2 > 8 || e1 < 0 || e2 < 0 || o1 < 0 || o2 < 0)
        return -2;
    const int pB = pos[B], pE = pos[E];
    if (pE <= pB) return -1;
    const int span = pE - pB + 1;
    /* window rows: as align_window (forward reachability from B, backward from E) */
    uint8_t *fl = (uint8_t *)calloc((size_t)span, 1);
    for (int r = pB; r <= pE; ++r) {
        const int v = order[r];
        if (v == B) { fl[r - pB] |= 1; continue; }
        for (int k = 0; k < g->in[v].n; ++k) {
            const int pu = pos[g->in[v].a[k]];
            if (pu >= pB && (fl[pu - pB] & 1)) { fl[r - pB] |= 1; break; }
        }
    }
    for (int r = pE; r >= pB; --r) {
        const int v = order[r];
        if (v == E) { fl[r - pB] |= 2; continue; }
        for (int k = 0; k < g->out[v].n; ++k) {
            const int pu = pos[g->out[v].a[k]];
            if (pu <= pE && pu > r && (fl[pu - pB] & 2)) { fl[r - pB] |= 2; break; }
        }
    }
    int m = 0;
    int *wrow = (int *)malloc(sizeof(int) * (size_t)span);
    int *rowv = (int *)malloc(sizeof(int) * (size_t)span);
    for (int x = 0; x < span; ++x) {
        wrow[x] = (fl[x] == 3) ? m : -1;
        if (fl[x] == 3) rowv[m++] = order[pB + x];
    }
    free(fl);
#define WROW(node_) ((pos[node_] >= pB && pos[node_] <= pE) ? wrow[pos[node_] - pB] : -1)
    const int remE = remain[E];
    const int w = band_w(p, qlen);

    /* score profile: prof[b][j] = score of node base b against query column j (j >= 1: q[j - 1]; j = 0
     * and past qlen: 0) */
    const int plen = qlen + 64;
    int16_t *prof = (int16_t *)malloc(sizeof(int16_t) * (size_t)plen * 5);
    for (int b = 0; b < 5; ++b) {
        int16_t *pr = prof + (size_t)b * plen;
        pr[0] = 0;
        for (int j = 1; j <= qlen; ++j) pr[j] = (int16_t)sc->mat[b][q[j - 1]];
        for (int j = qlen + 1; j < plen; ++j) pr[j] = 0;
    }

    srow *ri = (srow *)malloc(sizeof(srow) * (size_t)m);
    sarena *ar = arena_get();
    int64_t used = 0;
    if (ar->cap == 0) ar->cap = (int64_t)m * (2 * w + 2 * SPAD + 48) + 4096;
    int16_t *H = ar->pl[0], *E1 = ar->pl[1], *E2 = ar->pl[2];
#define SGROW(need)                                                                    \
    do {                                                                               \
        if (H == NULL || used + (need) > ar->cap) {                                    \
            while (used + (need) > ar->cap) ar->cap *= 2;                              \
            for (int k_ = 0; k_ < 3; ++k_)                                             \
                ar->pl[k_] = (int16_t *)realloc(ar->pl[k_], sizeof(int16_t) * (size_t)ar->cap); \
            H = ar->pl[0], E1 = ar->pl[1], E2 = ar->pl[2];                            \
        }                                                                              \
    } while (0)
    /* a row of band [beg, end]: SPAD -inf cells, the band rounded up to whole vectors, SPAD more */
#define ROWLEN(beg_, end_) (((((end_) - (beg_) + 1) + 15) & ~15) + 2 * SPAD)
#define SCELL(r_, col_) (ri[r_].off + SPAD + ((col_)-ri[r_].beg))
    int bad = 0;
    int64_t cells = 0;
    const __m256i negv = _mm256_set1_epi16(NEG16);
    {
        /* source row (B) */
        const int remB = remain[B] - remE - 1;
        const int end = imin(qlen, imax(0, qlen - remB) + w);
        const int L = ROWLEN(0, end);
        SGROW(L);
        ri[0].beg = 0;
        ri[0].end = end;
        ri[0].off = 0;
        ri[0].argmax = 0;
        for (int x = 0; x < L; ++x) H[x] = E1[x] = E2[x] = NEG16;
        for (int j = 0; j <= end; ++j) {
            const int64_t c = SPAD + j;
            int h, f1 = 0, f2 = 0;
            if (j == 0) {
                h = 0;
            } else {
                f1 = -(o1 + e1 * j);
                f2 = -(o2 + e2 * j);
                h = imax(f1, f2);
                if (f1 < T_HI || f2 < T_HI) bad = 1;
            }
            if (h - imax(oe1, oe2) < T_HI) bad = 1;
            H[c] = (int16_t)imax(h, -32768);
            E1[c] = (int16_t)imax(h - oe1, -32768);
            E2[c] = (int16_t)imax(h - oe2, -32768);
        }
        used = L;
        cells += end + 1;
    }
    /* per-lane constants: lane index, and the F ramps e * (lane) */
    const __m256i lanei = _mm256_setr_epi16(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
    const __m256i vcls = _mm256_set1_epi16(T_LO + 1);
    const __m256i ve1 = _mm256_set1_epi16((int16_t)e1), ve2 = _mm256_set1_epi16((int16_t)e2);
    const __m256i voe1 = _mm256_set1_epi16((int16_t)oe1), voe2 = _mm256_set1_epi16((int16_t)oe2);
    __m256i *ramps = NULL;
    int rcap = 0;
    int pr_list[64];
    for (int i = 1; i < m - 1 && !bad; ++i) {
        const int v = rowv[i];
        const ivec *in = &g->in[v];
        int posL = 2147483647, posR = -2147483647 - 1, np = 0;
        for (int k = 0; k < in->n; ++k) {
            const int pr = WROW(in->a[k]);
            if (pr < 0) continue;
            posL = imin(posL, ri[pr].argmax + 1);
            posR = imax(posR, ri[pr].argmax + 1);
            if (np < 64) pr_list[np] = pr;
            ++np;
        }
        if (np > 64) { bad = 1; break; }
        const int x = qlen - (remain[v] - remE - 1);
        const int beg = imax(0, imin(posL, x) - w);
        const int end = imin(qlen, imax(posR, x) + w);
        const int width = end - beg + 1;
        const int nv = (width + 15) >> 4;
        /* F's ramps e (j - beg) on top of the largest finite score must not saturate */
        if ((int64_t)p->match * qlen + (int64_t)imax(e1, e2) * 16 * nv >= 32000) { bad = 1; break; }
        /* every predecessor's padded storage must cover columns [beg - 1, beg + 16 nv) */
        for (int k = 0; k < np; ++k) {
            const srow *pi = &ri[pr_list[k]];
            const int lo = beg - 1 - pi->beg, hi = beg + 16 * nv - 1 - pi->beg;
            if (lo < -SPAD || hi >= ROWLEN(pi->beg, pi->end) - SPAD) bad = 1;
        }
        if (bad) break;
        const int L = ROWLEN(beg, end);
        SGROW(L);
        ri[i].beg = beg;
        ri[i].end = end;
        ri[i].off = used;
        const int64_t o = used + SPAD;
        used += L;
        cells += width;
        for (int x2 = 0; x2 < SPAD; x2 += 16) {
            const int64_t a = o - SPAD + x2, b = o + 16 * nv + x2;
            int16_t *const planes[3] = {H, E1, E2};
            for (int k = 0; k < 3; ++k) {
                _mm256_storeu_si256((__m256i *)(planes[k] + a), negv);
                _mm256_storeu_si256((__m256i *)(planes[k] + b), negv);
            }
        }
        const int16_t *sp = prof + (size_t)g->base[v] * plen;
        if (nv > rcap) {  /* F ramps e (j - beg) and oe + e (j - 1 - beg) of lane columns, per vector */
            rcap = 2 * nv;
            free(ramps);
            if (posix_memalign((void **)&ramps, 32, sizeof(__m256i) * 4 * (size_t)rcap)) { ramps = NULL; bad = 1; break; }
            for (int t = 0; t < rcap; ++t) {
                const __m256i col = _mm256_add_epi16(lanei, _mm256_set1_epi16((int16_t)(16 * t)));
                const __m256i a = _mm256_mullo_epi16(col, _mm256_set1_epi16((int16_t)e1));
                const __m256i b = _mm256_mullo_epi16(col, _mm256_set1_epi16((int16_t)e2));
                _mm256_store_si256(ramps + 4 * t, a);
                _mm256_store_si256(ramps + 4 * t + 1, b);
                _mm256_store_si256(ramps + 4 * t + 2, _mm256_add_epi16(a, _mm256_set1_epi16((int16_t)(oe1 - e1))));
                _mm256_store_si256(ramps + 4 * t + 3, _mm256_add_epi16(b, _mm256_set1_epi16((int16_t)(oe2 - e2))));
            }
        }
        __m256i c1 = negv, c2 = negv, vmax = negv, vmin = _mm256_set1_epi16(-1);
        for (int t = 0; t < nv; ++t) {
            const int j0 = beg + 16 * t;
            __m256i mv = negv, a1 = negv, a2 = negv;
            for (int k = 0; k < np; ++k) {
                const srow *pi = &ri[pr_list[k]];
                const int64_t b = pi->off + SPAD + (j0 - pi->beg);
                mv = _mm256_max_epi16(mv, _mm256_loadu_si256((const __m256i *)(H + b - 1)));
                a1 = _mm256_max_epi16(a1, _mm256_loadu_si256((const __m256i *)(E1 + b)));
                a2 = _mm256_max_epi16(a2, _mm256_loadu_si256((const __m256i *)(E2 + b)));
            }
            const __m256i s = _mm256_loadu_si256((const __m256i *)(sp + j0));
            /* the last vector's lanes past the band end hold -inf (stored and read as out-of-band cells) */
            const int tail = t == nv - 1;
            const __m256i valid = _mm256_cmpgt_epi16(_mm256_set1_epi16((int16_t)(width - 16 * t)), lanei);
            __m256i h0 = _mm256_max_epi16(_mm256_adds_epi16(mv, s), _mm256_max_epi16(a1, a2));
            if (tail) h0 = _mm256_blendv_epi8(negv, h0, valid);
            /* F: F[j] = max_{beg <= k < j} (H0[k] + e (k - beg)) - oe - e (j - 1 - beg) */
            const __m256i *rp = ramps + 4 * t;
            const __m256i p1 = _mm256_max_epi16(pmax16(_mm256_adds_epi16(h0, rp[0]), negv), c1);
            const __m256i p2 = _mm256_max_epi16(pmax16(_mm256_adds_epi16(h0, rp[1]), negv), c2);
            const __m256i f1 = _mm256_subs_epi16(shift1(p1, c1), rp[2]);
            const __m256i f2 = _mm256_subs_epi16(shift1(p2, c2), rp[3]);
            c1 = last16(p1);
            c2 = last16(p2);
            __m256i h = _mm256_max_epi16(h0, _mm256_max_epi16(f1, f2));
            __m256i ee1 = _mm256_max_epi16(_mm256_subs_epi16(a1, ve1), _mm256_subs_epi16(h, voe1));
            __m256i ee2 = _mm256_max_epi16(_mm256_subs_epi16(a2, ve2), _mm256_subs_epi16(h, voe2));
            if (tail) {
                h = _mm256_blendv_epi8(negv, h, valid);
                ee1 = _mm256_blendv_epi8(negv, ee1, valid);
                ee2 = _mm256_blendv_epi8(negv, ee2, valid);
            }
            const int64_t c = o + 16 * t;
            _mm256_storeu_si256((__m256i *)(H + c), h);
            _mm256_storeu_si256((__m256i *)(E1 + c), ee1);
            _mm256_storeu_si256((__m256i *)(E2 + c), ee2);
            vmax = _mm256_max_epi16(vmax, h);
            /* class check: T_LO < z < T_HI  <=>  (uint16)(z - T_LO - 1) < T_HI - T_LO - 1 */
            vmin = _mm256_min_epu16(vmin, _mm256_sub_epi16(h, vcls));
            vmin = _mm256_min_epu16(vmin, _mm256_sub_epi16(ee1, vcls));
            vmin = _mm256_min_epu16(vmin, _mm256_sub_epi16(ee2, vcls));
        }
        /* horizontal: the row's smallest class offset and its maximum */
        vmin = _mm256_min_epu16(vmin, _mm256_permute2x128_si256(vmin, vmin, 0x01));
        const int minoff = _mm_extract_epi16(_mm_minpos_epu16(_mm256_castsi256_si128(vmin)), 0);
        if (minoff < T_HI - T_LO - 1) { bad = 1; break; }
        /* leftmost maximum of H over the row */
        __m256i mx = _mm256_max_epi16(vmax, _mm256_alignr_epi8(vmax, vmax, 2));
        mx = _mm256_max_epi16(mx, _mm256_alignr_epi8(mx, mx, 4));
        mx = _mm256_max_epi16(mx, _mm256_alignr_epi8(mx, mx, 8));
        mx = _mm256_max_epi16(mx, _mm256_permute2x128_si256(mx, mx, 0x01));
        const __m256i best = mx; /* every lane: the row maximum */
        if (_mm256_extract_epi16(mx, 0) > T_TOP) { bad = 1; break; }
        int besti = beg;
        for (int t = 0; t < nv; ++t) {
            const __m256i hv = _mm256_loadu_si256((const __m256i *)(H + o + 16 * t));
            const unsigned msk = (unsigned)_mm256_movemask_epi8(_mm256_cmpeq_epi16(hv, best));
            if (msk) {
                besti = beg + 16 * t + (__builtin_ctz(msk) >> 1);
                break;
            }
        }
        ri[i].argmax = besti;
    }

    int fail = 0;
    if (!bad) {
        /* end: best predecessor of E at column qlen (first in in-edge order on ties) */
        int bi = -1, bs = -2147483647 - 1;
        for (int k = 0; k < g->in[E].n; ++k) {
            const int pr = WROW(g->in[E].a[k]);
            if (pr < 0) continue;
            if (qlen < ri[pr].beg || qlen > ri[pr].end) continue;
            const int h = H[SCELL(pr, qlen)];
            if (h > bs) {
                bs = h;
                bi = pr;
            }
        }
        if (bi < 0) fail = 1;
        /* backtrack by score comparison: poa_ref.c's, on the int16 planes.  H0, F1 and F2 are not
         * stored (half the store traffic of the rows): the row the walk reaches in an F test is
         * recomputed from its predecessors' stored H / E1 / E2 with the DP's own int16 operations */
        int frow = -1, fcap = 0;
        int16_t *rh0 = NULL, *rf1 = NULL, *rf2 = NULL;
#define RECOMPUTE(i_)                                                                                     \
    do {                                                                                                  \
        if (frow != (i_)) {                                                                               \
            frow = (i_);                                                                                  \
            const int rb = ri[frow].beg, rw = ri[frow].end - rb + 1;                                      \
            if (rw > fcap) {                                                                              \
                fcap = 2 * rw;                                                                            \
                rh0 = (int16_t *)realloc(rh0, sizeof(int16_t) * (size_t)fcap);                            \
                rf1 = (int16_t *)realloc(rf1, sizeof(int16_t) * (size_t)fcap);                            \
                rf2 = (int16_t *)realloc(rf2, sizeof(int16_t) * (size_t)fcap);                            \
            }                                                                                             \
            recompute_row(g, rowv[frow], pos, pB, pE, wrow, ri, H, E1, E2, prof + (size_t)g->base[rowv[frow]] * plen, \
                          rb, rw, e1, e2, oe1, oe2, rh0, rf1, rf2);                                       \
        }                                                                                                 \
    } while (0)
#define RH0(col_) ((col_) < ri[frow].beg ? -32768 : (int)rh0[(col_)-ri[frow].beg])
#define RF1(col_) ((col_) < ri[frow].beg ? -32768 : (int)rf1[(col_)-ri[frow].beg])
#define RF2(col_) ((col_) < ri[frow].beg ? -32768 : (int)rf2[(col_)-ri[frow].beg])
        int i = bi, j = qlen;
        enum { ST_H = 0, ST_E1, ST_E2, ST_F1, ST_F2 } st = ST_H;
        while (!fail && i > 0 && j > 0) {
            const int v = rowv[i];
            const ivec *in = &g->in[v];
            if (st == ST_H) {
                const int hcur = H[SCELL(i, j)];
                const int s = sc->mat[g->base[v]][q[j - 1]];
                int hit = 0;
                for (int k = 0; k < in->n && !hit; ++k) {
                    const int pr = WROW(in->a[k]);
                    if (pr < 0) continue;
                    if (j - 1 < ri[pr].beg || j - 1 > ri[pr].end) continue;
                    if (H[SCELL(pr, j - 1)] + s == hcur) {
                        qnode[j - 1] = v;
                        i = pr;
                        --j;
                        hit = 1;
                    }
                }
                if (hit) continue;
                for (int k = 0; k < in->n && !hit; ++k) {
                    const int pr = WROW(in->a[k]);
                    if (pr < 0) continue;
                    if (j < ri[pr].beg || j > ri[pr].end) continue;
                    const int64_t pc = SCELL(pr, j);
                    if (E1[pc] == hcur) {
                        st = (H[pc] - oe1 == E1[pc]) ? ST_H : ST_E1;
                        i = pr;
                        hit = 1;
                    } else if (E2[pc] == hcur) {
                        st = (H[pc] - oe2 == E2[pc]) ? ST_H : ST_E2;
                        i = pr;
                        hit = 1;
                    }
                }
                if (hit) continue;
                RECOMPUTE(i);
                if (RF1(j) == hcur)
                    st = ST_F1;
                else if (RF2(j) == hcur)
                    st = ST_F2;
                else {
                    fail = 1;
                    break;
                }
            }
            if (st == ST_E1 || st == ST_E2) {
                const int64_t cc = SCELL(i, j);
                const int want = (st == ST_E1) ? E1[cc] + e1 : E2[cc] + e2;
                int hit = 0;
                for (int k = 0; k < in->n && !hit; ++k) {
                    const int pr = WROW(in->a[k]);
                    if (pr < 0) continue;
                    if (j < ri[pr].beg || j > ri[pr].end) continue;
                    const int64_t pc = SCELL(pr, j);
                    if (st == ST_E1 && E1[pc] == want) {
                        st = (H[pc] - oe1 == E1[pc]) ? ST_H : ST_E1;
                        i = pr;
                        hit = 1;
                    } else if (st == ST_E2 && E2[pc] == want) {
                        st = (H[pc] - oe2 == E2[pc]) ? ST_H : ST_E2;
                        i = pr;
                        hit = 1;
                    }
                }
                if (!hit) {
                    fail = 1;
                    break;
                }
                continue;
            }
            if (st == ST_F1 || st == ST_F2) {
                RECOMPUTE(i);
                qnode[j - 1] = -1;
                if (st == ST_F1) {
                    if (RH0(j - 1) - oe1 == RF1(j))
                        st = ST_H;
                    else if (RF1(j - 1) - e1 == RF1(j))
                        st = ST_F1;
                    else {
                        fail = 1;
                        break;
                    }
                } else {
                    if (RH0(j - 1) - oe2 == RF2(j))
                        st = ST_H;
                    else if (RF2(j - 1) - e2 == RF2(j))
                        st = ST_F2;
                    else {
                        fail = 1;
                        break;
                    }
                }
                --j;
            }
        }
        for (int t = 0; t < j && !fail; ++t) qnode[t] = -1; /* leading insertions (right after B) */
        free(rh0);
        free(rf1);
        free(rf2);
#undef RECOMPUTE
#undef RH0
#undef RF1
#undef RF2
    }
    free(ri);
    free(ramps);
    free(prof);
    free(wrow);
    free(rowv);
    if (bad) return -2; /* the scalar window alignment takes it */
    return fail ? -1 : cells;
#undef SGROW
#undef ROWLEN
#undef SCELL
#undef WROW
}
