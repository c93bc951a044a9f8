/*
 * oracle/poa_ref.c — TEST INFRASTRUCTURE ONLY.  Imported by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py as the CHECKER; never linked into or called by the product path
 * (mandalorion_amd/ and libmando.so do not reference this file).
 *
 * What it restates
 * ----------------
 * The D module hands each isoform's oriented read group to the abPOA CLI:
 *     /root/reference/utils/SpliceDefineConsensus.py:915-923   `abpoa -M 5 -r 0 [-S] root.fasta`
 * and reads back the last FASTA record (:921-925).  abPOA v1.4.1 (pinned by
 * /root/reference/setup.sh:17-20, path /root/reference/Mando.py:257) is a third-party dependency that
 * is NOT vendored in the reference and NOT present in this container (no source, binary or wheel),
 * and the reference holds no fixture of its output.  This file therefore restates abPOA's published
 * algorithm (Gao et al., Bioinformatics 2021; abPOA README) for the default global / convex-gap /
 * heaviest-bundling mode:
 *   - scoring: match +M, mismatch -X, any pair with N scores 0; gap of length g costs
 *     min(o1 + g*e1, o2 + g*e2)  (five DP states H, E1, E2, F1, F2);
 *   - graph rows in BFS topological order with aligned-node grouping (abPOA's BFS);
 *   - adaptive band: w = b + (int)(f * qlen); row v spans
 *       [max(0, min(posL_v, qlen - remain_v) - w),  min(qlen, max(posR_v, qlen - remain_v) + w)]
 *     posL/posR = min/max over predecessors of (leftmost row-argmax of H) + 1, remain_v = length of the
 *     heaviest-out-edge path from v to the sink (sink = -1);
 *   - backtrack from the best predecessor of the sink at column qlen (first in in-edge order on
 *     ties), checking M (predecessors in in-edge order), then E1/E2 per predecessor, then F1, F2, with
 *     gap-open preferred over gap-extend on ties;
 *   - graph update: match reuses the node, mismatch reuses an aligned node of the same base or adds a
 *     new aligned node, insertions add nodes; edge weight +1 per read;
 *   - consensus: heaviest bundling (max out-edge weight, ties to the larger downstream score, later
 *     edge on equal score).
 * PARITY UNPINNED against real abPOA: the policy details above are reconstructed, not read from the
 * abPOA source; DESIGN.md §POA lists them.  The product HIP kernel must equal THIS restatement
 * byte-for-byte (tests/test_poa_gpu.py); it is written independently (different topological order,
 * aligned-group tables instead of lists, flag-based traceback instead of score re-comparison), so
 * agreement also checks those design claims.
 *
 * -S (minimizer-seeded window partition) is restated below ("-S: ..."), with its reconstructed choices
 * listed there; also PARITY UNPINNED.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/mando.h"

#define SRC 0
#define SINK 1
#define NEG_INF (-(1 << 28))

static uint8_t enc_tab[256];
static int enc_init = 0;

static void init_enc(void) {
    if (enc_init) return;
    for (int i = 0; i < 256; ++i) enc_tab[i] = 4;
    enc_tab['A'] = enc_tab['a'] = 0;
    enc_tab['C'] = enc_tab['c'] = 1;
    enc_tab['G'] = enc_tab['g'] = 2;
    enc_tab['T'] = enc_tab['t'] = 3;
    enc_init = 1;
}

typedef struct {
    int *a;
    int n, m;
} ivec;

static void iv_push(ivec *v, int x) {
    if (v->n == v->m) {
        v->m = v->m ? v->m * 2 : 4;
        v->a = (int *)realloc(v->a, sizeof(int) * (size_t)v->m);
    }
    v->a[v->n++] = x;
}

typedef struct {
    int n, m;
    uint8_t *base;
    ivec *in, *out, *outw, *aln;
} graph_t;

static int g_add_node(graph_t *g, uint8_t b) {
    if (g->n == g->m) {
        int nm = g->m ? g->m * 2 : 64;
        g->base = (uint8_t *)realloc(g->base, (size_t)nm);
        g->in = (ivec *)realloc(g->in, sizeof(ivec) * (size_t)nm);
        g->out = (ivec *)realloc(g->out, sizeof(ivec) * (size_t)nm);
        g->outw = (ivec *)realloc(g->outw, sizeof(ivec) * (size_t)nm);
        g->aln = (ivec *)realloc(g->aln, sizeof(ivec) * (size_t)nm);
        memset(g->in + g->m, 0, sizeof(ivec) * (size_t)(nm - g->m));
        memset(g->out + g->m, 0, sizeof(ivec) * (size_t)(nm - g->m));
        memset(g->outw + g->m, 0, sizeof(ivec) * (size_t)(nm - g->m));
        memset(g->aln + g->m, 0, sizeof(ivec) * (size_t)(nm - g->m));
        g->m = nm;
    }
    g->base[g->n] = b;
    return g->n++;
}

static void g_free(graph_t *g) {
    for (int i = 0; i < g->m; ++i) {
        free(g->in[i].a);
        free(g->out[i].a);
        free(g->outw[i].a);
        free(g->aln[i].a);
    }
    free(g->base);
    free(g->in);
    free(g->out);
    free(g->outw);
    free(g->aln);
}

/* abPOA add-edge semantics: with check, an existing from->to edge gets +1 weight; otherwise a new edge
 * is appended to from's out list and to's in list (insertion order is kept). */
static void g_add_edge(graph_t *g, int from, int to, int check) {
    if (check) {
        for (int i = 0; i < g->out[from].n; ++i)
            if (g->out[from].a[i] == to) {
                g->outw[from].a[i] += 1;
                return;
            }
    }
    iv_push(&g->out[from], to);
    iv_push(&g->outw[from], 1);
    iv_push(&g->in[to], from);
}

/* aligned-node list update as abPOA keeps it: every existing member learns the new node and the new
 * node learns every existing member, then the pair (node, new) is linked. */
static void g_add_aligned(graph_t *g, int node, int nw) {
    for (int i = 0; i < g->aln[node].n; ++i) {
        int x = g->aln[node].a[i];
        iv_push(&g->aln[x], nw);
        iv_push(&g->aln[nw], x);
    }
    iv_push(&g->aln[node], nw);
    iv_push(&g->aln[nw], node);
}

static int g_aligned_with_base(const graph_t *g, int node, uint8_t b) {
    for (int i = 0; i < g->aln[node].n; ++i) {
        int x = g->aln[node].a[i];
        if (g->base[x] == b) return x;
    }
    return -1;
}

/* BFS topological order with aligned-node grouping (a node is queued only once every member of its
 * aligned group has in-degree 0, and then the whole group is queued together). */
static int topo_bfs(const graph_t *g, int *order, int *pos) {
    int n = g->n;
    int *indeg = (int *)malloc(sizeof(int) * (size_t)n);
    int *q = (int *)malloc(sizeof(int) * (size_t)(n + 1));
    for (int i = 0; i < n; ++i) indeg[i] = g->in[i].n;
    int qh = 0, qt = 0, idx = 0;
    q[qt++] = SRC;
    int ok = 0;
    while (qh < qt) {
        int cur = q[qh++];
        order[idx] = cur;
        pos[cur] = idx++;
        if (cur == SINK) {
            ok = (idx == n);
            break;
        }
        for (int i = 0; i < g->out[cur].n; ++i) {
            int o = g->out[cur].a[i];
            if (--indeg[o] == 0) {
                int ready = 1;
                for (int k = 0; k < g->aln[o].n; ++k)
                    if (indeg[g->aln[o].a[k]] != 0) {
                        ready = 0;
                        break;
                    }
                if (!ready) continue;
                q[qt++] = o;
                for (int k = 0; k < g->aln[o].n; ++k) q[qt++] = g->aln[o].a[k];
            }
        }
    }
    free(indeg);
    free(q);
    return ok ? 0 : -1;
}

/* remain[v] = remain[heaviest out-neighbour] + 1 (first maximum in out-edge order), remain[sink] = -1,
 * evaluated in reverse topological order. */
static void set_remain(const graph_t *g, const int *order, int *remain) {
    int n = g->n;
    for (int r = n - 1; r >= 0; --r) {
        int v = order[r];
        if (v == SINK) {
            remain[v] = -1;
            continue;
        }
        int best_w = -2147483647 - 1, best = -1;
        for (int i = 0; i < g->out[v].n; ++i)
            if (g->outw[v].a[i] > best_w) {
                best_w = g->outw[v].a[i];
                best = g->out[v].a[i];
            }
        remain[v] = remain[best] + 1;
    }
}

static inline int imax(int a, int b) { return a > b ? a : b; }
static inline int imin(int a, int b) { return a < b ? a : b; }

typedef struct {
    int beg, end;
    int64_t off; /* into the per-read cell pools */
    int argmax;
} rowinfo;

enum { OP_M = 0, OP_D = 1, OP_I = 2 };

typedef struct {
    const mando_poa_params *p;
    int oe1, oe2;
    int mat[5][5];
} scorer;

static void make_scorer(scorer *s, const mando_poa_params *p) {
    s->p = p;
    s->oe1 = p->gap_open1 + p->gap_ext1;
    s->oe2 = p->gap_open2 + p->gap_ext2;
    for (int a = 0; a < 5; ++a)
        for (int b = 0; b < 5; ++b)
            s->mat[a][b] = (a == 4 || b == 4) ? 0 : (a == b ? p->match : -p->mismatch);
}

static int band_w(const mando_poa_params *p, int qlen) {
    float f = p->band_f * (float)qlen;
    return p->band_b + (int)f;
}

/* Banded DP of q[0..qlen) against the subgraph between node B and node E (both included): the rows
 * are the nodes v with B ~> v ~> E in topological order, B is the source row (row 0) and E the sink
 * (not a DP row).  remain relative to E: rem(v) = remain[v] - remain[E] - 1 (= remain[v] for E = SINK).
 * Predecessors outside the subgraph are ignored.  Fills qnode[0..qlen) with the aligned node of every
 * query position (-1 = inserted).  B = SRC, E = SINK is the whole-graph alignment of the default mode.
 * Returns the number of DP cells evaluated, or -1 on an internal inconsistency. */
#ifdef POA_SIMD
/* oracle/poa_simd.c (the cpu_baseline's vectorised build of this file): the same window alignment with
 * the DP rows in AVX2 int16 lanes; returns -2 when the window must take the scalar code below */
static int64_t align_window_simd(const graph_t *g, const int *order, const int *pos, const int *remain, int B,
                                 int E, const uint8_t *q, int qlen, const scorer *sc, int *qnode);
#endif
static int64_t align_window(const graph_t *g, const int *order, const int *pos, const int *remain, int B, int E,
                            const uint8_t *q, int qlen, const scorer *sc, int *qnode) {
#ifdef POA_SIMD
    {
        const int64_t c = align_window_simd(g, order, pos, remain, B, E, q, qlen, sc, qnode);
        if (c != -2) return c;
    }
#endif
    const int pB = pos[B], pE = pos[E];
    if (pE <= pB) return -1;
    const int span = pE - pB + 1;
    /* rows: forward reachability from B, backward from E, inside the topological range [pB, pE] */
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
    int *wrow = (int *)malloc(sizeof(int) * (size_t)span); /* window row of topological row pB + x, -1 if not in */
    int *rowv = (int *)malloc(sizeof(int) * (size_t)span); /* node of window row */
    for (int x = 0; x < span; ++x) {
        wrow[x] = (fl[x] == 3) ? m : -1;
        if (fl[x] == 3) rowv[m++] = order[pB + x];
    }
    free(fl);
#define WROW(node_) ((pos[node_] >= pB && pos[node_] <= pE) ? wrow[pos[node_] - pB] : -1)
    const int remE = remain[E];
    int w = band_w(sc->p, qlen);
    const int e1 = sc->p->gap_ext1, e2 = sc->p->gap_ext2, o1 = sc->p->gap_open1,
              o2 = sc->p->gap_open2;
    const int oe1 = sc->oe1, oe2 = sc->oe2;

    rowinfo *ri = (rowinfo *)malloc(sizeof(rowinfo) * (size_t)m);
    int64_t cap = (int64_t)(m) * (2 * w + 64) + 1024, used = 0;
    int *H = (int *)malloc(sizeof(int) * (size_t)cap), *H0 = (int *)malloc(sizeof(int) * (size_t)cap);
    int *E1 = (int *)malloc(sizeof(int) * (size_t)cap), *E2 = (int *)malloc(sizeof(int) * (size_t)cap);
    int *F1 = (int *)malloc(sizeof(int) * (size_t)cap), *F2 = (int *)malloc(sizeof(int) * (size_t)cap);
#define GROW(need)                                                                  \
    do {                                                                            \
        if (used + (need) > cap) {                                                  \
            while (used + (need) > cap) cap *= 2;                                   \
            H = (int *)realloc(H, sizeof(int) * (size_t)cap);                       \
            H0 = (int *)realloc(H0, sizeof(int) * (size_t)cap);                     \
            E1 = (int *)realloc(E1, sizeof(int) * (size_t)cap);                     \
            E2 = (int *)realloc(E2, sizeof(int) * (size_t)cap);                     \
            F1 = (int *)realloc(F1, sizeof(int) * (size_t)cap);                     \
            F2 = (int *)realloc(F2, sizeof(int) * (size_t)cap);                     \
        }                                                                           \
    } while (0)

    int64_t cells = 0;
    /* source row (B) */
    {
        const int remB = remain[B] - remE - 1;
        int end = imin(qlen, imax(0, qlen - remB) + w);
        ri[0].beg = 0;
        ri[0].end = end;
        ri[0].off = 0;
        GROW(end + 1);
        for (int j = 0; j <= end; ++j) {
            int h;
            if (j == 0) {
                h = 0;
                H0[j] = 0;
                F1[j] = NEG_INF;
                F2[j] = NEG_INF;
            } else {
                F1[j] = -(o1 + e1 * j);
                F2[j] = -(o2 + e2 * j);
                H0[j] = NEG_INF;
                h = imax(F1[j], F2[j]);
            }
            H[j] = h;
            E1[j] = h - oe1;
            E2[j] = h - oe2;
        }
        ri[0].argmax = 0;
        used = end + 1;
        cells += end + 1;
    }

    for (int i = 1; i < m - 1; ++i) {
        int v = rowv[i];
        const ivec *in = &g->in[v];
        int posL = 2147483647, posR = -2147483647 - 1;
        for (int k = 0; k < in->n; ++k) {
            int pr = WROW(in->a[k]);
            if (pr < 0) continue;
            posL = imin(posL, ri[pr].argmax + 1);
            posR = imax(posR, ri[pr].argmax + 1);
        }
        int x = qlen - (remain[v] - remE - 1);
        int beg = imax(0, imin(posL, x) - w);
        int end = imin(qlen, imax(posR, x) + w);
        int width = end - beg + 1;
        GROW(width);
        ri[i].beg = beg;
        ri[i].end = end;
        ri[i].off = used;
        int64_t o = used;
        used += width;
        cells += width;
        uint8_t vb = g->base[v];
        int best = -2147483647 - 1, besti = beg; /* leftmost maximum of H over the row */
        for (int j = beg; j <= end; ++j) {
            int64_t c = o + (j - beg);
            int mv = NEG_INF, e1in = NEG_INF, e2in = NEG_INF;
            for (int k = 0; k < in->n; ++k) {
                int pr = WROW(in->a[k]);
                if (pr < 0) continue;
                const rowinfo *pi = &ri[pr];
                if (j - 1 >= pi->beg && j - 1 <= pi->end) mv = imax(mv, H[pi->off + (j - 1 - pi->beg)]);
                if (j >= pi->beg && j <= pi->end) {
                    e1in = imax(e1in, E1[pi->off + (j - pi->beg)]);
                    e2in = imax(e2in, E2[pi->off + (j - pi->beg)]);
                }
            }
            int s = (j >= 1) ? sc->mat[vb][q[j - 1]] : 0;
            int mm = mv + s;
            int h0 = imax(mm, imax(e1in, e2in));
            int f1, f2;
            if (j == beg) {
                f1 = NEG_INF;
                f2 = NEG_INF;
            } else {
                f1 = imax(H0[c - 1] - oe1, F1[c - 1] - e1);
                f2 = imax(H0[c - 1] - oe2, F2[c - 1] - e2);
            }
            int h = imax(h0, imax(f1, f2));
            H0[c] = h0;
            F1[c] = f1;
            F2[c] = f2;
            H[c] = h;
            E1[c] = imax(e1in - e1, h - oe1);
            E2[c] = imax(e2in - e2, h - oe2);
            if (h > best) {
                best = h;
                besti = j;
            }
        }
        ri[i].argmax = besti;
    }

    /* end: best predecessor of E at column qlen (first in in-edge order on ties) */
    int bi = -1, bs = -2147483647 - 1;
    for (int k = 0; k < g->in[E].n; ++k) {
        int pr = WROW(g->in[E].a[k]);
        if (pr < 0) continue;
        if (qlen < ri[pr].beg || qlen > ri[pr].end) continue;
        int h = H[ri[pr].off + (qlen - ri[pr].beg)];
        if (h > bs) {
            bs = h;
            bi = pr;
        }
    }
    int fail = 0;
    if (bi < 0) fail = 1;

    /* backtrack by score comparison (abPOA style) */
#define CELL(r_, col_) (ri[r_].off + ((col_)-ri[r_].beg))
    int i = bi, j = qlen;
    enum { ST_H = 0, ST_E1, ST_E2, ST_F1, ST_F2 } st = ST_H;
    while (!fail && i > 0 && j > 0) {
        int v = rowv[i];
        const ivec *in = &g->in[v];
        if (st == ST_H) {
            int hcur = H[CELL(i, j)];
            int s = sc->mat[g->base[v]][q[j - 1]];
            int hit = 0;
            for (int k = 0; k < in->n && !hit; ++k) {
                int pr = WROW(in->a[k]);
                if (pr < 0) continue;
                if (j - 1 < ri[pr].beg || j - 1 > ri[pr].end) continue;
                if (H[CELL(pr, j - 1)] + s == hcur) {
                    qnode[j - 1] = v;
                    i = pr;
                    --j;
                    hit = 1;
                }
            }
            if (hit) continue;
            for (int k = 0; k < in->n && !hit; ++k) {
                int pr = WROW(in->a[k]);
                if (pr < 0) continue;
                if (j < ri[pr].beg || j > ri[pr].end) continue;
                int64_t pc = CELL(pr, j);
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
            if (F1[CELL(i, j)] == hcur)
                st = ST_F1;
            else if (F2[CELL(i, j)] == hcur)
                st = ST_F2;
            else {
                fail = 1;
                break;
            }
        }
        if (st == ST_E1 || st == ST_E2) {
            int64_t cc = CELL(i, j);
            int want = (st == ST_E1) ? E1[cc] + e1 : E2[cc] + e2;
            int hit = 0;
            for (int k = 0; k < in->n && !hit; ++k) {
                int pr = WROW(in->a[k]);
                if (pr < 0) continue;
                if (j < ri[pr].beg || j > ri[pr].end) continue;
                int64_t pc = CELL(pr, j);
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
            int64_t cc = CELL(i, j);
            qnode[j - 1] = -1;
            if (st == ST_F1) {
                if (H0[cc - 1] - oe1 == F1[cc])
                    st = ST_H;
                else if (F1[cc - 1] - e1 == F1[cc])
                    st = ST_F1;
                else {
                    fail = 1;
                    break;
                }
            } else {
                if (H0[cc - 1] - oe2 == F2[cc])
                    st = ST_H;
                else if (F2[cc - 1] - e2 == F2[cc])
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
    free(H); free(H0); free(E1); free(E2); free(F1); free(F2);
    free(ri);
    free(wrow);
    free(rowv);
    return fail ? -1 : cells;
#undef GROW
#undef CELL
#undef WROW
}

/* Graph update from the per-position path (abPOA add_graph_alignment): query position t joins node
 * qnode[t] (match: that node; mismatch: the aligned node of the same base, else a new aligned node) or
 * becomes a new node (qnode[t] = -1); consecutive positions are linked from SRC to SINK, edge weight +1.
 * tnode (optional) receives the node each position ended up on. */
static void apply_path(graph_t *g, const uint8_t *q, int qlen, const int *qnode, int *tnode) {
    int last = SRC, last_new = 0;
    for (int t = 0; t < qlen; ++t) {
        const int node = qnode[t];
        const uint8_t b = q[t];
        if (node < 0) {
            int nw = g_add_node(g, b);
            g_add_edge(g, last, nw, 0);
            last = nw;
            last_new = 1;
        } else if (g->base[node] == b) {
            g_add_edge(g, last, node, !last_new);
            last = node;
            last_new = 0;
        } else {
            int a = g_aligned_with_base(g, node, b);
            if (a >= 0) {
                g_add_edge(g, last, a, !last_new);
                last = a;
                last_new = 0;
            } else {
                int nw = g_add_node(g, b);
                g_add_edge(g, last, nw, 0);
                g_add_aligned(g, node, nw);
                last = nw;
                last_new = 1;
            }
        }
        if (tnode) tnode[t] = last;
    }
    g_add_edge(g, last, SINK, !last_new);
}

/* ---------------------------------------------------------------------------------------------
 * -S: minimizer-seeded window partition (abPOA v1.4.1 `-S`, SpliceDefineConsensus.py:915-919 when the
 * median subsample length is >= 8000).  Restated from abPOA's published description (seeding with
 * (k, w) minimizers, anchors chained by a longest increasing subsequence, the read split at anchors at
 * least min_w apart, each window aligned to the subgraph between its bounding anchor nodes, the whole
 * read's path added to the graph at once).  PARITY UNPINNED; the choices below are this restatement's
 * and the HIP kernel follows them exactly:
 *   - anchors pair read r with the previous non-empty read r' of the group: minimizers (minimap2's
 *     canonical k-mer hash, ambiguous and strand-symmetric k-mers skipped, every window minimum kept)
 *     with equal hash and strand; hashes occurring more than SEED_MAX_OCC times in r' are skipped;
 *   - anchors in (start in r ascending, start in r' descending) order -- the order in which r's
 *     minimizers meet r''s sorted index; the chain is the longest strictly increasing subsequence of
 *     the r' starts (hence strictly increasing in both reads; patience sorting, leftmost pile, traced
 *     back from the last pile);
 *   - partition: walking the chain, an anchor (t, q) (k-mer starts) is kept when t - T >= min_w,
 *     q - Q >= min_w, len(r') - (t + k) >= min_w and len(r) - (q + k) >= min_w, with (T, Q) the end of
 *     the last kept anchor's k-mer (initially 0, 0);
 *   - the kept k-mers are pinned: q + i joins node(r', t + i) (the node position t + i of r' was
 *     assigned to), i < k; the stretch between two kept k-mers (or the read ends) is aligned to the
 *     subgraph between node(r', last base of the left k-mer) (SRC at the start) and node(r', first base
 *     of the right k-mer) (SINK at the end), with that stretch's length as qlen of the adaptive band.
 * --------------------------------------------------------------------------------------------- */
#define SEED_MAX_OCC 8

typedef struct {
    uint64_t h;
    int32_t pos; /* k-mer start */
    int32_t z;
} seed_mm;

/* minimizers of encoded s[0..L) (codes 0..4), in position order */
static int seed_minimizers(const uint8_t *s, int L, int k, int w, seed_mm **out) {
    *out = NULL;
    if (L < k || k <= 0 || k > 28 || w <= 0) return 0;
    const uint64_t mask = (1ull << (2 * k)) - 1;
    const int np = L - k + 1;
    uint64_t *H = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)np);
    uint8_t *z = (uint8_t *)malloc((size_t)np);
    uint8_t *mark = (uint8_t *)calloc((size_t)np, 1);
    for (int p = 0; p < np; ++p) {
        uint64_t f = 0, r = 0;
        int bad = 0;
        for (int t = 0; t < k; ++t) {
            const int c = s[p + t];
            if (c > 3) { bad = 1; break; }
            f = (f << 2) | (uint64_t)c;
            r |= (uint64_t)(3 - c) << (2 * t);
        }
        if (bad || f == r) {
            H[p] = UINT64_MAX;
            z[p] = 0;
        } else {
            uint64_t key = f < r ? f : r;
            key = (~key + (key << 21)) & mask;
            key = key ^ key >> 24;
            key = ((key + (key << 3)) + (key << 8)) & mask;
            key = key ^ key >> 14;
            key = ((key + (key << 2)) + (key << 4)) & mask;
            key = key ^ key >> 28;
            key = (key + (key << 31)) & mask;
            H[p] = key;
            z[p] = f < r ? 0 : 1;
        }
    }
    const int nw = np <= w ? 1 : np - w + 1;
    const int ww = np <= w ? np : w;
    for (int w0 = 0; w0 < nw; ++w0) {
        uint64_t mn = UINT64_MAX;
        for (int t = 0; t < ww; ++t) if (H[w0 + t] < mn) mn = H[w0 + t];
        if (mn == UINT64_MAX) continue;
        for (int t = 0; t < ww; ++t) if (H[w0 + t] == mn) mark[w0 + t] = 1;
    }
    int n = 0;
    for (int p = 0; p < np; ++p) n += mark[p];
    seed_mm *o = (seed_mm *)malloc(sizeof(seed_mm) * (size_t)(n ? n : 1));
    n = 0;
    for (int p = 0; p < np; ++p)
        if (mark[p]) {
            o[n].h = H[p];
            o[n].pos = p;
            o[n].z = z[p];
            ++n;
        }
    free(H); free(z); free(mark);
    *out = o;
    return n;
}

static int cmp_mm_key(const void *a, const void *b) {
    const seed_mm *x = (const seed_mm *)a, *y = (const seed_mm *)b;
    if (x->h != y->h) return x->h < y->h ? -1 : 1;
    if (x->z != y->z) return x->z - y->z;
    return x->pos - y->pos;
}

typedef struct { int32_t t, q; } seed_anchor;

/* the kept partition anchors (k-mer starts in t and q) of read q against the previous read t */
int poa_ref_seed_partition(const uint8_t *t, int tlen, const uint8_t *q, int qlen, int k, int w, int min_w,
                           int32_t *par_t, int32_t *par_q, int cap) {
    seed_mm *mt = NULL, *mq = NULL;
    const int nt = seed_minimizers(t, tlen, k, w, &mt);
    const int nq = seed_minimizers(q, qlen, k, w, &mq);
    int np = 0;
    if (nt > 0 && nq > 0) {
        qsort(mt, (size_t)nt, sizeof(seed_mm), cmp_mm_key);
        seed_anchor *an = (seed_anchor *)malloc(sizeof(seed_anchor) * (size_t)nq * SEED_MAX_OCC + 1);
        int na = 0;
        for (int i = 0; i < nq; ++i) {
            int lo = 0, hi = nt; /* first entry >= (h, z) */
            while (lo < hi) {
                const int mid = (lo + hi) / 2;
                if (mt[mid].h < mq[i].h || (mt[mid].h == mq[i].h && mt[mid].z < mq[i].z)) lo = mid + 1;
                else hi = mid;
            }
            int e = lo;
            while (e < nt && mt[e].h == mq[i].h && mt[e].z == mq[i].z) ++e;
            if (e - lo == 0 || e - lo > SEED_MAX_OCC) continue;
            for (int x = e - 1; x >= lo; --x) { /* anchors in (q ascending, t descending) order */
                an[na].t = mt[x].pos;
                an[na].q = mq[i].pos;
                ++na;
            }
        }
        /* longest strictly increasing subsequence of t (q is strictly increasing along it by the order) */
        int *tail = (int *)malloc(sizeof(int) * (size_t)(na + 1));
        int *prev = (int *)malloc(sizeof(int) * (size_t)(na + 1));
        int L = 0;
        for (int i = 0; i < na; ++i) {
            int lo = 0, hi = L; /* leftmost pile whose tail t >= an[i].t */
            while (lo < hi) {
                const int mid = (lo + hi) / 2;
                if (an[tail[mid]].t < an[i].t) lo = mid + 1;
                else hi = mid;
            }
            prev[i] = lo > 0 ? tail[lo - 1] : -1;
            tail[lo] = i;
            if (lo == L) ++L;
        }
        int *chain = (int *)malloc(sizeof(int) * (size_t)(L + 1));
        for (int x = L - 1, c = L ? tail[L - 1] : -1; x >= 0; --x, c = prev[c]) chain[x] = c;
        int T = 0, Q = 0;
        for (int x = 0; x < L; ++x) {
            const seed_anchor *a = &an[chain[x]];
            if (a->t - T >= min_w && a->q - Q >= min_w && tlen - (a->t + k) >= min_w && qlen - (a->q + k) >= min_w) {
                if (np < cap) {
                    par_t[np] = a->t;
                    par_q[np] = a->q;
                }
                ++np;
                T = a->t + k;
                Q = a->q + k;
            }
        }
        free(chain); free(tail); free(prev); free(an);
    }
    free(mt);
    free(mq);
    return np;
}

static void add_chain(graph_t *g, const uint8_t *q, int qlen) {
    int last = SRC;
    for (int t = 0; t < qlen; ++t) {
        int nw = g_add_node(g, q[t]);
        g_add_edge(g, last, nw, 0);
        last = nw;
    }
    g_add_edge(g, last, SINK, 0);
}

/* heaviest bundling from the sink (reverse BFS by out-degree) */
static int hb_consensus(const graph_t *g, uint8_t *out, int cap) {
    int n = g->n;
    int *outdeg = (int *)malloc(sizeof(int) * (size_t)n);
    int *score = (int *)malloc(sizeof(int) * (size_t)n);
    int *nxt = (int *)malloc(sizeof(int) * (size_t)n);
    int *q = (int *)malloc(sizeof(int) * (size_t)(n + 1));
    for (int i = 0; i < n; ++i) outdeg[i] = g->out[i].n;
    int qh = 0, qt = 0;
    q[qt++] = SINK;
    int done = 0;
    while (qh < qt) {
        int cur = q[qh++];
        if (cur == SINK) {
            score[cur] = 0;
            nxt[cur] = -1;
        } else {
            int maxw = -1, maxid = -1;
            for (int k = 0; k < g->out[cur].n; ++k) {
                int o = g->out[cur].a[k], ow = g->outw[cur].a[k];
                if (maxw < ow) {
                    maxw = ow;
                    maxid = o;
                } else if (maxw == ow && score[maxid] <= score[o]) {
                    maxid = o;
                }
            }
            score[cur] = maxw + score[maxid];
            nxt[cur] = maxid;
        }
        if (cur == SRC) {
            done = 1;
            break;
        }
        for (int k = 0; k < g->in[cur].n; ++k) {
            int p = g->in[cur].a[k];
            if (--outdeg[p] == 0) q[qt++] = p;
        }
    }
    int len = 0;
    if (done) {
        int cur = nxt[SRC];
        while (cur != SINK && cur >= 0) {
            if (len < cap) out[len] = g->base[cur];
            ++len;
            cur = nxt[cur];
        }
    } else {
        len = -1;
    }
    free(outdeg);
    free(score);
    free(nxt);
    free(q);
    return len;
}

static int64_t align_read(graph_t *g, const uint8_t *q, int qlen, const scorer *sc, int seeding, const uint8_t *t,
                          int tlen, const int *tnode, int *qnode) {
    int n = g->n;
    int *order = (int *)malloc(sizeof(int) * (size_t)n);
    int *pos = (int *)malloc(sizeof(int) * (size_t)n);
    int *remain = (int *)malloc(sizeof(int) * (size_t)n);
    int64_t cells = 0;
    if (topo_bfs(g, order, pos) != 0) {
        cells = -1;
    } else {
        set_remain(g, order, remain);
        const mando_poa_params *p = sc->p;
        int np = 0, cap = qlen / (p->min_w > 0 ? p->min_w : 1) + 2;
        int32_t *pt = (int32_t *)malloc(sizeof(int32_t) * (size_t)cap), *pq = (int32_t *)malloc(sizeof(int32_t) * (size_t)cap);
        if (seeding && t) np = poa_ref_seed_partition(t, tlen, q, qlen, p->k, p->w, p->min_w, pt, pq, cap);
        if (np > cap) np = -1;
        if (np < 0) cells = -1;
        int B = SRC, q0 = 0;
        for (int x = 0; x <= np && cells >= 0; ++x) {
            const int E = x < np ? tnode[pt[x]] : SINK;
            const int q1 = x < np ? pq[x] : qlen;
            if (q1 > q0) {
                const int64_t c = align_window(g, order, pos, remain, B, E, q + q0, q1 - q0, sc, qnode + q0);
                cells = c < 0 ? -1 : cells + c;
            }
            if (x < np) {
                for (int i = 0; i < p->k; ++i) qnode[pq[x] + i] = tnode[pt[x] + i];
                B = tnode[pt[x] + p->k - 1];
                q0 = pq[x] + p->k;
            }
        }
        free(pt);
        free(pq);
    }
    free(order);
    free(pos);
    free(remain);
    return cells;
}

/* One group: encoded reads (0..4).  Writes the encoded consensus; returns its length, -1 on an
 * internal error.  seeding != 0 runs the -S path (see above).  *cells_out gets the DP cell count. */
int poa_ref_group_encoded(const uint8_t *const *reads, const int *lens, int n_reads,
                          const mando_poa_params *p, int seeding, uint8_t *cons, int cap,
                          int64_t *cells_out) {
    scorer sc;
    make_scorer(&sc, p);
    graph_t g;
    memset(&g, 0, sizeof(g));
    g_add_node(&g, 4); /* SRC */
    g_add_node(&g, 4); /* SINK */
    int64_t cells = 0;
    int have_graph = 0;
    int maxlen = 1;
    for (int r = 0; r < n_reads; ++r) maxlen = imax(maxlen, lens[r]);
    int *tnode = (int *)malloc(sizeof(int) * (size_t)maxlen), *qnode = (int *)malloc(sizeof(int) * (size_t)maxlen);
    const uint8_t *t = NULL;
    int tlen = 0;
    for (int r = 0; r < n_reads; ++r) {
        if (lens[r] <= 0) continue;
        if (!have_graph) {
            add_chain(&g, reads[r], lens[r]);
            for (int i = 0; i < lens[r]; ++i) tnode[i] = 2 + i;
            have_graph = 1;
        } else {
            int64_t c = align_read(&g, reads[r], lens[r], &sc, seeding, t, tlen, tnode, qnode);
            if (c < 0) {
                g_free(&g);
                free(tnode); free(qnode);
                return -1;
            }
            cells += c;
            apply_path(&g, reads[r], lens[r], qnode, tnode);
        }
        t = reads[r];
        tlen = lens[r];
    }
    int len = have_graph ? hb_consensus(&g, cons, cap) : 0;
    g_free(&g);
    free(tnode);
    free(qnode);
    if (cells_out) *cells_out = cells;
    return len;
}

/* Batch entry mirroring mando_poa_batch (ASCII in, ASCII out). */
int poa_ref_batch(const mando_poa_params *params, const uint8_t *seqs, const int64_t *seq_off,
                  const int64_t *grp_off, int64_t n_groups, const uint8_t *seeding_per_group,
                  uint8_t *cons_out, int64_t cons_cap, int64_t *cons_off, int64_t *cells_out) {
    init_enc();
    int64_t used = 0;
    cons_off[0] = 0;
    for (int64_t gi = 0; gi < n_groups; ++gi) {
        int64_t r0 = grp_off[gi], r1 = grp_off[gi + 1];
        int nr = (int)(r1 - r0);
        const uint8_t **rd = (const uint8_t **)malloc(sizeof(uint8_t *) * (size_t)(nr + 1));
        int *ln = (int *)malloc(sizeof(int) * (size_t)(nr + 1));
        uint8_t **own = (uint8_t **)malloc(sizeof(uint8_t *) * (size_t)(nr + 1));
        int64_t maxcons = 16;
        for (int r = 0; r < nr; ++r) {
            int64_t a = seq_off[r0 + r], b = seq_off[r0 + r + 1];
            int L = (int)(b - a);
            own[r] = (uint8_t *)malloc((size_t)(L + 1));
            for (int t = 0; t < L; ++t) own[r][t] = enc_tab[seqs[a + t]];
            rd[r] = own[r];
            ln[r] = L;
            maxcons += L;
        }
        uint8_t *tmp = (uint8_t *)malloc((size_t)maxcons);
        int64_t cells = 0;
        int len = poa_ref_group_encoded(rd, ln, nr, params,
                                        seeding_per_group ? seeding_per_group[gi] : 0, tmp,
                                        (int)maxcons, &cells);
        for (int r = 0; r < nr; ++r) free(own[r]);
        free(own);
        free(rd);
        free(ln);
        if (len < 0) {
            free(tmp);
            return len == -5 ? MANDO_E_UNSUPPORTED : MANDO_E_INTERNAL;
        }
        if (used + len <= cons_cap) {
            static const char dec[5] = {'A', 'C', 'G', 'T', 'N'};
            for (int t = 0; t < len; ++t) cons_out[used + t] = (uint8_t)dec[tmp[t]];
        }
        free(tmp);
        used += len;
        cons_off[gi + 1] = used;
        if (cells_out) cells_out[gi] = cells;
    }
    return used <= cons_cap ? MANDO_OK : MANDO_E_CAP;
}
