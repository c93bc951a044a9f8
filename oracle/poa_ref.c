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
 * The -S (minimizer seeding) window partition is not restated: seeded groups run the same full
 * adaptive-band DP, exactly like the HIP kernel (DESIGN.md "Known gaps").
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

/* Align one encoded read to the graph and add it (abPOA align + add_graph_alignment).
 * Returns the number of DP cells evaluated, or -1 on an internal inconsistency. */
static int64_t align_and_add(graph_t *g, const uint8_t *q, int qlen, const scorer *sc) {
    int n = g->n;
    int *order = (int *)malloc(sizeof(int) * (size_t)n);
    int *pos = (int *)malloc(sizeof(int) * (size_t)n);
    int *remain = (int *)malloc(sizeof(int) * (size_t)n);
    if (topo_bfs(g, order, pos) != 0) {
        free(order);
        free(pos);
        free(remain);
        return -1;
    }
    set_remain(g, order, remain);
    int w = band_w(sc->p, qlen);
    const int e1 = sc->p->gap_ext1, e2 = sc->p->gap_ext2, o1 = sc->p->gap_open1,
              o2 = sc->p->gap_open2;
    const int oe1 = sc->oe1, oe2 = sc->oe2;

    rowinfo *ri = (rowinfo *)malloc(sizeof(rowinfo) * (size_t)n);
    int64_t cap = (int64_t)(n) * (2 * w + 64) + 1024, used = 0;
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
    /* source row */
    {
        int end = imin(qlen, imax(0, qlen - remain[SRC]) + w);
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

    for (int i = 1; i < n - 1; ++i) {
        int v = order[i];
        const ivec *in = &g->in[v];
        int posL = 2147483647, posR = -2147483647 - 1;
        for (int k = 0; k < in->n; ++k) {
            int pr = pos[in->a[k]];
            posL = imin(posL, ri[pr].argmax + 1);
            posR = imax(posR, ri[pr].argmax + 1);
        }
        int x = qlen - remain[v];
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
                int pr = pos[in->a[k]];
                const rowinfo *pi = &ri[pr];
                if (j - 1 >= pi->beg && j - 1 <= pi->end) mv = imax(mv, H[pi->off + (j - 1 - pi->beg)]);
                if (j >= pi->beg && j <= pi->end) {
                    e1in = imax(e1in, E1[pi->off + (j - pi->beg)]);
                    e2in = imax(e2in, E2[pi->off + (j - pi->beg)]);
                }
            }
            int s = (j >= 1) ? sc->mat[vb][q[j - 1]] : 0;
            int m = mv + s;
            int h0 = imax(m, imax(e1in, e2in));
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

    /* global end: best predecessor of the sink at column qlen */
    int bi = -1, bs = -2147483647 - 1;
    for (int k = 0; k < g->in[SINK].n; ++k) {
        int pr = pos[g->in[SINK].a[k]];
        if (qlen < ri[pr].beg || qlen > ri[pr].end) continue;
        int h = H[ri[pr].off + (qlen - ri[pr].beg)];
        if (h > bs) {
            bs = h;
            bi = pr;
        }
    }
    if (bi < 0) {
        free(order); free(pos); free(remain); free(ri);
        free(H); free(H0); free(E1); free(E2); free(F1); free(F2);
        return -1;
    }

    /* backtrack by score comparison (abPOA style); ops recorded in reverse */
    int opcap = qlen + n + 16, nops = 0;
    int *opk = (int *)malloc(sizeof(int) * (size_t)opcap);
    int *opn = (int *)malloc(sizeof(int) * (size_t)opcap);
    int *opq = (int *)malloc(sizeof(int) * (size_t)opcap);
#define PUSHOP(k_, n_, q_)   \
    do {                     \
        opk[nops] = (k_);    \
        opn[nops] = (n_);    \
        opq[nops] = (q_);    \
        ++nops;              \
    } while (0)
#define CELL(r_, col_) (ri[r_].off + ((col_)-ri[r_].beg))
    int i = bi, j = qlen;
    enum { ST_H = 0, ST_E1, ST_E2, ST_F1, ST_F2 } st = ST_H;
    int fail = 0;
    while (i > 0 && j > 0) {
        int v = order[i];
        const ivec *in = &g->in[v];
        if (st == ST_H) {
            int hcur = H[CELL(i, j)];
            int s = sc->mat[g->base[v]][q[j - 1]];
            int hit = 0;
            for (int k = 0; k < in->n && !hit; ++k) {
                int pr = pos[in->a[k]];
                if (j - 1 < ri[pr].beg || j - 1 > ri[pr].end) continue;
                if (H[CELL(pr, j - 1)] + s == hcur) {
                    PUSHOP(OP_M, v, j - 1);
                    i = pr;
                    --j;
                    hit = 1;
                }
            }
            if (hit) continue;
            for (int k = 0; k < in->n && !hit; ++k) {
                int pr = pos[in->a[k]];
                if (j < ri[pr].beg || j > ri[pr].end) continue;
                int64_t pc = CELL(pr, j);
                if (E1[pc] == hcur) {
                    PUSHOP(OP_D, v, -1);
                    st = (H[pc] - oe1 == E1[pc]) ? ST_H : ST_E1;
                    i = pr;
                    hit = 1;
                } else if (E2[pc] == hcur) {
                    PUSHOP(OP_D, v, -1);
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
            PUSHOP(OP_D, v, -1);
            for (int k = 0; k < in->n && !hit; ++k) {
                int pr = pos[in->a[k]];
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
            PUSHOP(OP_I, -1, j - 1);
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
    int lead_ins = j;
    free(H); free(H0); free(E1); free(E2); free(F1); free(F2);
    free(ri);
    free(order); free(pos); free(remain);
    if (fail) {
        free(opk); free(opn); free(opq);
        return -1;
    }

    /* graph update, forward order: leading insertions then the reversed op list */
    int last = SRC, last_new = 0;
    for (int t = 0; t < lead_ins; ++t) {
        int nw = g_add_node(g, q[t]);
        g_add_edge(g, last, nw, 0);
        last = nw;
        last_new = 1;
    }
    for (int t = nops - 1; t >= 0; --t) {
        if (opk[t] == OP_D) continue;
        if (opk[t] == OP_I) {
            int nw = g_add_node(g, q[opq[t]]);
            g_add_edge(g, last, nw, 0);
            last = nw;
            last_new = 1;
            continue;
        }
        int node = opn[t];
        uint8_t b = q[opq[t]];
        if (g->base[node] == b) {
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
    }
    g_add_edge(g, last, SINK, !last_new);
    free(opk); free(opn); free(opq);
    return cells;
#undef GROW
#undef PUSHOP
#undef CELL
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

/* One group: encoded reads (0..4).  Writes the encoded consensus; returns its length, -1 on an
 * internal error.  `seeding` (-S) is accepted and ignored (see header).  *cells_out gets the DP cell count. */
int poa_ref_group_encoded(const uint8_t *const *reads, const int *lens, int n_reads,
                          const mando_poa_params *p, int seeding, uint8_t *cons, int cap,
                          int64_t *cells_out) {
    (void)seeding;
    scorer sc;
    make_scorer(&sc, p);
    graph_t g;
    memset(&g, 0, sizeof(g));
    g_add_node(&g, 4); /* SRC */
    g_add_node(&g, 4); /* SINK */
    int64_t cells = 0;
    int have_graph = 0;
    for (int r = 0; r < n_reads; ++r) {
        if (lens[r] <= 0) continue;
        if (!have_graph) {
            add_chain(&g, reads[r], lens[r]);
            have_graph = 1;
            continue;
        }
        int64_t c = align_and_add(&g, reads[r], lens[r], &sc);
        if (c < 0) {
            g_free(&g);
            return -1;
        }
        cells += c;
    }
    int len = have_graph ? hb_consensus(&g, cons, cap) : 0;
    g_free(&g);
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
