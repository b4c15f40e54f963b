/*
 * refcpu.c — CPU restatement of bn-pp's VE hot path (see refcpu.h).
 * TEST INFRASTRUCTURE ONLY: the parity oracle and the "port" CPU baseline.
 * Single-threaded fp64, per-entry position computation, sequential sums —
 * the same arithmetic, in the same order, as the reference.
 */
#define _POSIX_C_SOURCE 199309L
#include "refcpu.h"

#include <ctype.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static void *xmalloc(size_t n) {
    void *p = malloc(n ? n : 1);
    if (!p) { fprintf(stderr, "refcpu: out of memory (%zu bytes)\n", n); abort(); }
    return p;
}
static void *xcalloc(size_t n, size_t s) {
    void *p = calloc(n ? n : 1, s ? s : 1);
    if (!p) { fprintf(stderr, "refcpu: out of memory\n"); abort(); }
    return p;
}

static double now_ms(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
}

/* ---------------------------------------------------------------- domain */
/* offsets: row-major, last scope variable fastest (domain.cpp:15-26) */
static void compute_offsets(int width, const int *cards, uint64_t *off, uint64_t *size) {
    uint64_t s = 1;
    for (int i = width - 1; i >= 0; --i) { off[i] = s; s *= (uint64_t)cards[i]; }
    *size = s;
}

static int scope_index(int width, const int *vars, int v) {
    for (int i = 0; i < width; ++i) if (vars[i] == v) return i;
    return -1;
}

/* Domain::next_valuation (domain.cpp:113-123) */
static void next_valuation(int width, const int *cards, unsigned *val) {
    int j;
    for (j = width - 1; j >= 0 && val[j] == (unsigned)cards[j] - 1; --j) val[j] = 0;
    if (j >= 0) val[j]++;
}

static rc_factor *factor_alloc(int width, const int *vars, const int *cards) {
    rc_factor *f = (rc_factor *)xcalloc(1, sizeof(rc_factor));
    f->width = width;
    f->vars = (int *)xmalloc(sizeof(int) * (size_t)width);
    f->cards = (int *)xmalloc(sizeof(int) * (size_t)width);
    uint64_t size = 1;
    for (int i = 0; i < width; ++i) {
        f->vars[i] = vars[i];
        f->cards[i] = cards[i];
        size *= (uint64_t)cards[i];
    }
    f->size = size;
    f->values = (double *)xcalloc((size_t)size, sizeof(double));
    f->partition = 0.0;
    return f;
}

rc_factor *rc_factor_new(int width, const int *vars, const int *cards, const double *values) {
    rc_factor *f = factor_alloc(width, vars, cards);
    double p = 0.0;
    for (uint64_t i = 0; i < f->size; ++i) {
        f->values[i] = values ? values[i] : 0.0;
        p += f->values[i];                 /* io.cpp:92-97 */
    }
    f->partition = p;
    return f;
}

rc_factor *rc_factor_copy(const rc_factor *f) {
    rc_factor *g = factor_alloc(f->width, f->vars, f->cards);
    memcpy(g->values, f->values, sizeof(double) * (size_t)f->size);
    g->partition = f->partition;
    return g;
}

void rc_factor_free(rc_factor *f) {
    if (!f) return;
    free(f->vars); free(f->cards); free(f->values); free(f);
}

int rc_factor_width(const rc_factor *f) { return f->width; }
uint64_t rc_factor_size(const rc_factor *f) { return f->size; }
void rc_factor_scope(const rc_factor *f, int *out) { memcpy(out, f->vars, sizeof(int) * (size_t)f->width); }
void rc_factor_values(const rc_factor *f, double *out) { memcpy(out, f->values, sizeof(double) * (size_t)f->size); }
double rc_factor_partition(const rc_factor *f) { return f->partition; }

/* Factor(1.0) (factor.cpp:25-30) */
static rc_factor *unit_factor(void) {
    rc_factor *f = factor_alloc(0, NULL, NULL);
    f->values[0] = 1.0;
    f->partition = 1.0;
    return f;
}

/* Domain(d1,d2) scope (domain.cpp:32-41): d1 order, then d2 vars not in d1 */
static rc_factor *alloc_union(const rc_factor *a, const rc_factor *b) {
    int w = a->width;
    int *vars = (int *)xmalloc(sizeof(int) * (size_t)(a->width + b->width));
    int *cards = (int *)xmalloc(sizeof(int) * (size_t)(a->width + b->width));
    for (int i = 0; i < a->width; ++i) { vars[i] = a->vars[i]; cards[i] = a->cards[i]; }
    for (int j = 0; j < b->width; ++j) {
        if (scope_index(a->width, a->vars, b->vars[j]) < 0) { vars[w] = b->vars[j]; cards[w] = b->cards[j]; ++w; }
    }
    rc_factor *out = factor_alloc(w, vars, cards);
    free(vars); free(cards);
    return out;
}

/* Factor::product / Factor::divide (factor.cpp:117-180).  Per output entry
   the positions in both inputs are recomputed from the odometer valuation
   (position_consistent_valuation, domain.cpp:162-179). */
static rc_factor *product_or_divide(const rc_factor *a, const rc_factor *b, int divide) {
    rc_factor *out = alloc_union(a, b);
    int w = out->width;
    uint64_t *offa = (uint64_t *)xmalloc(sizeof(uint64_t) * (size_t)(a->width + 1));
    uint64_t *offb = (uint64_t *)xmalloc(sizeof(uint64_t) * (size_t)(b->width + 1));
    uint64_t sa, sb;
    compute_offsets(a->width, a->cards, offa, &sa);
    compute_offsets(b->width, b->cards, offb, &sb);
    int *mapa = (int *)xmalloc(sizeof(int) * (size_t)(a->width + 1));
    int *mapb = (int *)xmalloc(sizeof(int) * (size_t)(b->width + 1));
    for (int j = 0; j < a->width; ++j) mapa[j] = scope_index(w, out->vars, a->vars[j]);
    for (int j = 0; j < b->width; ++j) mapb[j] = scope_index(w, out->vars, b->vars[j]);
    unsigned *val = (unsigned *)xcalloc((size_t)w + 1, sizeof(unsigned));
    double partition = 0;
    for (uint64_t i = 0; i < out->size; ++i) {
        uint64_t pos1 = 0, pos2 = 0;
        for (int j = 0; j < a->width; ++j) pos1 += offa[j] * val[mapa[j]];
        for (int j = 0; j < b->width; ++j) pos2 += offb[j] * val[mapb[j]];
        double value;
        if (divide) {
            if (b->values[pos2] == 0) { fprintf(stderr, "refcpu: divide by zero (factor.cpp:169 assert)\n"); abort(); }
            value = a->values[pos1] / b->values[pos2];
        } else {
            value = a->values[pos1] * b->values[pos2];
        }
        out->values[i] = value;
        partition += value;
        next_valuation(w, out->cards, val);
    }
    out->partition = partition;
    free(offa); free(offb); free(mapa); free(mapb); free(val);
    return out;
}

rc_factor *rc_product(const rc_factor *a, const rc_factor *b) { return product_or_divide(a, b, 0); }
rc_factor *rc_divide(const rc_factor *a, const rc_factor *b) { return product_or_divide(a, b, 1); }

/* Factor::sum_out (factor.cpp:182-212) */
rc_factor *rc_sum_out(const rc_factor *f, int var, int card) {
    int xi = scope_index(f->width, f->vars, var);
    if (xi < 0) return rc_factor_copy(f);          /* factor.cpp:185-188 */
    (void)card;
    int w = f->width - 1;
    int *vars = (int *)xmalloc(sizeof(int) * (size_t)(w + 1));
    int *cards = (int *)xmalloc(sizeof(int) * (size_t)(w + 1));
    int *map = (int *)xmalloc(sizeof(int) * (size_t)(w + 1));   /* new index -> old index */
    for (int i = 0, n = 0; i < f->width; ++i) {
        if (i == xi) continue;
        vars[n] = f->vars[i]; cards[n] = f->cards[i]; map[n] = i; ++n;
    }
    rc_factor *out = factor_alloc(w, vars, cards);
    uint64_t *off = (uint64_t *)xmalloc(sizeof(uint64_t) * (size_t)(f->width + 1));
    uint64_t s;
    compute_offsets(f->width, f->cards, off, &s);
    unsigned k = (unsigned)f->cards[xi];
    unsigned *val = (unsigned *)xcalloc((size_t)w + 1, sizeof(unsigned));
    double partition = 0;
    for (uint64_t i = 0; i < out->size; ++i) {
        for (unsigned v = 0; v < k; ++v) {
            uint64_t pos = 0;
            for (int j = 0; j < w; ++j) pos += off[map[j]] * val[j];
            pos += off[xi] * v;
            double value = f->values[pos];
            out->values[i] += value;
            partition += value;
        }
        next_valuation(w, out->cards, val);
    }
    out->partition = partition;
    free(vars); free(cards); free(map); free(off); free(val);
    return out;
}

/* Factor::conditioning (factor.cpp:214-242) with Domain(d, evidence)
   (domain.cpp:74-90) and next_valuation_with_evidence (domain.cpp:125-136). */
rc_factor *rc_conditioning(const rc_factor *f, int n_ev, const int *ev_vars, const int *ev_vals) {
    int *is_ev = (int *)xcalloc((size_t)f->width + 1, sizeof(int));
    unsigned *val = (unsigned *)xcalloc((size_t)f->width + 1, sizeof(unsigned));
    int w = 0;
    int *vars = (int *)xmalloc(sizeof(int) * (size_t)(f->width + 1));
    int *cards = (int *)xmalloc(sizeof(int) * (size_t)(f->width + 1));
    for (int i = 0; i < f->width; ++i) {
        int e = -1;
        for (int q = 0; q < n_ev; ++q) if (ev_vars[q] == f->vars[i]) e = q;
        if (e >= 0) { is_ev[i] = 1; val[i] = (unsigned)ev_vals[e]; }
        else { vars[w] = f->vars[i]; cards[w] = f->cards[i]; ++w; }
    }
    rc_factor *out = factor_alloc(w, vars, cards);
    uint64_t *off = (uint64_t *)xmalloc(sizeof(uint64_t) * (size_t)(f->width + 1));
    uint64_t s;
    compute_offsets(f->width, f->cards, off, &s);
    double partition = 0;
    for (uint64_t i = 0; i < out->size; ++i) {
        uint64_t pos = 0;
        for (int j = f->width - 1; j >= 0; --j) pos += val[j] * off[j];   /* position_valuation */
        double value = f->values[pos];
        out->values[i] = value;
        partition += value;
        int j;
        for (j = f->width - 1; j >= 0 && (is_ev[j] || val[j] == (unsigned)f->cards[j] - 1); --j) {
            if (is_ev[j]) continue;
            val[j] = 0;
        }
        if (j >= 0) val[j]++;
    }
    out->partition = partition;
    free(is_ev); free(val); free(vars); free(cards); free(off);
    return out;
}

/* Factor::normalize (factor.cpp:244-255) */
rc_factor *rc_normalize(const rc_factor *f) {
    rc_factor *g = rc_factor_copy(f);
    for (uint64_t i = 0; i < g->size; ++i) g->values[i] = g->values[i] / g->partition;
    g->partition = 1.0;
    return g;
}

/* model.cpp:414-418 */
rc_factor *rc_bucket(int n_in, const rc_factor *const *in, int var, int card) {
    rc_factor *prod = unit_factor();
    for (int i = 0; i < n_in; ++i) {
        rc_factor *p = rc_product(prod, in[i]);
        rc_factor_free(prod);
        prod = p;
    }
    rc_factor *msg = rc_sum_out(prod, var, card);
    rc_factor_free(prod);
    return msg;
}

/* ------------------------------------------------------------------- I/O */
typedef struct { FILE *fp; } tok_reader;

/* read_next_token (io.cpp:14-23): whitespace tokens; a token starting with
   '#' discards the rest of its line */
static int next_token(tok_reader *r, char *buf, size_t cap) {
    for (;;) {
        int c;
        do { c = fgetc(r->fp); } while (c != EOF && isspace(c));
        if (c == EOF) return 0;
        size_t n = 0;
        while (c != EOF && !isspace(c)) {
            if (n + 1 < cap) buf[n++] = (char)c;
            c = fgetc(r->fp);
        }
        buf[n] = 0;
        if (buf[0] != '#') return 1;
        while (c != EOF && c != '\n') c = fgetc(r->fp);
    }
}
static int next_int(tok_reader *r, long *out) {
    char buf[256];
    if (!next_token(r, buf, sizeof buf)) return 0;
    *out = strtol(buf, NULL, 10);
    return 1;
}
static int next_double(tok_reader *r, double *out) {
    char buf[256];
    if (!next_token(r, buf, sizeof buf)) return 0;
    *out = strtod(buf, NULL);
    return 1;
}

/* read_file_header / read_variables / read_factors (io.cpp:43-100) */
rc_model *rc_model_load_uai(const char *path) {
    FILE *fp = fopen(path, "r");
    if (!fp) return NULL;
    tok_reader r = {fp};
    char hdr[64];
    rc_model *m = NULL;
    if (!next_token(&r, hdr, sizeof hdr)) goto fail;
    int is_bayes;
    if (strcmp(hdr, "BAYES") == 0) is_bayes = 1;
    else if (strcmp(hdr, "MARKOV") == 0) is_bayes = 0;
    else goto fail;
    long nv, nf, w, id, sz;
    if (!next_int(&r, &nv) || nv < 0) goto fail;
    m = (rc_model *)xcalloc(1, sizeof(rc_model));
    m->is_bayes = is_bayes;
    m->n_vars = (int)nv;
    m->cards = (int *)xmalloc(sizeof(int) * (size_t)(nv + 1));
    for (long i = 0; i < nv; ++i) { if (!next_int(&r, &sz)) goto fail; m->cards[i] = (int)sz; }
    if (!next_int(&r, &nf) || nf < 0) goto fail;
    m->n_factors = (int)nf;
    m->factors = (rc_factor **)xcalloc((size_t)nf + 1, sizeof(rc_factor *));
    int **scopes = (int **)xcalloc((size_t)nf + 1, sizeof(int *));
    int *widths = (int *)xcalloc((size_t)nf + 1, sizeof(int));
    for (long i = 0; i < nf; ++i) {
        if (!next_int(&r, &w)) goto fail_sc;
        widths[i] = (int)w;
        scopes[i] = (int *)xmalloc(sizeof(int) * (size_t)(w + 1));
        for (long j = 0; j < w; ++j) {
            if (!next_int(&r, &id) || id < 0 || id >= nv) goto fail_sc;
            scopes[i][j] = (int)id;
        }
    }
    for (long i = 0; i < nf; ++i) {
        int *cards = (int *)xmalloc(sizeof(int) * (size_t)(widths[i] + 1));
        for (int j = 0; j < widths[i]; ++j) cards[j] = m->cards[scopes[i][j]];
        rc_factor *f = factor_alloc(widths[i], scopes[i], cards);
        free(cards);
        m->factors[i] = f;
        long fs;
        if (!next_int(&r, &fs) || (uint64_t)fs != f->size) goto fail_sc;
        double p = 0;
        for (long j = 0; j < fs; ++j) {
            double v;
            if (!next_double(&r, &v)) goto fail_sc;
            f->values[j] = v;
            p += v;
        }
        f->partition = p;
    }
    for (long i = 0; i < nf; ++i) free(scopes[i]);
    free(scopes); free(widths);
    fclose(fp);
    return m;
fail_sc:
    for (long i = 0; i < nf; ++i) free(scopes[i]);
    free(scopes); free(widths);
fail:
    fclose(fp);
    rc_model_free(m);
    return NULL;
}

rc_model *rc_model_new(int is_bayes, int n_vars, const int *cards, int n_factors,
                       const int *widths, const int *scopes, const double *values) {
    rc_model *m = (rc_model *)xcalloc(1, sizeof(rc_model));
    m->is_bayes = is_bayes;
    m->n_vars = n_vars;
    m->cards = (int *)xmalloc(sizeof(int) * (size_t)(n_vars + 1));
    memcpy(m->cards, cards, sizeof(int) * (size_t)n_vars);
    m->n_factors = n_factors;
    m->factors = (rc_factor **)xcalloc((size_t)n_factors + 1, sizeof(rc_factor *));
    const int *sc = scopes;
    const double *vals = values;
    for (int i = 0; i < n_factors; ++i) {
        int fc[64];
        for (int j = 0; j < widths[i]; ++j) fc[j] = cards[sc[j]];
        m->factors[i] = rc_factor_new(widths[i], sc, fc, vals);
        vals += m->factors[i]->size;
        sc += widths[i];
    }
    return m;
}

void rc_model_free(rc_model *m) {
    if (!m) return;
    if (m->factors) for (int i = 0; i < m->n_factors; ++i) rc_factor_free(m->factors[i]);
    free(m->factors); free(m->cards); free(m);
}
int rc_model_n_vars(const rc_model *m) { return m->n_vars; }
int rc_model_n_factors(const rc_model *m) { return m->n_factors; }
int rc_model_card(const rc_model *m, int v) { return m->cards[v]; }

/* read_uai_evidence (io.cpp:157-180): only read when the first integer is 1 */
int rc_load_evidence(const char *path, int cap, int *vars, int *vals) {
    FILE *fp = fopen(path, "r");
    if (!fp) return -1;
    tok_reader r = {fp};
    long n, size, id, v;
    int count = 0;
    if (next_int(&r, &n) && n == 1 && next_int(&r, &size)) {
        for (long i = 0; i < size; ++i) {
            if (!next_int(&r, &id) || !next_int(&r, &v)) break;
            int slot = -1;                       /* evidence[id] = val: last write wins */
            for (int q = 0; q < count; ++q) if (vars[q] == id) slot = q;
            if (slot < 0) { if (count >= cap) { fclose(fp); return -1; } slot = count++; }
            vars[slot] = (int)id; vals[slot] = (int)v;
        }
    }
    fclose(fp);
    return count;
}

/* ------------------------------------------------------- moral graph */
typedef struct {
    int n;            /* model variables */
    int words;
    uint64_t *adj;    /* n x words bitset */
    unsigned char *present;
    int n_present;
} graph;

static void bit_set(uint64_t *row, int j) { row[j >> 6] |= (uint64_t)1 << (j & 63); }
static void bit_clr(uint64_t *row, int j) { row[j >> 6] &= ~((uint64_t)1 << (j & 63)); }
static int popcount_row(const uint64_t *row, int words) {
    int c = 0;
    for (int i = 0; i < words; ++i) c += __builtin_popcountll(row[i]);
    return c;
}

/* Graph::Graph (graph.cpp:9-35) */
static graph graph_build(const rc_model *m, int nf, const rc_factor *const *fs) {
    graph g;
    g.n = m->n_vars;
    g.words = (g.n + 63) / 64;
    g.adj = (uint64_t *)xcalloc((size_t)g.n * (size_t)g.words + 1, sizeof(uint64_t));
    g.present = (unsigned char *)xcalloc((size_t)g.n + 1, 1);
    g.n_present = 0;
    for (int f = 0; f < nf; ++f) {
        const rc_factor *pf = fs[f];
        for (int i = 0; i < pf->width; ++i) {
            if (!g.present[pf->vars[i]]) { g.present[pf->vars[i]] = 1; g.n_present++; }
        }
        for (int i = 0; i + 1 < pf->width; ++i)
            for (int j = i + 1; j < pf->width; ++j) {
                int a = pf->vars[i], b = pf->vars[j];
                if (a == b) continue;
                bit_set(g.adj + (size_t)a * g.words, b);
                bit_set(g.adj + (size_t)b * g.words, a);
            }
    }
    return g;
}
static void graph_free(graph *g) { free(g->adj); free(g->present); }

static int degree(const graph *g, int v) {
    if (!g->present[v]) return 0;
    return popcount_row(g->adj + (size_t)v * g->words, g->words);
}

/* number of non-adjacent neighbour pairs (graph.cpp:131-138); weighted form
   sums card(id1)*card(id2) in unsigned arithmetic (graph.cpp:174-180) */
static unsigned fill_in(const graph *g, const rc_model *m, int v, int weighted) {
    if (!g->present[v]) return 0;
    const uint64_t *row = g->adj + (size_t)v * g->words;
    unsigned fill = 0;
    for (int wi = 0; wi < g->words; ++wi) {
        uint64_t bits = row[wi];
        while (bits) {
            int a = wi * 64 + __builtin_ctzll(bits);
            bits &= bits - 1;
            const uint64_t *ra = g->adj + (size_t)a * g->words;
            for (int wj = wi; wj < g->words; ++wj) {
                uint64_t cand = row[wj] & ~ra[wj];
                if (wj == wi) cand &= ~((((uint64_t)2) << (a & 63)) - 1);   /* id2 > id1 */
                while (cand) {
                    int b = wj * 64 + __builtin_ctzll(cand);
                    cand &= cand - 1;
                    fill += weighted ? (unsigned)m->cards[a] * (unsigned)m->cards[b] : 1u;
                }
            }
        }
    }
    return fill;
}

static void eliminate_vertex(graph *g, int v) {
    if (!g->present[v]) return;
    uint64_t *row = g->adj + (size_t)v * g->words;
    int nb[4096 * 4];
    int nn = 0;
    for (int wi = 0; wi < g->words; ++wi) {
        uint64_t bits = row[wi];
        while (bits) { nb[nn++] = wi * 64 + __builtin_ctzll(bits); bits &= bits - 1; }
    }
    for (int i = 0; i < nn; ++i) bit_clr(g->adj + (size_t)nb[i] * g->words, v);
    for (int i = 0; i < nn; ++i)
        for (int j = 0; j < nn; ++j)
            if (i != j) bit_set(g->adj + (size_t)nb[i] * g->words, nb[j]);
    memset(row, 0, sizeof(uint64_t) * (size_t)g->words);
    g->present[v] = 0;
    g->n_present--;
}

/* Graph::ordering (graph.cpp:41-101) with min_fill (122-153),
   weighted_min_fill (155-195), min_degree (103-120).  Candidates are visited
   in ascending id order. */
int rc_ordering(const rc_model *m, int nf, const rc_factor *const *fs,
                int n_vars, const int *vars, int heuristic, int *order_out) {
    graph g = graph_build(m, nf, fs);
    unsigned char *cand = (unsigned char *)xcalloc((size_t)m->n_vars + 1, 1);
    int remaining = 0;
    for (int i = 0; i < n_vars; ++i) if (!cand[vars[i]]) { cand[vars[i]] = 1; remaining++; }
    int width = 0, pos = 0;
    while (remaining > 0) {
        int first = -1;
        for (int v = 0; v < m->n_vars; ++v) if (cand[v]) { first = v; break; }
        int next = first;
        if (heuristic == RC_MIN_DEGREE) {
            unsigned best = (unsigned)g.n_present + 1;
            for (int v = first; v < m->n_vars; ++v) {
                if (!cand[v]) continue;
                unsigned d = (unsigned)degree(&g, v);
                if (d < best) { next = v; best = d; }
            }
        } else {
            int weighted = heuristic == RC_WEIGHTED_MIN_FILL;
            unsigned best = weighted ? fill_in(&g, m, first, 1) : (unsigned)g.n_present + 1;
            for (int v = first; v < m->n_vars; ++v) {
                if (!cand[v]) continue;
                unsigned f = fill_in(&g, m, v, weighted);
                if (f < best) { next = v; best = f; }
                else if (f == best && degree(&g, v) < degree(&g, next)) { next = v; best = f; }
            }
        }
        order_out[pos++] = next;
        int d = degree(&g, next);
        if (d > width) width = d;
        eliminate_vertex(&g, next);
        cand[next] = 0;
        remaining--;
    }
    free(cand);
    graph_free(&g);
    return width;
}

/* Graph::order_width (graph.cpp:197-237) */
int rc_order_width(const rc_model *m, int nf, const rc_factor *const *fs, int n, const int *order) {
    graph g = graph_build(m, nf, fs);
    int width = 0;
    for (int i = 0; i < n; ++i) {
        int d = degree(&g, order[i]);
        if (d > width) width = d;
        eliminate_vertex(&g, order[i]);
    }
    graph_free(&g);
    return width;
}

/* ------------------------------------------------- variable elimination */
typedef struct { const rc_factor **items; int n, cap; } fvec;
static void fvec_push(fvec *v, const rc_factor *f) {
    if (v->n == v->cap) {
        v->cap = v->cap ? 2 * v->cap : 4;
        v->items = (const rc_factor **)realloc((void *)v->items, sizeof(*v->items) * (size_t)v->cap);
        if (!v->items) abort();
    }
    v->items[v->n++] = f;
}

/* BN::variable_elimination (model.cpp:348-446) */
rc_factor *rc_variable_elimination(const rc_model *m, int n_vars, const int *vars,
                                   int nf, const rc_factor *const *fs, int heuristic) {
    rc_factor *result = unit_factor();
    int *order = (int *)xmalloc(sizeof(int) * (size_t)(n_vars + 1));
    if (heuristic != RC_ORDER_GIVEN) rc_ordering(m, nf, fs, n_vars, vars, heuristic, order);
    else memcpy(order, vars, sizeof(int) * (size_t)n_vars);

    /* position of each variable in the remaining ordering (-1: not in it) */
    int *rank = (int *)xmalloc(sizeof(int) * (size_t)(m->n_vars + 1));
    for (int v = 0; v < m->n_vars; ++v) rank[v] = -1;
    for (int i = n_vars - 1; i >= 0; --i) rank[order[i]] = i;
    fvec *buckets = (fvec *)xcalloc((size_t)n_vars + 1, sizeof(fvec));
    fvec owned = {0, 0, 0};

    /* first variable of the ordering that is in the factor's scope */
    #define FIRST_BUCKET(pf, from, out_b) do {                                   \
        int _b = -1;                                                             \
        for (int _j = 0; _j < (pf)->width; ++_j) {                               \
            int _r = rank[(pf)->vars[_j]];                                       \
            if (_r >= (from) && (_b < 0 || _r < _b)) _b = _r;                    \
        }                                                                        \
        (out_b) = _b;                                                            \
    } while (0)

    for (int f = 0; f < nf; ++f) {                 /* model.cpp:394-406 */
        int b;
        FIRST_BUCKET(fs[f], 0, b);
        if (b >= 0) fvec_push(&buckets[b], fs[f]);
        else { rc_factor *r = rc_product(result, fs[f]); rc_factor_free(result); result = r; }
    }
    for (int i = 0; i < n_vars; ++i) {             /* model.cpp:409-439 */
        int var = order[i];
        rc_factor *msg = rc_bucket(buckets[i].n, buckets[i].items, var, m->cards[var]);
        fvec_push(&owned, msg);
        int b;
        FIRST_BUCKET(msg, i + 1, b);
        if (b >= 0) fvec_push(&buckets[b], msg);
        else { rc_factor *r = rc_product(result, msg); rc_factor_free(result); result = r; }
    }
    #undef FIRST_BUCKET
    for (int i = 0; i < owned.n; ++i) rc_factor_free((rc_factor *)owned.items[i]);
    free((void *)owned.items);
    for (int i = 0; i < n_vars; ++i) free((void *)buckets[i].items);
    free(buckets); free(rank); free(order);
    return result;
}

static rc_factor **condition_all(const rc_model *m, int n_ev, const int *ev_vars, const int *ev_vals) {
    rc_factor **fs = (rc_factor **)xmalloc(sizeof(rc_factor *) * (size_t)(m->n_factors + 1));
    for (int i = 0; i < m->n_factors; ++i) fs[i] = rc_conditioning(m->factors[i], n_ev, ev_vars, ev_vals);
    return fs;
}
static void free_all(rc_factor **fs, int n) {
    for (int i = 0; i < n; ++i) rc_factor_free(fs[i]);
    free(fs);
}

/* BN::partition (model.cpp:250-301), VE branch */
double rc_partition(const rc_model *m, int n_ev, const int *ev_vars, const int *ev_vals,
                    int heuristic, double *uptime_ms) {
    double t0 = now_ms();
    int *vars = (int *)xmalloc(sizeof(int) * (size_t)(m->n_vars + 1));
    int n = 0;
    for (int v = 0; v < m->n_vars; ++v) {
        int is_ev = 0;
        for (int q = 0; q < n_ev; ++q) if (ev_vars[q] == v) is_ev = 1;
        if (!is_ev) vars[n++] = v;
    }
    rc_factor **fs = condition_all(m, n_ev, ev_vars, ev_vals);
    rc_factor *part = rc_variable_elimination(m, n, vars, m->n_factors, (const rc_factor *const *)fs, heuristic);
    double p = part->partition;
    rc_factor_free(part);
    free_all(fs, m->n_factors);
    free(vars);
    if (uptime_ms) *uptime_ms = now_ms() - t0;
    return p;
}

static void write_marginal(const rc_model *m, const rc_factor *nf, int target,
                           int n_ev, const int *ev_vars, const int *ev_vals, double *out) {
    int k = m->cards[target];
    if (nf->width == 1) {
        for (int s = 0; s < k; ++s) out[s] = nf->values[s];
        return;
    }
    /* width-0 marginal: evidence variable (printed one-hot in the UAI MAR
       format) or a variable in no factor (uniform) */
    int ev = -1;
    for (int q = 0; q < n_ev; ++q) if (ev_vars[q] == target) ev = ev_vals[q];
    for (int s = 0; s < k; ++s) out[s] = ev >= 0 ? (s == ev ? 1.0 : 0.0) : 1.0 / k;
}

int rc_marginal_one(const rc_model *m, int n_ev, const int *ev_vars, const int *ev_vals,
                    int heuristic, int target, double *out) {
    rc_factor **fs = condition_all(m, n_ev, ev_vars, ev_vals);
    int *vars = (int *)xmalloc(sizeof(int) * (size_t)(m->n_vars + 1));
    int n = 0;
    for (int v = 0; v < m->n_vars; ++v) if (v != target) vars[n++] = v;
    rc_factor *r = rc_variable_elimination(m, n, vars, m->n_factors, (const rc_factor *const *)fs, heuristic);
    rc_factor *nf = rc_normalize(r);
    write_marginal(m, nf, target, n_ev, ev_vars, ev_vals, out);
    rc_factor_free(r); rc_factor_free(nf);
    free(vars);
    free_all(fs, m->n_factors);
    return 0;
}

/* BN::marginals (model.cpp:303-346), VE branch */
int rc_marginals(const rc_model *m, int n_ev, const int *ev_vars, const int *ev_vals,
                 int heuristic, double *out, double *uptime_ms) {
    double t0 = now_ms();
    rc_factor **fs = condition_all(m, n_ev, ev_vars, ev_vals);
    int *vars = (int *)xmalloc(sizeof(int) * (size_t)(m->n_vars + 1));
    size_t o = 0;
    for (int t = 0; t < m->n_vars; ++t) {
        int n = 0;
        for (int v = 0; v < m->n_vars; ++v) if (v != t) vars[n++] = v;
        rc_factor *r = rc_variable_elimination(m, n, vars, m->n_factors, (const rc_factor *const *)fs, heuristic);
        rc_factor *nf = rc_normalize(r);
        write_marginal(m, nf, t, n_ev, ev_vars, ev_vals, out + o);
        o += (size_t)m->cards[t];
        rc_factor_free(r); rc_factor_free(nf);
    }
    free(vars);
    free_all(fs, m->n_factors);
    if (uptime_ms) *uptime_ms = now_ms() - t0;
    return 0;
}

/* ------------------------------------------------------ bucket micro */
double rc_micro_bucket(int k, int w, int reps, double *seconds_out) {
    int vm[64], cm[64], vf[2] = {0, w + 1}, cf[2] = {k, k};
    vm[0] = 0; cm[0] = k;
    for (int i = 1; i <= w; ++i) { vm[i] = i; cm[i] = k; }
    rc_factor *mf = rc_factor_new(w + 1, vm, cm, NULL);
    rc_factor *ff = rc_factor_new(2, vf, cf, NULL);
    uint64_t s = 0x9E3779B97F4A7C15ull;
    for (uint64_t i = 0; i < mf->size; ++i) { s = s * 6364136223846793005ull + 1442695040888963407ull; mf->values[i] = 0.5 + 1.5 * (double)(s >> 11) / 9007199254740992.0; }
    for (uint64_t i = 0; i < ff->size; ++i) { s = s * 6364136223846793005ull + 1442695040888963407ull; ff->values[i] = 0.5 + 1.5 * (double)(s >> 11) / 9007199254740992.0; }
    const rc_factor *in[2] = {mf, ff};
    double entries = (double)mf->size * k;     /* prod(card) over (x, S, y) */
    double t0 = now_ms();
    double sink = 0;
    for (int r = 0; r < reps; ++r) {
        rc_factor *msg = rc_bucket(2, in, 0, k);
        sink += msg->partition;
        rc_factor_free(msg);
    }
    double sec = (now_ms() - t0) * 1e-3;
    if (seconds_out) *seconds_out = sec;
    rc_factor_free(mf); rc_factor_free(ff);
    if (sink < 0) fprintf(stderr, "impossible\n");
    return entries * reps / sec;
}

/* ------------------------------------------------------ loopy BP (-sp) */
/* FactorGraph (graph.cpp:256-403) as driven by BN::sum_product + marginals
   (model.cpp:313-317, 736-753): flooding schedule, every variable->factor
   message, then every factor->variable message, convergence on the largest
   relative change |old - new| / old of the iteration (graph.cpp:298-332).
   Restated with this file's factor algebra.  Deviation: the reference walks
   unordered_maps keyed by id (graph.hh:50-51), so its products run in hash
   order; here they run by ascending factor id (variable side) and in scope
   order (factor side) -- the same values up to rounding. */
static double sp_replace(rc_factor **slot, rc_factor *raw) {
    rc_factor *nw = rc_normalize(raw);                               /* graph.cpp:345, 374 */
    rc_factor_free(raw);
    const rc_factor *old = *slot;
    double maxerror = 0.0;
    for (uint64_t i = 0; i < old->size; ++i) {                        /* graph.cpp:348-356 */
        double err = fabs(old->values[i] - nw->values[i]) / old->values[i];
        if (err > maxerror) maxerror = err;
    }
    rc_factor_free(*slot);
    *slot = nw;
    return maxerror;
}

int rc_sum_product(const rc_model *m, int max_iter, double eps, double *out, int *iterations, double *uptime_ms) {
    double t0 = now_ms();
    int n_edges = 0;
    for (int f = 0; f < m->n_factors; ++f) n_edges += m->factors[f]->width;
    int *e_off = (int *)xmalloc(sizeof(int) * (size_t)(m->n_factors + 1));
    rc_factor **v2f = (rc_factor **)xcalloc((size_t)n_edges, sizeof(rc_factor *));
    rc_factor **f2v = (rc_factor **)xcalloc((size_t)n_edges, sizeof(rc_factor *));
    e_off[0] = 0;
    for (int f = 0; f < m->n_factors; ++f) {
        const rc_factor *F = m->factors[f];
        e_off[f + 1] = e_off[f] + F->width;
        for (int j = 0; j < F->width; ++j) {                          /* graph.cpp:265-273 */
            int v = F->vars[j], r = F->cards[j];
            double *u = (double *)xmalloc(sizeof(double) * (size_t)r);
            for (int x = 0; x < r; ++x) u[x] = 1.0 / r;
            f2v[e_off[f] + j] = rc_factor_new(1, &v, &r, u);
            v2f[e_off[f] + j] = rc_factor_new(1, &v, &r, u);
            free(u);
        }
    }
    int it;
    for (it = 0; it < max_iter; ++it) {
        double maxerror = 0.0;
        for (int f = 0; f < m->n_factors; ++f)                        /* graph.cpp:306-315 */
            for (int j = 0; j < m->factors[f]->width; ++j) {
                int v = m->factors[f]->vars[j], r = m->factors[f]->cards[j];
                rc_factor *nw = rc_factor_new(1, &v, &r, NULL);       /* Factor(sc, 1.0), graph.cpp:339 */
                for (uint64_t x = 0; x < nw->size; ++x) nw->values[x] = 1.0;
                nw->partition = (double)r;                            /* factor.cpp:18-23 */
                for (int g = 0; g < m->n_factors; ++g) {
                    if (g == f) continue;
                    for (int k = 0; k < m->factors[g]->width; ++k)
                        if (m->factors[g]->vars[k] == v) {
                            rc_factor *p = rc_product(nw, f2v[e_off[g] + k]);
                            rc_factor_free(nw);
                            nw = p;
                        }
                }
                double err = sp_replace(&v2f[e_off[f] + j], nw);
                if (err > maxerror) maxerror = err;
            }
        for (int f = 0; f < m->n_factors; ++f)                        /* graph.cpp:317-326 */
            for (int j = 0; j < m->factors[f]->width; ++j) {
                const rc_factor *F = m->factors[f];
                rc_factor *nw = rc_factor_copy(F);                    /* graph.cpp:367-373 */
                for (int k = 0; k < F->width; ++k) {
                    if (k == j) continue;
                    rc_factor *p = rc_product(nw, v2f[e_off[f] + k]);
                    rc_factor_free(nw);
                    nw = rc_sum_out(p, F->vars[k], F->cards[k]);
                    rc_factor_free(p);
                }
                double err = sp_replace(&f2v[e_off[f] + j], nw);
                if (err > maxerror) maxerror = err;
            }
        if (maxerror < eps) break;                                    /* graph.cpp:328 */
    }
    /* FactorGraph::marginal (graph.cpp:393-403), var-major output */
    size_t o = 0;
    for (int v = 0; v < m->n_vars; ++v) {
        rc_factor *mg = rc_factor_new(0, NULL, NULL, NULL);
        mg->values[0] = 1.0;
        mg->partition = 1.0;
        for (int g = 0; g < m->n_factors; ++g)
            for (int k = 0; k < m->factors[g]->width; ++k)
                if (m->factors[g]->vars[k] == v) {
                    rc_factor *p = rc_product(mg, f2v[e_off[g] + k]);
                    rc_factor_free(mg);
                    mg = p;
                }
        rc_factor *nm = rc_normalize(mg);
        for (int x = 0; x < m->cards[v]; ++x) out[o++] = nm->size == (uint64_t)m->cards[v] ? nm->values[x] : 1.0 / m->cards[v];
        rc_factor_free(mg);
        rc_factor_free(nm);
    }
    for (int e = 0; e < n_edges; ++e) { rc_factor_free(v2f[e]); rc_factor_free(f2v[e]); }
    free(v2f); free(f2v); free(e_off);
    if (iterations) *iterations = it;
    if (uptime_ms) *uptime_ms = now_ms() - t0;
    return 0;
}
