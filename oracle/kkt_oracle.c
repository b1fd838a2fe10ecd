/*
 * kkt_oracle.c -- TEST INFRASTRUCTURE ONLY (parity checker; never linked into the product).
 *
 * Multifrontal LDL^T with threshold 1x1/2x2 pivoting, delayed pivots, null-pivot detection and
 * inertia: a CPU restatement of what uno/ingredients/subproblem_solvers/MUMPS/MUMPSSolver.cpp asks
 * MUMPS 5.8.0 to compute (see kkt_oracle.h for the option-by-option citation).  Plain C99, single
 * threaded, written for clarity rather than speed.
 *
 * Pipeline:
 *   analyze   : canonical lower pattern (duplicates merged)            COOFormat.hpp:92-99 semantics
 *               -> reverse Cuthill-McKee ordering, dense nodes last
 *               -> column structures of L, fundamental supernodes, assembly tree
 *   factorize : sum duplicates, equilibrate (ICNTL(8)=8, MUMPSSolver.cpp:82),
 *               null threshold eps*1e-5*||A_pre|| (ICNTL(24)=1, MUMPSSolver.cpp:36),
 *               fronts in postorder with delayed pivots, inertia (MUMPSSolver.cpp:124-147)
 *   solve     : forward, block-diagonal, backward, unscale (MUMPSSolver.cpp:91-96)
 */
#include "kkt_oracle.h"

#include <float.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

enum { PIV_NULL = 0, PIV_1X1 = 1, PIV_2X2_A = 2, PIV_2X2_B = 3 };

struct oracle_kkt {
    int64_t n, nnz;
    int analyzed, factored;
    double u;
    int scale_iters;
    int ordering;  /* 0: reverse Cuthill-McKee (default), 1: Cuthill-McKee (not reversed) -- a second valid ordering */
    double null_fac;
    char err[256];
    /* canonical pattern */
    int64_t nu;
    int64_t *map;      /* COO position -> unique entry */
    int64_t *ur, *uc;  /* unique entry: row >= col, original numbering */
    int64_t *dup_ptr, *dup_pos; /* unique entry -> COO positions (ascending) */
    /* ordering */
    int64_t *perm, *iperm;
    /* supernodes */
    int64_t nsn;
    int64_t *sn_first, *sn_parent, *sn_sptr, *sn_struct, *col2sn;
    int64_t *sn_eptr, *sn_ent; /* unique entries assembled at each supernode */
    /* numeric */
    double *scale, *uval;
    double thres;
    int64_t *f_m, *f_npiv;
    int64_t **f_vars;
    double **f_L;
    signed char **f_piv;
    int64_t npos, nneg, nzero;
    double stats[7];
};

static int fail(oracle_kkt_t h, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(h->err, sizeof(h->err), fmt, ap);
    va_end(ap);
    return -1;
}

static void* xcalloc(size_t n, size_t s) {
    void* p = calloc(n ? n : 1, s);
    if (!p) { fprintf(stderr, "oracle: out of memory\n"); abort(); }
    return p;
}

static void free_numeric(oracle_kkt_t h) {
    if (h->f_vars) {
        for (int64_t s = 0; s < h->nsn; ++s) { free(h->f_vars[s]); free(h->f_L[s]); free(h->f_piv[s]); }
    }
    free(h->f_vars); free(h->f_L); free(h->f_piv); free(h->f_m); free(h->f_npiv);
    free(h->scale); free(h->uval);
    h->f_vars = NULL; h->f_L = NULL; h->f_piv = NULL; h->f_m = NULL; h->f_npiv = NULL;
    h->scale = NULL; h->uval = NULL;
    h->factored = 0;
}

static void free_symbolic(oracle_kkt_t h) {
    free_numeric(h);
    free(h->map); free(h->ur); free(h->uc); free(h->dup_ptr); free(h->dup_pos);
    free(h->perm); free(h->iperm);
    free(h->sn_first); free(h->sn_parent); free(h->sn_sptr); free(h->sn_struct); free(h->col2sn);
    free(h->sn_eptr); free(h->sn_ent);
    h->map = h->ur = h->uc = h->dup_ptr = h->dup_pos = NULL;
    h->perm = h->iperm = NULL;
    h->sn_first = h->sn_parent = h->sn_sptr = h->sn_struct = h->col2sn = NULL;
    h->sn_eptr = h->sn_ent = NULL;
    h->analyzed = 0;
}

oracle_kkt_t oracle_kkt_create(void) {
    oracle_kkt_t h = (oracle_kkt_t)xcalloc(1, sizeof(*h));
    h->u = 0.01;
    h->scale_iters = 3;
    h->null_fac = 1e-5;
    return h;
}

void oracle_kkt_destroy(oracle_kkt_t h) {
    if (!h) return;
    free_symbolic(h);
    free(h);
}

int oracle_kkt_set_option(oracle_kkt_t h, const char* name, double value) {
    if (!strcmp(name, "pivot_threshold")) { h->u = value; return 0; }
    if (!strcmp(name, "scale_iters")) { h->scale_iters = (int)value; return 0; }
    if (!strcmp(name, "ordering")) { h->ordering = (int)value; return 0; }
    if (!strcmp(name, "null_tol_factor")) { h->null_fac = value; return 0; }
    return fail(h, "unknown option '%s'", name);
}

const char* oracle_kkt_last_error(oracle_kkt_t h) { return h->err; }

/* ------------------------------------------------------------------------------------------ */
/* analysis                                                                                    */
/* ------------------------------------------------------------------------------------------ */

typedef struct { int64_t a, k; } pair_t;
static int cmp_pair(const void* x, const void* y) {
    const pair_t* p = (const pair_t*)x; const pair_t* q = (const pair_t*)y;
    if (p->a != q->a) return p->a < q->a ? -1 : 1;
    return p->k < q->k ? -1 : (p->k > q->k);
}
static int cmp_i64(const void* x, const void* y) {
    int64_t a = *(const int64_t*)x, b = *(const int64_t*)y;
    return a < b ? -1 : (a > b);
}

/* BFS over the non-dense subgraph restricted to unvisited nodes; returns number of levels */
static int64_t bfs_levels(int64_t start, const int64_t* ap, const int64_t* ai, const char* skip,
                          int64_t* level, int64_t* queue, int64_t* qlen, int64_t stamp, int64_t* seen) {
    int64_t head = 0, tail = 0, nlev = 0;
    queue[tail++] = start; seen[start] = stamp; level[start] = 0;
    while (head < tail) {
        int64_t v = queue[head++];
        if (level[v] + 1 > nlev) nlev = level[v] + 1;
        for (int64_t p = ap[v]; p < ap[v + 1]; ++p) {
            int64_t w = ai[p];
            if (skip[w] || seen[w] == stamp) continue;
            seen[w] = stamp; level[w] = level[v] + 1; queue[tail++] = w;
        }
    }
    *qlen = tail;
    return nlev;
}

int oracle_kkt_analyze(oracle_kkt_t h, int64_t n, int64_t nnz, const int64_t* row, const int64_t* col) {
    free_symbolic(h);
    h->err[0] = 0;
    if (n < 0 || nnz < 0) return fail(h, "negative size");
    h->n = n; h->nnz = nnz;
    for (int64_t k = 0; k < nnz; ++k)
        if (row[k] < 0 || row[k] >= n || col[k] < 0 || col[k] >= n)
            return fail(h, "entry %lld (%lld,%lld) out of range for n=%lld", (long long)k,
                        (long long)row[k], (long long)col[k], (long long)n);

    /* ---- canonical lower pattern: bucket by min index, sort by max index then position ---- */
    int64_t* cnt = (int64_t*)xcalloc((size_t)n + 1, sizeof(int64_t));
    for (int64_t k = 0; k < nnz; ++k) cnt[(row[k] < col[k] ? row[k] : col[k]) + 1]++;
    for (int64_t i = 0; i < n; ++i) cnt[i + 1] += cnt[i];
    pair_t* pr = (pair_t*)xcalloc((size_t)nnz, sizeof(pair_t));
    int64_t* fill = (int64_t*)xcalloc((size_t)n + 1, sizeof(int64_t));
    memcpy(fill, cnt, sizeof(int64_t) * (size_t)(n + 1));
    for (int64_t k = 0; k < nnz; ++k) {
        int64_t b = row[k] < col[k] ? row[k] : col[k];
        int64_t a = row[k] < col[k] ? col[k] : row[k];
        pr[fill[b]].a = a; pr[fill[b]].k = k; fill[b]++;
    }
    h->map = (int64_t*)xcalloc((size_t)nnz, sizeof(int64_t));
    h->ur = (int64_t*)xcalloc((size_t)nnz, sizeof(int64_t));
    h->uc = (int64_t*)xcalloc((size_t)nnz, sizeof(int64_t));
    h->dup_ptr = (int64_t*)xcalloc((size_t)nnz + 1, sizeof(int64_t));
    h->dup_pos = (int64_t*)xcalloc((size_t)nnz, sizeof(int64_t));
    int64_t nu = 0;
    for (int64_t b = 0; b < n; ++b) {
        int64_t s = cnt[b], e = cnt[b + 1];
        if (e - s > 1) qsort(pr + s, (size_t)(e - s), sizeof(pair_t), cmp_pair);
        for (int64_t q = s; q < e; ++q) {
            if (q == s || pr[q].a != pr[q - 1].a) {
                h->ur[nu] = pr[q].a; h->uc[nu] = b; h->dup_ptr[nu] = q; nu++;
            }
            h->map[pr[q].k] = nu - 1;
            h->dup_pos[q] = pr[q].k;
        }
    }
    h->dup_ptr[nu] = nnz;
    h->nu = nu;
    free(pr); free(fill); free(cnt);

    /* ---- symmetric adjacency (no diagonal) ---- */
    int64_t* ap = (int64_t*)xcalloc((size_t)n + 1, sizeof(int64_t));
    for (int64_t u = 0; u < nu; ++u)
        if (h->ur[u] != h->uc[u]) { ap[h->ur[u] + 1]++; ap[h->uc[u] + 1]++; }
    for (int64_t i = 0; i < n; ++i) ap[i + 1] += ap[i];
    int64_t* ai = (int64_t*)xcalloc((size_t)ap[n] + 1, sizeof(int64_t));
    int64_t* pos = (int64_t*)xcalloc((size_t)n + 1, sizeof(int64_t));
    memcpy(pos, ap, sizeof(int64_t) * (size_t)n);
    for (int64_t u = 0; u < nu; ++u)
        if (h->ur[u] != h->uc[u]) { ai[pos[h->ur[u]]++] = h->uc[u]; ai[pos[h->uc[u]]++] = h->ur[u]; }
    free(pos);

    /* ---- ordering: RCM on the non-dense subgraph, dense nodes last ---- */
    double dense_thr = 10.0 * sqrt((double)n);
    if (dense_thr < 16) dense_thr = 16;
    char* dense = (char*)xcalloc((size_t)n + 1, 1);
    for (int64_t i = 0; i < n; ++i) dense[i] = (double)(ap[i + 1] - ap[i]) > dense_thr;
    int64_t* deg = (int64_t*)xcalloc((size_t)n + 1, sizeof(int64_t));
    for (int64_t i = 0; i < n; ++i) {
        if (dense[i]) continue;
        for (int64_t p = ap[i]; p < ap[i + 1]; ++p) deg[i] += !dense[ai[p]];
    }
    int64_t* order = (int64_t*)xcalloc((size_t)n + 1, sizeof(int64_t));
    int64_t* level = (int64_t*)xcalloc((size_t)n + 1, sizeof(int64_t));
    int64_t* queue = (int64_t*)xcalloc((size_t)n + 1, sizeof(int64_t));
    int64_t* seen = (int64_t*)xcalloc((size_t)n + 1, sizeof(int64_t));
    char* done = (char*)xcalloc((size_t)n + 1, 1);
    int64_t* nbr = (int64_t*)xcalloc((size_t)n + 1, sizeof(int64_t));
    for (int64_t i = 0; i < n; ++i) seen[i] = -1;
    int64_t norder = 0, stamp = 0;
    for (int64_t root = 0; root < n; ++root) {
        if (dense[root] || done[root]) continue;
        /* pseudo-peripheral start node of this component (George-Liu) */
        int64_t start = root, qlen = 0;
        int64_t ecc = bfs_levels(start, ap, ai, dense, level, queue, &qlen, stamp++, seen);
        for (int it = 0; it < 8; ++it) {
            int64_t best = -1;
            for (int64_t q = 0; q < qlen; ++q) {
                int64_t v = queue[q];
                if (level[v] == ecc - 1 && (best < 0 || deg[v] < deg[best])) best = v;
            }
            int64_t e2 = bfs_levels(best, ap, ai, dense, level, queue, &qlen, stamp++, seen);
            if (e2 <= ecc) break;
            ecc = e2; start = best;
        }
        /* Cuthill-McKee from start: neighbours in increasing degree */
        int64_t head = norder;
        order[norder++] = start; done[start] = 1;
        while (head < norder) {
            int64_t v = order[head++];
            int64_t k = 0;
            for (int64_t p = ap[v]; p < ap[v + 1]; ++p) {
                int64_t w = ai[p];
                if (dense[w] || done[w]) continue;
                done[w] = 1; nbr[k++] = w;
            }
            for (int64_t a = 1; a < k; ++a) { /* insertion sort by (deg, index) */
                int64_t w = nbr[a], b = a - 1;
                while (b >= 0 && (deg[nbr[b]] > deg[w] || (deg[nbr[b]] == deg[w] && nbr[b] > w))) {
                    nbr[b + 1] = nbr[b]; b--;
                }
                nbr[b + 1] = w;
            }
            for (int64_t a = 0; a < k; ++a) order[norder++] = nbr[a];
        }
    }
    /* reverse the Cuthill-McKee order, then dense nodes */
    h->perm = (int64_t*)xcalloc((size_t)n + 1, sizeof(int64_t));
    h->iperm = (int64_t*)xcalloc((size_t)n + 1, sizeof(int64_t));
    for (int64_t q = 0; q < norder; ++q) h->perm[q] = h->ordering == 1 ? order[q] : order[norder - 1 - q];
    int64_t nq = norder;
    for (int64_t i = 0; i < n; ++i) if (dense[i]) h->perm[nq++] = i;
    for (int64_t q = 0; q < n; ++q) h->iperm[h->perm[q]] = q;
    free(order); free(level); free(queue); free(seen); free(done); free(nbr); free(deg); free(dense);

    /* ---- column structures of L, fundamental supernodes ---- */
    int64_t** cs = (int64_t**)xcalloc((size_t)n + 1, sizeof(int64_t*));
    int64_t* clen = (int64_t*)xcalloc((size_t)n + 1, sizeof(int64_t));
    int64_t* parent = (int64_t*)xcalloc((size_t)n + 1, sizeof(int64_t));
    int64_t* chead = (int64_t*)xcalloc((size_t)n + 1, sizeof(int64_t));
    int64_t* cnext = (int64_t*)xcalloc((size_t)n + 1, sizeof(int64_t));
    int64_t* nchild = (int64_t*)xcalloc((size_t)n + 1, sizeof(int64_t));
    int64_t* mark = (int64_t*)xcalloc((size_t)n + 1, sizeof(int64_t));
    int64_t* buf = (int64_t*)xcalloc((size_t)n + 1, sizeof(int64_t));
    int64_t* col2sn = (int64_t*)xcalloc((size_t)n + 1, sizeof(int64_t));
    int64_t* snf = (int64_t*)xcalloc((size_t)n + 2, sizeof(int64_t));
    for (int64_t i = 0; i < n; ++i) { chead[i] = -1; mark[i] = -1; }
    int64_t nsn = 0;
    for (int64_t j = 0; j < n; ++j) {
        int64_t len = 0;
        mark[j] = j;
        int64_t old = h->perm[j];
        for (int64_t p = ap[old]; p < ap[old + 1]; ++p) {
            int64_t i = h->iperm[ai[p]];
            if (i > j && mark[i] != j) { mark[i] = j; buf[len++] = i; }
        }
        for (int64_t c = chead[j]; c >= 0; c = cnext[c]) {
            for (int64_t q = 0; q < clen[c]; ++q) {
                int64_t i = cs[c][q];
                if (i > j && mark[i] != j) { mark[i] = j; buf[len++] = i; }
            }
        }
        qsort(buf, (size_t)len, sizeof(int64_t), cmp_i64);
        cs[j] = (int64_t*)xcalloc((size_t)len + 1, sizeof(int64_t));
        memcpy(cs[j], buf, sizeof(int64_t) * (size_t)len);
        clen[j] = len;
        parent[j] = len ? buf[0] : -1;
        if (parent[j] >= 0) { cnext[j] = chead[parent[j]]; chead[parent[j]] = j; nchild[parent[j]]++; }
        /* fundamental supernode: j continues j-1's supernode */
        int merge = j > 0 && parent[j - 1] == j && nchild[j] == 1 && clen[j - 1] == clen[j] + 1;
        if (merge) {
            free(cs[j - 1]); cs[j - 1] = NULL; /* struct(first cols) = later cols U struct(last) */
        } else {
            snf[nsn++] = j;
        }
        col2sn[j] = nsn - 1;
    }
    snf[nsn] = n;
    h->nsn = nsn;
    h->sn_first = snf;
    h->col2sn = col2sn;
    h->sn_parent = (int64_t*)xcalloc((size_t)nsn + 1, sizeof(int64_t));
    h->sn_sptr = (int64_t*)xcalloc((size_t)nsn + 1, sizeof(int64_t));
    for (int64_t s = 0; s < nsn; ++s) {
        int64_t last = snf[s + 1] - 1;
        h->sn_sptr[s + 1] = h->sn_sptr[s] + clen[last];
        h->sn_parent[s] = parent[last] >= 0 ? col2sn[parent[last]] : -1;
    }
    h->sn_struct = (int64_t*)xcalloc((size_t)h->sn_sptr[nsn] + 1, sizeof(int64_t));
    for (int64_t s = 0; s < nsn; ++s) {
        int64_t last = snf[s + 1] - 1;
        memcpy(h->sn_struct + h->sn_sptr[s], cs[last], sizeof(int64_t) * (size_t)clen[last]);
    }
    for (int64_t j = 0; j < n; ++j) free(cs[j]);
    free(cs); free(clen); free(parent); free(chead); free(cnext); free(nchild); free(mark); free(buf);
    free(ap); free(ai);

    /* ---- unique entries per supernode ---- */
    h->sn_eptr = (int64_t*)xcalloc((size_t)nsn + 2, sizeof(int64_t));
    h->sn_ent = (int64_t*)xcalloc((size_t)nu + 1, sizeof(int64_t));
    for (int64_t u = 0; u < nu; ++u) {
        int64_t a = h->iperm[h->ur[u]], b = h->iperm[h->uc[u]];
        h->sn_eptr[col2sn[a < b ? a : b] + 1]++;
    }
    for (int64_t s = 0; s < nsn; ++s) h->sn_eptr[s + 1] += h->sn_eptr[s];
    int64_t* fp = (int64_t*)xcalloc((size_t)nsn + 1, sizeof(int64_t));
    memcpy(fp, h->sn_eptr, sizeof(int64_t) * (size_t)nsn);
    for (int64_t u = 0; u < nu; ++u) {
        int64_t a = h->iperm[h->ur[u]], b = h->iperm[h->uc[u]];
        h->sn_ent[fp[col2sn[a < b ? a : b]]++] = u;
    }
    free(fp);
    h->analyzed = 1;
    return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* numerical factorization                                                                     */
/* ------------------------------------------------------------------------------------------ */

typedef struct {
    int64_t m, ndel;
    int64_t* vars;
    double* F; /* m x m full symmetric, row-major */
} cblock_t;

static void swap_sym(double* F, int64_t m, int64_t s, int64_t t, int64_t* vars) {
    if (s == t) return;
    for (int64_t j = 0; j < m; ++j) { double x = F[s * m + j]; F[s * m + j] = F[t * m + j]; F[t * m + j] = x; }
    for (int64_t i = 0; i < m; ++i) { double x = F[i * m + s]; F[i * m + s] = F[i * m + t]; F[i * m + t] = x; }
    int64_t v = vars[s]; vars[s] = vars[t]; vars[t] = v;
}

/* Threshold pivot test for candidate `c` at elimination step k (MUMPS/Duff-Reid rule).
 * Returns 0 none, 1 null, 2 1x1, 3 2x2 (partner in *r_out). */
static int test_pivot(const double* F, int64_t m, int64_t k, int64_t nfs, int64_t c, double u, double thres,
                      int64_t* r_out) {
    double acc = fabs(F[c * m + c]);
    double gamma = 0.0, rmax = 0.0;
    int64_t r = -1;
    for (int64_t i = k; i < m; ++i) {
        if (i == c) continue;
        double v = fabs(F[i * m + c]);
        if (v > gamma) gamma = v;
        if (i < nfs && v > rmax) { rmax = v; r = i; }
    }
    if ((acc > gamma ? acc : gamma) <= thres) return 1;
    if (acc != 0.0 && acc >= u * gamma) return 2;
    if (r >= 0 && rmax > 0.0) {
        double gc = 0.0, gr = 0.0;
        for (int64_t i = k; i < m; ++i) {
            if (i == c || i == r) continue;
            double vc = fabs(F[i * m + c]), vr = fabs(F[i * m + r]);
            if (vc > gc) gc = vc;
            if (vr > gr) gr = vr;
        }
        double a = F[c * m + c], b = F[r * m + c], d = F[r * m + r];
        double det = a * d - b * b;
        if (det != 0.0) {
            double lim = u > 0 ? fabs(det) / u : INFINITY;
            if (fabs(d) * gc + fabs(b) * gr <= lim && fabs(b) * gc + fabs(a) * gr <= lim) {
                *r_out = r;
                return 3;
            }
        }
    }
    return 0;
}

static void elim_1x1(double* F, int64_t m, int64_t k, double* colv) {
    double d = F[k * m + k];
    for (int64_t i = k + 1; i < m; ++i) colv[i] = F[i * m + k];
    for (int64_t i = k + 1; i < m; ++i) {
        double li = colv[i] / d;
        double* Fi = F + i * m;
        for (int64_t j = k + 1; j <= i; ++j) Fi[j] -= li * colv[j];
    }
    for (int64_t i = k + 1; i < m; ++i) {
        F[i * m + k] = colv[i] / d;
        for (int64_t j = k + 1; j < i; ++j) F[j * m + i] = F[i * m + j];
    }
}

static void elim_2x2(double* F, int64_t m, int64_t k, double* c0, double* c1) {
    double a = F[k * m + k], b = F[(k + 1) * m + k], d = F[(k + 1) * m + k + 1];
    double det = a * d - b * b;
    for (int64_t i = k + 2; i < m; ++i) { c0[i] = F[i * m + k]; c1[i] = F[i * m + k + 1]; }
    for (int64_t i = k + 2; i < m; ++i) {
        double l0 = (d * c0[i] - b * c1[i]) / det;
        double l1 = (a * c1[i] - b * c0[i]) / det;
        double* Fi = F + i * m;
        for (int64_t j = k + 2; j <= i; ++j) Fi[j] -= l0 * c0[j] + l1 * c1[j];
    }
    for (int64_t i = k + 2; i < m; ++i) {
        F[i * m + k] = (d * c0[i] - b * c1[i]) / det;
        F[i * m + k + 1] = (a * c1[i] - b * c0[i]) / det;
        for (int64_t j = k + 2; j < i; ++j) F[j * m + i] = F[i * m + j];
    }
}

int oracle_kkt_factorize(oracle_kkt_t h, const double* values) {
    if (!h->analyzed) return fail(h, "factorize before analyze");
    free_numeric(h);
    const int64_t n = h->n, nu = h->nu, nsn = h->nsn;
    h->err[0] = 0;

    /* sum duplicates in COO order (COOFormat keeps duplicates; MUMPS sums them) */
    h->uval = (double*)xcalloc((size_t)nu + 1, sizeof(double));
    for (int64_t u = 0; u < nu; ++u) {
        double s = 0.0;
        for (int64_t q = h->dup_ptr[u]; q < h->dup_ptr[u + 1]; ++q) s += values[h->dup_pos[q]];
        h->uval[u] = s;
    }
    /* symmetric infinity-norm equilibration (ICNTL(8)=8 restated) */
    double* s = (double*)xcalloc((size_t)n + 1, sizeof(double));
    double* r = (double*)xcalloc((size_t)n + 1, sizeof(double));
    for (int64_t i = 0; i < n; ++i) s[i] = 1.0;
    for (int it = 0; it < h->scale_iters; ++it) {
        for (int64_t i = 0; i < n; ++i) r[i] = 0.0;
        for (int64_t u = 0; u < nu; ++u) {
            int64_t a = h->ur[u], b = h->uc[u];
            double w = fabs(s[a] * h->uval[u] * s[b]);
            if (w > r[a]) r[a] = w;
            if (w > r[b]) r[b] = w;
        }
        for (int64_t i = 0; i < n; ++i) if (r[i] > 0.0) s[i] = s[i] / sqrt(r[i]);
    }
    h->scale = s;
    /* ||A_pre||_inf of the scaled matrix, null-pivot threshold */
    for (int64_t i = 0; i < n; ++i) r[i] = 0.0;
    double* sv = (double*)xcalloc((size_t)nu + 1, sizeof(double));
    for (int64_t u = 0; u < nu; ++u) {
        int64_t a = h->ur[u], b = h->uc[u];
        sv[u] = s[a] * h->uval[u] * s[b];
        r[a] += fabs(sv[u]);
        if (a != b) r[b] += fabs(sv[u]);
    }
    double anorm = 0.0;
    for (int64_t i = 0; i < n; ++i) if (r[i] > anorm) anorm = r[i];
    h->thres = DBL_EPSILON * h->null_fac * anorm;
    free(r);

    h->f_m = (int64_t*)xcalloc((size_t)nsn + 1, sizeof(int64_t));
    h->f_npiv = (int64_t*)xcalloc((size_t)nsn + 1, sizeof(int64_t));
    h->f_vars = (int64_t**)xcalloc((size_t)nsn + 1, sizeof(int64_t*));
    h->f_L = (double**)xcalloc((size_t)nsn + 1, sizeof(double*));
    h->f_piv = (signed char**)xcalloc((size_t)nsn + 1, sizeof(signed char*));
    cblock_t* cb = (cblock_t*)xcalloc((size_t)nsn + 1, sizeof(cblock_t));
    int64_t* loc = (int64_t*)xcalloc((size_t)n + 1, sizeof(int64_t));
    for (int64_t i = 0; i < n; ++i) loc[i] = -1;
    /* children lists of the assembly tree */
    int64_t* chead = (int64_t*)xcalloc((size_t)nsn + 1, sizeof(int64_t));
    int64_t* cnext = (int64_t*)xcalloc((size_t)nsn + 1, sizeof(int64_t));
    for (int64_t t = 0; t < nsn; ++t) chead[t] = -1;
    for (int64_t t = nsn - 1; t >= 0; --t)
        if (h->sn_parent[t] >= 0) { cnext[t] = chead[h->sn_parent[t]]; chead[h->sn_parent[t]] = t; }

    h->npos = h->nneg = h->nzero = 0;
    memset(h->stats, 0, sizeof(h->stats));
    int64_t nnzL = 0, n2x2 = 0, ndelay = 0, nnull = 0, maxm = 0;
    double flops = 0.0;
    int status = 0;
    const double ulist_root[] = {h->u, h->u * 0.1, h->u * 0.01, 1e-6, 1e-10, 0.0};

    for (int64_t t = 0; t < nsn && status == 0; ++t) {
        int64_t width = h->sn_first[t + 1] - h->sn_first[t];
        int64_t slen = h->sn_sptr[t + 1] - h->sn_sptr[t];
        int64_t ndel = 0;
        for (int64_t c = chead[t]; c >= 0; c = cnext[c]) ndel += cb[c].ndel;
        int64_t nfs = ndel + width, m = nfs + slen;
        if (m > maxm) maxm = m;
        int64_t* vars = (int64_t*)xcalloc((size_t)m + 1, sizeof(int64_t));
        int64_t q = 0;
        for (int64_t c = chead[t]; c >= 0; c = cnext[c])
            for (int64_t a = 0; a < cb[c].ndel; ++a) vars[q++] = cb[c].vars[a];
        for (int64_t j = h->sn_first[t]; j < h->sn_first[t + 1]; ++j) vars[q++] = j;
        for (int64_t a = 0; a < slen; ++a) vars[q++] = h->sn_struct[h->sn_sptr[t] + a];
        for (int64_t a = 0; a < m; ++a) loc[vars[a]] = a;
        double* F = (double*)xcalloc((size_t)(m * m) + 1, sizeof(double));
        /* assemble original entries */
        for (int64_t e = h->sn_eptr[t]; e < h->sn_eptr[t + 1]; ++e) {
            int64_t u = h->sn_ent[e];
            int64_t pa = loc[h->iperm[h->ur[u]]], pb = loc[h->iperm[h->uc[u]]];
            F[pa * m + pb] += sv[u];
            if (pa != pb) F[pb * m + pa] += sv[u];
        }
        /* extend-add children contribution blocks */
        for (int64_t c = chead[t]; c >= 0; c = cnext[c]) {
            int64_t cm = cb[c].m;
            for (int64_t a = 0; a < cm; ++a) {
                int64_t pa = loc[cb[c].vars[a]];
                for (int64_t b = 0; b < cm; ++b) F[pa * m + loc[cb[c].vars[b]]] += cb[c].F[a * cm + b];
            }
            free(cb[c].F); free(cb[c].vars); cb[c].F = NULL; cb[c].vars = NULL;
        }
        /* eliminate */
        signed char* piv = (signed char*)xcalloc((size_t)m + 1, 1);
        double* c0 = (double*)xcalloc((size_t)m + 1, sizeof(double));
        double* c1 = (double*)xcalloc((size_t)m + 1, sizeof(double));
        int is_root = h->sn_parent[t] < 0;
        int64_t k = 0;
        while (k < nfs) {
            int found = 0;
            int nu_try = is_root ? (int)(sizeof(ulist_root) / sizeof(double)) : 1;
            for (int ut = 0; ut < nu_try && !found; ++ut) {
                double uu = ulist_root[ut];
                for (int64_t c = k; c < nfs && !found; ++c) {
                    int64_t rr = -1;
                    int kind = test_pivot(F, m, k, nfs, c, uu, h->thres, &rr);
                    if (kind == 0) continue;
                    found = 1;
                    swap_sym(F, m, k, c, vars);
                    int64_t rem;
                    if (kind == 1) {
                        for (int64_t i = k + 1; i < m; ++i) { F[i * m + k] = 0.0; F[k * m + i] = 0.0; }
                        piv[k] = PIV_NULL; h->nzero++; nnull++;
                        k += 1;
                    } else if (kind == 2) {
                        rem = m - k - 1;
                        elim_1x1(F, m, k, c0);
                        piv[k] = PIV_1X1;
                        if (F[k * m + k] > 0) h->npos++; else h->nneg++;
                        flops += (double)rem + (double)rem * (double)(rem + 1);
                        nnzL += rem;
                        k += 1;
                    } else {
                        if (rr == k) rr = c; /* candidate moved into k's old slot */
                        swap_sym(F, m, k + 1, rr, vars);
                        rem = m - k - 2;
                        elim_2x2(F, m, k, c0, c1);
                        piv[k] = PIV_2X2_A; piv[k + 1] = PIV_2X2_B;
                        double a = F[k * m + k], b = F[(k + 1) * m + k], d = F[(k + 1) * m + k + 1];
                        double det = a * d - b * b;
                        if (det < 0) { h->npos++; h->nneg++; }
                        else if (a + d > 0) h->npos += 2;
                        else h->nneg += 2;
                        n2x2++;
                        flops += 6.0 * (double)rem + 2.0 * (double)rem * (double)(rem + 1);
                        nnzL += 2 * rem + 1;
                        k += 2;
                    }
                }
            }
            if (!found) break; /* remaining fully-summed columns are delayed */
        }
        if (k < nfs && is_root) { status = fail(h, "root front could not be eliminated"); }
        ndelay += nfs - k;
        /* keep L (first k columns) for the solve */
        double* L = (double*)xcalloc((size_t)(m * (k > 0 ? k : 1)), sizeof(double));
        for (int64_t j = 0; j < k; ++j)
            for (int64_t i = 0; i < m; ++i) L[j * m + i] = F[i * m + j];
        h->f_m[t] = m; h->f_npiv[t] = k; h->f_L[t] = L; h->f_piv[t] = piv;
        h->f_vars[t] = (int64_t*)xcalloc((size_t)m + 1, sizeof(int64_t));
        memcpy(h->f_vars[t], vars, sizeof(int64_t) * (size_t)m);
        /* contribution block */
        int64_t cm = m - k;
        cb[t].m = cm; cb[t].ndel = nfs - k;
        cb[t].vars = (int64_t*)xcalloc((size_t)cm + 1, sizeof(int64_t));
        cb[t].F = (double*)xcalloc((size_t)(cm * cm) + 1, sizeof(double));
        for (int64_t a = 0; a < cm; ++a) {
            cb[t].vars[a] = vars[k + a];
            for (int64_t b = 0; b < cm; ++b) cb[t].F[a * cm + b] = F[(k + a) * m + k + b];
        }
        for (int64_t a = 0; a < m; ++a) loc[vars[a]] = -1;
        free(F); free(vars); free(c0); free(c1);
    }
    for (int64_t t = 0; t < nsn; ++t) { free(cb[t].F); free(cb[t].vars); }
    free(cb); free(loc); free(chead); free(cnext); free(sv);
    h->stats[0] = (double)nnzL; h->stats[1] = (double)nsn; h->stats[2] = (double)n2x2;
    h->stats[3] = (double)ndelay; h->stats[4] = (double)nnull; h->stats[5] = flops; h->stats[6] = (double)maxm;
    if (status) return status;
    h->factored = 1;
    return 0;
}

int oracle_kkt_inertia(oracle_kkt_t h, int64_t* pos, int64_t* neg, int64_t* zero) {
    if (!h->factored) return fail(h, "inertia before factorize");
    *pos = h->npos; *neg = h->nneg; *zero = h->nzero;
    return 0;
}

int oracle_kkt_scaling(oracle_kkt_t h, double* scale, double* thres) {
    if (!h->factored) return fail(h, "scaling before factorize");
    memcpy(scale, h->scale, sizeof(double) * (size_t)h->n);
    *thres = h->thres;
    return 0;
}

int oracle_kkt_stats(oracle_kkt_t h, double* out7) {
    memcpy(out7, h->stats, sizeof(h->stats));
    return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* solve                                                                                       */
/* ------------------------------------------------------------------------------------------ */

int oracle_kkt_solve(oracle_kkt_t h, const double* rhs, double* x) {
    if (!h->factored) return fail(h, "solve before factorize");
    const int64_t n = h->n, nsn = h->nsn;
    double* w = (double*)xcalloc((size_t)n + 1, sizeof(double));
    for (int64_t i = 0; i < n; ++i) w[h->iperm[i]] = h->scale[i] * rhs[i];
    /* forward: L y = b */
    for (int64_t t = 0; t < nsn; ++t) {
        const int64_t m = h->f_m[t], np = h->f_npiv[t];
        const int64_t* v = h->f_vars[t];
        const double* L = h->f_L[t];
        const signed char* piv = h->f_piv[t];
        for (int64_t c = 0; c < np; ++c) {
            if (piv[c] == PIV_1X1) {
                double y = w[v[c]];
                for (int64_t i = c + 1; i < m; ++i) w[v[i]] -= L[c * m + i] * y;
            } else if (piv[c] == PIV_2X2_A) {
                double y0 = w[v[c]], y1 = w[v[c + 1]];
                for (int64_t i = c + 2; i < m; ++i) w[v[i]] -= L[c * m + i] * y0 + L[(c + 1) * m + i] * y1;
                c++;
            }
        }
    }
    /* diagonal: D z = y (null pivots contribute 0) */
    for (int64_t t = 0; t < nsn; ++t) {
        const int64_t m = h->f_m[t], np = h->f_npiv[t];
        const int64_t* v = h->f_vars[t];
        const double* L = h->f_L[t];
        const signed char* piv = h->f_piv[t];
        for (int64_t c = 0; c < np; ++c) {
            if (piv[c] == PIV_NULL) w[v[c]] = 0.0;
            else if (piv[c] == PIV_1X1) w[v[c]] /= L[c * m + c];
            else if (piv[c] == PIV_2X2_A) {
                double a = L[c * m + c], b = L[c * m + c + 1], d = L[(c + 1) * m + c + 1];
                double det = a * d - b * b;
                double y0 = w[v[c]], y1 = w[v[c + 1]];
                w[v[c]] = (d * y0 - b * y1) / det;
                w[v[c + 1]] = (a * y1 - b * y0) / det;
                c++;
            }
        }
    }
    /* backward: L^T x = z */
    for (int64_t t = nsn - 1; t >= 0; --t) {
        const int64_t m = h->f_m[t], np = h->f_npiv[t];
        const int64_t* v = h->f_vars[t];
        const double* L = h->f_L[t];
        const signed char* piv = h->f_piv[t];
        for (int64_t c = np - 1; c >= 0; --c) {
            if (piv[c] == PIV_1X1) {
                double acc = 0.0;
                for (int64_t i = c + 1; i < m; ++i) acc += L[c * m + i] * w[v[i]];
                w[v[c]] -= acc;
            } else if (piv[c] == PIV_2X2_B) {
                int64_t c0 = c - 1;
                double a0 = 0.0, a1 = 0.0;
                for (int64_t i = c + 1; i < m; ++i) { a0 += L[c0 * m + i] * w[v[i]]; a1 += L[c * m + i] * w[v[i]]; }
                w[v[c0]] -= a0; w[v[c]] -= a1;
                c--;
            }
        }
    }
    for (int64_t i = 0; i < n; ++i) x[i] = h->scale[i] * w[h->iperm[i]];
    free(w);
    return 0;
}
