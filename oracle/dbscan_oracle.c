/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into, loaded by, or called
 * from the product path (pypardis_amd/); only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg use it, as the checker.
 *
 * Plain-C restatement of the arithmetic the reference delegates to
 * scikit-learn 1.7.2 inside dbscan_partition (R:dbscan/dbscan.py:28-30):
 *
 *   sklearn.cluster.DBSCAN(eps, min_samples, metric, algorithm='kd_tree').fit
 *     SK:cluster/_dbscan.py:410-446
 *   radius query, kd_tree leaf predicate      SK:neighbors/_binary_tree.pxi.tp:1949-1958
 *     euclidean: rdist = sum_j (x_j - y_j)^2, fp64, j ascending, no FMA,
 *                accepted iff rdist <= eps*eps      SK:metrics/_dist_metrics.pxd.tp:39-53
 *     cityblock: sum_j |x_j - y_j| <= eps
 *   core  = (neighbour count incl. self) >= min_samples   SK:cluster/_dbscan.py:423-434
 *   labels = depth-first expansion in index order           SK:cluster/_dbscan_inner.pyx:11-41
 *
 * Pinned against sklearn itself and the shim-run reference by
 * the fixtures in tests/golden/ (see tests/test_oracle.py).
 *
 * Neighbour search is deliberately NOT the GPU's: candidates come from a sort
 * along axis 0 and a window sweep of half-width eps*(1+2^-20), so the oracle
 * shares no binning logic with the HIP kernels it checks.
 *
 * Build: gcc -O2 -ffp-contract=off -fPIC -shared (oracle/Makefile).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    double key;
    int64_t idx;
} kv_t;

static int kv_cmp(const void* a, const void* b) {
    const kv_t* x = (const kv_t*)a;
    const kv_t* y = (const kv_t*)b;
    if (x->key < y->key) return -1;
    if (x->key > y->key) return 1;
    return (x->idx < y->idx) ? -1 : (x->idx > y->idx);
}

/* kd_tree leaf predicate (SK:neighbors/_binary_tree.pxi.tp:1951-1955). */
static inline int within(const double* a, const double* b, int d, double r,
                         double r2, int metric) {
    double acc = 0.0;
    if (metric == 0) {
        for (int j = 0; j < d; ++j) {
            double t = a[j] - b[j];
            double sq = t * t;     /* separate rounding: no contraction */
            acc = acc + sq;
        }
        return acc <= r2;
    }
    for (int j = 0; j < d; ++j) acc = acc + fabs(a[j] - b[j]);
    return acc <= r;
}

/* Sorted-axis-0 candidate enumeration.  For each point i (in sorted order
 * position p), candidates are sorted positions q with |x0_q - x0_i| <= w.
 * Calls visit(i, j) for every accepted neighbour j (self included). */
typedef void (*visit_fn)(void* ctx, int64_t i, int64_t j);

static int sweep(const double* X, int64_t n, int d, double eps, int metric,
                 void* ctx, visit_fn visit, const uint8_t* only) {
    kv_t* s = (kv_t*)malloc(sizeof(kv_t) * (size_t)(n > 0 ? n : 1));
    if (!s) return -1;
    for (int64_t i = 0; i < n; ++i) {
        s[i].key = X[i * d];
        s[i].idx = i;
    }
    qsort(s, (size_t)n, sizeof(kv_t), kv_cmp);
    const double r2 = eps * eps;
    const double w = eps * (1.0 + 1.0 / 1048576.0);
    int64_t lo = 0;
    for (int64_t p = 0; p < n; ++p) {
        const int64_t i = s[p].idx;
        const double x0 = s[p].key;
        while (s[lo].key < x0 - w) ++lo;
        if (only && !only[i]) continue;
        const double* a = X + i * d;
        for (int64_t q = lo; q < n && s[q].key <= x0 + w; ++q) {
            const int64_t j = s[q].idx;
            if (within(a, X + j * d, d, eps, r2, metric)) visit(ctx, i, j);
        }
    }
    free(s);
    return 0;
}

static void count_visit(void* ctx, int64_t i, int64_t j) {
    (void)j;
    ((int64_t*)ctx)[i] += 1;
}

typedef struct {
    int64_t* fill;      /* next write slot per point */
    int64_t* nbr;       /* CSR column array */
} csr_ctx;

static void csr_visit(void* ctx, int64_t i, int64_t j) {
    csr_ctx* c = (csr_ctx*)ctx;
    c->nbr[c->fill[i]++] = j;
}

/* Neighbour counts only (SK:cluster/_dbscan.py:421-427). */
int oracle_counts(const double* X, int64_t n, int32_t d, double eps,
                  int32_t metric, int64_t* counts) {
    memset(counts, 0, sizeof(int64_t) * (size_t)n);
    return sweep(X, n, d, eps, metric, counts, count_visit, NULL);
}

/* Full CSR neighbourhoods (radius_neighbors(X) of SK:cluster/_dbscan.py:421);
 * offsets has n+1 entries, nbr has offsets[n] entries, each row sorted. */
static int cmp_i64(const void* a, const void* b) {
    int64_t x = *(const int64_t*)a, y = *(const int64_t*)b;
    return (x > y) - (x < y);
}

int oracle_neighbors(const double* X, int64_t n, int32_t d, double eps,
                     int32_t metric, const int64_t* offsets, int64_t* nbr) {
    csr_ctx c;
    c.fill = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
    if (!c.fill) return -1;
    memcpy(c.fill, offsets, sizeof(int64_t) * (size_t)n);
    c.nbr = nbr;
    int rc = sweep(X, n, d, eps, metric, &c, csr_visit, NULL);
    free(c.fill);
    for (int64_t i = 0; rc == 0 && i < n; ++i)
        qsort(nbr + offsets[i], (size_t)(offsets[i + 1] - offsets[i]),
              sizeof(int64_t), cmp_i64);
    return rc;
}

/* Neighbour counts of nq query points against a candidate set (brute force,
 * same predicate), stopping at `cap` (cap <= 0: no cap).  Used by the
 * windowed full-size checks where a window is too dense for the sweep: with
 * the candidates = every point within eps of the queries, out = min(count,
 * cap) exactly (SK:cluster/_dbscan.py:421-434, the count the core test uses). */
int oracle_counts_capped(const double* Q, int64_t nq, const double* C, int64_t nc, int32_t d,
                         double eps, int32_t metric, int64_t cap, int64_t* out) {
    const double r2 = eps * eps;
    for (int64_t i = 0; i < nq; ++i) {
        int64_t c = 0;
        for (int64_t j = 0; j < nc; ++j) {
            if (within(Q + i * d, C + j * d, d, eps, r2, metric)) {
                ++c;
                if (cap > 0 && c >= cap) break;
            }
        }
        out[i] = c;
    }
    return 0;
}

/* DBSCAN.fit: counts -> core -> dbscan_inner DFS.  labels int64[n],
 * core uint8[n], counts int64[n].  Returns number of clusters (>= 0) or -1. */
int64_t oracle_dbscan(const double* X, int64_t n, int32_t d, double eps,
                      int64_t min_samples, int32_t metric, int64_t* labels,
                      uint8_t* core, int64_t* counts) {
    if (oracle_counts(X, n, d, eps, metric, counts) != 0) return -1;
    for (int64_t i = 0; i < n; ++i) core[i] = counts[i] >= min_samples;
    /* neighbourhoods of core points only: the DFS never expands others */
    int64_t* off = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n + 1));
    if (!off) return -1;
    off[0] = 0;
    for (int64_t i = 0; i < n; ++i) off[i + 1] = off[i] + (core[i] ? counts[i] : 0);
    int64_t* nbr = (int64_t*)malloc(sizeof(int64_t) * (size_t)(off[n] > 0 ? off[n] : 1));
    int64_t* stack = (int64_t*)malloc(sizeof(int64_t) * (size_t)(off[n] + n + 1));
    if (!nbr || !stack) { free(off); free(nbr); free(stack); return -1; }
    csr_ctx c;
    c.fill = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
    if (!c.fill) { free(off); free(nbr); free(stack); return -1; }
    memcpy(c.fill, off, sizeof(int64_t) * (size_t)n);
    c.nbr = nbr;
    if (sweep(X, n, d, eps, metric, &c, csr_visit, core) != 0) {
        free(off); free(nbr); free(stack); free(c.fill);
        return -1;
    }
    free(c.fill);

    /* SK:cluster/_dbscan_inner.pyx:19-41 */
    for (int64_t i = 0; i < n; ++i) labels[i] = -1;
    int64_t label_num = 0;
    for (int64_t s = 0; s < n; ++s) {
        if (labels[s] != -1 || !core[s]) continue;
        int64_t top = 0;
        int64_t i = s;
        for (;;) {
            if (labels[i] == -1) {
                labels[i] = label_num;
                if (core[i]) {
                    for (int64_t q = off[i]; q < off[i + 1]; ++q) {
                        int64_t v = nbr[q];
                        if (labels[v] == -1) stack[top++] = v;
                    }
                }
            }
            if (top == 0) break;
            i = stack[--top];
        }
        ++label_num;
    }
    free(off); free(nbr); free(stack);
    return label_num;
}
