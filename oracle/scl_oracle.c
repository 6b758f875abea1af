/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C restatement of the reference's polar SC/SCL algorithms (heimrih/polar_code,
 * package dl_scl_polar), used by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg as the CHECKER / CPU baseline.  Nothing in polar_code_amd/ links,
 * loads or calls this file; the product path is the HIP library (libpolar_mi355x.so).
 *
 * Pinned against golden vectors produced by running the reference itself in the survey
 * container (tests/golden/make_golden.py -> tests/golden/*.npz; tests/test_oracle_golden.py).
 *
 * Arithmetic follows the reference exactly:
 *   f(a,b) = sign(a) sign(b) min(|a|,|b|)              polar.py:122-123
 *   g(a,b,c) = b + (1-2c) a                           polar.py:126-127
 *   metric += logaddexp(0, bit ? llr : -llr)          scl.py:102-105 (numpy npy_logaddexp,
 *            computed here with the platform libm exp/log1p, as numpy does)
 *   list: frozen -> bit 0; forced -> one child; free -> children (bit0, bit1) in list order;
 *         Python-stable sort by metric; keep first M       scl.py:133-174
 * The LLR values equal the reference's recompute-from-root schedule (_ensure_alpha,
 * scl.py:64-78) because every ancestor depends only on the channel LLRs and on
 * left-sibling partial sums that are final once written; this file evaluates each node
 * once per path (standard SC schedule), which produces the same doubles.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define OR_MAXN 1024
#define OR_MAXM 64

/* ------------------------------------------------------------------ CRC (crc.py) */

/* _poly_to_bits crc.py:10-16: MSB-first bits of the hex value; returns degree. */
static int poly_bits(uint64_t poly, uint8_t* bits) {
    int len = 0;
    for (uint64_t v = poly; v; v >>= 1) len++;
    for (int i = 0; i < len; i++) bits[i] = (uint8_t)((poly >> (len - 1 - i)) & 1);
    return len - 1;
}

/* attach_crc crc.py:19-37. out has len+deg entries. returns deg or -1. */
int oracle_attach_crc(const int8_t* msg, int len, uint64_t poly, int8_t* out) {
    uint8_t pb[65];
    int deg = poly_bits(poly, pb);
    if (deg <= 0) return -1;
    uint8_t* buf = (uint8_t*)calloc((size_t)(len + deg), 1);
    for (int i = 0; i < len; i++) buf[i] = (uint8_t)(msg[i] & 1);
    for (int i = 0; i < len; i++) {
        if (!buf[i]) continue;
        for (int j = 0; j <= deg; j++) buf[i + j] ^= pb[j];
    }
    for (int i = 0; i < len; i++) out[i] = (int8_t)(msg[i] & 1);
    for (int j = 0; j < deg; j++) out[len + j] = (int8_t)buf[len + j];
    free(buf);
    return deg;
}

/* check_crc crc.py:40-56. returns 1 pass, 0 fail, -1 error (too short). */
int oracle_check_crc(const int8_t* msg, int len, uint64_t poly) {
    uint8_t pb[65];
    int deg = poly_bits(poly, pb);
    if (len <= deg) return -1;
    uint8_t buf[OR_MAXN + 65];
    for (int i = 0; i < len; i++) buf[i] = (uint8_t)(msg[i] & 1);
    for (int i = 0; i < len - deg; i++) {
        if (!buf[i]) continue;
        for (int j = 0; j <= deg; j++) buf[i + j] ^= pb[j];
    }
    for (int j = 0; j < deg; j++)
        if (buf[len - deg + j]) return 0;
    return 1;
}

/* ------------------------------------------------------------ polar core (polar.py) */

/* _polar_transform polar.py:17-29 (in place). */
void oracle_polar_transform(int8_t* x, int N) {
    for (int step = 1; step < N; step <<= 1)
        for (int start = 0; start < N; start += 2 * step)
            for (int i = 0; i < step; i++) x[start + i] ^= x[start + step + i];
}

static double phi_inv(double x) { /* polar.py:51-58 */
    if (x > 12.0) return 0.9861 * x - 2.3152;
    if (x > 3.5) return x * (0.009005 * x + 0.7694) - 0.9507;
    if (x > 1.0) return x * (0.062883 * x + 0.3678) - 0.1627;
    return x * (0.2202 * x + 0.06448);
}

/* construct_info_set(N, K, "gaussian", design_snr_db) polar.py:61-103. */
int oracle_construct_info_set(int N, int K, double design_snr_db, int32_t* info) {
    if (N <= 0 || (N & (N - 1)) || K <= 0 || K > N || N > OR_MAXN) return -1;
    double rate = (double)K / N;
    double snr = pow(10.0, design_snr_db / 10.0);
    double sigma_sq = 1.0 / (2.0 * rate * snr);
    double m[OR_MAXN], pe[OR_MAXN];
    memset(m, 0, sizeof(m));
    m[0] = 2.0 / sigma_sq;
    int stages = 0;
    while ((1 << stages) < N) stages++;
    for (int level = 1; level <= stages; level++) {
        int half = (1 << level) >> 1;
        for (int j = 0; j < half; j++) {
            double T = m[j];
            m[j] = phi_inv(T);
            m[half + j] = 2.0 * T;
        }
    }
    for (int i = 0; i < N; i++) {
        double val = m[i] > 1e-12 ? m[i] : 1e-12;
        pe[i] = 0.5 - 0.5 * erf(sqrt(val) / 2.0);
    }
    /* stable argsort of pe, first K, sorted */
    int order[OR_MAXN];
    for (int i = 0; i < N; i++) order[i] = i;
    for (int i = 1; i < N; i++) { /* insertion sort: stable */
        int v = order[i], j = i - 1;
        while (j >= 0 && pe[order[j]] > pe[v]) {
            order[j + 1] = order[j];
            j--;
        }
        order[j + 1] = v;
    }
    uint8_t sel[OR_MAXN];
    memset(sel, 0, sizeof(sel));
    for (int i = 0; i < K; i++) sel[order[i]] = 1;
    int k = 0;
    for (int i = 0; i < N; i++)
        if (sel[i]) info[k++] = i;
    return 0;
}

static inline double f_fn(double a, double b) { /* polar.py:122-123 */
    double sa = (a > 0) - (a < 0), sb = (b > 0) - (b < 0);
    double aa = fabs(a), ab = fabs(b);
    return sa * sb * (aa < ab ? aa : ab);
}

static inline double g_fn(double a, double b, int c) { /* polar.py:126-127 */
    return b + (double)(1 - 2 * c) * a;
}

/* sc_decode polar.py:130-168 (recursive, hard decisions llr < 0). */
static void sc_rec(const double* llr, int w, int start, const uint8_t* frozen, int8_t* u_hat,
                   int8_t* out_bits) {
    if (w == 1) {
        int8_t bit = frozen[start] ? 0 : (int8_t)(llr[0] < 0);
        u_hat[start] = bit;
        out_bits[0] = bit;
        return;
    }
    int h = w / 2;
    double* tmp = (double*)malloc(sizeof(double) * (size_t)h);
    int8_t* lb = (int8_t*)malloc((size_t)h);
    int8_t* rb = (int8_t*)malloc((size_t)h);
    for (int i = 0; i < h; i++) tmp[i] = f_fn(llr[i], llr[h + i]);
    sc_rec(tmp, h, start, frozen, u_hat, lb);
    for (int i = 0; i < h; i++) tmp[i] = g_fn(llr[i], llr[h + i], lb[i]);
    sc_rec(tmp, h, start + h, frozen, u_hat, rb);
    for (int i = 0; i < h; i++) {
        out_bits[i] = lb[i] ^ rb[i];
        out_bits[h + i] = rb[i];
    }
    free(tmp);
    free(lb);
    free(rb);
}

int oracle_sc_decode(const double* llr, int N, const int32_t* info, int K, int8_t* out) {
    if (N <= 0 || (N & (N - 1)) || N > OR_MAXN) return -1;
    uint8_t frozen[OR_MAXN];
    for (int i = 0; i < N; i++) frozen[i] = 1;
    for (int i = 0; i < K; i++) {
        if (info[i] < 0 || info[i] >= N) return -2;
        frozen[info[i]] = 0;
    }
    int8_t u_hat[OR_MAXN], bits[OR_MAXN];
    memset(u_hat, 0, sizeof(u_hat));
    sc_rec(llr, N, 0, frozen, u_hat, bits);
    for (int i = 0; i < K; i++) out[i] = u_hat[info[i]];
    return 0;
}

/* --------------------------------------------------------------------- SCL (scl.py) */

/* np.logaddexp(0.0, v) via npy_logaddexp with libm exp/log1p. */
static inline double logaddexp0(double v) {
    const double x = 0.0, y = v;
    if (x == y) return x + 0.693147180559945309417232121458176568;
    double tmp = x - y;
    if (tmp > 0) return x + log1p(exp(-tmp));
    if (tmp <= 0) return y + log1p(exp(tmp));
    return tmp;
}

typedef struct {
    double* alpha;  /* depths 1..n: offsets off[d], width N>>d */
    uint8_t* bleft; /* left-sibling partial sums per depth, same layout */
    int8_t* u;      /* decided bits, N */
    double* illr;   /* decision LLR at each info phase, K */
    int n_illr;
    double metric;
} opath;

typedef struct {
    int N, n, K;
    int off[12];
    int alen; /* total alpha entries for depths 1..n */
} otree;

static void path_alloc(opath* p, const otree* t) {
    p->alpha = (double*)malloc(sizeof(double) * (size_t)t->alen);
    p->bleft = (uint8_t*)malloc((size_t)t->alen);
    p->u = (int8_t*)malloc((size_t)t->N);
    p->illr = (double*)malloc(sizeof(double) * (size_t)(t->K > 0 ? t->K : 1));
}

static void path_free(opath* p) {
    free(p->alpha);
    free(p->bleft);
    free(p->u);
    free(p->illr);
}

static void path_copy(opath* dst, const opath* src, const otree* t) {
    memcpy(dst->alpha, src->alpha, sizeof(double) * (size_t)t->alen);
    memcpy(dst->bleft, src->bleft, (size_t)t->alen);
    memcpy(dst->u, src->u, (size_t)t->N);
    memcpy(dst->illr, src->illr, sizeof(double) * (size_t)src->n_illr);
    dst->n_illr = src->n_illr;
    dst->metric = src->metric;
}

/* leaf LLR at phase phi (standard SC schedule == scl.py:_ensure_alpha values) */
static double path_leaf_llr(opath* p, const double* ch, const otree* t, int phi) {
    int n = t->n;
    int start;
    if (phi == 0) {
        start = 1;
    } else {
        int tz = 0;
        while (!((phi >> tz) & 1)) tz++;
        start = n - tz;
    }
    for (int d = start; d <= n; d++) {
        int w = t->N >> d;
        const double* par = (d == 1) ? ch : p->alpha + t->off[d - 1];
        double* out = p->alpha + t->off[d];
        if (d == start && phi != 0) {
            const uint8_t* c = p->bleft + t->off[d];
            for (int e = 0; e < w; e++) out[e] = g_fn(par[e], par[w + e], c[e]);
        } else {
            for (int e = 0; e < w; e++) out[e] = f_fn(par[e], par[w + e]);
        }
    }
    return p->alpha[t->off[n]];
}

/* set_bit scl.py:84-99 equivalent: propagate partial sums of completed right children */
static void path_set_bit(opath* p, const otree* t, int phi, int bit) {
    int n = t->n;
    uint8_t cur[OR_MAXN], nxt[OR_MAXN];
    p->u[phi] = (int8_t)(bit & 1);
    cur[0] = (uint8_t)(bit & 1);
    int w = 1;
    for (int d = n; d >= 1; d--) {
        int node = phi >> (n - d);
        if ((node & 1) == 0) { /* left child completed: remember for the sibling's g */
            memcpy(p->bleft + t->off[d], cur, (size_t)w);
            return;
        }
        const uint8_t* l = p->bleft + t->off[d];
        for (int e = 0; e < w; e++) {
            nxt[e] = l[e] ^ cur[e];
            nxt[w + e] = cur[e];
        }
        w *= 2;
        memcpy(cur, nxt, (size_t)w);
    }
}

/*
 * decode_scl scl.py:108-209.
 * force: NULL or K entries in {-1,0,1}.  crc_poly: 0 = no CRC.
 * Outputs (M-major, only n_out rows written):
 *   cands[M*K], metrics[M], info_llrs[M*K] (may be NULL), best_index (-1 if none).
 * Returns number of surviving paths (>0), or negative error:
 *   -1 bad args, -2 bad force value, -3 all paths pruned.
 */
int oracle_decode_scl(const double* llr, int N, const int32_t* info, int K, int M, uint64_t crc_poly,
                      const int8_t* force, int8_t* cands, double* metrics, double* info_llrs,
                      int32_t* best_index) {
    if (M <= 0 || M > OR_MAXM || N <= 1 || (N & (N - 1)) || N > OR_MAXN) return -1;
    otree t;
    t.N = N;
    t.K = K;
    t.n = 0;
    while ((1 << t.n) < N) t.n++;
    t.off[0] = 0;
    int acc = 0;
    for (int d = 1; d <= t.n; d++) {
        t.off[d] = acc;
        acc += N >> d;
    }
    t.alen = acc;
    uint8_t is_info[OR_MAXN];
    memset(is_info, 0, sizeof(is_info));
    for (int i = 0; i < K; i++) {
        if (info[i] < 0 || info[i] >= N) return -1;
        is_info[info[i]] = 1;
    }
    int cap = 2 * M;
    opath* pool = (opath*)malloc(sizeof(opath) * (size_t)(2 * cap));
    for (int i = 0; i < 2 * cap; i++) path_alloc(&pool[i], &t);
    opath* cur[2 * OR_MAXM];
    opath* nxt[2 * OR_MAXM];
    opath* freel[4 * OR_MAXM];
    int nfree = 0;
    for (int i = 1; i < 2 * cap; i++) freel[nfree++] = &pool[i];
    int count = 1;
    cur[0] = &pool[0];
    memset(cur[0]->alpha, 0, sizeof(double) * (size_t)t.alen);
    memset(cur[0]->bleft, 0, (size_t)t.alen);
    memset(cur[0]->u, 0, (size_t)N);
    cur[0]->n_illr = 0;
    cur[0]->metric = 0.0;
    int info_index = 0;
    int rc = 0;
    for (int phi = 0; phi < N; phi++) {
        int frozen = !is_info[phi];
        int forced = -1;
        if (!frozen && force) {
            int v = force[info_index];
            if (v == 0 || v == 1)
                forced = v;
            else if (v != -1) {
                rc = -2;
                goto done;
            }
        }
        int nn = 0;
        for (int i = 0; i < count; i++) {
            opath* p = cur[i];
            double lv = path_leaf_llr(p, llr, &t, phi);
            if (frozen) {
                p->metric = p->metric + logaddexp0(-lv);
                path_set_bit(p, &t, phi, 0);
                nxt[nn++] = p;
            } else if (forced >= 0) {
                p->metric = p->metric + logaddexp0(forced ? lv : -lv);
                path_set_bit(p, &t, phi, forced);
                p->illr[p->n_illr++] = lv;
                nxt[nn++] = p;
            } else {
                opath* b1 = freel[--nfree];
                path_copy(b1, p, &t);
                /* bit 0 reuses p (clone semantics: both children are independent copies) */
                p->metric = p->metric + logaddexp0(-lv);
                path_set_bit(p, &t, phi, 0);
                p->illr[p->n_illr++] = lv;
                b1->metric = b1->metric + logaddexp0(lv);
                path_set_bit(b1, &t, phi, 1);
                b1->illr[b1->n_illr++] = lv;
                nxt[nn++] = p;
                nxt[nn++] = b1;
            }
        }
        if (!frozen) info_index++;
        if (nn == 0) {
            rc = -3;
            goto done;
        }
        /* Python list.sort(key=metric): stable, uses only '<' */
        for (int i = 1; i < nn; i++) {
            opath* v = nxt[i];
            int j = i - 1;
            while (j >= 0 && v->metric < nxt[j]->metric) {
                nxt[j + 1] = nxt[j];
                j--;
            }
            nxt[j + 1] = v;
        }
        count = nn < M ? nn : M;
        for (int i = count; i < nn; i++) freel[nfree++] = nxt[i];
        for (int i = 0; i < count; i++) cur[i] = nxt[i];
    }
    {
        int bi = -1;
        for (int i = 0; i < count; i++) {
            for (int j = 0; j < K; j++) cands[(size_t)i * K + j] = cur[i]->u[info[j]];
            metrics[i] = cur[i]->metric;
            if (info_llrs)
                for (int j = 0; j < K; j++) info_llrs[(size_t)i * K + j] = cur[i]->illr[j];
        }
        if (crc_poly)
            for (int i = 0; i < count; i++)
                if (oracle_check_crc(cands + (size_t)i * K, K, crc_poly) == 1) {
                    bi = i;
                    break;
                }
        if (bi < 0 && count > 0) bi = 0;
        *best_index = bi;
        rc = count;
    }
done:
    for (int i = 0; i < 2 * cap; i++) path_free(&pool[i]);
    free(pool);
    return rc;
}

/* ------------------------------------------------------------- DL-SCL (dlscl/flip.py) */

/* stable argsort of q (ascending). Tie order of numpy's default argsort is not pinned. */
static void argsort_stable(const double* q, int n, int* order) {
    for (int i = 0; i < n; i++) order[i] = i;
    for (int i = 1; i < n; i++) {
        int v = order[i], j = i - 1;
        while (j >= 0 && q[order[j]] > q[v]) {
            order[j + 1] = order[j];
            j--;
        }
        order[j + 1] = v;
    }
}

/*
 * decode_with_retries flip.py:65-141.  beta: NULL or K*K float32 row-major (q = |L0| @ beta).
 * Outputs: final best bits (K), success flag, attempts (1 + retries used), tried[] indices.
 * Returns 0 or negative error.
 */
int oracle_decode_with_retries(const double* llr, int N, const int32_t* info, int K, int M, int retries,
                               uint64_t crc_poly, const float* beta, int8_t* best_bits, int32_t* success,
                               int32_t* attempts, int32_t* tried, int32_t* n_tried) {
    int8_t* cands = (int8_t*)malloc((size_t)M * K);
    double* mets = (double*)malloc(sizeof(double) * (size_t)M);
    double* illr = (double*)malloc(sizeof(double) * (size_t)M * K);
    int8_t* ref_bits = (int8_t*)malloc((size_t)K);
    double* absl0 = (double*)malloc(sizeof(double) * (size_t)K);
    double* q = (double*)malloc(sizeof(double) * (size_t)K);
    int* order = (int*)malloc(sizeof(int) * (size_t)K);
    int8_t* forced = (int8_t*)malloc((size_t)K);
    int32_t bi;
    int rc = oracle_decode_scl(llr, N, info, K, M, crc_poly, NULL, cands, mets, illr, &bi);
    int nt = 0;
    int att = 1;
    int ok;
    if (rc <= 0) goto fail;
#define PASSES(bits_) (crc_poly ? (oracle_check_crc((bits_), K, crc_poly) == 1) : 1)
    memcpy(best_bits, cands + (size_t)bi * K, (size_t)K);
    ok = PASSES(best_bits);
    if (!ok && retries > 0) {
        memcpy(ref_bits, cands + (size_t)bi * K, (size_t)K);
        for (int j = 0; j < K; j++) absl0[j] = fabs(illr[(size_t)bi * K + j]);
        while (nt < retries && nt < K) {
            if (beta) {
                for (int j = 0; j < K; j++) {
                    double s = 0.0;
                    for (int k = 0; k < K; k++) s += absl0[k] * (double)beta[(size_t)k * K + j];
                    q[j] = s;
                }
                argsort_stable(q, K, order);
            } else {
                argsort_stable(absl0, K, order);
            }
            int idx = -1;
            for (int r = 0; r < K && idx < 0; r++) {
                int cand = order[r], seen = 0;
                for (int s2 = 0; s2 < nt; s2++) seen |= (tried[s2] == cand);
                if (!seen) idx = cand;
            }
            if (idx < 0) break;
            tried[nt++] = idx;
            /* _force_vector flip.py:30-34 */
            for (int j = 0; j < K; j++) forced[j] = -1;
            for (int j = 0; j < idx; j++) forced[j] = ref_bits[j];
            forced[idx] = (int8_t)(1 - ref_bits[idx]);
            rc = oracle_decode_scl(llr, N, info, K, M, crc_poly, forced, cands, mets, illr, &bi);
            att++;
            if (rc <= 0) goto fail;
            memcpy(best_bits, cands + (size_t)bi * K, (size_t)K);
            memcpy(ref_bits, best_bits, (size_t)K);
            for (int j = 0; j < K; j++) absl0[j] = fabs(illr[(size_t)bi * K + j]);
            if (PASSES(best_bits)) break;
        }
        ok = PASSES(best_bits);
    }
#undef PASSES
    *success = ok;
    *attempts = att;
    *n_tried = nt;
    rc = 0;
fail:
    free(cands);
    free(mets);
    free(illr);
    free(ref_bits);
    free(absl0);
    free(q);
    free(order);
    free(forced);
    return rc < 0 ? rc : 0;
}

/* --------------------------------------------- batch helpers (CPU baseline, tests) */

/*
 * Decode B frames (row-major llr[B][N]); writes best bits (K per frame) and CRC pass flag.
 * Parallel over frames with OpenMP when built with -fopenmp (threads = OMP_NUM_THREADS).
 */
int oracle_decode_batch(const double* llr, int64_t B, int N, const int32_t* info, int K, int M,
                        uint64_t crc_poly, int8_t* best_bits, uint8_t* crc_pass, int32_t* best_idx) {
    int err = 0;
#pragma omp parallel for schedule(dynamic, 4) reduction(| : err)
    for (int64_t b = 0; b < B; b++) {
        int8_t cands[OR_MAXM * OR_MAXN];
        double mets[OR_MAXM];
        int32_t bi;
        int rc = oracle_decode_scl(llr + b * N, N, info, K, M, crc_poly, NULL, cands, mets, NULL, &bi);
        if (rc <= 0) {
            err |= 1;
            continue;
        }
        memcpy(best_bits + b * K, cands + (size_t)bi * K, (size_t)K);
        crc_pass[b] = (uint8_t)(crc_poly ? oracle_check_crc(cands + (size_t)bi * K, K, crc_poly) == 1 : 1);
        if (best_idx) best_idx[b] = bi;
    }
    return err ? -1 : 0;
}

/*
 * decode_with_retries over B frames (OpenMP over frames): final best bits [B][K], success
 * [B], attempts [B].  beta: NULL or K*K float32.  Returns 0 or -1.
 */
int oracle_dl_batch(const double* llr, int64_t B, int N, const int32_t* info, int K, int M, int retries,
                    uint64_t crc_poly, const float* beta, int8_t* best_bits, int32_t* success, int32_t* attempts) {
    int err = 0;
#pragma omp parallel for schedule(dynamic, 4) reduction(| : err)
    for (int64_t b = 0; b < B; b++) {
        int32_t tried[OR_MAXN];
        int32_t nt;
        if (oracle_decode_with_retries(llr + b * N, N, info, K, M, retries > K ? K : retries, crc_poly, beta,
                                       best_bits + b * K, success + b, attempts + b, tried, &nt))
            err |= 1;
    }
    return err ? -1 : 0;
}

int oracle_num_threads(void) {
#ifdef _OPENMP
    extern int omp_get_max_threads(void);
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* thread count of the batch entry points (bench.py's cpu_baseline: one per CPU of the affinity mask) */
void oracle_set_num_threads(int n) {
#ifdef _OPENMP
    extern void omp_set_num_threads(int);
    if (n > 0) omp_set_num_threads(n);
#else
    (void)n;
#endif
}

/* np.logaddexp(0, v) as the reference computes it (for host checks of the device port) */
void oracle_logaddexp0_batch(const double* v, int64_t n, double* out) {
    for (int64_t i = 0; i < n; i++) out[i] = logaddexp0(v[i]);
}
