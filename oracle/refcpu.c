/*
 * oracle/refcpu.c -- TEST INFRASTRUCTURE ONLY.
 *
 * A loop-faithful C restatement of the reference decoders of
 * B1ear/PolarCode_and_LDPC (pure Python/NumPy).  It is the parity checker for
 * the HIP decoders and the timed CPU baseline in bench.py ("kind": "port").
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * it; the product path (polarcode_and_ldpc_amd) never does.
 *
 * Parity of this restatement is pinned against golden vectors produced by the
 * reference itself (tests/golden/make_golden.py -> tests/golden/ *.npz;
 * tests/test_oracle_golden.py).
 *
 * Every function mirrors the reference data layout and loop order:
 *   SC   : src/polar/decoder.py:38-170   (L,B matrices of shape N x (n+1))
 *   SCL  : src/polar/decoder.py:225-441  (per-path L/B, full snapshot copies,
 *                                          CPython's list.sort order (pysort.h:
 *                                          stable descending for finite metrics,
 *                                          exact for NaN ones), np.argmax)
 *   BP   : src/ldpc/decoder.py:62-202    (flooding, tanh rule, clip +-0.999999)
 *   MS   : src/ldpc/decoder.py:257-352
 * Arithmetic dependencies: NumPy ufuncs in the reference -> libm here
 * (exp, log1p, tanh, atanh may differ by <=2 ulp).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#include "pysort.h" /* CPython 3.10 list.sort restated (NaN metrics) */

#define ORC_OK 0
#define ORC_EINVAL -1
#define ORC_ENOMEM -2
#define ORC_EDEGREE -4 /* MSDecoder on a degree-1 check: np.min([]) raises */

/* src/polar/utils.py:11-26 */
static int bit_reverse(int v, int nb) {
    int r = 0;
    for (int i = 0; i < nb; i++) { r = (r << 1) | (v & 1); v >>= 1; }
    return r;
}

/* src/polar/decoder.py:146-157 (_active_llr_level) */
static int active_llr_level(int i, int n) {
    int mask = 1 << (n - 1), count = 1;
    for (int k = 0; k < n; k++) {
        if ((mask & i) == 0) { count++; mask >>= 1; } else break;
    }
    return count < n ? count : n;
}

/* src/polar/decoder.py:159-170 (_active_bit_level) */
static int active_bit_level(int i, int n) {
    int mask = 1 << (n - 1), count = 1;
    for (int k = 0; k < n; k++) {
        if ((mask & i) > 0) { count++; mask >>= 1; } else break;
    }
    return count < n ? count : n;
}

static inline double npsign(double x) { return x > 0 ? 1.0 : (x < 0 ? -1.0 : (x == 0 ? 0.0 : x)); }

/* decoder.py:121-127 f = sign(a)*sign(b)*min(|a|,|b|)  (Python min keeps the
 * first argument on ties / when the comparison is false) */
static inline double f_upper(double a, double b) {
    double x = fabs(a), y = fabs(b);
    double mn = (y < x) ? y : x;
    return npsign(a) * npsign(b) * mn;
}

/* decoder.py:129-144 g */
static inline double g_lower(double btm, double top, double bit) {
    return (bit == 0.0) ? btm + top : btm - top;
}

static int log2i(int N) { int n = 0; while ((1 << n) < N) n++; return n; }

/* ---------------------------------------------------------------- SC ---- */
/* Decode one frame; writes u_hat[N] (0/1).  frozen_mask[N] != 0 => frozen. */
int orc_sc_decode(int N, const uint8_t* frozen_mask, const double* llr, uint8_t* u_hat) {
    if (N < 2 || (N & (N - 1))) return ORC_EINVAL;
    const int n = log2i(N), W = n + 1;
    double* Lm = (double*)malloc(sizeof(double) * N * W);
    double* Bm = (double*)malloc(sizeof(double) * N * W);
    if (!Lm || !Bm) { free(Lm); free(Bm); return ORC_ENOMEM; }
    for (int k = 0; k < N * W; k++) { Lm[k] = NAN; Bm[k] = NAN; }
#define LL(j, s) Lm[(j) * W + (s)]
#define BB(j, s) Bm[(j) * W + (s)]
    for (int j = 0; j < N; j++) LL(j, 0) = llr[j];
    for (int i = 0; i < N; i++) {
        const int l = bit_reverse(i, n);
        for (int s = n - active_llr_level(l, n); s < n; s++) {       /* :73-94 */
            const int bs = 1 << (s + 1), br = bs / 2;
            for (int j = l; j < N; j += bs) {
                if (j % bs < br) LL(j, s + 1) = f_upper(LL(j, s), LL(j + br, s));
                else LL(j, s + 1) = g_lower(LL(j, s), LL(j - br, s), BB(j - br, s + 1));
            }
        }
        BB(l, n) = frozen_mask[l] ? 0.0 : (LL(l, n) >= 0 ? 0.0 : 1.0);  /* :61-64 */
        if (!(l < N / 2.0)) {                                           /* :96-115 */
            for (int s = n; s > n - active_bit_level(l, n); s--) {
                const int bs = 1 << s, br = bs / 2;
                for (int j = l; j >= 0; j -= bs) {
                    if (j % bs >= br) {
                        BB(j - br, s - 1) = (double)((int)BB(j, s) ^ (int)BB(j - br, s));
                        BB(j, s - 1) = BB(j, s);
                    }
                }
            }
        }
    }
    for (int j = 0; j < N; j++) u_hat[j] = (uint8_t)(int)BB(j, n);
#undef LL
#undef BB
    free(Lm); free(Bm);
    return ORC_OK;
}

/* --------------------------------------------------------------- SCL ---- */
/* decoder.py:374-406 */
static inline double log_likelihood(double llr, int bit) {
    if (bit == 0) {
        if (llr >= 0) return -log1p(exp(-llr));
        return llr - log1p(exp(llr));
    } else {
        if (llr >= 0) return -llr - log1p(exp(-llr));
        return -log1p(exp(llr));
    }
}

typedef struct { double m; int p; int bit; } cand_t;

uint32_t orc_crc(const uint8_t* bits, int nbits, int crc_len, uint32_t poly);

/* crc_len > 0: CRC-aided selection (build-defined extension, SURVEY.md §8f rank 2;
 * the reference stores use_crc but never reads it, decoder.py:202-203,259): the
 * first path, in the stable descending order of the final metrics, whose
 * u_hat[info bits] passes crc_check (src/polar/utils.py:128-163); none -> argmax. */
static int scl_decode_impl(int N, int Lsz, const uint8_t* frozen_mask, const double* llr, uint8_t* u_hat,
                           int crc_len, uint32_t poly) {
    if (N < 2 || (N & (N - 1)) || Lsz < 1) return ORC_EINVAL;
    const int n = log2i(N), W = n + 1;
    const size_t per = (size_t)N * W;
    double* Lp = (double*)malloc(sizeof(double) * per * Lsz);
    double* Bp = (double*)malloc(sizeof(double) * per * Lsz);
    double* oL = (double*)malloc(sizeof(double) * per * Lsz);
    double* oB = (double*)malloc(sizeof(double) * per * Lsz);
    double* pm = (double*)malloc(sizeof(double) * Lsz);
    uint8_t* act = (uint8_t*)malloc(Lsz);
    cand_t* cand = (cand_t*)malloc(sizeof(cand_t) * 2 * Lsz);
    int* aidx = (int*)malloc(sizeof(int) * Lsz);
    cand_t* cand2 = (cand_t*)malloc(sizeof(cand_t) * 2 * Lsz);
    ps_item* srt = (ps_item*)malloc(sizeof(ps_item) * 2 * Lsz);
    ps_item* stmp = (ps_item*)malloc(sizeof(ps_item) * (Lsz + 1));
    if (!Lp || !Bp || !oL || !oB || !pm || !act || !cand || !aidx || !cand2 || !srt || !stmp) {
        free(Lp); free(Bp); free(oL); free(oB); free(pm); free(act); free(cand); free(aidx);
        free(cand2); free(srt); free(stmp);
        return ORC_ENOMEM;
    }
    for (size_t k = 0; k < per * Lsz; k++) { Lp[k] = NAN; Bp[k] = NAN; }
#define PL(p, j, s) Lp[(size_t)(p) * per + (size_t)(j) * W + (s)]
#define PB(p, j, s) Bp[(size_t)(p) * per + (size_t)(j) * W + (s)]
    for (int p = 0; p < Lsz; p++) { act[p] = 0; pm[p] = -INFINITY; }     /* :238-241 */
    act[0] = 1; pm[0] = 0.0;
    for (int p = 0; p < Lsz; p++) for (int j = 0; j < N; j++) PL(p, j, 0) = llr[j];

    for (int i = 0; i < N; i++) {
        const int l = bit_reverse(i, n);
        const int s0 = n - active_llr_level(l, n);
        const int upd_bits = !(l < N / 2.0);
        const int sb = n - active_bit_level(l, n);
        /* _update_llrs_for_path :341-356 */
#define UPD_LLR(p)                                                                    \
        for (int s = s0; s < n; s++) {                                                \
            const int bs = 1 << (s + 1), br = bs / 2;                                 \
            for (int j = l; j < N; j += bs) {                                         \
                if (j % bs < br) PL(p, j, s + 1) = f_upper(PL(p, j, s), PL(p, j + br, s)); \
                else PL(p, j, s + 1) = g_lower(PL(p, j, s), PL(p, j - br, s), PB(p, j - br, s + 1)); \
            }                                                                         \
        }
        /* _update_bits_for_path :358-372 */
#define UPD_BITS(p)                                                                   \
        if (upd_bits) {                                                               \
            for (int s = n; s > sb; s--) {                                            \
                const int bs = 1 << s, br = bs / 2;                                   \
                for (int j = l; j >= 0; j -= bs)                                      \
                    if (j % bs >= br) {                                               \
                        PB(p, j - br, s - 1) = (double)((int)PB(p, j, s) ^ (int)PB(p, j - br, s)); \
                        PB(p, j, s - 1) = PB(p, j, s);                                \
                    }                                                                 \
            }                                                                         \
        }
        if (frozen_mask[l]) {                                              /* :264-281 */
            for (int p = 0; p < Lsz; p++) {
                if (!act[p]) continue;
                UPD_LLR(p);
                PB(p, l, n) = 0.0;
                pm[p] += log_likelihood(PL(p, l, n), 0);
                UPD_BITS(p);
            }
        } else {                                                           /* :283-339 */
            int na = 0;
            for (int p = 0; p < Lsz; p++) if (act[p]) aidx[na++] = p;
            for (int a = 0; a < na; a++) {
                const int p = aidx[a];
                UPD_LLR(p);
                const double lv = PL(p, l, n);
                cand[a].m = pm[p] + log_likelihood(lv, 0); cand[a].p = p; cand[a].bit = 0;
                cand[na + a].m = pm[p] + log_likelihood(lv, 1); cand[na + a].p = p; cand[na + a].bit = 1;
            }
            /* all_candidates.sort(key=lambda x: x[0], reverse=True) (:306-307): CPython's
             * algorithm (pysort.h) -- stable descending for finite metrics, and the
             * interpreter's own order when NaN metrics compare false both ways */
            const int nc = 2 * na;
            for (int a = 0; a < nc; a++) { srt[a].k = cand[a].m; srt[a].v = a; }
            ps_sort_desc(srt, nc, stmp);
            for (int a = 0; a < nc; a++) cand2[a] = cand[srt[a].v];
            memcpy(cand, cand2, sizeof(cand_t) * nc);
            const int ns = nc < Lsz ? nc : Lsz;
            memcpy(oL, Lp, sizeof(double) * per * Lsz);                  /* :314-316 */
            memcpy(oB, Bp, sizeof(double) * per * Lsz);
            for (int p = 0; p < Lsz; p++) { act[p] = 0; pm[p] = -INFINITY; }
            for (int k = 0; k < ns; k++) {
                const int op = cand[k].p;
                memcpy(&Lp[(size_t)k * per], &oL[(size_t)op * per], sizeof(double) * per);
                memcpy(&Bp[(size_t)k * per], &oB[(size_t)op * per], sizeof(double) * per);
                PB(k, l, n) = (double)cand[k].bit;
                pm[k] = cand[k].m;
                act[k] = 1;
                UPD_BITS(k);
            }
        }
#undef UPD_LLR
#undef UPD_BITS
    }
    /* np.argmax (:258): the first NaN if there is one, else the first maximum */
    int best = 0;
    for (int p = 1; p < Lsz && !isnan(pm[best]); p++) if (isnan(pm[p]) || pm[p] > pm[best]) best = p;
    if (crc_len > 0) {
        /* build-defined CA-SCL: active paths in the order list.sort(key=metric,
         * reverse=True) leaves them (stable descending; CPython's order with NaN) */
        int na = 0;
        for (int p = 0; p < Lsz; p++) if (act[p]) { srt[na].k = pm[p]; srt[na].v = p; na++; }
        ps_sort_desc(srt, na, stmp);
        for (int a = 0; a < na; a++) aidx[a] = srt[a].v;
        uint8_t* msg = (uint8_t*)malloc((size_t)N);
        for (int a = 0; a < na && msg; a++) {
            int k = 0;
            for (int j = 0; j < N; j++) if (!frozen_mask[j]) msg[k++] = (uint8_t)(int)PB(aidx[a], j, n);
            if (orc_crc(msg, k, crc_len, poly) == 0) { best = aidx[a]; break; }
        }
        free(msg);
    }
    for (int j = 0; j < N; j++) u_hat[j] = (uint8_t)(int)PB(best, j, n);
#undef PL
#undef PB
    free(Lp); free(Bp); free(oL); free(oB); free(pm); free(act); free(cand); free(aidx);
    free(cand2); free(srt); free(stmp);
    return ORC_OK;
}

/* test hook: the permutation list.sort(key=k, reverse=True) applies (pysort.h) */
int orc_pysort_desc(const double* keys, int n, int32_t* perm) {
    ps_item* a = (ps_item*)malloc(sizeof(ps_item) * (size_t)(n > 0 ? n : 1));
    ps_item* t = (ps_item*)malloc(sizeof(ps_item) * (size_t)(n / 2 + 1));
    if (!a || !t) { free(a); free(t); return ORC_ENOMEM; }
    for (int i = 0; i < n; i++) { a[i].k = keys[i]; a[i].v = i; }
    ps_sort_desc(a, n, t);
    for (int i = 0; i < n; i++) perm[i] = a[i].v;
    free(a); free(t);
    return ORC_OK;
}

int orc_scl_decode(int N, int Lsz, const uint8_t* frozen_mask, const double* llr, uint8_t* u_hat) {
    return scl_decode_impl(N, Lsz, frozen_mask, llr, u_hat, 0, 0);
}

/* --------------------------------------------------------------- LDPC --- */
/* numpy add.reduce over float64 (pairwise_sum, numpy/_core/src/umath/loops_utils.h.src):
 * verified equal to np.sum on lists for n = 1..128 in the build container. */
static double np_pairwise_sum(const double* a, int n) {
    if (n < 8) {
        double res = 0.;
        for (int i = 0; i < n; i++) res += a[i];
        return res;
    } else if (n <= 128) {
        double r[8];
        int i;
        for (int j = 0; j < 8; j++) r[j] = a[j];
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; j++) r[j] += a[i + j];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; i++) res += a[i];
        return res;
    } else {
        int n2 = n / 2;
        n2 -= n2 % 8;
        return np_pairwise_sum(a, n2) + np_pairwise_sum(a + n2, n - n2);
    }
}

static inline double clip999(double x) {
    const double c = 0.999999;
    return x < -c ? -c : (x > c ? c : x);
}

typedef struct {
    int m, n, E, maxdv, maxdc;
    const int32_t *row_ptr, *col_idx;
    int32_t *var_ptr, *var_edge; /* var-major lists of check-major edge ids, ascending check */
} tanner_t;

static int tanner_build(tanner_t* t, int m, int n, const int32_t* row_ptr, const int32_t* col_idx) {
    t->m = m; t->n = n; t->E = row_ptr[m];
    t->row_ptr = row_ptr; t->col_idx = col_idx;
    t->var_ptr = (int32_t*)calloc(n + 1, sizeof(int32_t));
    t->var_edge = (int32_t*)malloc(sizeof(int32_t) * (t->E > 0 ? t->E : 1));
    if (!t->var_ptr || !t->var_edge) return ORC_ENOMEM;
    for (int e = 0; e < t->E; e++) {
        if (col_idx[e] < 0 || col_idx[e] >= n) return ORC_EINVAL;
        t->var_ptr[col_idx[e] + 1]++;
    }
    for (int v = 0; v < n; v++) t->var_ptr[v + 1] += t->var_ptr[v];
    int32_t* fill = (int32_t*)malloc(sizeof(int32_t) * (n > 0 ? n : 1));
    memcpy(fill, t->var_ptr, sizeof(int32_t) * n);
    t->maxdc = 0;
    for (int c = 0; c < m; c++) {          /* rows scanned ascending: decoder.py:43-47 */
        int d = row_ptr[c + 1] - row_ptr[c];
        if (d > t->maxdc) t->maxdc = d;
        for (int e = row_ptr[c]; e < row_ptr[c + 1]; e++) t->var_edge[fill[col_idx[e]]++] = e;
    }
    t->maxdv = 0;
    for (int v = 0; v < n; v++) {
        int d = t->var_ptr[v + 1] - t->var_ptr[v];
        if (d > t->maxdv) t->maxdv = d;
    }
    free(fill);
    return ORC_OK;
}
static void tanner_free(tanner_t* t) { free(t->var_ptr); free(t->var_edge); }

/* algo 0 = BP (BPDecoder, decoder.py:124-202), 1 = MS (MSDecoder, :289-352) */
static int ldpc_decode_one(const tanner_t* t, int algo, int max_iter, int early_stop, double norm,
                           const double* llr, uint8_t* bits, int32_t* iters, double* work) {
    const int m = t->m, n = t->n, E = t->E;
    double* v2c = work;            /* E, indexed by check-major edge id */
    double* c2v = v2c + E;         /* E */
    double* tv = c2v + E;          /* maxdc */
    double* msg = tv + (t->maxdc > 0 ? t->maxdc : 1); /* maxdv */
    for (int e = 0; e < E; e++) v2c[e] = llr[t->col_idx[e]];           /* :144-146 */
    int actual = max_iter;
    for (int v = 0; v < n; v++) bits[v] = 0;
    for (int it = 0; it < max_iter; it++) {
        for (int c = 0; c < m; c++) {
            const int e0 = t->row_ptr[c], d = t->row_ptr[c + 1] - e0;
            if (algo == 0) {                                              /* :62-96 */
                for (int k = 0; k < d; k++) tv[k] = clip999(tanh(v2c[e0 + k] / 2.0));
                for (int i = 0; i < d; i++) {
                    double p = 1.0;
                    for (int k = 0; k < d; k++) if (k != i) p *= tv[k];
                    p = clip999(p);
                    double o = 2.0 * atanh(p);
                    if (isnan(o)) o = 0.0;
                    else if (isinf(o)) o = o > 0 ? 20.0 : -20.0;
                    c2v[e0 + i] = o;
                }
            } else {                                                      /* :257-287 */
                if (d == 1) return ORC_EDEGREE;
                for (int i = 0; i < d; i++) {
                    double sp = 1.0, mn = INFINITY;
                    int first = 1;
                    for (int k = 0; k < d; k++) {
                        if (k == i) continue;
                        const double x = v2c[e0 + k];
                        sp *= npsign(x);
                        const double ax = fabs(x);
                        if (first) { mn = ax; first = 0; }
                        else if (isnan(ax) || isnan(mn)) mn = NAN;  /* np.min propagates NaN */
                        else if (ax < mn) mn = ax;
                    }
                    c2v[e0 + i] = sp * mn * norm;
                }
            }
        }
        for (int v = 0; v < n; v++) {                                     /* :98-122 */
            const int a0 = t->var_ptr[v], dv = t->var_ptr[v + 1] - a0;
            for (int k = 0; k < dv; k++) msg[k] = c2v[t->var_edge[a0 + k]];
            const double total = llr[v] + np_pairwise_sum(msg, dv);
            for (int k = 0; k < dv; k++) v2c[t->var_edge[a0 + k]] = total - msg[k];
            bits[v] = (total <= 0) ? 1 : 0;                                /* :191 */
        }
        if (early_stop) {                                                 /* :194-198 */
            int ok = 1;
            for (int c = 0; c < m && ok; c++) {
                int s = 0;
                for (int e = t->row_ptr[c]; e < t->row_ptr[c + 1]; e++) s += bits[t->col_idx[e]];
                if (s % 2) ok = 0;
            }
            if (ok) { actual = it + 1; break; }
        }
    }
    if (iters) *iters = actual;
    return ORC_OK;
}

int orc_ldpc_decode_batch(int m, int n, const int32_t* row_ptr, const int32_t* col_idx, int algo,
                          int max_iter, int early_stop, double norm, const double* llr,
                          int64_t batch, int64_t ld, uint8_t* bits, int32_t* iters, int threads) {
    tanner_t t;
    int rc = tanner_build(&t, m, n, row_ptr, col_idx);
    if (rc) { tanner_free(&t); return rc; }
    if (algo == 1) {
        for (int c = 0; c < m; c++)
            if (row_ptr[c + 1] - row_ptr[c] == 1 && max_iter > 0) { tanner_free(&t); return ORC_EDEGREE; }
    }
    const size_t wsz = 2 * (size_t)t.E + t.maxdc + t.maxdv + 2;
    int err = 0;
#ifdef _OPENMP
    if (threads < 1) threads = 1;
#pragma omp parallel num_threads(threads) reduction(| : err)
#endif
    {
        double* work = (double*)malloc(sizeof(double) * wsz);
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
        for (int64_t b = 0; b < batch; b++)
            err |= ldpc_decode_one(&t, algo, max_iter, early_stop, norm, llr + b * ld, bits + b * n,
                                   iters ? iters + b : NULL, work) ? 1 : 0;
        free(work);
    }
    (void)threads;
    tanner_free(&t);
    return err ? ORC_EINVAL : ORC_OK;
}

/* list_size <= 0 -> SC, else SCL(list_size).  u_hat: [batch, N] */
int orc_polar_decode_batch(int N, int list_size, const uint8_t* frozen_mask, const double* llr,
                           int64_t batch, int64_t ld, uint8_t* u_hat, int threads) {
    int err = 0;
#ifdef _OPENMP
    if (threads < 1) threads = 1;
#pragma omp parallel for num_threads(threads) schedule(dynamic, 1) reduction(| : err)
#endif
    for (int64_t b = 0; b < batch; b++) {
        int rc = list_size <= 0 ? orc_sc_decode(N, frozen_mask, llr + b * ld, u_hat + b * N)
                                : orc_scl_decode(N, list_size, frozen_mask, llr + b * ld, u_hat + b * N);
        err |= rc ? 1 : 0;
    }
    (void)threads;
    return err ? ORC_EINVAL : ORC_OK;
}

/* CA-SCL batch (see scl_decode_impl): u_hat [batch, N] */
int orc_cascl_decode_batch(int N, int list_size, const uint8_t* frozen_mask, const double* llr, int64_t batch,
                           int64_t ld, uint8_t* u_hat, int threads, int crc_len, uint32_t poly) {
    int err = 0;
#ifdef _OPENMP
    if (threads < 1) threads = 1;
#pragma omp parallel for num_threads(threads) schedule(dynamic, 1) reduction(| : err)
#endif
    for (int64_t b = 0; b < batch; b++)
        err |= scl_decode_impl(N, list_size, frozen_mask, llr + b * ld, u_hat + b * N, crc_len, poly) ? 1 : 0;
    (void)threads;
    return err ? ORC_EINVAL : ORC_OK;
}

/* src/polar/utils.py:86-125 crc_encode (bit-serial, MSB first) -> crc value */
uint32_t orc_crc(const uint8_t* bits, int nbits, int crc_len, uint32_t poly) {
    uint32_t crc = 0, top = 1u << (crc_len - 1), mask = (crc_len == 32) ? 0xffffffffu : ((1u << crc_len) - 1);
    for (int i = 0; i < nbits; i++) {
        crc ^= ((uint32_t)(bits[i] & 1)) << (crc_len - 1);
        crc = (crc & top) ? ((crc << 1) ^ poly) : (crc << 1);
        crc &= mask;
    }
    return crc;
}
