/*
 * mmre_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity oracle).
 *
 * A plain-C, single-threaded restatement of the reference's CPU path for the KG
 * scoring hot path. Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker. The product
 * (multimodal-relation-extrapolation_amd/) never links or calls it.
 *
 * Pinning: every function below is checked against golden vectors produced in
 * the build container by the reference itself (tests/golden/make_golden.py:
 * the reference OpenKE Python models + the reference Base.so compiled from
 * /root/reference/OpenKE/openke/base/Base.cpp by oracle/Makefile).
 *
 * Canonical arithmetic ("CA", shared *specification* with the HIP kernels, but
 * written independently here). Built with -ffp-contract=off, no fast-math:
 *   TransE  L1 : s = 0; for k: s = s + |q_k - e_k|
 *   TransE  L2 : s = 0; for k: x = q_k - e_k; s = s + x*x;  s = sqrtf(s)
 *   DistMult   : s = 0; for k: s = fmaf(e_k, q_k, s)
 *   ComplEx    : s = 0; for k: s = fmaf(re_k, qa_k, s); for k: s = fmaf(im_k, qb_k, s)
 *   RotatE     : s = 0; for k: dr = qa_k - x_k; di = qb_k - y_k; s = s + sqrtf(fmaf(di, di, dr*dr))
 * Query vectors (element-wise, same rounding as the reference's torch ops):
 *   TransE  head: q = -(r - t)   tail: q = h + r          (TransE.py:71-74)
 *   DistMult head: q = r * t     tail: q = h * r          (DistMult.py:37-42)
 *   ComplEx head: qa = t_re r_re + t_im r_im, qb = t_im r_re - t_re r_im
 *           tail: qa = h_re r_re - h_im r_im, qb = h_im r_re + h_re r_im   (ComplEx.py:20-27)
 *   RotatE  head: qa = c t_re + s t_im, qb = c t_im - s t_re
 *           tail: qa = h_re c - h_im s, qb = h_re s + h_im c   (RotatE.py:63-72)
 *           c, s = canonical cos/sin of phase = r / denom   (RotatE.py:51-54)
 * Prediction transform (what model.predict returns, TransE.py:88-94, DistMult.py:70-72,
 * ComplEx.py:60-62, RotatE.py:86-91):
 *   0: p = s   1: p = m - (m - s)   2: p = -s   3: p = -(m - s)
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

enum { M_TRANSE_L1 = 0, M_TRANSE_L2 = 1, M_DISTMULT = 2, M_COMPLEX = 3, M_ROTATE = 4 };
enum { HEAD_BATCH = 0, TAIL_BATCH = 1 };

/* ---------------------------------------------------------------- sincos -- */
/* Canonical single-precision sin/cos: Cody-Waite reduction by pi/2 (fma form)
 * + cephes minimax polynomials on [-pi/4, pi/4]. Restated in csrc/ for HIP.  */
static void orc_sincos(float x, float *s_out, float *c_out) {
    const float TWO_OVER_PI = 0.636619772367581343f;
    const float P1 = 1.57079637050628662109375f;
    const float P2 = -4.37113900018624283e-8f;
    const float P3 = -1.71512986e-15f;
    float j = rintf(x * TWO_OVER_PI);
    float r = fmaf(-j, P1, x);
    r = fmaf(-j, P2, r);
    r = fmaf(-j, P3, r);
    float z = r * r;
    float sp = fmaf(fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f);
    float sv = fmaf(sp * z, r, r);
    float cp = fmaf(fmaf(2.443315711809948e-5f, z, -1.388731625493765e-3f), z, 4.166664568298827e-2f);
    float cv = fmaf(cp * z, z, fmaf(-0.5f, z, 1.0f));
    int q = ((int)j) & 3;
    float s, c;
    switch (q) {
        case 0: s = sv; c = cv; break;
        case 1: s = cv; c = -sv; break;
        case 2: s = -sv; c = -cv; break;
        default: s = -cv; c = sv; break;
    }
    *s_out = s;
    *c_out = c;
}

void orc_sincos_vec(const float *x, int64_t n, float *s, float *c) {
    for (int64_t i = 0; i < n; ++i) orc_sincos(x[i], &s[i], &c[i]);
}

/* ------------------------------------------------------------ normalize -- */
/* F.normalize(x, 2, -1) with eps 1e-12 (TransE.py:63-66): x / max(||x||, eps) */
static void orc_normalize_row(const float *x, int d, float *out) {
    float ss = 0.0f;
    for (int k = 0; k < d; ++k) ss = ss + x[k] * x[k];
    float n = sqrtf(ss);
    if (n < 1e-12f) n = 1e-12f;
    for (int k = 0; k < d; ++k) out[k] = x[k] / n;
}

void orc_normalize_rows(const float *x, int64_t n, int d, float *out) {
    for (int64_t i = 0; i < n; ++i) orc_normalize_row(x + i * d, d, out + i * d);
}

/* ------------------------------------------------------------ scoring ---- */
static float apply_pred(int pred_kind, float m, float s) {
    switch (pred_kind) {
        case 0: return s;
        case 1: return m - (m - s);
        case 2: return -s;
        default: return -(m - s);
    }
}

/* Build the query vectors for one query (h, r, t) in mode; K = row width. */
static void build_query(int model, int mode, int norm_flag, const float *ent, const float *ent_im,
                        const float *rel, const float *rel_im, int d, float phase_denom, int64_t h,
                        int64_t r, int64_t t, float *qa, float *qb, float *tmp) {
    if (model == M_TRANSE_L1 || model == M_TRANSE_L2) {
        float *hv = tmp, *rv = tmp + d, *tv = tmp + 2 * d;
        if (norm_flag) {
            orc_normalize_row(ent + h * d, d, hv);
            orc_normalize_row(rel + r * d, d, rv);
            orc_normalize_row(ent + t * d, d, tv);
        } else {
            memcpy(hv, ent + h * d, d * sizeof(float));
            memcpy(rv, rel + r * d, d * sizeof(float));
            memcpy(tv, ent + t * d, d * sizeof(float));
        }
        for (int k = 0; k < d; ++k)
            qa[k] = (mode == HEAD_BATCH) ? -(rv[k] - tv[k]) : (hv[k] + rv[k]);
    } else if (model == M_DISTMULT) {
        const float *hv = ent + h * d, *rv = rel + r * d, *tv = ent + t * d;
        for (int k = 0; k < d; ++k) qa[k] = (mode == HEAD_BATCH) ? (rv[k] * tv[k]) : (hv[k] * rv[k]);
    } else if (model == M_COMPLEX) {
        const float *hr = ent + h * d, *hi = ent_im + h * d, *tr = ent + t * d, *ti = ent_im + t * d;
        const float *rr = rel + r * d, *ri = rel_im + r * d;
        for (int k = 0; k < d; ++k) {
            if (mode == HEAD_BATCH) {
                qa[k] = tr[k] * rr[k] + ti[k] * ri[k];
                qb[k] = ti[k] * rr[k] - tr[k] * ri[k];
            } else {
                qa[k] = hr[k] * rr[k] - hi[k] * ri[k];
                qb[k] = hi[k] * rr[k] + hr[k] * ri[k];
            }
        }
    } else { /* RotatE: entity rows are (2d) = [re | im], relation rows are (d) phases */
        const float *hrow = ent + h * 2 * d, *trow = ent + t * 2 * d, *rv = rel + r * d;
        for (int k = 0; k < d; ++k) {
            float ph = rv[k] / phase_denom, s, c;
            orc_sincos(ph, &s, &c);
            if (mode == HEAD_BATCH) {
                float tre = trow[k], tim = trow[d + k];
                qa[k] = c * tre + s * tim;
                qb[k] = c * tim - s * tre;
            } else {
                float hre = hrow[k], him = hrow[d + k];
                qa[k] = hre * c - him * s;
                qb[k] = hre * s + him * c;
            }
        }
    }
}

static float score_one(int model, const float *ent, const float *ent_im, const float *ent_n, int d,
                       int64_t e, const float *qa, const float *qb) {
    float s = 0.0f;
    if (model == M_TRANSE_L1) {
        const float *ev = ent_n + e * d;
        for (int k = 0; k < d; ++k) s = s + fabsf(qa[k] - ev[k]);
    } else if (model == M_TRANSE_L2) {
        const float *ev = ent_n + e * d;
        for (int k = 0; k < d; ++k) { float x = qa[k] - ev[k]; s = s + x * x; }
        s = sqrtf(s);
    } else if (model == M_DISTMULT) {
        const float *ev = ent + e * d;
        for (int k = 0; k < d; ++k) s = fmaf(ev[k], qa[k], s);
    } else if (model == M_COMPLEX) {
        const float *re = ent + e * d, *im = ent_im + e * d;
        for (int k = 0; k < d; ++k) s = fmaf(re[k], qa[k], s);
        for (int k = 0; k < d; ++k) s = fmaf(im[k], qb[k], s);
    } else {
        const float *row = ent + e * 2 * d;
        for (int k = 0; k < d; ++k) {
            float dr = qa[k] - row[k], di = qb[k] - row[d + k];
            s = s + sqrtf(fmaf(di, di, dr * dr));
        }
    }
    return s;
}

/* model.predict over all E candidates for each query (Tester.test_one_step,
 * Tester.py:62-68 + Test.h:36-53 getHeadBatch/getTailBatch).
 * out: (Q, E) row-major predicted values. For TransE with norm_flag the entity
 * table is normalised once (identical values to per-query normalisation). */
int orc_link_predict(int model, int mode, int norm_flag, int pred_kind, float margin,
                     const float *ent, const float *ent_im, const float *rel, const float *rel_im,
                     int64_t n_ent, int dim, float phase_denom, const int64_t *qh, const int64_t *qr,
                     const int64_t *qt, int64_t n_query, float *out) {
    int d = dim;
    float *qa = (float *)malloc(sizeof(float) * d);
    float *qb = (float *)malloc(sizeof(float) * d);
    float *tmp = (float *)malloc(sizeof(float) * 3 * d);
    float *ent_n = NULL;
    if (model == M_TRANSE_L1 || model == M_TRANSE_L2) {
        ent_n = (float *)malloc(sizeof(float) * n_ent * d);
        if (norm_flag) orc_normalize_rows(ent, n_ent, d, ent_n);
        else memcpy(ent_n, ent, sizeof(float) * n_ent * d);
    }
    for (int64_t q = 0; q < n_query; ++q) {
        build_query(model, mode, norm_flag, ent, ent_im, rel, rel_im, d, phase_denom, qh[q], qr[q], qt[q],
                    qa, qb, tmp);
        for (int64_t e = 0; e < n_ent; ++e)
            out[q * n_ent + e] = apply_pred(pred_kind, margin, score_one(model, ent, ent_im, ent_n, d, e, qa, qb));
    }
    free(qa); free(qb); free(tmp); free(ent_n);
    return 0;
}

/* --------------------------------------------------------------- ranking -- */
/* Triple set lookup: (h, r, t) sorted lexicographically as int64 triples.
 * Restates _find (Corrupt.h:166-177) as a binary search over cmp_head order. */
static int triple_less(const int64_t *a, int64_t h, int64_t r, int64_t t) {
    if (a[0] != h) return a[0] < h;
    if (a[1] != r) return a[1] < r;
    return a[2] < t;
}

static int orc_find(const int64_t *hrt_sorted, int64_t n, int64_t h, int64_t r, int64_t t) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        int64_t mid = (lo + hi) >> 1;
        if (triple_less(hrt_sorted + 3 * mid, h, r, t)) lo = mid + 1; else hi = mid;
    }
    if (lo < n) {
        const int64_t *a = hrt_sorted + 3 * lo;
        return a[0] == h && a[1] == r && a[2] == t;
    }
    return 0;
}

/* testHead / testTail (Test.h:65-192): per query counts.
 * out[4*q + {0,1,2,3}] = raw, filtered, raw_constrained, filtered_constrained.
 * type lists: sorted allowed entity ids per relation (Reader.h:266-317),
 * CSR (type_off[r]..type_off[r+1]); pass NULL for no type constraint. */
int orc_test_rank(int mode, const float *pred, int64_t n_ent, const int64_t *qh, const int64_t *qr,
                  const int64_t *qt, int64_t n_query, const int64_t *hrt_sorted, int64_t n_triples,
                  const int64_t *type_off, const int64_t *type_ids, int64_t *out) {
    for (int64_t q = 0; q < n_query; ++q) {
        int64_t h = qh[q], r = qr[q], t = qt[q];
        int64_t truth = (mode == HEAD_BATCH) ? h : t;
        const float *con = pred + q * n_ent;
        float minimal = con[truth];
        int64_t raw = 0, filt = 0, rawc = 0, filtc = 0;
        int64_t lef = 0, rig = 0;
        if (type_off) { lef = type_off[r]; rig = type_off[r + 1]; }
        for (int64_t j = 0; j < n_ent; ++j) {
            if (j == truth) continue;
            float value = con[j];
            int better = value < minimal;
            int known = 0;
            if (better) {
                known = (mode == HEAD_BATCH) ? orc_find(hrt_sorted, n_triples, j, r, t)
                                             : orc_find(hrt_sorted, n_triples, h, r, j);
                raw += 1;
                if (!known) filt += 1;
            }
            if (type_off) {
                while (lef < rig && type_ids[lef] < j) lef++;
                if (lef < rig && j == type_ids[lef] && better) {
                    rawc += 1;
                    if (!known) filtc += 1;
                }
            }
        }
        out[4 * q + 0] = raw;
        out[4 * q + 1] = filt;
        out[4 * q + 2] = rawc;
        out[4 * q + 3] = filtc;
    }
    return 0;
}

/* test_link_prediction (Test.h:232-327) float accumulation semantics (P14).
 * head/tail: (Q, 4) counts from orc_test_rank, in testList order.
 * out: [mrr, mr, hit10, hit3, hit1] (filtered, averaged l/r) then the same for
 * raw, then constrained-filtered, constrained-raw (20 floats). */
static void acc_side(const int64_t *c, int64_t n, int col, float tot, float acc[5]) {
    float t10 = 0, t3 = 0, t1 = 0, rank = 0, reci = 0;
    for (int64_t i = 0; i < n; ++i) {
        int64_t s = c[4 * i + col];
        if (s < 10) t10 += 1;
        if (s < 3) t3 += 1;
        if (s < 1) t1 += 1;
        rank += (float)(s + 1);
        reci = (float)((double)reci + 1.0 / (double)(s + 1));
    }
    acc[0] = reci / tot; acc[1] = rank / tot; acc[2] = t10 / tot; acc[3] = t3 / tot; acc[4] = t1 / tot;
}

int orc_link_metrics(const int64_t *head, const int64_t *tail, int64_t n, float *out) {
    float tot = (float)n;
    const int cols[4] = {1, 0, 3, 2};
    for (int g = 0; g < 4; ++g) {
        float l[5], r[5];
        acc_side(head, n, cols[g], tot, l);
        acc_side(tail, n, cols[g], tot, r);
        for (int i = 0; i < 5; ++i) out[5 * g + i] = (l[i] + r[i]) / 2;
    }
    return 0;
}

/* ------------------------------------------------------------ sampling ---- */
/* glibc rand() after the default srand(1) (Random.h:11-15 randReset): the
 * TYPE_3 additive feedback generator, restated. */
void orc_glibc_rand(int64_t n, int64_t *out) {
    int32_t r[34 + 400];
    int64_t total = 344 + n;
    int32_t *v = (int32_t *)malloc(sizeof(int32_t) * (total + 1));
    v[0] = 1;
    for (int i = 1; i < 31; ++i) {
        int64_t hi = v[i - 1] / 127773, lo = v[i - 1] % 127773;
        int64_t word = 16807 * lo - 2836 * hi;
        if (word < 0) word += 2147483647;
        v[i] = (int32_t)word;
    }
    for (int i = 31; i < 34; ++i) v[i] = v[i - 31];
    for (int64_t i = 34; i < total; ++i) v[i] = (int32_t)((uint32_t)v[i - 31] + (uint32_t)v[i - 3]);
    for (int64_t i = 0; i < n; ++i) out[i] = (int64_t)(((uint32_t)v[344 + i]) >> 1);
    free(v);
    (void)r;
}

static uint64_t lcg_next(uint64_t *st) {
    *st = *st * 25214903917ULL + 11ULL;
    return *st;
}
static int64_t rand_max(uint64_t *st, int64_t x) { return (int64_t)(lcg_next(st) % (uint64_t)x); }

typedef struct {
    const int64_t *head_hrt; /* train triples sorted (h, r, t) -- trainHead   */
    const int64_t *tail_hrt; /* train triples sorted (t, r, h) -- trainTail   */
    const int64_t *rel_hrt;  /* train triples sorted (h, t, r) -- trainRel    */
    const int64_t *lef_head, *rig_head, *lef_tail, *rig_tail, *lef_rel, *rig_rel;
    int64_t n_ent, n_rel;
} orc_train_index;

/* corrupt_head (Corrupt.h:7-43): a replacement TAIL for (h, r). */
static int64_t corrupt_head(const orc_train_index *ix, uint64_t *st, int64_t h, int64_t r) {
    const int64_t *T = ix->head_hrt; /* fields: [3*i+0]=h, +1=r, +2=t */
    int64_t lef = ix->lef_head[h] - 1, rig = ix->rig_head[h], mid, ll, rr;
    while (lef + 1 < rig) { mid = (lef + rig) >> 1; if (T[3 * mid + 1] >= r) rig = mid; else lef = mid; }
    ll = rig;
    lef = ix->lef_head[h]; rig = ix->rig_head[h] + 1;
    while (lef + 1 < rig) { mid = (lef + rig) >> 1; if (T[3 * mid + 1] <= r) lef = mid; else rig = mid; }
    rr = lef;
    int64_t tmp = rand_max(st, ix->n_ent - (rr - ll + 1));
    if (tmp < T[3 * ll + 2]) return tmp;
    if (tmp > T[3 * rr + 2] - rr + ll - 1) return tmp + rr - ll + 1;
    lef = ll; rig = rr + 1;
    while (lef + 1 < rig) { mid = (lef + rig) >> 1; if (T[3 * mid + 2] - mid + ll - 1 < tmp) lef = mid; else rig = mid; }
    return tmp + lef - ll + 1;
}

/* corrupt_tail (Corrupt.h:45-81): a replacement HEAD for (t, r).
 * tail_hrt rows hold (h, r, t) sorted by (t, r, h). */
static int64_t corrupt_tail(const orc_train_index *ix, uint64_t *st, int64_t t, int64_t r) {
    const int64_t *T = ix->tail_hrt;
    int64_t lef = ix->lef_tail[t] - 1, rig = ix->rig_tail[t], mid, ll, rr;
    while (lef + 1 < rig) { mid = (lef + rig) >> 1; if (T[3 * mid + 1] >= r) rig = mid; else lef = mid; }
    ll = rig;
    lef = ix->lef_tail[t]; rig = ix->rig_tail[t] + 1;
    while (lef + 1 < rig) { mid = (lef + rig) >> 1; if (T[3 * mid + 1] <= r) lef = mid; else rig = mid; }
    rr = lef;
    int64_t tmp = rand_max(st, ix->n_ent - (rr - ll + 1));
    if (tmp < T[3 * ll + 0]) return tmp;
    if (tmp > T[3 * rr + 0] - rr + ll - 1) return tmp + rr - ll + 1;
    lef = ll; rig = rr + 1;
    while (lef + 1 < rig) { mid = (lef + rig) >> 1; if (T[3 * mid + 0] - mid + ll - 1 < tmp) lef = mid; else rig = mid; }
    return tmp + lef - ll + 1;
}

/* corrupt_rel (Corrupt.h:85-162): rel_hrt rows (h, r, t) sorted by (h, t, r). prob NULL: p == false
 * (uniform draw); else importProb's table, p == true (Corrupt.h:111-147): the cumulative list of
 * prob / sum over the relations outside the (h, t) block (r's own column excluded), binary-searched
 * for m = rand_max(10000) / 10000, with the reference's record / prob_tmp arrays. */
static int64_t corrupt_rel(const orc_train_index *ix, uint64_t *st, int64_t h, int64_t t, int64_t r,
                           const float *prob) {
    const int64_t *T = ix->rel_hrt;
    int64_t lef = ix->lef_rel[h] - 1, rig = ix->rig_rel[h], mid, ll, rr;
    while (lef + 1 < rig) { mid = (lef + rig) >> 1; if (T[3 * mid + 2] >= t) rig = mid; else lef = mid; }
    ll = rig;
    lef = ix->lef_rel[h]; rig = ix->rig_rel[h] + 1;
    while (lef + 1 < rig) { mid = (lef + rig) >> 1; if (T[3 * mid + 2] <= t) lef = mid; else rig = mid; }
    rr = lef;
    int64_t tmp;
    if (!prob) {
        tmp = rand_max(st, ix->n_rel - (rr - ll + 1));
    } else {
        const int64_t R = ix->n_rel, start = r * (R - 1);
        float sum = 1;
        unsigned char *record = (unsigned char *)calloc((size_t)(R - 1), 1);
        for (int64_t i = ll; i <= rr; ++i) {
            const int64_t rel = T[3 * i + 1];
            if (rel > r) { sum -= prob[start + rel - 1]; record[rel - 1] = 1; }
            else if (rel < r) { sum -= prob[start + rel]; record[rel] = 1; }
        }
        float *prob_tmp = (float *)calloc((size_t)(R - (rr - ll + 1)) + 1, sizeof(float));
        int64_t cnt = 0;
        float rec = 0;
        for (int64_t i = start; i < start + R - 1; ++i) {
            if (record[i - start]) continue;
            rec += prob[i] / sum;
            prob_tmp[cnt++] = rec;
        }
        const float m = (float)((double)rand_max(st, 10000) / 10000.0);
        lef = 0; rig = cnt - 1;
        while (lef < rig) { mid = (lef + rig) >> 1; if (prob_tmp[mid] < m) lef = mid + 1; else rig = mid; }
        tmp = rig;
        free(prob_tmp);
        free(record);
    }
    if (tmp < T[3 * ll + 1]) return tmp;
    if (tmp > T[3 * rr + 1] - rr + ll - 1) return tmp + rr - ll + 1;
    lef = ll; rig = rr + 1;
    while (lef + 1 < rig) { mid = (lef + rig) >> 1; if (T[3 * mid + 1] - mid + ll - 1 < tmp) lef = mid; else rig = mid; }
    return tmp + lef - ll + 1;
}

/* importProb (Reader.h:26-49): kl_prob.txt (n_rel x (n_rel - 1) floats) -> exp(-kl / temp)
 * normalised per relation row, in float. Returns -1 when the file cannot be opened. */
int orc_import_prob(const char *path, int64_t n_rel, float temp, float *prob) {
    FILE *fin = fopen(path, "r");
    if (!fin) return -1;
    const int64_t n = n_rel * (n_rel - 1);
    for (int64_t i = 0; i < n; ++i) prob[i] = 0.0f;
    for (int64_t i = 0; i < n; ++i)
        if (fscanf(fin, "%f", &prob[i]) != 1) break;
    fclose(fin);
    float sum = 0.0f;
    for (int64_t i = 0; i < n_rel; ++i) {
        for (int64_t j = 0; j < n_rel - 1; ++j) {
            /* Reader.h:40: unqualified exp(float) with <cmath> only = (float)exp((double)x) */
            float e = (float)exp((double)(-prob[i * (n_rel - 1) + j] / temp));
            sum += e;
            prob[i * (n_rel - 1) + j] = e;
        }
        for (int64_t j = 0; j < n_rel - 1; ++j) prob[i * (n_rel - 1) + j] /= sum;
        sum = 0;
    }
    return 0;
}

/* sampling / getBatch (Base.cpp:78-197), run thread-by-thread sequentially.
 * seeds[work_threads]: per-thread LCG state, advanced in place.
 * train_list: deduplicated training triples (h, r, t) in cmp_head order.
 * bern: right_mean / left_mean per relation (NULL when bern is off). */
int orc_sampling(const int64_t *train_list, int64_t train_total, const int64_t *head_hrt,
                 const int64_t *tail_hrt, const int64_t *rel_hrt, const int64_t *lef_head,
                 const int64_t *rig_head, const int64_t *lef_tail, const int64_t *rig_tail,
                 const int64_t *lef_rel, const int64_t *rig_rel, const float *left_mean,
                 const float *right_mean, int64_t n_ent, int64_t n_rel, uint64_t *seeds, int64_t work_threads,
                 int64_t *batch_h, int64_t *batch_t, int64_t *batch_r, float *batch_y, int64_t batch_size,
                 int64_t neg_rate, int64_t neg_rel_rate, int64_t mode, const float *rel_prob) {
    orc_train_index ix = {head_hrt, tail_hrt, rel_hrt, lef_head, rig_head, lef_tail, rig_tail,
                          lef_rel, rig_rel, n_ent, n_rel};
    for (int64_t id = 0; id < work_threads; ++id) {
        int64_t lef, rig;
        if (batch_size % work_threads == 0) {
            lef = id * (batch_size / work_threads);
            rig = (id + 1) * (batch_size / work_threads);
        } else {
            lef = id * (batch_size / work_threads + 1);
            rig = (id + 1) * (batch_size / work_threads + 1);
            if (rig > batch_size) rig = batch_size;
        }
        uint64_t *st = &seeds[id];
        for (int64_t b = lef; b < rig; ++b) {
            int64_t i = rand_max(st, train_total);
            int64_t h = train_list[3 * i], r = train_list[3 * i + 1], t = train_list[3 * i + 2];
            batch_h[b] = h; batch_t[b] = t; batch_r[b] = r; batch_y[b] = 1;
            int64_t last = batch_size;
            for (int64_t k = 0; k < neg_rate; ++k) {
                if (mode == 0) {
                    float prob = 500;
                    if (left_mean) prob = 1000 * right_mean[r] / (right_mean[r] + left_mean[r]);
                    if ((float)(lcg_next(st) % 1000) < prob) {
                        batch_h[b + last] = h; batch_t[b + last] = corrupt_head(&ix, st, h, r); batch_r[b + last] = r;
                    } else {
                        batch_h[b + last] = corrupt_tail(&ix, st, t, r); batch_t[b + last] = t; batch_r[b + last] = r;
                    }
                } else if (mode == -1) {
                    batch_h[b + last] = corrupt_tail(&ix, st, t, r); batch_t[b + last] = t; batch_r[b + last] = r;
                } else {
                    batch_h[b + last] = h; batch_t[b + last] = corrupt_head(&ix, st, h, r); batch_r[b + last] = r;
                }
                batch_y[b + last] = -1;
                last += batch_size;
            }
            for (int64_t k = 0; k < neg_rel_rate; ++k) {
                batch_h[b + last] = h; batch_t[b + last] = t; batch_r[b + last] = corrupt_rel(&ix, st, h, t, r, rel_prob);
                batch_y[b + last] = -1;
                last += batch_size;
            }
        }
    }
    return 0;
}

/* -------------------------------------------------- candidate-list ranks -- */
/* main.evaluate (main.py:232-250): TransE L1 without normalisation
 * (module/NegativeSampling.py:294-302), score = |(h + r) - t|_1 per candidate,
 * rank = #(n < p) + #(n == p) // 2 + 1 ; candidates CSR, true tail first. */
int orc_candidate_rank_transe(const float *ent, const float *rel, int dim, const int64_t *qh,
                              const int64_t *qr, const int64_t *cand_off, const int64_t *cand_ids,
                              int64_t n_query, float *scores_out, int64_t *rank_out) {
    int d = dim;
    float *hr = (float *)malloc(sizeof(float) * d);
    for (int64_t q = 0; q < n_query; ++q) {
        const float *h = ent + qh[q] * d, *r = rel + qr[q] * d;
        for (int k = 0; k < d; ++k) hr[k] = h[k] + r[k];
        int64_t a = cand_off[q], b = cand_off[q + 1];
        float p = 0.0f;
        int64_t less = 0, eq = 0;
        for (int64_t c = a; c < b; ++c) {
            const float *t = ent + cand_ids[c] * d;
            float s = 0.0f;
            for (int k = 0; k < d; ++k) s = s + fabsf(hr[k] - t[k]);
            if (scores_out) scores_out[c] = s;
            if (c == a) p = s;
            else { less += (s < p); eq += (s == p); }
        }
        rank_out[q] = less + eq / 2 + 1;
    }
    free(hr);
    return 0;
}
