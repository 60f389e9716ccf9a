/*
 * oracle.c — TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Serial C restatement of the reference's canonical integer forward pass.  Each function cites
 * the reference lines it follows (paths relative to /root/reference/edge-eegnet_wolf).
 * Arithmetic: int32 accumulators, C '/' (truncation toward zero), '>>' arithmetic shift,
 * clip to [-128, 127] (__CLIP_R(x, 127) of the PULP SDK, clip_balanced=False in the golden model;
 * or_params_t.clip_lo = -127 gives the golden model's clip_balanced=True).
 */
#include "oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define L2_TAPS 64
#define L2_PAD_START 31 /* gen_net_header.py:142 */
#define L2_PAD_END 32   /* gen_net_header.py:143 */
#define L3_TAPS 16
#define L3_PAD_START 7 /* gen_net_header.py:162 */
#define L3_PAD_END 8   /* gen_net_header.py:163 */

/* clip to [p->clip_lo, 127]: clip_lo = -128 is the C's __CLIP_R(x, 127); -127 is the golden
 * model's clip_balanced=True (functional.py:89-91), which has no C build */
static inline int32_t clipq(const or_params_t* p, int32_t v) {
    return v < p->clip_lo ? p->clip_lo : (v > 127 ? 127 : v);
}

static inline int32_t clip8(int32_t v) { return v < -128 ? -128 : (v > 127 ? 127 : v); }

/* ---- func primitives (src/cl/func/{dotp,xcorr,conv,transform,flip}.c) ------------------------
 * Each is pinned by the reference's own func test (test/cl/func/<name>/testcase.py: NumPy
 * expectations at the sizes listed there) in tests/test_oracle_func.py, and the layers below
 * are built from them. */

/* func_dotp (dotp.c:45, and the SIMD form :82): int8 dot product into int32 */
int32_t or_func_dotp(const int8_t* a, const int8_t* b, unsigned len) {
    int32_t acc = 0;
    for (unsigned i = 0; i < len; i++) acc += (int32_t)a[i] * (int32_t)b[i];
    return acc;
}

static inline int32_t dotp(const int8_t* a, const int8_t* b, int len) { return or_func_dotp(a, b, (unsigned)len); }

/* func_dotp_slow (dotp.c:172-210): scalar dot product over strided vectors, sum_i a[i as] b[i bs]
 * (two interleaved accumulators in the reference; the same int32 sum) */
int32_t or_func_dotp_slow(const int8_t* a, unsigned as, const int8_t* b, unsigned bs, unsigned len) {
    int32_t acc = 0;
    for (unsigned i = 0; i < len; i++) acc += (int32_t)a[(size_t)i * as] * (int32_t)b[(size_t)i * bs];
    return acc;
}

/* The longer vector is the signal (xcorr.c:44-57, conv.c:67-80 swap a and b when a is shorter). */
static void order_ab(const int8_t** a, unsigned* la, const int8_t** b, unsigned* lb) {
    if (*la < *lb) {
        const int8_t* t = *a; *a = *b; *b = t;
        unsigned n = *la; *la = *lb; *lb = n;
    }
}

/* func_xcorr (xcorr.c:44): valid cross-correlation, r[i] = sum_j a[i + j] * b[j], la - lb + 1 outputs */
void or_func_xcorr(const int8_t* a, unsigned la, const int8_t* b, unsigned lb, int32_t* r) {
    order_ab(&a, &la, &b, &lb);
    for (unsigned i = 0; i + lb <= la; i++) r[i] = or_func_dotp(a + i, b, lb);
}

/* func_xcorr_scale (xcorr.c:346): clip((xcorr + offset) / div) */
void or_func_xcorr_scale(const int8_t* a, unsigned la, const int8_t* b, unsigned lb, int32_t div, int32_t offset,
                         int8_t* r) {
    order_ab(&a, &la, &b, &lb);
    for (unsigned i = 0; i + lb <= la; i++) r[i] = (int8_t)clip8((or_func_dotp(a + i, b, lb) + offset) / div);
}

static inline int32_t conv_at(const int8_t* a, const int8_t* b, unsigned lb, unsigned i) {
    int32_t acc = 0;
    for (unsigned j = 0; j < lb; j++) acc += (int32_t)a[i + j] * (int32_t)b[lb - 1 - j];
    return acc;
}

/* func_conv (conv.c:67): valid true convolution, r[i] = sum_j a[i + j] * b[lb - 1 - j] */
void or_func_conv(const int8_t* a, unsigned la, const int8_t* b, unsigned lb, int32_t* r) {
    order_ab(&a, &la, &b, &lb);
    for (unsigned i = 0; i + lb <= la; i++) r[i] = conv_at(a, b, lb, i);
}

/* func_conv_scale (conv.c:105): acc = offset + conv; clip(acc / div) */
void or_func_conv_scale(const int8_t* a, unsigned la, const int8_t* b, unsigned lb, int32_t div, int32_t offset,
                        int8_t* r) {
    order_ab(&a, &la, &b, &lb);
    for (unsigned i = 0; i + lb <= la; i++) r[i] = (int8_t)clip8((offset + conv_at(a, b, lb, i)) / div);
}

/* func_transform_32to8 (transform.c:47): r[k] = clip(in[k * stride] / div).  Writes whole
 * 4-byte packs: a partial last pack is zero-filled (transform.c:95-121), so r holds
 * ceil(len / 4) * 4 bytes. */
void or_func_transform_32to8(const int32_t* in, unsigned len, int32_t div, unsigned stride, int8_t* r) {
    for (unsigned k = 0; k < (len + 3) / 4 * 4; k++) r[k] = k < len ? (int8_t)clip8(in[(size_t)k * stride] / div) : 0;
}

/* func_transform_32to8_bias (transform.c:138): r[k] = clip((in[k * stride] + bias) / div), same packing */
void or_func_transform_32to8_bias(const int32_t* in, unsigned len, int32_t div, int32_t bias, unsigned stride,
                                  int8_t* r) {
    for (unsigned k = 0; k < (len + 3) / 4 * 4; k++)
        r[k] = k < len ? (int8_t)clip8((in[(size_t)k * stride] + bias) / div) : 0;
}

/* func_flip_2d_axis (flip.c:92): in [outer][align4(inner)] -> r [inner][align4(outer)], the
 * alignment padding of each output row zero (flip.c:161-300 writes whole 4-byte parts). */
void or_func_flip_2d_axis(const int8_t* in, unsigned outer, unsigned inner, int8_t* r) {
    const unsigned ia = (inner + 3) / 4 * 4, oa = (outer + 3) / 4 * 4;
    for (unsigned i = 0; i < inner; i++)
        for (unsigned o = 0; o < oa; o++) r[(size_t)i * oa + o] = o < outer ? in[(size_t)o * ia + i] : 0;
}

/* Layer 1: layer1.c:53-101 (_net_layer1_kernel) — per filter, per time sample:
 * y[f][t] = clip((dotp(x[t], W1[f], C_ALIGN) + off[f]) / fac[f]) */
void or_layer1(const or_params_t* p, const int8_t* x, int8_t* y1) {
    memset(y1, 0, (size_t)p->F1 * p->T_ALIGN);
    for (int f = 0; f < p->F1; f++) {
        const int8_t* w = p->l1_weight_align + (size_t)f * p->C_ALIGN;
        int32_t fac = p->l1_factor[f], off = p->l1_offset[f];
        for (int t = 0; t < p->T; t++) {
            int32_t e = dotp(x + (size_t)t * p->C_ALIGN, w, p->C_ALIGN);
            e = (e + off) / fac;
            y1[(size_t)f * p->T_ALIGN + t] = (int8_t)clipq(p, e);
        }
    }
}

/* Layer 2, REORDER_BN branch: layer2.c:56-118 (kernel) and :231-326 (driver).
 * Row padded with 31 leading / 32 trailing zeros (:262-275), func_xcorr with the torch-order
 * weights net_l2_weight_reverse (xcorr.c:44: r[i] = sum_j a[i+j] * b[j]), then for each of the
 * T/8 output samples: sum_{8} max(a, -(off >> 3)), + off, / fac, clip (:97-117). */
void or_layer2(const or_params_t* p, const int8_t* y1, int8_t* y2) {
    const int pad_len = p->T + L2_PAD_START + L2_PAD_END;
    int8_t* row = (int8_t*)calloc((size_t)pad_len, 1);
    int32_t* xc = (int32_t*)malloc(sizeof(int32_t) * (size_t)(pad_len - L2_TAPS + 1));
    int8_t* xs = (int8_t*)malloc((size_t)(pad_len - L2_TAPS + 1));
    memset(y2, 0, (size_t)p->F2 * p->T8_ALIGN);
    for (int f = 0; f < p->F2; f++) {
        memset(row, 0, (size_t)pad_len);
        memcpy(row + L2_PAD_START, y1 + (size_t)f * p->T_ALIGN, (size_t)p->T);
        const int8_t* w = p->l2_weight_reverse + (size_t)f * L2_TAPS;
        or_func_xcorr(row, (unsigned)pad_len, w, L2_TAPS, xc); /* pad_len - 63 == T outputs */
        const int32_t fac = p->l2_factor[f], off = p->l2_offset[f];
        const int32_t* it = xc;
        if (p->reorder_bn) {
            const int32_t thr = -(off >> 3);
            for (int u = 0; u < p->T8; u++) {
                int32_t sum = 0;
                for (int k = 0; k < 8; k++) {
                    int32_t v = *(it++);
                    sum += v > thr ? v : thr; /* __MAX */
                }
                sum = sum + off;
                sum = sum / fac;
                y2[(size_t)f * p->T8_ALIGN + u] = (int8_t)clipq(p, sum);
            }
        } else {
            /* layer2.c:139-210: factor and offset >> 3, func_xcorr_scale (xcorr.c:346 ->
             * transform.c:224: clip((x + offset) / factor) to int8), then sum of 8 ReLUs >> 3, clip */
            const int32_t fac3 = fac >> 3, off3 = off >> 3;
            or_func_xcorr_scale(row, (unsigned)pad_len, w, L2_TAPS, fac3, off3, xs);
            const int8_t* is = xs;
            for (int u = 0; u < p->T8; u++) {
                int32_t sum = 0;
                for (int k = 0; k < 8; k++) {
                    int32_t v = *(is++); /* the ReLU makes the lower clip bound irrelevant */
                    sum += v > 0 ? v : 0;
                }
                sum = sum >> 3;
                y2[(size_t)f * p->T8_ALIGN + u] = (int8_t)clipq(p, sum);
            }
        }
    }
    free(xs);
    free(xc);
    free(row);
}

/* Layer 3: layer3.c:49-79 (kernel) + :100-159 (driver).  Row padded 7/8 (:122-131),
 * func_conv_scale(row, 155, net_l3_weight[f], 16, NET_L3_FACTOR, 0) — a TRUE convolution
 * (conv.c:105-146: acc = offset + sum_i a[i_out+i] * b[len-1-i]; acc / div; clip). */
void or_layer3(const or_params_t* p, const int8_t* y2, int8_t* y3) {
    const int pad_len = p->T8 + L3_PAD_START + L3_PAD_END;
    int8_t* row = (int8_t*)calloc((size_t)pad_len, 1);
    memset(y3, 0, (size_t)p->F2 * p->T8_ALIGN);
    for (int f = 0; f < p->F2; f++) {
        memset(row, 0, (size_t)pad_len);
        memcpy(row + L3_PAD_START, y2 + (size_t)f * p->T8_ALIGN, (size_t)p->T8);
        const int8_t* w = p->l3_weight + (size_t)f * L3_TAPS;
        int8_t* out = y3 + (size_t)f * p->T8_ALIGN;
        or_func_conv_scale(row, (unsigned)pad_len, w, L3_TAPS, p->l3_factor, 0, out); /* offset 0: layer3.c:70 */
        for (int i = 0; i < p->T8; i++) out[i] = (int8_t)clipq(p, out[i]);  /* balanced clipping */
    }
    free(row);
}

/* net_layer3_flip_inplace: layer3.c:243-268 -> func_flip_2d_axis (flip.c:92):
 * [F2][T8_ALIGN] -> [T8][F2] */
void or_layer3_flip_inplace(const or_params_t* p, int8_t* y3) {
    int8_t* tmp = (int8_t*)malloc((size_t)p->F2 * p->T8_ALIGN);
    memcpy(tmp, y3, (size_t)p->F2 * p->T8_ALIGN);
    memset(y3, 0, (size_t)p->F2 * p->T8_ALIGN);
    or_func_flip_2d_axis(tmp, (unsigned)p->F2, (unsigned)p->T8, y3); /* F2 = 16: rows of F2 bytes */
    free(tmp);
}

/* Layer 4, FLIP_LAYERS + REORDER_BN: layer4.c:51-149.  For each output filter k and each of the
 * T64 pooled samples: sum_{8} max(dotp(x[t], W4[k], F2), -(off >> 3)); + off; / fac; clip. */
void or_layer4(const or_params_t* p, const int8_t* y3t, int8_t* y4) {
    memset(y4, 0, (size_t)p->F2 * p->T64_ALIGN);
    for (int k = 0; k < p->F2; k++) {
        const int32_t fac = p->l4_factor[k], off = p->l4_offset[k];
        const int32_t thr = -(off >> 3);
        const int32_t fac3 = fac >> 3, off3 = off >> 3;
        const int8_t* w = p->l4_weight + (size_t)k * p->F2;
        const int8_t* it = y3t;
        for (int v = 0; v < p->T64; v++) {
            int32_t sum = 0;
            for (int i = 0; i < 8; i++) {
                int32_t e = dotp(it, w, p->F2);
                if (p->reorder_bn) {
                    e = e > thr ? e : thr;
                } else {
                    /* layer4.c:113-118: BN per element (no clip), then ReLU */
                    e = (e + off3) / fac3;
                    e = e > 0 ? e : 0;
                }
                sum += e;
                it += p->F2;
            }
            if (p->reorder_bn) {
                sum = sum + off;
                sum = sum / fac;
            } else {
                sum = sum >> 3;  /* layer4.c:130 */
            }
            y4[(size_t)k * p->T64_ALIGN + v] = (int8_t)clipq(p, sum);
        }
    }
}

/* Layer 4 without FLIP_LAYERS: layer4.c:380-505.  The same arithmetic as or_layer4 on the
 * unflipped [F2][T8_ALIGN] layer-3 output: each element is func_dotp_slow down a column (stride
 * T8_ALIGN) against the weight row.  A second restatement of layer 4 from the reference's other
 * build branch, used to cross-check or_layer4 (tests/test_oracle_func.py). */
void or_layer4_noflip(const or_params_t* p, const int8_t* y3, int8_t* y4) {
    memset(y4, 0, (size_t)p->F2 * p->T64_ALIGN);
    for (int k = 0; k < p->F2; k++) {
        int32_t fac = p->l4_factor[k], off = p->l4_offset[k], thr = 0;
        if (p->reorder_bn) thr = -(off >> 3);
        else { fac = fac >> 3; off = off >> 3; }
        const int8_t* w = p->l4_weight + (size_t)k * p->F2;
        const int8_t* it = y3;
        for (int v = 0; v < p->T64; v++) {
            int32_t sum = 0;
            for (int i = 0; i < 8; i++) {
                int32_t e = or_func_dotp_slow(it, (unsigned)p->T8_ALIGN, w, 1, (unsigned)p->F2);
                if (p->reorder_bn) e = e > thr ? e : thr;
                else { e = (e + off) / fac; e = e > 0 ? e : 0; }
                sum += e;
                it += 1;
            }
            if (p->reorder_bn) sum = (sum + off) / fac;
            else sum = sum >> 3;
            y4[(size_t)k * p->T64_ALIGN + v] = (int8_t)clipq(p, sum);
        }
    }
}

/* Layer 5: layer5.c:43-89.  z[n] = dotp(y4, W5[n], F2*T64_ALIGN) + bias[n] (the weight's pad
 * positions are zero), then func_transform_32to8 (transform.c:47-121): z / NET_L5_FACTOR, clip. */
void or_layer5(const or_params_t* p, const int8_t* y4, int8_t* out) {
    const int len = p->F2 * p->T64_ALIGN;
    int8_t* xin = (int8_t*)malloc((size_t)len);
    /* the reference leaves the T64..T64_ALIGN tail of each row uninitialised; the weight is zero
     * there, so zero it for a deterministic product */
    for (int k = 0; k < p->F2; k++)
        for (int v = 0; v < p->T64_ALIGN; v++)
            xin[k * p->T64_ALIGN + v] = v < p->T64 ? y4[(size_t)k * p->T64_ALIGN + v] : 0;
    int32_t* z = (int32_t*)malloc(sizeof(int32_t) * (size_t)p->N);
    int8_t* zq = (int8_t*)malloc((size_t)(p->N + 3) / 4 * 4);
    for (int n = 0; n < p->N; n++) z[n] = dotp(xin, p->l5_weight + (size_t)n * len, len) + (int32_t)p->l5_bias[n];
    or_func_transform_32to8(z, (unsigned)p->N, p->l5_factor, 1, zq);
    for (int n = 0; n < p->N; n++) out[n] = (int8_t)clipq(p, zq[n]);
    free(zq);
    free(z);
    free(xin);
}

/* net_model_compute: model.c:84-148 */
void or_model_compute(const or_params_t* p, const int8_t* x, int8_t* out) {
    int8_t* y1 = (int8_t*)malloc((size_t)p->F1 * p->T_ALIGN);
    int8_t* y2 = (int8_t*)malloc((size_t)p->F2 * p->T8_ALIGN);
    int8_t* y3 = (int8_t*)malloc((size_t)p->F2 * p->T8_ALIGN);
    int8_t* y4 = (int8_t*)malloc((size_t)p->F2 * p->T64_ALIGN);
    or_layer1(p, x, y1);
    or_layer2(p, y1, y2);
    or_layer3(p, y2, y3);
    or_layer3_flip_inplace(p, y3);
    or_layer4(p, y3, y4);
    or_layer5(p, y4, out);
    free(y1); free(y2); free(y3); free(y4);
}

typedef struct {
    const or_params_t* p;
    const int8_t* x;
    size_t stride;
    int8_t* out;
    size_t b0, b1;
} or_job_t;

static void* or_worker(void* arg) {
    or_job_t* j = (or_job_t*)arg;
    const or_params_t* p = j->p;
    int8_t* xa = (int8_t*)calloc((size_t)p->T * p->C_ALIGN, 1);
    for (size_t b = j->b0; b < j->b1; b++) {
        const int8_t* xt = j->x + b * j->stride;
        for (int t = 0; t < p->T; t++)
            memcpy(xa + (size_t)t * p->C_ALIGN, xt + (size_t)t * p->C, (size_t)p->C);
        or_model_compute(p, xa, j->out + b * (size_t)p->N);
    }
    free(xa);
    return NULL;
}

void or_model_compute_batch(const or_params_t* p, const int8_t* x, size_t trial_stride,
                            int8_t* out, size_t B, int nthreads) {
    if (nthreads <= 1 || B < 2) {
        or_job_t j = {p, x, trial_stride, out, 0, B};
        or_worker(&j);
        return;
    }
    if ((size_t)nthreads > B) nthreads = (int)B;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
    or_job_t* jobs = (or_job_t*)malloc(sizeof(or_job_t) * (size_t)nthreads);
    for (int i = 0; i < nthreads; i++) {
        jobs[i].p = p; jobs[i].x = x; jobs[i].stride = trial_stride; jobs[i].out = out;
        jobs[i].b0 = B * (size_t)i / (size_t)nthreads;
        jobs[i].b1 = B * (size_t)(i + 1) / (size_t)nthreads;
        pthread_create(&th[i], NULL, or_worker, &jobs[i]);
    }
    for (int i = 0; i < nthreads; i++) pthread_join(th[i], NULL);
    free(th);
    free(jobs);
}
