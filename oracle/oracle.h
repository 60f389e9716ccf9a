/*
 * oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C restatement of the reference's canonical integer forward pass
 * (edge-eegnet_wolf/src/cl/net/layer{1..5}.c with -DPARALLEL -DCROSS_CORRELATE -DFLIP_LAYERS, and
 * either -DREORDER_BN (canonical) or not (or_params_t.reorder_bn), serialised).  It is the checker for the HIP path: only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load it.  The product library (libmibminet.so) never links or
 * calls it.
 *
 * Parity pin: the restatement is checked against SURVEY.md Appendix B's known answer
 * (logits [-2, -7, -11, 18] and the derived factors, produced once by the reference golden model)
 * and against an independent NumPy restatement of python_utils/golden_model.py
 * (oracle/golden_np.py) on every committed fixture (tests/golden/).
 *
 * All buffers use the reference layouts documented in src/cl/net/layers.h / model.h:
 *   input  x   [T][C_ALIGN]     int8 (model.c:81)
 *   layer1 y1  [F1][T_ALIGN]    int8 (layer1.c:116)
 *   layer2 y2  [F2][T8_ALIGN]   int8 (layer2.c:225)
 *   layer3 y3  [F2][T8_ALIGN]   int8 (layer3.c:95); after net_layer3_flip_inplace [T8][F2]
 *   layer4 y4  [F2][T64_ALIGN]  int8 (layer4.c:168)
 *   layer5 out [N]              int8 (layer5.c:41)
 * Padding bytes of every output are written as zero.
 */
#ifndef MIBMINET_ORACLE_H
#define MIBMINET_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    int32_t C, T, F1, F2, N;
    int32_t C_ALIGN, T_ALIGN, T8, T8_ALIGN, T64, T64_ALIGN;
    const int32_t* l1_factor;       /* [F2] */
    const int32_t* l1_offset;       /* [F2] */
    const int8_t*  l1_weight_align; /* [F2][C_ALIGN] */
    const int32_t* l2_factor;       /* [F2] */
    const int32_t* l2_offset;       /* [F2] */
    const int8_t*  l2_weight_reverse; /* [F2][64] */
    int32_t        l3_factor;
    const int8_t*  l3_weight;       /* [F2][16], flipped */
    const int32_t* l4_factor;       /* [F2] */
    const int32_t* l4_offset;       /* [F2] */
    const int8_t*  l4_weight;       /* [F2][F2] */
    int32_t        l5_factor;
    const int8_t*  l5_bias;         /* [N] */
    const int8_t*  l5_weight;       /* [N][F2*T64_ALIGN] */
    int32_t        reorder_bn;      /* 1: -DREORDER_BN branches (canonical), 0: the plain ones */
    int32_t        clip_lo;         /* lower clip bound: -128 (the C's __CLIP_R) or -127 (golden
                                       model clip_balanced=True, functional.py:89-91) */
} or_params_t;

/* func primitives (src/cl/func/{dotp,xcorr,conv,transform,flip}.c), clip to [-128, 127] as the C's __CLIP_R */
int32_t or_func_dotp_slow(const int8_t* a, unsigned as, const int8_t* b, unsigned bs, unsigned len);
int32_t or_func_dotp(const int8_t* a, const int8_t* b, unsigned len);
void or_func_xcorr(const int8_t* a, unsigned la, const int8_t* b, unsigned lb, int32_t* r);
void or_func_xcorr_scale(const int8_t* a, unsigned la, const int8_t* b, unsigned lb, int32_t div, int32_t offset,
                         int8_t* r);
void or_func_conv(const int8_t* a, unsigned la, const int8_t* b, unsigned lb, int32_t* r);
void or_func_conv_scale(const int8_t* a, unsigned la, const int8_t* b, unsigned lb, int32_t div, int32_t offset,
                        int8_t* r);
void or_func_transform_32to8(const int32_t* in, unsigned len, int32_t div, unsigned stride, int8_t* r);
void or_func_transform_32to8_bias(const int32_t* in, unsigned len, int32_t div, int32_t bias, unsigned stride,
                                  int8_t* r);
void or_func_flip_2d_axis(const int8_t* in, unsigned outer, unsigned inner, int8_t* r);

void or_layer1(const or_params_t* p, const int8_t* x, int8_t* y1);
void or_layer2(const or_params_t* p, const int8_t* y1, int8_t* y2);
void or_layer3(const or_params_t* p, const int8_t* y2, int8_t* y3);
void or_layer3_flip_inplace(const or_params_t* p, int8_t* y3);
void or_layer4(const or_params_t* p, const int8_t* y3t, int8_t* y4);
void or_layer5(const or_params_t* p, const int8_t* y4, int8_t* out);
/* layer 4 of the non-FLIP_LAYERS build (layer4.c:380-505) on the unflipped [F2][T8_ALIGN] input */
void or_layer4_noflip(const or_params_t* p, const int8_t* y3, int8_t* y4);

/* net_model_compute restated (model.c:84-148); x is [T][C_ALIGN]. */
void or_model_compute(const or_params_t* p, const int8_t* x, int8_t* out);

/* Batched driver over the device layout used by the GPU path: trial b starts at
 * x + b*trial_stride and is stored [T][C] (no channel padding).  out is [B][N].
 * nthreads <= 1 runs serially; otherwise trials are split over pthreads. */
void or_model_compute_batch(const or_params_t* p, const int8_t* x, size_t trial_stride,
                            int8_t* out, size_t B, int nthreads);

#ifdef __cplusplus
}
#endif
#endif
