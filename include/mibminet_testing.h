/*
 * mibminet_testing.h — test hooks of libmibminet (not part of the reference's interface).
 *
 * The library turns every C truncating division of the path, y = clip(trunc(v / fac)), into a
 * float multiply by a reciprocal r that it chooses and verifies on the host (DESIGN.md §3,
 * "Exact requantisation"), or, for parameter sets outside that envelope, into an exact integer
 * division by a magic multiplier.  These hooks expose both so the tests can check them against
 * exhaustive integer division.
 */
#ifndef MIBMINET_TESTING_H
#define MIBMINET_TESTING_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* The reciprocal the library would use for factor `fac` when |v| <= vmax and outputs must be
 * exact up to step kmax (128 for int8 clipping).  magic != 0 also requires and returns
 * c = -1.5 * 2^23 * r exact (the layer-1/3 fma form).  Returns 0, or NET_ERR_RANGE when no
 * float reciprocal is exact over that range. */
int mibminet_test_reciprocal(int32_t fac, int64_t vmax, int32_t kmax, int32_t magic, float* r, float* c);

/* The floor-form constants of the plain-BN branches (layer2.c:139-210, layer4.c:113-130: every
 * element requantised, then the ReLU): for |x| <= vmax, e = clamp(floor(x / fac), 0, emax) is
 * computed as bits(fmed3(fma(f32 bits (mbits + x), r, c), K, K + emax)) - bits(K), K = 1.5 * 2^23.
 * Returns 0 with mbits (the magic the MFMA C-init adds to the offset), r and c, or NET_ERR_RANGE. */
int mibminet_test_floor_form(int32_t fac, int64_t emax, int64_t vmax, int32_t* mbits, float* r, float* c);

/* The float32 input quantiser of net_model_compute_batch_f32 (in-kernel, Markstein-corrected
 * quotient) on a flat device array: q[i] = quantize(x[i]) for i < n.  Enqueued on `stream`. */
int mibminet_test_quantize_f32(const float* x, int8_t* q, size_t n, float scale, int device, void* stream);

/* The multi-device driver of net_model_compute_batch_multi[_ct] run with recording stand-ins
 * instead of device work (no device needed): writes the order of its steps into `log` as
 * "P<device>" (parameter image made resident), "E<shard>" (shard enqueued) and "W<n>" (the first
 * n shards waited for), with the enqueue of shard `fail_at` failing (-1: none).  Returns what the
 * driver returns. */
int mibminet_test_multi_order(int ndev, const int* devices, int fail_at, char* log, size_t len);

/* Parameter-image uploads so far, and how many of them happened while the multi-device entry
 * points were enqueueing shards (0 when every device is prepared before the first enqueue). */
int mibminet_test_upload_stats(int64_t* uploads, int64_t* uploads_while_enqueueing);

/* Number of parameter-image copies resident on `device`. */
int mibminet_test_device_images(int device);

/* Exact-division builds (Cfg::XR, parameter sets outside the float requant envelope): the
 * integer division the kernels use at layers 1, 2 and 4 (forward_common.hpp, xdiv; constants from
 * mibminet.hip, xdiv_consts).  _host: the device instruction sequence emulated on the host,
 * q[i] = xdiv(e[i], d) for i < n (no device needed).  _gpu: the device function itself over
 * e = e0 .. e0 + count - 1 against C division in 64 bits, on `device`; *mismatches = the number of
 * e where they differ.  d != 0 (NET_ERR_INVALID otherwise). */
int mibminet_test_xdiv_host(const int32_t* e, size_t n, int32_t d, int32_t* q);
int mibminet_test_xdiv_gpu(int32_t d, int64_t e0, int64_t count, int64_t* mismatches, int device);

/* The REORDER_BN pooling constants of layer 2 or 4 for offset `off`: the threshold as the kernels
 * use it (thr = -(off >> 3) clamped to the layer's conv range [-V, V], V = 2^20 / 2^18) and the
 * offset term, so that sum_8 max(v - thr_c, 0) + offm (mod 2^32) = sum_8 max(v, thr) + off for
 * every reachable v. */
int mibminet_test_pool_consts(int32_t off, int32_t layer, int32_t* thr, int32_t* offm);

/* 1 when the loaded parameter set runs the exact-division kernels, 0 when the float requant
 * kernels, NET_ERR_NO_PARAMS when none is loaded. */
int mibminet_test_params_xr(void);

/* on != 0: every parameter set loaded after this call runs the run-time-dimension kernels
 * (forward_gen.hpp), the compiled geometries included, so that both kernel families can be
 * checked against the oracle on the same set; 0 restores the normal choice. */
int mibminet_test_force_general(int on);

/* FNV-1a digest of the loaded set's device parameter image (the bytes uploaded to every device):
 * equal digests mean the two loads produce the same kernels' inputs. */
int mibminet_test_image_digest(uint64_t* digest);

/* Number of constant filters the loaded set had folded (zero weights, offset +-y, factor +-1) to
 * stay on the float requant kernels: 0 unless the set as given needed exact division. */
int mibminet_test_folded_filters(int32_t* count);

#ifdef __cplusplus
}
#endif
#endif
