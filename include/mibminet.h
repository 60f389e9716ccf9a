/*
 * mibminet.h — C ABI of the MI355X-native int8 MI-BMInet (edgeEEGNet) inference path.
 *
 * Drop-in for the reference's model/layer call API (pulp-platform/MI-BMInet,
 * edge-eegnet_wolf/src/cl/net/model.h and layers.h): same symbols, same argument meaning and the
 * same single-trial buffer layouts, backed by hand-written CDNA4 (gfx950) HIP kernels.  Everything
 * the reference links in as generated C globals (src/cl/net/net.{h,c}) is loaded at run time from
 * a versioned parameter blob instead (net_params_load).
 *
 * Layout conventions (reference layouts, "_ALIGN" = rounded up to a multiple of 4):
 *   input       [T][C_ALIGN]   int8   (model.h:37 / model.c:81, gen_input_header.py:74-75)
 *   layer1 out  [F1][T_ALIGN]  int8   (layer1.c:116)
 *   layer2 out  [F2][T8_ALIGN] int8   (layer2.c:225)
 *   layer3 out  [F2][T8_ALIGN] int8   (layer3.c:95), [T8][F2] after net_layer3_flip_inplace
 *   layer4 out  [F2][T64_ALIGN] int8  (layer4.c:168)
 *   output      [N]            int8   (model.h:38)
 * Padding bytes of every produced buffer are written as zero.
 *
 * Batched layout (net_model_compute_batch): trial b starts at x + b * net_trial_stride(); each
 * trial is time-major [T][C] without channel padding, trial stride = C*T rounded up to 16 bytes.
 * Output is [B][N] int8.  Both pointers are DEVICE pointers on `device`.
 *
 * Errors: functions returning int return NET_OK (0) or a negative code; the reference's void
 * entry points keep their void signature and record the status for net_last_error().
 * Thread safety: every entry point may be called from any host thread; calls on one device are
 * serialised internally, different devices run concurrently.
 */
#ifndef MIBMINET_H
#define MIBMINET_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MIBMINET_VERSION 1

#define NET_OK 0
#define NET_ERR_INVALID (-1)     /* bad argument (null pointer, bad size, bad device) */
#define NET_ERR_NO_PARAMS (-2)   /* no parameter blob loaded */
#define NET_ERR_UNSUPPORTED (-3) /* network dimensions outside what the kernels take: F1 = F2 = 16, D = 1,
                                    C <= 64, 64 <= T <= 4096, N <= 16 */
#define NET_ERR_BLOB (-4)        /* malformed parameter blob */
#define NET_ERR_RANGE (-5)       /* parameters on which the reference's int32 arithmetic is undefined
                                    (overflow, zero divisor), or a float-input scale outside
                                    [2^-60, 2^60] (net_model_compute_batch_f32) */
#define NET_ERR_HIP (-100)       /* HIP runtime error: code = NET_ERR_HIP - hipError_t */

/* ---- reference entry points (host pointers, single trial) -------------------------------- */

/* edge-eegnet_wolf/src/cl/net/model.h:40 — whole forward pass of one trial.
 * p_data: [T][C_ALIGN] int8, p_output: [N] int8 (host memory). */
void net_model_compute(const int8_t* p_data, int8_t* p_output);

/* north_star name for the same entry, with a status return. */
int net_forward(const int8_t* p_data, int8_t* p_output);

/* edge-eegnet_wolf/src/cl/net/layers.h:46 (layer1.c:121): [T][C_ALIGN] -> [F1][T_ALIGN] */
void net_layer1(const int8_t* p_data, int8_t* p_result);
/* layers.h:74 (layer2.c:228): [F1][T_ALIGN] -> [F2][T8_ALIGN] */
void net_layer2(const int8_t* p_data, int8_t* p_result);
/* layers.h:97 (layer3.c:98): [F2][T8_ALIGN] -> [F2][T8_ALIGN] */
void net_layer3(const int8_t* p_data, int8_t* p_result);
/* layers.h:107 (layer3.c:243): [F2][T8_ALIGN] -> [T8][F2] in place */
void net_layer3_flip_inplace(int8_t* p_data);
/* layers.h:123 (layer4.c:172, FLIP_LAYERS): [T8][F2] -> [F2][T64_ALIGN] */
void net_layer4(const int8_t* p_data, int8_t* p_result);
/* layers.h:134 (layer5.c:43): [F2][T64_ALIGN] -> [N] */
void net_layer5(const int8_t* p_data, int8_t* p_result);

/* Status of the last void entry point called on this host thread. */
int net_last_error(void);

/* ---- parameters (replace the link-time globals of the generated net.h/net.c) ------------- */

/* Load a parameter blob (format: net_params_load_arrays below; mibminet/params.py, ParamSet.to_blob): the
 * net.h arrays net_l1_factor ... net_l5_weight with their dimensions, int8 or packed int4
 * weights, and the build variant (flag bit 0: -DREORDER_BN, the canonical build; clear: the plain
 * BN branches of layer2.c:139-210 / layer4.c:91-133.  Flag bit 1: clip every requantised output to
 * [-127, 127], the golden model's clip_balanced=True, functional.py:89-91; clear: [-128, 127] as
 * the C's __CLIP_R).  Other flag bits are rejected (NET_ERR_BLOB).  Validates, precomputes the gfx950 operand fragments and exact requantisation
 * constants, and uploads lazily to each device on first use.  Geometry: F1 = F2 = 16 and D = 1
 * (layer2.c:246), any C <= 64, 64 <= T <= 4096 and 1 <= N <= 16 (the channel-selected and 2- or
 * 3-class networks of QuantLab's loaders included); 22 x 1125, 64 x 1000 and 64 x 480 with N = 4
 * run kernels compiled for those shapes, every other geometry the run-time-dimension kernels
 * (net_params_info reports which).  Every set on which the reference's
 * own int32 arithmetic is defined for every int8 input loads: sets inside the float requant
 * envelope run the float-requant kernels, the others (e.g. large folded BN offsets) kernels that
 * divide exactly in integers.  NET_ERR_RANGE only where the reference's arithmetic is undefined:
 * a zero factor (or factor >> 3 in the plain branches), INT_MIN / -1, or an int32 overflow of
 * acc + offset (layer1.c:90-91), of the pooled sum or sum + offset (layer2.c:97-111,
 * layer4.c:99-130), or of the plain layer 4's sum of eight elements (layer4.c:113-130).  Replaces any previous set.  Pad
 * bytes of net_l1_weight_align (channels C..C_ALIGN-1) and of net_l5_weight (columns
 * T64..T64_ALIGN-1 of every row) must be zero, as gen_net_header.py writes them (NET_ERR_BLOB
 * otherwise).  Each distinct set gets its own device copy (about 144 KB per set and device), which
 * is never overwritten: launches already enqueued, and launches captured into a HIP graph, keep
 * running the set (and build variant) they were enqueued with, whatever is loaded later.  A load
 * never waits for the device.  When a device already holds 8 copies, the least recently used
 * copies whose launches have all completed are freed first (a copy is freed only once no launch
 * can still read it); if none is idle, the device keeps more than 8.  A copy used by a launch
 * under stream capture (which a HIP graph may replay at any time) is pinned until
 * net_params_unload, so captured graphs stay valid across any number of later loads.  A set
 * loaded again reuses its copy. */
int net_params_load(const void* blob, size_t len);

/* Which kernels the loaded set runs, for integrators who need to see a slower path coming:
 * info[0] = NET_PATH_FLOAT (compiled geometry, float requant proven exact on every reachable
 * value), NET_PATH_EXACT (compiled geometry, exact division at layers 1, 2 and 4: about
 * 1.1x the float kernels' time on 22 x 1125) or NET_PATH_GENERAL (run-time-dimension kernels,
 * float or exact requant as info[4] says); info[1] = the layer (1, 2 or 4) of the first requant that has no
 * proven float form (NET_PATH_EXACT), else 0; info[2] = its filter, else -1; info[3] = the
 * compiled geometry (0: 22 x 1125, 1: 64 x 1000, 2: 64 x 480), -1 on the general path; info[4] = 1
 * when the set divides exactly at layers 1-4 (NET_PATH_EXACT, or NET_PATH_GENERAL without a proven
 * float form for every requant), 0 when it runs the proven float requant.  info holds 5 entries.
 * A layer-1, -2 or -4 filter whose output is one constant over its whole reachable range (an
 * offset past the weights' reach, a factor that sends every sum to zero, a suppressed ReLU) is
 * folded into an equivalent constant filter before the choice, so such filters alone never force
 * exact division; info[1] / info[2] name a filter whose output varies. */
#define NET_PATH_FLOAT 0
#define NET_PATH_EXACT 1
#define NET_PATH_GENERAL 2
int net_params_info(int32_t* info);

/* The reference's generated globals (edge-eegnet_wolf/data/gen_net_header.py:78-224, written by
 * python_utils/header_file.py as src/cl/net/net.{h,c}), by pointer, in their own layouts: a C host
 * that links the reference's net.c loads them with net_params_load_arrays and needs no blob file
 * and no Python.  include/mibminet_net_h.h fills this struct from the NET_* macros and net_l*
 * arrays of an included net.h (and the build variant from -DREORDER_BN, as the reference's
 * Makefile selects it).  Weights are int8, as net.c holds them. */
typedef struct {
    int32_t C, T, F1, F2, D, N;         /* NET_C, NET_T, NET_F1, NET_F2, NET_D, NET_N */
    uint32_t flags;                     /* NET_FLAG_REORDER_BN | NET_FLAG_CLIP_BALANCED (blob flag bits) */
    const int32_t* l1_factor;           /* net_l1_factor [F2] */
    const int32_t* l1_offset;           /* net_l1_offset [F2] */
    const int8_t* l1_weight_align;      /* net_l1_weight_align [F2][C_ALIGN], zero pad */
    const int32_t* l2_factor;           /* net_l2_factor [F2] (pool 8 folded in) */
    const int32_t* l2_offset;           /* net_l2_offset [F2] */
    const int8_t* l2_weight_reverse;    /* net_l2_weight_reverse [F2][64] (torch order) */
    int32_t l3_factor;                  /* NET_L3_FACTOR */
    const int8_t* l3_weight;            /* net_l3_weight [F2][16] (flipped) */
    const int32_t* l4_factor;           /* net_l4_factor [F2] */
    const int32_t* l4_offset;           /* net_l4_offset [F2] */
    const int8_t* l4_weight;            /* net_l4_weight [F2][F2] */
    int32_t l5_factor;                  /* NET_L5_FACTOR */
    const int8_t* l5_bias;              /* net_l5_bias [N] */
    const int8_t* l5_weight;            /* net_l5_weight [N][F2 * T64_ALIGN], zero pad per row */
} net_arrays_t;
#define NET_FLAG_REORDER_BN 1u
#define NET_FLAG_CLIP_BALANCED 2u

/* Loads the arrays of `a` exactly as net_params_load loads a blob holding them (same checks,
 * codes and device images; the arrays are copied, so they may go away after the call).  A blob
 * is the same fields serialised: a 64-byte header "MIBMINET", then uint32 version = 1, C, T, F1,
 * F2, D, N, weight_bits (8, or 4 for packed nibbles: element 2i in the low nibble of byte i),
 * l2_taps = 64, l3_taps = 16, flags, zero to byte 64; then l1_factor, l1_offset, l1_weight_align,
 * l2_factor, l2_offset, l2_weight_reverse, l3_factor, l3_weight, l4_factor, l4_offset, l4_weight,
 * l5_factor, l5_bias, l5_weight in that order, little endian, each section zero-padded to a
 * multiple of 4 bytes (mibminet/params.py, ParamSet.to_blob, writes it). */
int net_params_load_arrays(const net_arrays_t* a);

/* dims[0..6] = C, T, F1, F2, N, weight_bits, loaded(0/1). */
int net_params_dims(int32_t* dims);

/* Drops the loaded set and frees every device copy of every set, after synchronising each device
 * that holds copies (HIP graphs capturing launches must be dropped first: this is the one call
 * after which a captured launch may no longer be replayed). */
void net_params_unload(void);

/* ---- batched device entry points ---------------------------------------------------------- */

/* Bytes between consecutive trials of the batched input for the loaded network (0 if none). */
size_t net_trial_stride(void);

/* Forward B trials resident on `device`; x: device pointer [B][trial_stride], y: device pointer
 * [B][N].  x must be 16-byte aligned and y 4-byte aligned (NET_ERR_INVALID otherwise; hipMalloc
 * and torch allocations are).  Launches on the device's null stream and waits for completion.
 * TIME-MAJOR trials ([T][C] each, the reference's own single-trial orientation): a caller holding
 * channel-major [B][C][T] trials (SURVEY §8(b)'s layout, input.npz before gen_input_header.py:74
 * transposes it) must call net_model_compute_batch_ct_sync / net_model_compute_batch_ct instead;
 * the pointers carry no layout, and a [B][C][T] buffer passed here returns wrong logits. */
int net_model_compute_batch(const int8_t* x, int8_t* y, size_t B, int device);

/* SURVEY §8(b)'s batched signature, channel-major: x: DEVICE pointer to B trials [B][C][T] int8,
 * contiguous (trial stride C*T bytes, any alignment); y: DEVICE pointer [B][N], 4-byte aligned.
 * Launches on the device's null stream and waits for completion (net_model_compute_batch_ct is
 * the stream-ordered form). */
int net_model_compute_batch_ct_sync(const int8_t* x, int8_t* y, size_t B, int device);

/* Same, enqueued on `stream` (a hipStream_t of `device`, NULL = null stream), no host sync. */
int net_model_compute_batch_async(const int8_t* x, int8_t* y, size_t B, int device, void* stream);

/* Channel-major trials (SURVEY §8(b)'s batched signature; the layout of the reference's
 * input.npz before gen_input_header.py:74 transposes it): x: DEVICE pointer to B trials
 * [B][C][T] int8, contiguous (trial stride C*T bytes, any alignment); y: DEVICE pointer [B][N],
 * 4-byte aligned.  The same fused forward, with each layer-1 block transposed through LDS inside
 * the kernel (no separate pack pass).  Enqueued on `stream` (NULL = null stream), no host sync. */
int net_model_compute_batch_ct(const int8_t* x, int8_t* y, size_t B, int device, void* stream);

/* Float EEG straight into the forward: x: DEVICE pointer to B float32 trials [B][C][T] (the
 * reference's input.npz, 4-byte aligned), y: DEVICE pointer [B][N].  Each layer-1 block is
 * quantised in the kernel exactly as net_quantize_input_f32 does it (x / scale, clip to [-1, 1],
 * * 127, truncate, in float32; gen_input_header.py:66-76), then staged as in
 * net_model_compute_batch_ct: no int8 copy of the batch in memory.  scale = absMaxValue of quant1,
 * in [2^-60, 2^60] (NET_ERR_RANGE otherwise: the in-kernel quotient is exact there; use
 * net_quantize_input_f32 + net_model_compute_batch_async beyond).  Enqueued on `stream` (NULL =
 * null stream), no host sync. */
int net_model_compute_batch_f32(const float* x, int8_t* y, size_t B, float scale, int device, void* stream);

/* Several devices from one host thread (static split, no collectives): shard i is
 * x[i] / y[i] / B[i] on devices[i] (DEVICE pointers of that device).  Every shard is enqueued
 * before any is waited for, so the devices run concurrently.  streams == NULL: each device's null
 * stream, and the call returns when all shards are done; otherwise streams[i] (a hipStream_t of
 * devices[i]) and no host sync.  Returns the first error; the shards enqueued before it have
 * finished by then (in both modes). */
int net_model_compute_batch_multi(int ndev, const int* devices, const int8_t* const* x, int8_t* const* y,
                                  const size_t* B, void* const* streams);

/* The same split over channel-major shards: x[i] is [B[i]][C][T] int8 on devices[i] (as
 * net_model_compute_batch_ct takes it). */
int net_model_compute_batch_multi_ct(int ndev, const int* devices, const int8_t* const* x, int8_t* const* y,
                                     const size_t* B, void* const* streams);

/* Input quantiser / transposer (the step before the path; reference
 * edge-eegnet_wolf/data/gen_input_header.py:66-76 with python_utils/functional.py:308-334):
 * x: DEVICE pointer to B float trials [B][C][T]; y: DEVICE pointer to the batched int8 layout
 * ([B][stride], stride = C*T rounded up to 16, each trial [T][C], pad bytes zero), computed as
 * trunc(clip(x / scale, -1, 1) * 127) in the input's precision.  scale = absMaxValue of the
 * network's quant1 activation.  Enqueued on `stream` (NULL = null stream), no host sync.
 * Any B up to INT32_MAX - 65,535 in one call (batches past 65,535 trials loop inside the kernel).  y must be
 * 16-byte aligned (as net_model_compute_batch requires of its input) and one trial's input must
 * stay below 2 GiB (C * T * sizeof(element) < 2^31); NET_ERR_INVALID otherwise. */
int net_quantize_input_f32(const float* x, int8_t* y, size_t B, int C, int T, float scale, int device,
                           void* stream);
int net_quantize_input_f64(const double* x, int8_t* y, size_t B, int C, int T, double scale, int device,
                           void* stream);

/* The step after the path: cls[b] = index of the largest of the N int8 logits of trial b, the
 * first one on ties (torch.max(pr_outs, dim=1) of the reference's accuracy meter,
 * QuantLab/quantlab/BCI-CompIV-2a/edgeEEGNet/postprocess.py:6-8).  logits: DEVICE pointer [B][N]
 * (as net_model_compute_batch writes it), cls: DEVICE pointer [B].  1 <= N <= 64,
 * B <= INT32_MAX - 1024 (NET_ERR_INVALID otherwise).  Enqueued on
 * `stream` (NULL = null stream), no host sync. */
int net_argmax_batch(const int8_t* logits, int32_t* cls, size_t B, int N, int device, void* stream);

/* Already-quantised int8 trials in channel-major [B][C][T] (the layout of the reference's
 * input.npz, transposed by gen_input_header.py:74 on the host): the same GPU transpose into the
 * batched [B][stride] layout, without the quantisation.  DEVICE pointers, B <= INT32_MAX - 65,535,
 * C <= 64, y 16-byte aligned, enqueued on `stream`, no host sync. */
int net_pack_trials_i8(const int8_t* x, int8_t* y, size_t B, int C, int T, int device, void* stream);

/* Device used by the single-trial API (default 0). */
int net_set_device(int device);

/* Kernel launch geometry used for a batch of B trials (for profiling/roofline bookkeeping):
 * out[0] = grid size (workgroups), out[1] = threads per workgroup, out[2] = LDS bytes. */
int net_launch_info(size_t B, int device, int32_t* out);
/* The same for the channel-major kernel (net_model_compute_batch_ct). */
int net_launch_info_ct(size_t B, int device, int32_t* out);

const char* net_error_string(int code);
int net_version(void);

#ifdef __cplusplus
}
#endif
#endif /* MIBMINET_H */
