// quantize.hpp — gfx950 input quantiser / transposer: float EEG trials [B][C][T] -> the batched
// int8 layout of the forward kernel ([B][trial stride], each trial time-major [T][C]).
//
// Restates the reference's input preparation (edge-eegnet_wolf/data/gen_input_header.py:66-76:
// quantize_to_int(data, absMaxValue of quant1) then transpose (0, 2, 1)) with
// python_utils/functional.py:308-334 semantics, in the input's own precision:
//     q = trunc(clip(x / s, -1, 1) * (255 - 1) / 2)        (x / s, * 254 and / 2 each rounded
//                                                           to nearest in that precision)
// (* 254 then / 2 equals * 127 exactly: scaling by 2 commutes with rounding.)
//
// HBM-bound streaming transpose: one workgroup per (64-sample time tile, trial; batches past
// 65,535 trials loop over trials in the workgroup); reads the
// C rows of the tile coalesced along time, quantises, transposes through LDS and writes the
// tile's 64 * C output bytes as contiguous dwords.  The trial's pad bytes (stride - C * T) are
// written as zeros by the last tile.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mib {
namespace quant {

constexpr int TT = 64;          // time samples per tile
constexpr int QTHREADS = 256;
constexpr int CMAX = 64;
constexpr int YMAX = 65535;   // grid.y limit: trials per launch row (larger batches loop)

template <class F>
__device__ __forceinline__ int quantize_one(F x, F s);

template <>
__device__ __forceinline__ int quantize_one<float>(float x, float s) {
  float q = __fdiv_rn(x, s);
  q = fminf(fmaxf(q, -1.0f), 1.0f);
  return (int)__fmul_rn(q, 127.0f);  // trunc toward zero
}

template <>
__device__ __forceinline__ int quantize_one<double>(double x, double s) {
  double q = __ddiv_rn(x, s);
  q = fmin(fmax(q, -1.0), 1.0);
  return (int)__dmul_rn(q, 127.0);
}

// int8 EEG already quantised ([B][C][T], the layout of SURVEY §8(b)'s batched signature): the same
// kernel is then only the transpose into the forward's [T][C] trial layout
template <>
__device__ __forceinline__ int quantize_one<int8_t>(int8_t x, int8_t) {
  return x;
}

template <class F>
__global__ __launch_bounds__(QTHREADS) void k_quantize(const F* __restrict__ x, int8_t* __restrict__ y,
                                                       int C, int T, int stride, F s, int B) {
  __shared__ __attribute__((aligned(16))) int8_t tile[TT * CMAX];
  const int t0 = blockIdx.x * TT;
  const int nt = min(TT, T - t0);
  // trials: grid.y is capped at YMAX, so a workgroup walks trials blockIdx.y + k gridDim.y
  for (int b = blockIdx.y; b < B; b += gridDim.y) {
    const F* xb = x + (size_t)b * C * T;
    if (b != (int)blockIdx.y) __syncthreads();  // the previous trial's tile has been written out
    // read: consecutive threads walk time within a channel row (coalesced)
    for (int i = threadIdx.x; i < C * TT; i += QTHREADS) {
      const int c = i / TT, t = i - c * TT;
      if (t < nt) tile[t * C + c] = (int8_t)quantize_one<F>(xb[(size_t)c * T + t0 + t], s);
    }
    __syncthreads();
    // write: the tile's nt * C bytes are contiguous in the output; dwords when aligned
    int8_t* yb = y + (size_t)b * stride + (size_t)t0 * C;
    const int nbytes = nt * C;
    if (((t0 * C) & 3) == 0) {
      const int nd = nbytes >> 2;
      for (int i = threadIdx.x; i < nd; i += QTHREADS) ((int*)yb)[i] = ((const int*)tile)[i];
      for (int i = (nd << 2) + threadIdx.x; i < nbytes; i += QTHREADS) yb[i] = tile[i];
    } else {
      for (int i = threadIdx.x; i < nbytes; i += QTHREADS) yb[i] = tile[i];
    }
    // trial pad bytes
    if (t0 + TT >= T) {
      int8_t* pad = y + (size_t)b * stride + (size_t)C * T;
      for (int i = threadIdx.x; i < stride - C * T; i += QTHREADS) pad[i] = 0;
    }
  }
}

}  // namespace quant
}  // namespace mib
