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
// HBM-bound streaming transpose.  One workgroup (4 waves) per (tile of TT = 256 time samples,
// trial); batches past 65,535 trials loop over trials in the workgroup.  Each lane loads 4
// consecutive samples of one channel row with one wide raw buffer load (float: 16 B, double:
// 2 x 16 B, int8: 8 B at a 4-byte-aligned offset and a byte align), so a row's 256 samples are one
// coalesced wave-instruction (two for double); the waves take rows w, w + 4, ... and issue the
// loads of 4 rows before using any.  The buffer view of a trial ends at its own bytes (rounded up to
// a dword), so loads past the last row's end read zeros instead of the next trial's samples.  Quantised bytes go into the
// tile in LDS at [t][c]; the tile, which is contiguous in the output, then leaves as 16-byte
// stores.  The last tile of a trial also writes the trial's pad bytes (stride - C T) as zeros.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mib {
namespace quant {

constexpr int TT = 256;         // time samples per tile (4 per lane)
constexpr int QTHREADS = 256;   // 4 waves
constexpr int QWAVES = QTHREADS / 64;
constexpr int CMAX = 64;
constexpr int YMAX = 65535;     // grid.y limit: trials per launch row (larger batches loop)
constexpr int RCHUNK = 4;       // rows per wave whose loads are in flight together

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

typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef unsigned v2u __attribute__((ext_vector_type(2)));

// 4 consecutive samples of one row as raw bits, loaded from byte offset `off` of the trial's view
template <class F>
struct Row4;

template <>
struct Row4<float> {
  v4u v;
  __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t r, int off) {
    v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
  }
  __device__ __forceinline__ float get(int j) const { return __uint_as_float(v[j]); }
};

template <>
struct Row4<double> {
  v4u lo, hi;
  __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t r, int off) {
    lo = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
    hi = __builtin_amdgcn_raw_buffer_load_b128(r, off + 16, 0, 0);
  }
  __device__ __forceinline__ double get(int j) const {
    const v4u& w = j < 2 ? lo : hi;
    const int k = 2 * (j & 1);
    return __hiloint2double((int)w[k + 1], (int)w[k]);
  }
};

template <>
struct Row4<int8_t> {
  unsigned w;
  __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t r, int off) {
    // 8 bytes from the 4-byte-aligned offset below, then the 4 wanted bytes by a byte align
    const v2u d = __builtin_amdgcn_raw_buffer_load_b64(r, off & ~3, 0, 0);
    w = __builtin_amdgcn_alignbyte(d[1], d[0], (unsigned)(off & 3));
  }
  __device__ __forceinline__ int8_t get(int j) const { return (int8_t)(w >> (8 * j)); }
};

template <class F>
__global__ __launch_bounds__(QTHREADS) void k_quantize(const F* __restrict__ x, int8_t* __restrict__ y,
                                                       int C, int T, int stride, F s, int B) {
  __shared__ __attribute__((aligned(16))) int8_t tile[TT * CMAX + 16];
  const int t0 = blockIdx.x * TT;
  const int nt = min(TT, T - t0);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int tl = 4 * lane;  // the lane's first sample in the tile
  const bool last = t0 + TT >= T;
  // bytes this tile writes: its nt * C samples, and for the last tile the pad up to the stride
  const int nout = last ? stride - t0 * C : TT * C;
  // trials: grid.y is capped at YMAX, so a workgroup walks trials blockIdx.y + k gridDim.y
  for (int b = blockIdx.y; b < B; b += gridDim.y) {
    if (b != (int)blockIdx.y) __syncthreads();  // the previous trial's tile has been written out
    // the view starts at the trial's first byte rounded down to 4 (int8 trials are byte-aligned),
    // so every load address below is 4-byte aligned; `d` is that rounding.  Its end is rounded up
    // to a whole dword: the range check is per dword, so a dword holding the trial's last bytes
    // would read as zeros otherwise.  The up to 3 bytes past the trial share that dword's page.
    const uintptr_t a = (uintptr_t)(x + (size_t)b * C * T);
    const int d = (int)(a & 3);
    const int nrec = ((int)((size_t)C * T * sizeof(F)) + d + 3) & ~3;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)(a - d), (short)0, nrec, 0x00020000);
    for (int c0 = wave; c0 < C; c0 += QWAVES * RCHUNK) {
      Row4<F> v[RCHUNK];
#pragma unroll
      for (int k = 0; k < RCHUNK; k++) {
        const int c = c0 + QWAVES * k;
        if (c < C) v[k].load(r, d + (int)(((size_t)c * T + t0 + tl) * sizeof(F)));
      }
#pragma unroll
      for (int k = 0; k < RCHUNK; k++) {
        const int c = c0 + QWAVES * k;
        if (c < C) {
#pragma unroll
          for (int j = 0; j < 4; j++)
            if (tl + j < nt) tile[(tl + j) * C + c] = (int8_t)quantize_one<F>(v[k].get(j), s);
        }
      }
    }
    if (last)  // the trial's pad bytes follow its last sample in the tile
      for (int i = nt * C + threadIdx.x; i < nout; i += QTHREADS) tile[i] = 0;
    __syncthreads();
    // the tile is contiguous in the output and both ends are 16-byte aligned (t0 C = 256 k C, the
    // stride is a multiple of 16)
    v4u* yb = (v4u*)(y + (size_t)b * stride + (size_t)t0 * C);
    for (int i = threadIdx.x; i < nout / 16; i += QTHREADS) yb[i] = ((const v4u*)tile)[i];
  }
}

}  // namespace quant
}  // namespace mib
