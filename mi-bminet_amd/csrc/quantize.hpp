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
// HBM-bound streaming transpose.  A workgroup (4 waves) owns one tile column of TT = 256 time
// samples and walks trials blockIdx.y + k gridDim.y (2 per workgroup for float / double, 4 for
// int8; grid y is capped at 65,535).  Each lane loads 4 consecutive samples of one channel row with
// one wide raw buffer load (float: 16 B, double: 2 x 16 B, int8: 8 B at a 4-byte-aligned offset and
// a byte align at use), so a row's 256 samples are one coalesced wave-instruction (two for
// double).  The waves take rows w, w + 4, ...; the loads carry no branch (rows past C read zeros
// from outside the trial's view), so a wave's first rows are all in flight together, and they are
// issued one trial ahead, while the previous tile leaves.  The buffer view of a trial ends at its
// own bytes (rounded up to a dword), so loads past the last row's end read zeros instead of the
// next trial's samples.  Quantised bytes go into the tile in LDS at [t][c]; the tile, which is
// contiguous in the output, then leaves as 16-byte stores.  The last tile of a trial also writes
// the trial's pad bytes (stride - C T) as zeros.
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
// rows per wave whose loads are in flight together (measured best: float / double 8, int8 4)
template <class F>
constexpr int rchunk() { return sizeof(F) == 1 ? 4 : 8; }
// trials per workgroup (the grid covers B / qtrials rows): measured best, float / double 2, int8 4
// (profiles/r03_steps.json)
template <class F>
constexpr int qtrials() { return sizeof(F) == 1 ? 4 : 2; }

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
  v2u d;
  unsigned sh;
  __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t r, int off) {
    // 8 bytes from the 4-byte-aligned offset below; the 4 wanted bytes come out by a byte align
    // at use, so the load does not wait here
    d = __builtin_amdgcn_raw_buffer_load_b64(r, off & ~3, 0, 0);
    sh = (unsigned)(off & 3);
  }
  __device__ __forceinline__ int8_t get(int j) const {
    return (int8_t)(__builtin_amdgcn_alignbyte(d[1], d[0], sh) >> (8 * j));
  }
};

// A trial's view: its first byte rounded down to 4 (int8 trials are byte-aligned), so every load
// address is 4-byte aligned (`d` is that rounding), and its end rounded up to a whole dword: the
// range check is per dword, so a dword holding the trial's last bytes would read as zeros otherwise
// (the up to 3 bytes past the trial share that dword's page).  `live` false gives an empty view
// (every load reads zeros, no memory access).
template <class F>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t trial_view(const F* x, int b, int C, int T, bool live, int& d) {
  const uintptr_t a = (uintptr_t)(x + (size_t)b * C * T);
  d = (int)(a & 3);
  const int nrec = live ? ((int)((size_t)C * T * sizeof(F)) + d + 3) & ~3 : 0;
  return __builtin_amdgcn_make_buffer_rsrc((void*)(a - d), (short)0, nrec, 0x00020000);
}

constexpr int NOWHERE = 0x7fffff00;  // a view offset past any trial: the load reads zeros

template <class F>
__global__ __launch_bounds__(QTHREADS) void k_quantize(const F* __restrict__ x, int8_t* __restrict__ y,
                                                       int C, int T, int stride, F s, int B) {
  constexpr int RCHUNK = rchunk<F>();
  __shared__ __attribute__((aligned(16))) int8_t tile[TT * CMAX + 16];
  const int t0 = blockIdx.x * TT;
  const int nt = min(TT, T - t0);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int tl = 4 * lane;  // the lane's first sample in the tile
  const bool last = t0 + TT >= T;
  // bytes this tile writes: its nt * C samples, and for the last tile the pad up to the stride
  const int nout = last ? stride - t0 * C : TT * C;
  // the lane's byte offset in row c of a trial's view, or NOWHERE for the rows past C (their loads
  // are issued all the same, so no load sits behind a branch and they all stay in flight together)
  auto row_off = [&](int c, int d) {
    return c < C ? d + (int)(((size_t)c * T + t0 + tl) * sizeof(F)) : NOWHERE;
  };
  // The wave's rows are wave, wave + 4, ...; its first RCHUNK rows (all of them for C <= 4 RCHUNK)
  // are loaded one trial ahead, while the previous tile leaves; further rows load when used.
  Row4<F> v[RCHUNK];
  int b = blockIdx.y;  // < B: the grid has at most B rows
  int d = 0;
  __amdgpu_buffer_rsrc_t r = trial_view<F>(x, b, C, T, true, d);
#pragma unroll
  for (int k = 0; k < RCHUNK; k++) v[k].load(r, row_off(wave + QWAVES * k, d));
  // trials: a workgroup walks trials blockIdx.y + k gridDim.y
  for (; b < B; b += gridDim.y) {
    for (int c0 = wave; c0 < C; c0 += QWAVES * RCHUNK) {
      if (c0 != wave) {  // rows past the first chunk: load now
#pragma unroll
        for (int k = 0; k < RCHUNK; k++) v[k].load(r, row_off(c0 + QWAVES * k, d));
      }
#pragma unroll
      for (int k = 0; k < RCHUNK; k++) {
        const int c = c0 + QWAVES * k;  // wave-uniform
        if (c < C) {
          // samples past the trial's end (the last tile) become the zeros of rows t >= nt
#pragma unroll
          for (int j = 0; j < 4; j++)
            tile[(tl + j) * C + c] = tl + j < nt ? (int8_t)quantize_one<F>(v[k].get(j), s) : (int8_t)0;
        }
      }
    }
    // rows t < TT are all written above; the pad can reach past them when nt = TT
    if (last)
      for (int i = TT * C + threadIdx.x; i < nout; i += QTHREADS) tile[i] = 0;
    __syncthreads();
    // the next trial's first rows load while this tile leaves (an empty view past the last trial)
    const int bn = b + gridDim.y;
    r = trial_view<F>(x, bn < B ? bn : b, C, T, bn < B, d);
#pragma unroll
    for (int k = 0; k < RCHUNK; k++) v[k].load(r, row_off(wave + QWAVES * k, d));
    // the tile is contiguous in the output and both ends are 16-byte aligned (t0 C = 256 k C, the
    // stride is a multiple of 16)
    v4u* yb = (v4u*)(y + (size_t)b * stride + (size_t)t0 * C);
    for (int i = threadIdx.x; i < nout / 16; i += QTHREADS) yb[i] = ((const v4u*)tile)[i];
    __syncthreads();  // the tile is read out before the next trial's bytes go in
  }
}

}  // namespace quant
}  // namespace mib
