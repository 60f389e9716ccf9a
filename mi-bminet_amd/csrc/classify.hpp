// classify.hpp — the step after the path: class = index of the largest int8 logit per trial.
//
// The reference's accuracy meter takes torch.max(pr_outs, dim=1) of the network output
// (QuantLab/quantlab/BCI-CompIV-2a/edgeEEGNet/postprocess.py:6-8, utils/meter.py:36-39); with
// int8 logits ties are common (both rails saturate), so the rule matters: the FIRST maximal
// index, as torch.max(dim) and np.argmax return it.  One thread per trial, or four trials per
// thread for N = 4 with 16-byte-aligned buffers (k_argmax4); B * (N + 4) bytes of HBM traffic,
// negligible next to the forward's input.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mib {
namespace cls {

constexpr int CTHREADS = 256;
constexpr int NMAX = 64;

__global__ __launch_bounds__(CTHREADS) void k_argmax(const int8_t* __restrict__ logits, int32_t* __restrict__ out,
                                                     int B, int N) {
  const int b = blockIdx.x * CTHREADS + threadIdx.x;
  if (b >= B) return;
  const int8_t* z = logits + (size_t)b * N;
  int best = z[0], arg = 0;
  for (int n = 1; n < N; n++) {
    const int v = z[n];
    if (v > best) {  // strict: the first maximal index wins ties
      best = v;
      arg = n;
    }
  }
  out[b] = arg;
}

// N = 4 (the network's classes), logits and classes 16-byte aligned: each thread takes 4 trials
// with one 16-byte load and one 16-byte store (the generic kernel reads byte by byte)
__device__ __forceinline__ int argmax4(unsigned w) {
  int best = (int)(int8_t)w, arg = 0;
#pragma unroll
  for (int n = 1; n < 4; n++) {
    const int v = (int)(int8_t)(w >> (8 * n));
    if (v > best) {
      best = v;
      arg = n;
    }
  }
  return arg;
}

__global__ __launch_bounds__(CTHREADS) void k_argmax4(const unsigned* __restrict__ logits, int32_t* __restrict__ out,
                                                      int B) {
  typedef unsigned v4u __attribute__((ext_vector_type(4)));
  typedef int v4i __attribute__((ext_vector_type(4)));
  const int q = blockIdx.x * CTHREADS + threadIdx.x;  // trials 4q .. 4q + 3
  if (4 * q + 3 < B) {
    const v4u w = ((const v4u*)logits)[q];
    ((v4i*)out)[q] = (v4i){argmax4(w[0]), argmax4(w[1]), argmax4(w[2]), argmax4(w[3])};
  } else {
    for (int b = 4 * q; b < B; b++) out[b] = argmax4(logits[b]);
  }
}

}  // namespace cls
}  // namespace mib
