// classify.hpp — the step after the path: class = index of the largest int8 logit per trial.
//
// The reference's accuracy meter takes torch.max(pr_outs, dim=1) of the network output
// (QuantLab/quantlab/BCI-CompIV-2a/edgeEEGNet/postprocess.py:6-8, utils/meter.py:36-39); with
// int8 logits ties are common (both rails saturate), so the rule matters: the FIRST maximal
// index, as torch.max(dim) and np.argmax return it.  One thread per trial; B * (N + 4) bytes of
// HBM traffic, negligible next to the forward's input.
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

}  // namespace cls
}  // namespace mib
