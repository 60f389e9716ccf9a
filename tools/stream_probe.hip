// Plain HBM read stream (diagnostic, not part of the product): every lane reads 16-byte chunks of a
// buffer with a grid stride (one wave-instruction = 1 KB contiguous, 16-byte aligned) and folds
// them into one XOR per lane, stored once.  tools/stream_energy.py times it and samples board
// power beside it, for comparison with the forward kernel's input stream (energy).
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef unsigned v4u __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(512) void k_stream(const v4u* __restrict__ x, size_t n16, unsigned* out) {
  const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  v4u acc = {0, 0, 0, 0};
  for (size_t i = tid; i < n16; i += 4 * stride) {
    v4u a = __builtin_nontemporal_load(x + i);
    v4u b = i + stride < n16 ? __builtin_nontemporal_load(x + i + stride) : (v4u){0, 0, 0, 0};
    v4u c = i + 2 * stride < n16 ? __builtin_nontemporal_load(x + i + 2 * stride) : (v4u){0, 0, 0, 0};
    v4u d = i + 3 * stride < n16 ? __builtin_nontemporal_load(x + i + 3 * stride) : (v4u){0, 0, 0, 0};
    acc ^= a ^ b ^ c ^ d;
  }
  out[tid] = acc[0] ^ acc[1] ^ acc[2] ^ acc[3];
}

extern "C" int stream_read(const void* x, size_t bytes, unsigned* out, int blocks, void* stream) {
  if (!x || !out || (bytes & 15) || blocks < 1) return -1;
  hipLaunchKernelGGL(k_stream, dim3(blocks), dim3(512), 0, (hipStream_t)stream, (const v4u*)x, bytes / 16, out);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
