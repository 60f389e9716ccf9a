// Byte-unaligned raw buffer loads on gfx950 (diagnostic for the channel-major input path):
//  1. correctness of buffer_load_dwordx4 at every byte offset (0..3 mod 4), via the VGPR offset
//     and via the immediate field, and what a load straddling num_records returns per byte;
//  2. read throughput of the channel-major pattern: trial [C][T] int8 (C = 22, T = 1125, rows
//     start at odd bytes), lane (c, h) of a block reads 16 B at c T + 32 blk + 16 h, against the
//     same bytes read as 16-byte-aligned chunks.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef unsigned v4u __attribute__((ext_vector_type(4)));

__global__ void k_off(const unsigned char* x, v4u* o, int nrec, int base) {
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)x, (short)0, nrec, 0x00020000);
  const int t = threadIdx.x;  // byte offset base + t
  o[t] = __builtin_amdgcn_raw_buffer_load_b128(r, base + t, 0, 2);
  o[64 + t] = __builtin_amdgcn_raw_buffer_load_b128(r, base - 48 + t + 48 * 0, 48, 2);
}

// channel-major stream: trial b, block blk, lane (c, h): 16 B at b * CT + c T + 32 blk + 16 h
__global__ void k_ct(const unsigned char* __restrict__ x, unsigned* __restrict__ out, int B, int C, int T, int mode) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = lane >> 1, h = lane & 1;
  const int nb = (T + 31) / 32;
  unsigned acc = 0;
  for (int b = blockIdx.x; b < B; b += gridDim.x) {
    const int CT = C * T;
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)(x + (size_t)b * CT), (short)0, CT, 0x00020000);
    for (int blk = wave; blk < nb; blk += 8) {
      if (c < C) {
        int off = mode == 0 ? c * T + 32 * blk + 16 * h : (c * T + 32 * blk + 16 * h) & ~15;
        v4u v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 2);
        acc += v[0] ^ v[1] ^ v[2] ^ v[3];
      }
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main() {
  const int N = 4096, nrec = 2001;
  std::vector<unsigned char> h(N);
  for (int i = 0; i < N; i++) h[i] = (unsigned char)(i * 7 + 1);
  unsigned char* d; v4u* o;
  hipMalloc(&d, N); hipMalloc(&o, 128 * 16);
  int bad = 0;
  for (int base = 64; base <= 1024; base += 64) {
    hipMemcpy(d, h.data(), N, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_off, 1, 64, 0, 0, d, o, nrec, base);
    v4u r[128]; hipMemcpy(r, o, sizeof(r), hipMemcpyDeviceToHost);
    for (int t = 0; t < 64; t++)
      for (int p = 0; p < 2; p++) {
        const unsigned char* got = (const unsigned char*)&r[64 * p + t];
        for (int i = 0; i < 16; i++) bad += got[i] != h[base + t + i];
      }
  }
  printf("unaligned b128 (VGPR offset / immediate 48), offsets 64..1087: %d wrong bytes\n", bad);
  // straddling num_records = 2001: per byte, data or zero?
  hipLaunchKernelGGL(k_off, 1, 64, 0, 0, d, o, nrec, nrec - 40);
  v4u r[128]; hipMemcpy(r, o, sizeof(r), hipMemcpyDeviceToHost);
  for (int t = 20; t < 44; t++) {
    const int off = nrec - 40 + t;
    printf("off %4d (mod 4 = %d, end %d):", off, off & 3, off + 16);
    const unsigned char* got = (const unsigned char*)&r[t];
    for (int i = 0; i < 16; i++) {
      const int a = off + i;
      printf("%c", got[i] == h[a] ? (a < nrec ? 'd' : 'D') : got[i] == 0 ? (a < nrec ? 'z' : '0') : '?');
    }
    printf("   (d data in range, 0 zero past end, z ZERO IN RANGE, D data past end)\n");
  }
  // throughput
  const int C = 22, T = 1125, B = 65536;
  size_t bytes = (size_t)B * C * T + 64;
  unsigned char* x; unsigned* out;
  hipMalloc(&x, bytes); hipMalloc(&out, 4 << 20);
  hipMemset(x, 1, bytes);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const char* nm[] = {"channel-major rows, byte-unaligned 16 B", "same bytes as 16-B-aligned chunks"};
  for (int mode = 0; mode < 2; mode++)
    for (int rep = 0; rep < 3; rep++) {
      hipEventRecord(e0);
      hipLaunchKernelGGL(k_ct, 512, 512, 0, 0, x, out, B, C, T, mode);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      if (rep == 2) printf("%-42s %.3f ms  %.0f GB/s\n", nm[mode], ms, (double)B * C * T / ms / 1e6);
    }
  return 0;
}
