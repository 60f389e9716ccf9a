// Micro-probe: are 4-byte-aligned global_load_dwordx4 loads correct and fast on gfx950?
// Pattern = layer-1 windows: lane (j,g) of block b reads 16 B at b*704 + 44j + 16g.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef int v4i __attribute__((ext_vector_type(4)));
__global__ void k_un(const int8_t* __restrict__ x, int* __restrict__ out, int nblk, int mode) {
  int lane = threadIdx.x & 63, j = lane & 15, g = lane >> 4;
  int acc = 0;
  for (int b = blockIdx.x * 4 + (threadIdx.x >> 6); b < nblk; b += gridDim.x * 4) {
    const int8_t* p = x + (size_t)b * 704 + (mode ? 44 * j + 16 * g : 16 * lane);
    v4i v;
    if (mode == 2) { const int* q = (const int*)p; v = (v4i){q[0], q[1], q[2], q[3]}; }
    else v = *(const v4i*)p;
    acc += v.x ^ v.y ^ v.z ^ v.w;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}
__global__ void k_chk(const int8_t* x, int* bad) {
  int lane = threadIdx.x, j = lane & 15, g = lane >> 4;
  const int8_t* p = x + 44 * j + 16 * g + 704 * blockIdx.x;
  v4i v = *(const v4i*)p;
  const int8_t* vb = (const int8_t*)&v;
  for (int i = 0; i < 16; i++) if (vb[i] != p[i]) atomicAdd(bad, 1);
}
int main() {
  size_t nblk = 1 << 21; size_t bytes = nblk * 704 + 64;
  int8_t* x; int* out; int* bad;
  hipMalloc(&x, bytes); hipMalloc(&out, 4 << 20); hipMalloc(&bad, 4);
  std::vector<int8_t> h(bytes); for (size_t i = 0; i < bytes; i++) h[i] = (int8_t)(i * 2654435761u >> 13);
  hipMemcpy(x, h.data(), bytes, hipMemcpyHostToDevice); hipMemset(bad, 0, 4);
  k_chk<<<1024, 64>>>(x, bad); int hb; hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
  printf("unaligned dwordx4 byte mismatches: %d\n", hb);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const char* nm[] = {"aligned 16B/lane (1KB/wave)", "4B-aligned windows dwordx4", "4B-aligned windows 4x dword"};
  for (int mode = 0; mode < 3; mode++) {
    for (int rep = 0; rep < 2; rep++) {
      hipEventRecord(e0); k_un<<<2048, 256>>>(x, out, (int)nblk, mode); hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      if (rep) printf("%-32s %.3f ms  %.0f GB/s (of %.2f GB span)\n", nm[mode], ms, nblk * 704 / ms / 1e6, nblk * 704 / 1e9);
    }
  }
  return 0;
}
