// Which SIMD does each wave of each workgroup land on? (diagnostic)  512-thread workgroups with
// 58 KB of LDS (two per CU, like k_forward); prints, for the CUs of XCC 0, the SIMD of waves 6
// and 7 of both resident workgroups.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <map>
#include <vector>
__global__ void k(unsigned* out) {
  __shared__ char pad[58 * 1024];
  unsigned id, xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(id));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  pad[threadIdx.x] = (char)id;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) {
    out[3 * (blockIdx.x * 8 + threadIdx.x / 64)] = id;
    out[3 * (blockIdx.x * 8 + threadIdx.x / 64) + 1] = xcc;
    out[3 * (blockIdx.x * 8 + threadIdx.x / 64) + 2] = pad[(threadIdx.x + 1) & 1023];
  }
  // keep the workgroup resident a while so that two share each CU
  long long t0 = __builtin_amdgcn_s_memtime();
  while (__builtin_amdgcn_s_memtime() - t0 < 200000) {}
}
int main() {
  const int G = 512;
  unsigned* d; hipMalloc(&d, G * 8 * 12);
  hipLaunchKernelGGL(k, G, 512, 0, 0, d);
  std::vector<unsigned> h(G * 8 * 3);
  hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
  // HW_ID (gfx9): wave[3:0] simd[5:4] pipe[7:6] cu[11:8] sh[12] se[15:13] tg[19:16]
  std::map<unsigned, std::vector<int>> bycu;
  for (int b = 0; b < G; b++) {
    unsigned id = h[3 * (b * 8)], xcc = h[3 * (b * 8) + 1] & 0xf;
    unsigned key = (xcc << 16) | (((id >> 13) & 7) << 8) | (((id >> 12) & 1) << 4) | ((id >> 8) & 15);
    bycu[key].push_back(b);
  }
  int shown = 0, same = 0, total = 0;
  for (auto& [key, bs] : bycu) {
    if (bs.size() < 2) continue;
    total++;
    unsigned s7a = (h[3 * (bs[0] * 8 + 7)] >> 4) & 3, s7b = (h[3 * (bs[1] * 8 + 7)] >> 4) & 3;
    same += s7a == s7b;
    if (shown++ < 12) {
      printf("cu key %05x: blocks", key);
      for (int b : bs) {
        printf(" %d(tg %u: w0..7 simd", b, (h[3 * (b * 8)] >> 16) & 15);
        for (int w = 0; w < 8; w++) printf(" %u", (h[3 * (b * 8 + w)] >> 4) & 3);
        printf(")");
      }
      printf("\n");
    }
  }
  printf("CUs with two workgroups: %d; wave 7 of both on the same SIMD: %d\n", total, same);
  return 0;
}
