// Semantics probe (diagnostic): v_sub_u32 with clamp (unsigned saturation) on gfx950, the relu of
// biased integers used by the layer-2/4 pooling: sat_u32((a + B) - (t + B)) == max(a - t, 0).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(const unsigned* a, const unsigned* b, unsigned* o) {
  int i = threadIdx.x;
  unsigned r;
  asm volatile("v_sub_u32_e64 %0, %1, %2 clamp" : "=v"(r) : "v"(a[i]), "v"(b[i]));
  o[i] = r;
}
int main() {
  const int n = 8;
  unsigned ha[n] = {5, 3, 0x80000000u, 0x7fffffffu, 0x3F800000u + 100, 0x3F800000u - 100, 0xffffffffu, 0};
  unsigned hb[n] = {3, 5, 0x7fffffffu, 0x80000000u, 0x3F800000u - 7, 0x3F800000u - 7, 1, 0xffffffffu};
  unsigned *da, *db, *dout, ho[n];
  hipMalloc(&da, 64); hipMalloc(&db, 64); hipMalloc(&dout, 64);
  hipMemcpy(da, ha, sizeof ha, hipMemcpyHostToDevice);
  hipMemcpy(db, hb, sizeof hb, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, 1, n, 0, 0, da, db, dout);
  hipMemcpy(ho, dout, sizeof ho, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < n; i++) {
    const unsigned want = ha[i] >= hb[i] ? ha[i] - hb[i] : 0u;
    printf("%08x - %08x clamp = %08x (want %08x)\n", ha[i], hb[i], ho[i], want);
    bad += ho[i] != want;
  }
  printf(bad ? "MISMATCH\n" : "ok\n");
  return bad;
}
