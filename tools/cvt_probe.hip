// Rounding of v_cvt_pk_u8_f32 / v_cvt_pknorm_i16_f32 / fma under the default and RTZ round modes (diagnostic).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(const float* in, unsigned* out, int n) {
  int i = threadIdx.x;
  if (i >= n) return;
  float x = in[i];
  unsigned d = 0, e = 0, m = 0, g;
  asm volatile("v_cvt_pk_u8_f32 %0, %1, 0, %0" : "+v"(d) : "v"(x));
  // RTZ for f32 (MODE.FP_ROUND[1:0] = 3)
  __builtin_amdgcn_s_setreg((1 << 0) | (0 << 6) | (1 << 11), 3);  // hwreg(HW_REG_MODE, 0, 2)
  asm volatile("v_cvt_pk_u8_f32 %0, %1, 0, %0" : "+v"(e) : "v"(x));
  float s; asm volatile("v_add_f32 %0, %1, %2" : "=v"(s) : "v"(x), "v"(12582912.0f));
  __builtin_amdgcn_s_setreg((1 << 0) | (0 << 6) | (1 << 11), 0);
  float t; asm volatile("v_add_f32 %0, %1, %2" : "=v"(t) : "v"(x), "v"(12582912.0f));
  out[4 * i] = d; out[4 * i + 1] = e; out[4 * i + 2] = __float_as_uint(s) - 0x4B400000u; out[4 * i + 3] = __float_as_uint(t) - 0x4B400000u;
}
int main() {
  float h[] = {0.f, 0.4f, 0.5f, 0.6f, 1.5f, 2.5f, 2.7f, 254.6f, 255.5f, 300.f, -0.3f, -1.f, -1.5f, -2.5f, 127.999f, 3.0000002f};
  int n = sizeof(h) / 4;
  float* d; unsigned* o; hipMalloc(&d, 256); hipMalloc(&o, 1024);
  hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, 1, 64, 0, 0, d, o, n);
  unsigned r[64]; hipMemcpy(r, o, 4 * 4 * n, hipMemcpyDeviceToHost);
  for (int i = 0; i < n; i++) printf("x=%-10g cvt_pk_u8 RNE-mode %3u RTZ-mode %3u | magic add RTZ %d RNE %d\n", h[i], r[4*i] & 255, r[4*i+1] & 255, (int)r[4*i+2], (int)r[4*i+3]);
  return 0;
}
