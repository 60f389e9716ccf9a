// Semantics probe (diagnostic): v_cvt_i32_f32 with SDWA byte destination, v_pk_fma_f32 clamp.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));
__global__ void k(const float* in, unsigned* out) {
  int t = threadIdx.x;
  float a = in[4 * t], b = in[4 * t + 1], c = in[4 * t + 2], d = in[4 * t + 3];
  unsigned r = 0xdeadbeefu;
  asm volatile("v_cvt_i32_f32_sdwa %0, %1 dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD\n"
               "v_cvt_i32_f32_sdwa %0, %2 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD\n"
               "v_cvt_i32_f32_sdwa %0, %3 dst_sel:BYTE_2 dst_unused:UNUSED_PRESERVE src0_sel:DWORD\n"
               "v_cvt_i32_f32_sdwa %0, %4 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:DWORD"
               : "+v"(r) : "v"(a), "v"(b), "v"(c), "v"(d));
  out[2 * t] = r;
  unsigned r2 = 0xdeadbeefu;
  asm volatile("v_cvt_i32_f32_sdwa %0, %1 dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD\n s_nop 0\n"
               "v_cvt_i32_f32_sdwa %0, %2 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD\n s_nop 0\n"
               "v_cvt_i32_f32_sdwa %0, %3 dst_sel:BYTE_2 dst_unused:UNUSED_PRESERVE src0_sel:DWORD\n s_nop 0\n"
               "v_cvt_i32_f32_sdwa %0, %4 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:DWORD"
               : "+v"(r2) : "v"(a), "v"(b), "v"(c), "v"(d));
  out[64 + t] = r2;
  unsigned r3 = 0xdeadbeefu, r4 = 0x12345678u;
  asm volatile("v_cvt_i32_f32_sdwa %0, %2 dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD\n"
               "v_cvt_i32_f32_sdwa %1, %2 dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD\n"
               "v_cvt_i32_f32_sdwa %0, %3 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD\n"
               "v_cvt_i32_f32_sdwa %1, %3 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD\n"
               "v_cvt_i32_f32_sdwa %0, %4 dst_sel:BYTE_2 dst_unused:UNUSED_PRESERVE src0_sel:DWORD\n"
               "v_cvt_i32_f32_sdwa %1, %4 dst_sel:BYTE_2 dst_unused:UNUSED_PRESERVE src0_sel:DWORD\n"
               "v_cvt_i32_f32_sdwa %0, %5 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:DWORD\n"
               "v_cvt_i32_f32_sdwa %1, %5 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:DWORD"
               : "+v"(r3), "+v"(r4) : "v"(a), "v"(b), "v"(c), "v"(d));
  out[128 + t] = r3; out[192 + t] = r4;
  unsigned r5 = 0xdeadbeefu;
  asm volatile("v_cvt_i32_f32_sdwa %0, %1 clamp dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD\n s_nop 0\n"
               "v_cvt_i32_f32_sdwa %0, %2 clamp dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD\n s_nop 0\n"
               "v_cvt_i32_f32_sdwa %0, %3 clamp dst_sel:BYTE_2 dst_unused:UNUSED_PRESERVE src0_sel:DWORD\n s_nop 0\n"
               "v_cvt_i32_f32_sdwa %0, %4 clamp dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:DWORD"
               : "+v"(r5) : "v"(a), "v"(b), "v"(c), "v"(d));
  out[256 + t] = r5;
  f2 x = {a, b}, y = {0.5f, 0.25f}, z = {0.1f, 0.2f};
  f2 w;
  asm volatile("v_pk_fma_f32 %0, %1, %2, %3 clamp" : "=v"(w) : "v"(x), "v"(y), "v"(z));
  out[2 * t + 1] = (unsigned)(int)(w.x * 1000.f) | ((unsigned)(int)(w.y * 1000.f) << 16);
}
int main() {
  float h[16] = {1.9f, -1.9f, 127.5f, -128.7f, 200.f, -300.f, 0.2f, -0.2f, 5.f, 3.f, -2.f, 0.f, 1e9f, -1e9f, 126.99f, -127.99f};
  float* d; unsigned* o; hipMalloc(&d, 64); hipMalloc(&o, 4096);
  hipMemcpy(d, h, 64, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, 1, 4, 0, 0, d, o);
  unsigned r[320]; hipMemcpy(r, o, 1280, hipMemcpyDeviceToHost);
  for (int t = 0; t < 4; t++) {
    printf("in %g %g %g %g -> bytes", h[4*t], h[4*t+1], h[4*t+2], h[4*t+3]);
    for (int b = 0; b < 4; b++) printf(" %d", (int)(signed char)(r[2*t] >> (8*b)));
    for (int v = 1; v < 5; v++) { printf(" | v%d", v); for (int b = 0; b < 4; b++) printf(" %d", (int)(signed char)(r[64 * v + t] >> (8*b))); }
    printf(" | pk_fma clamp (x*[.5,.25]+[.1,.2]) x1000: %u %u\n", r[2*t+1] & 0xffff, r[2*t+1] >> 16);
  }
  return 0;
}
