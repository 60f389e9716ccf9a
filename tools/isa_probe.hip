// ISA behaviour / throughput micro-probe for gfx950 (diagnostic, not part of the product).
//  1. misaligned ds_read_b128: correctness and cost vs aligned
//  2. v_ashr_pk_i8_i32 with op_sel dst-hi: does it preserve the low half?
//  3. v_cvt_pk_u8_f32 rounding / saturation
//  4. issue cost of v_pk_fma_f32 vs v_fma_f32, v_cvt_i32_f32, v_med3_f32, v_sad_u32
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef int v4i __attribute__((ext_vector_type(4)));

__global__ void k_lds(int* out, long long* cyc, int mis) {
  __shared__ __attribute__((aligned(16))) unsigned char s[8192];
  for (int i = threadIdx.x; i < 8192; i += 64) s[i] = (unsigned char)(i * 7 + 3);
  __syncthreads();
  const int lane = threadIdx.x;
  unsigned addr = (unsigned)(uintptr_t)s + lane * 32 + mis;
  v4i r;
  asm volatile("ds_read_b128 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(addr));
  // correctness
  int ok = 1;
  for (int k = 0; k < 16; k++) {
    unsigned char want = s[lane * 32 + mis + k];
    unsigned char got = (unsigned char)(((unsigned)r[k / 4]) >> (8 * (k % 4)));
    ok &= want == got;
  }
  out[lane] = ok;
  // timing: 256 independent reads
  long long t0 = __builtin_amdgcn_s_memtime();
  v4i acc = {0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < 64; i++) {
    v4i a, b, c, d;
    unsigned ad = addr + ((i * 512) & 4095);
    asm volatile("ds_read_b128 %0, %4\n ds_read_b128 %1, %4 offset:1024\n ds_read_b128 %2, %4 offset:2048\n ds_read_b128 %3, %4 offset:3072\n s_waitcnt lgkmcnt(0)"
                 : "=v"(a), "=v"(b), "=v"(c), "=v"(d) : "v"(ad));
    acc += a ^ b ^ c ^ d;
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) cyc[0] = t1 - t0;
  out[64 + lane] = acc[0] ^ acc[1] ^ acc[2] ^ acc[3];
}

__global__ void k_ashr(int* out) {
  const int lane = threadIdx.x;
  int a = lane * 37 - 1000, b = 300 - lane * 11, c = lane * 3 - 100, d = -lane * 5 + 50;
  unsigned r = 0xDEADBEEF;
  asm volatile("v_ashr_pk_i8_i32 %0, %1, %2, 0" : "+v"(r) : "v"(a), "v"(b));
  unsigned lo = r;
  asm volatile("v_ashr_pk_i8_i32 %0, %1, %2, 0 op_sel:[0,0,0,1]" : "+v"(r) : "v"(c), "v"(d));
  out[4 * lane + 0] = (int)lo;
  out[4 * lane + 1] = (int)r;
  out[4 * lane + 2] = a;
  out[4 * lane + 3] = b;
}

__global__ void k_cvtu8(const float* in, unsigned* out, int n) {
  const int i = threadIdx.x;
  if (i < n) {
    unsigned r = 0x11223344u;
    asm volatile("v_cvt_pk_u8_f32 %0, %1, 1, %0" : "+v"(r) : "v"(in[i]));
    out[i] = r;
  }
}

template <int OP>
__global__ void k_tput(float* out, long long* cyc) {
  float x[8];
  for (int k = 0; k < 8; k++) x[k] = threadIdx.x * 0.001f + k;
  const float m = 1.0001f, c = 0.5f;
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < 256; it++) {
    if constexpr (OP == 0) {  // 8 independent v_fma_f32
      asm volatile("v_fma_f32 %0, %0, %8, %9\n v_fma_f32 %1, %1, %8, %9\n v_fma_f32 %2, %2, %8, %9\n v_fma_f32 %3, %3, %8, %9\n"
                   "v_fma_f32 %4, %4, %8, %9\n v_fma_f32 %5, %5, %8, %9\n v_fma_f32 %6, %6, %8, %9\n v_fma_f32 %7, %7, %8, %9"
                   : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]) : "v"(m), "v"(c));
    } else if constexpr (OP == 1) {  // 4 independent v_pk_fma_f32 (same 8 FMAs)
      typedef float f2 __attribute__((ext_vector_type(2)));
      f2 p0 = {x[0], x[1]}, p1 = {x[2], x[3]}, p2 = {x[4], x[5]}, p3 = {x[6], x[7]};
      f2 mm = {m, m}, cc = {c, c};
      asm volatile("v_pk_fma_f32 %0, %0, %4, %5\n v_pk_fma_f32 %1, %1, %4, %5\n v_pk_fma_f32 %2, %2, %4, %5\n v_pk_fma_f32 %3, %3, %4, %5"
                   : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3) : "v"(mm), "v"(cc));
      x[0] = p0[0]; x[1] = p0[1]; x[2] = p1[0]; x[3] = p1[1]; x[4] = p2[0]; x[5] = p2[1]; x[6] = p3[0]; x[7] = p3[1];
    } else if constexpr (OP == 2) {  // 8 v_med3_f32
      asm volatile("v_med3_f32 %0, %0, %8, %9\n v_med3_f32 %1, %1, %8, %9\n v_med3_f32 %2, %2, %8, %9\n v_med3_f32 %3, %3, %8, %9\n"
                   "v_med3_f32 %4, %4, %8, %9\n v_med3_f32 %5, %5, %8, %9\n v_med3_f32 %6, %6, %8, %9\n v_med3_f32 %7, %7, %8, %9"
                   : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]) : "v"(m), "v"(c));
    } else if constexpr (OP == 3) {  // 8 v_cvt_i32_f32 (in place, bit pattern garbage is fine)
      asm volatile("v_cvt_i32_f32 %0, %0\n v_cvt_i32_f32 %1, %1\n v_cvt_i32_f32 %2, %2\n v_cvt_i32_f32 %3, %3\n"
                   "v_cvt_i32_f32 %4, %4\n v_cvt_i32_f32 %5, %5\n v_cvt_i32_f32 %6, %6\n v_cvt_i32_f32 %7, %7"
                   : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]));
    } else if constexpr (OP == 4) {  // 8 v_sad_u32
      asm volatile("v_sad_u32 %0, %0, %8, %9\n v_sad_u32 %1, %1, %8, %9\n v_sad_u32 %2, %2, %8, %9\n v_sad_u32 %3, %3, %8, %9\n"
                   "v_sad_u32 %4, %4, %8, %9\n v_sad_u32 %5, %5, %8, %9\n v_sad_u32 %6, %6, %8, %9\n v_sad_u32 %7, %7, %8, %9"
                   : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]) : "v"(m), "v"(c));
    } else if constexpr (OP == 5) {  // 8 v_cvt_i32_f32 SDWA byte writes
      asm volatile("v_cvt_i32_f32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD\n"
                   "v_cvt_i32_f32_sdwa %2, %3 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD\n"
                   "v_cvt_i32_f32_sdwa %4, %5 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD\n"
                   "v_cvt_i32_f32_sdwa %6, %7 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD\n"
                   : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]));
    } else if constexpr (OP == 6) {  // 8 v_ashr_pk_i8_i32
      asm volatile("v_ashr_pk_i8_i32 %0, %1, %2, 0\n v_ashr_pk_i8_i32 %1, %2, %3, 0\n v_ashr_pk_i8_i32 %2, %3, %4, 0\n v_ashr_pk_i8_i32 %3, %4, %5, 0\n"
                   "v_ashr_pk_i8_i32 %4, %5, %6, 0\n v_ashr_pk_i8_i32 %5, %6, %7, 0\n v_ashr_pk_i8_i32 %6, %7, %0, 0\n v_ashr_pk_i8_i32 %7, %0, %1, 0"
                   : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]));
    }
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0;
  for (int k = 0; k < 8; k++) s += x[k];
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

template <int OP>
static double tput(float* dout, long long* dcyc) {
  hipLaunchKernelGGL(k_tput<OP>, dim3(1), dim3(64), 0, 0, dout, dcyc);
  long long c;
  hipMemcpy(&c, dcyc, 8, hipMemcpyDeviceToHost);
  return (double)c / (256.0 * 8.0);
}

int main() {
  int* dout; long long* dcyc; float* dfo; unsigned* du;
  hipMalloc(&dout, 4096 * 4); hipMalloc(&dcyc, 64); hipMalloc(&dfo, 4096 * 4); hipMalloc(&du, 4096);
  int h[256];
  long long cyc;
  for (int mis : {0, 4, 1, 8}) {
    hipLaunchKernelGGL(k_lds, dim3(1), dim3(64), 0, 0, dout, dcyc, mis);
    hipMemcpy(h, dout, 64 * 4, hipMemcpyDeviceToHost);
    hipMemcpy(&cyc, dcyc, 8, hipMemcpyDeviceToHost);
    int ok = 1;
    for (int i = 0; i < 64; i++) ok &= h[i];
    printf("ds_read_b128 misalign %d: correct=%d  %.1f cycles per read (256 reads, 4 in flight)\n", mis, ok, cyc / 256.0);
  }
  hipLaunchKernelGGL(k_ashr, dim3(1), dim3(64), 0, 0, dout);
  hipMemcpy(h, dout, 256 * 4, hipMemcpyDeviceToHost);
  for (int l : {0, 5, 20, 40, 63})
    printf("ashr_pk lane %d: a=%d b=%d lo=%08x after-hi=%08x\n", l, h[4 * l + 2], h[4 * l + 3], (unsigned)h[4 * l], (unsigned)h[4 * l + 1]);
  float fin[12] = {0.5f, 1.5f, 2.5f, 2.7f, -0.5f, -1.7f, 127.9f, 254.6f, 255.5f, 300.0f, -300.0f, 3.49f};
  hipMemcpy(dfo, fin, sizeof(fin), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_cvtu8, dim3(1), dim3(64), 0, 0, dfo, du, 12);
  unsigned hu[12];
  hipMemcpy(hu, du, sizeof(hu), hipMemcpyDeviceToHost);
  for (int i = 0; i < 12; i++) printf("cvt_pk_u8(%g) byte1 = %u  (dword %08x)\n", fin[i], (hu[i] >> 8) & 255, hu[i]);
  printf("issue cost per instruction, one wave (cycles): fma %.2f  pk_fma %.2f (x2 work)  med3 %.2f  cvt_i32 %.2f  sad %.2f\n",
         tput<0>(dfo, dcyc), tput<1>(dfo, dcyc) * 2, tput<2>(dfo, dcyc), tput<3>(dfo, dcyc), tput<4>(dfo, dcyc));
  printf("  cvt sdwa (4 per loop, cost per instr) %.2f   ashr_pk %.2f\n", tput<5>(dfo, dcyc) * 2, tput<6>(dfo, dcyc));
  return 0;
}
