// VALU throughput probe for gfx950 (diagnostic, not part of the product).
// One workgroup of W waves on one CU (W/4 waves per SIMD), each wave runs 8 independent chains of
// one instruction, 64 iterations unrolled x 8.  Prints SIMD cycles per wave-instruction
// (= wave cycles / instructions issued per SIMD).
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHAIN8(OP) OP(a0) OP(a1) OP(a2) OP(a3) OP(a4) OP(a5) OP(a6) OP(a7)

#define DEFK(NAME, OPSTR)                                                                        \
  __global__ void NAME(int* out, long long* cyc) {                                             \
    int a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,      \
        a6 = a0 + 6, a7 = a0 + 7;                                                                \
    int k = threadIdx.x * 3 + 1;                                                                 \
    __syncthreads();                                                                             \
    long long t0 = __builtin_amdgcn_s_memtime();                                                 \
    for (int it = 0; it < 64; it++) {                                                            \
      _Pragma("unroll") for (int u = 0; u < 8; u++) {                                            \
        CHAIN8(OPSTR)                                                                            \
      }                                                                                          \
    }                                                                                            \
    __syncthreads();                                                                             \
    long long t1 = __builtin_amdgcn_s_memtime();                                                 \
    out[threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;                                    \
    if (threadIdx.x == 0) cyc[0] = t1 - t0;                                                      \
  }

#define OP_MAXI(x) asm volatile("v_max_i32 %0, %0, %1" : "+v"(x) : "v"(k));
DEFK(k_maxi, OP_MAXI)
#define OP_ADDU(x) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(k));
DEFK(k_addu, OP_ADDU)
#define OP_ADDU64(x) asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(x) : "v"(k));
DEFK(k_addu64, OP_ADDU64)
#define OP_SUBU(x) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(x) : "v"(k));
DEFK(k_subu, OP_SUBU)
#define OP_ADD3(x) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(x) : "v"(k));
DEFK(k_add3, OP_ADD3)
#define OP_CVTI(x) asm volatile("v_cvt_i32_f32 %0, %0" : "+v"(x) );
DEFK(k_cvti, OP_CVTI)
#define OP_CVTF(x) asm volatile("v_cvt_f32_i32 %0, %0" : "+v"(x) );
DEFK(k_cvtf, OP_CVTF)
#define OP_FMA(x) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(x) : "v"(k));
DEFK(k_fma, OP_FMA)
#define OP_MAXF(x) asm volatile("v_max_f32 %0, %0, %1" : "+v"(x) : "v"(k));
DEFK(k_maxf, OP_MAXF)
#define OP_MULF(x) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x) : "v"(k));
DEFK(k_mulf, OP_MULF)
#define OP_ADDF(x) asm volatile("v_add_f32 %0, %0, %1" : "+v"(x) : "v"(k));
DEFK(k_addf, OP_ADDF)
#define OP_ADDFABS(x) asm volatile("v_add_f32_e64 %0, %0, |%1|" : "+v"(x) : "v"(k));
DEFK(k_addfabs, OP_ADDFABS)
#define OP_ASHRPK(x) asm volatile("v_ashr_pk_i8_i32 %0, %0, %1, 0" : "+v"(x) : "v"(k));
DEFK(k_ashrpk, OP_ASHRPK)
#define OP_ASHRPKU(x) asm volatile("v_ashr_pk_u8_i32 %0, %0, %1, 0" : "+v"(x) : "v"(k));
DEFK(k_ashrpku, OP_ASHRPKU)
#define OP_PERM(x) asm volatile("v_perm_b32 %0, %0, %1, %1" : "+v"(x) : "v"(k));
DEFK(k_perm, OP_PERM)
#define OP_MED3(x) asm volatile("v_med3_i32 %0, %0, %1, %1" : "+v"(x) : "v"(k));
DEFK(k_med3, OP_MED3)
#define OP_MED3F(x) asm volatile("v_med3_f32 %0, %0, %1, %1" : "+v"(x) : "v"(k));
DEFK(k_med3f, OP_MED3F)
#define OP_PKMAXI16(x) asm volatile("v_pk_max_i16 %0, %0, %1" : "+v"(x) : "v"(k));
DEFK(k_pkmaxi16, OP_PKMAXI16)
#define OP_PKADDU16(x) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(x) : "v"(k));
DEFK(k_pkaddu16, OP_PKADDU16)
#define OP_MAX3I(x) asm volatile("v_max3_i32 %0, %0, %1, %1" : "+v"(x) : "v"(k));
DEFK(k_max3i, OP_MAX3I)
#define OP_LSHLOR(x) asm volatile("v_lshl_or_b32 %0, %0, 8, %1" : "+v"(x) : "v"(k));
DEFK(k_lshlor, OP_LSHLOR)
#define OP_ANDB(x) asm volatile("v_and_b32 %0, %0, %1" : "+v"(x) : "v"(k));
DEFK(k_andb, OP_ANDB)
#define OP_ORB(x) asm volatile("v_or_b32 %0, %0, %1" : "+v"(x) : "v"(k));
DEFK(k_orb, OP_ORB)
#define OP_XORB(x) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(k));
DEFK(k_xorb, OP_XORB)
#define OP_LSHL(x) asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(x) );
DEFK(k_lshl, OP_LSHL)
#define OP_ASHR(x) asm volatile("v_ashrrev_i32 %0, 3, %0" : "+v"(x) );
DEFK(k_ashr, OP_ASHR)
#define OP_CVTPKI16(x) asm volatile("v_cvt_pk_i16_i32 %0, %0, %1" : "+v"(x) : "v"(k));
DEFK(k_cvtpki16, OP_CVTPKI16)
#define OP_SATPKU8(x) asm volatile("v_sat_pk_u8_i16 %0, %0" : "+v"(x) );
DEFK(k_satpku8, OP_SATPKU8)
#define OP_CVTPKU8(x) asm volatile("v_cvt_pk_u8_f32 %0, %1, 1, %0" : "+v"(x) : "v"(k));
DEFK(k_cvtpku8, OP_CVTPKU8)
#define OP_CVTPKNORM(x) asm volatile("v_cvt_pknorm_i16_f32 %0, %0, %1" : "+v"(x) : "v"(k));
DEFK(k_cvtpknorm, OP_CVTPKNORM)
#define OP_SDOT4(x) asm volatile("v_dot4_i32_i8 %0, %1, %1, %0" : "+v"(x) : "v"(k));
DEFK(k_sdot4, OP_SDOT4)
#define OP_MAD24(x) asm volatile("v_mad_i32_i24 %0, %0, %1, %1" : "+v"(x) : "v"(k));
DEFK(k_mad24, OP_MAD24)
#define OP_MAXU(x) asm volatile("v_max_u32 %0, %0, %1" : "+v"(x) : "v"(k));
DEFK(k_maxu, OP_MAXU)
#define OP_MOVB(x) asm volatile("v_mov_b32 %0, %1" : "+v"(x) : "v"(k));
DEFK(k_movb, OP_MOVB)
#define OP_CNDM(x) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x) : "v"(k));
DEFK(k_cndm, OP_CNDM)
#define OP_BFE(x) asm volatile("v_bfe_i32 %0, %0, 8, 8" : "+v"(x) );
DEFK(k_bfe, OP_BFE)
#define OP_ADDI32(x) asm volatile("v_add_i32 %0, %0, %1" : "+v"(x) : "v"(k));
DEFK(k_addi32, OP_ADDI32)
#define OP_MAXIMUM3F(x) asm volatile("v_maximum3_f32 %0, %0, %1, %1" : "+v"(x) : "v"(k));
DEFK(k_maximum3f, OP_MAXIMUM3F)
#define OP_BITOP3(x) asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x12" : "+v"(x) : "v"(k));
DEFK(k_bitop3, OP_BITOP3)
#define OP_SUBREVU(x) asm volatile("v_subrev_u32 %0, %0, %1" : "+v"(x) : "v"(k));
DEFK(k_subrevu, OP_SUBREVU)
#define OP_MINF(x) asm volatile("v_min_f32 %0, %0, %1" : "+v"(x) : "v"(k));
DEFK(k_minf, OP_MINF)
#define OP_MINI(x) asm volatile("v_min_i32 %0, %0, %1" : "+v"(x) : "v"(k));
DEFK(k_mini, OP_MINI)
#define OP_SUBUCL(x) asm volatile("v_sub_u32_e64 %0, %0, %1 clamp" : "+v"(x) : "v"(k));
DEFK(k_subucl, OP_SUBUCL)
#define OP_MAXI64(x) asm volatile("v_max_i32_e64 %0, %0, %1" : "+v"(x) : "v"(k));
DEFK(k_maxi64, OP_MAXI64)
#define OP_SUBICL(x) asm volatile("v_sub_i32 %0, %0, %1 clamp" : "+v"(x) : "v"(k));
DEFK(k_subicl, OP_SUBICL)
#define OP_DPP(x) asm volatile("v_add_u32_dpp %0, %1, %0 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(x) : "v"(k));
DEFK(k_dpp, OP_DPP)


__global__ void k_cnd_vcc(int* out, long long* cyc) {
  int a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  int k = threadIdx.x * 3 + 1;
  asm volatile("v_cmp_gt_u32 vcc, 32, %0" :: "v"(a0));
  __syncthreads();
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < 64; it++) {
#pragma unroll
    for (int u = 0; u < 8; u++) {
#define OPC(x) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x) : "v"(k));
      CHAIN8(OPC)
    }
  }
  __syncthreads();
  long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
__global__ void k_cnd_sgpr(int* out, long long* cyc) {
  int a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  int k = threadIdx.x * 3 + 1;
  unsigned long long m;
  asm volatile("v_cmp_gt_u32 %0, 32, %1" : "=s"(m) : "v"(a0));
  __syncthreads();
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < 64; it++) {
#pragma unroll
    for (int u = 0; u < 8; u++) {
#define OPS(x) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(x) : "v"(k), "s"(m));
      CHAIN8(OPS)
    }
  }
  __syncthreads();
  long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}


#define OP_CVTSDWA(x) asm volatile("v_cvt_i32_f32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD" : "+v"(x) : "v"(k));
DEFK(k_cvtsdwa, OP_CVTSDWA)
#define OP_CVTSDWA0(x) asm volatile("v_cvt_i32_f32_sdwa %0, %1 dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD" : "=v"(x) : "v"(x));
DEFK(k_cvtsdwa0, OP_CVTSDWA0)

// packed f32 (64-bit register pairs)
typedef float f2 __attribute__((ext_vector_type(2)));
#define OP_PKFMA(x) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(x) : "v"(kk));
#define OP_PKADD(x) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(x) : "v"(kk));
#define OP_PKFMAC(x) asm volatile("v_pk_fma_f32 %0, %0, %1, %1 clamp" : "+v"(x) : "v"(kk));
#define DEFK2(NAME, OPSTR)                                                                       \
  __global__ void NAME(int* out, long long* cyc) {                                             \
    f2 a0 = {(float)threadIdx.x, 1.f}, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,      \
       a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;                                                    \
    f2 kk = {1.0f, 0.5f};                                                                        \
    __syncthreads();                                                                             \
    long long t0 = __builtin_amdgcn_s_memtime();                                                 \
    for (int it = 0; it < 64; it++) {                                                            \
      _Pragma("unroll") for (int u = 0; u < 8; u++) {                                            \
        CHAIN8(OPSTR)                                                                            \
      }                                                                                          \
    }                                                                                            \
    __syncthreads();                                                                             \
    long long t1 = __builtin_amdgcn_s_memtime();                                                 \
    f2 s = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;                                                \
    out[threadIdx.x] = (int)(s.x + s.y);                                                         \
    if (threadIdx.x == 0) cyc[0] = t1 - t0;                                                      \
  }
DEFK2(k_pkfma, OP_PKFMA)
DEFK2(k_pkadd, OP_PKADD)
DEFK2(k_pkfmac, OP_PKFMAC)

// MFMA + VALU mix: per iteration one MFMA 32x32x32 i8 and N int VALU (4 waves/SIMD)
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
template <int NV>
__global__ void k_mix(int* out, long long* cyc) {
  int a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  int k = threadIdx.x * 3 + 1;
  v4i A = {k, k + 1, k + 2, k + 3}, B = {k, 2, 3, 4};
  v16i acc = {};
  __syncthreads();
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < 64; it++) {
#pragma unroll
    for (int u = 0; u < 4; u++) {
      acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(A, B, acc, 0, 0, 0);
      if (NV > 0) { OP_MAXI(a0) }
      if (NV > 1) { OP_MAXI(a1) }
      if (NV > 2) { OP_MAXI(a2) }
      if (NV > 3) { OP_MAXI(a3) }
      if (NV > 4) { OP_MAXI(a4) }
      if (NV > 5) { OP_MAXI(a5) }
      if (NV > 6) { OP_MAXI(a6) }
      if (NV > 7) { OP_MAXI(a7) }
      if (NV > 8) { OP_MAXI(a0) }
      if (NV > 9) { OP_MAXI(a1) }
      if (NV > 10) { OP_MAXI(a2) }
      if (NV > 11) { OP_MAXI(a3) }
      if (NV > 12) { OP_MAXI(a4) }
      if (NV > 13) { OP_MAXI(a5) }
      if (NV > 14) { OP_MAXI(a6) }
      if (NV > 15) { OP_MAXI(a7) }
    }
  }
  __syncthreads();
  long long t1 = __builtin_amdgcn_s_memtime();
  int s = 0;
  for (int i = 0; i < 16; i++) s ^= acc[i];
  out[threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ s;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

typedef void (*KF)(int*, long long*);
static double run(KF f, int waves, double ninstr_per_wave, int* dout, long long* dcyc) {
  long long best = 1LL << 60;
  for (int r = 0; r < 5; r++) {
    hipLaunchKernelGGL(f, dim3(1), dim3(64 * waves), 0, 0, dout, dcyc);
    hipDeviceSynchronize();
    long long c;
    hipMemcpy(&c, dcyc, 8, hipMemcpyDeviceToHost);
    if (c < best) best = c;
  }
  // instructions per SIMD = ninstr_per_wave * waves / 4
  return (double)best / (ninstr_per_wave * (waves > 4 ? waves / 4.0 : 1.0));
}

int main() {
  int* dout;
  long long* dcyc;
  hipMalloc(&dout, 4096 * 4);
  hipMalloc(&dcyc, 64);
  struct { const char* n; KF f; } ks[] = {{"v_max_i32", k_maxi}, {"v_add_u32", k_addu}, {"v_add_u32_e64", k_addu64}, {"v_sub_u32", k_subu}, {"v_add3_u32", k_add3}, {"v_cvt_i32_f32", k_cvti}, {"v_cvt_f32_i32", k_cvtf}, {"v_fma_f32", k_fma}, {"v_max_f32", k_maxf}, {"v_mul_f32", k_mulf}, {"v_add_f32", k_addf}, {"v_add_f32_e64", k_addfabs}, {"v_ashr_pk_i8_i32", k_ashrpk}, {"v_ashr_pk_u8_i32", k_ashrpku}, {"v_perm_b32", k_perm}, {"v_med3_i32", k_med3}, {"v_med3_f32", k_med3f}, {"v_pk_max_i16", k_pkmaxi16}, {"v_pk_add_u16", k_pkaddu16}, {"v_max3_i32", k_max3i}, {"v_lshl_or_b32", k_lshlor}, {"v_and_b32", k_andb}, {"v_or_b32", k_orb}, {"v_xor_b32", k_xorb}, {"v_lshlrev_b32", k_lshl}, {"v_ashrrev_i32", k_ashr}, {"v_cvt_pk_i16_i32", k_cvtpki16}, {"v_sat_pk_u8_i16", k_satpku8}, {"v_cvt_pk_u8_f32", k_cvtpku8}, {"v_cvt_pknorm_i16_f32", k_cvtpknorm}, {"v_dot4_i32_i8", k_sdot4}, {"v_mad_i32_i24", k_mad24}, {"v_max_u32", k_maxu}, {"v_mov_b32", k_movb}, {"v_cndmask_b32", k_cndm}, {"v_bfe_i32", k_bfe}, {"v_add_i32", k_addi32}, {"v_maximum3_f32", k_maximum3f}, {"v_bitop3_b32", k_bitop3}, {"v_subrev_u32", k_subrevu}, {"v_min_f32", k_minf}, {"v_min_i32", k_mini}, {"v_add_u32_dpp", k_dpp}, {"v_sub_u32_e64 clamp", k_subucl}, {"v_max_i32_e64", k_maxi64}, {"v_sub_i32 clamp", k_subicl}, {"v_cndmask(vcc set)", k_cnd_vcc}, {"v_cndmask_e64(sgpr)", k_cnd_sgpr}, {"v_cvt_i32_f32_sdwa(byte1,preserve)", k_cvtsdwa}, {"v_cvt_i32_f32_sdwa(byte0,pad)", k_cvtsdwa0}, {"v_pk_fma_f32 clamp", k_pkfmac}, {"v_pk_fma_f32", k_pkfma}, {"v_pk_add_f32", k_pkadd}};
  const double n = 64.0 * 8 * 8;
  printf("SIMD cycles per wave-instruction (1 / 2 / 4 waves per SIMD)\n");
  for (auto& k : ks) {
    printf("%-18s", k.n);
    for (int w : {4, 8, 16}) printf(" %6.2f", run(k.f, w, n, dout, dcyc));
    printf("\n");
  }
  printf("MFMA 32x32x32 i8 + N v_max_i32 per MFMA, SIMD cycles per MFMA (1/2/4 waves per SIMD)\n");
  KF mix[] = {k_mix<0>, k_mix<2>, k_mix<4>, k_mix<6>, k_mix<8>, k_mix<12>, k_mix<16>};
  int nv[] = {0, 2, 4, 6, 8, 12, 16};
  for (int i = 0; i < 7; i++) {
    printf("N=%2d            ", nv[i]);
    for (int w : {4, 8, 16}) printf(" %6.2f", run(mix[i], w, 64.0 * 4, dout, dcyc));
    printf("\n");
  }
  return 0;
}
