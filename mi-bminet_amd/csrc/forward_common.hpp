// forward_common.hpp — types, parameter images and helpers of the gfx950 forward kernel
// (forward_wg.hpp).
//
// Requantisation y = clip(trunc((acc + off) / fac), -128, 127) is computed as
// clip(int(float(acc + off) * r)) with r chosen on the host (mibminet.hip: choose_reciprocal) and
// verified at every step boundary of the clipped output range, so it is bit-exact to C's integer
// division for every reachable accumulator.  Parameter sets outside that float envelope run the
// exact-division builds (Cfg::XR: xdiv below) at layers 1, 2 and 4.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace mib {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef float f2 __attribute__((ext_vector_type(2)));

constexpr int F2 = 16;          // filters (F1 == F2, D == 1)
constexpr int N_OUT = 4;        // classes
constexpr int L2_TAPS = 64;
constexpr int L3_TAPS = 16;
constexpr int ND5_MAX = 96;     // dwords of the layer-4 output [F2][T64_ALIGN] (F2*T64_ALIGN <= 384)
constexpr int FMAGIC_I = 0x4B400000;   // bit pattern of 1.5 * 2^23
constexpr float FMAGIC_F = 12582912.0f; // 1.5 * 2^23
// REORDER_BN pooling bias: the layer-2 MFMA chains start from a bias B (the bits of a
// float MFMA srcC inline constant), so every conv value a lies at a + B with no wrap (|a| < 2^22),
// and max(a, thr) - thr = sat_u32((a + B) - (thr + B)): one full-rate v_sub_u32 clamp per element
// instead of a quarter-rate v_max_i32 (tools/vthru.hip: 2.45 vs 4.21 SIMD cycles).  Each chain
// gets a constant of its own (filter slot 0: 1.0, slot 1: 2.0, the tail: 4.0): a constant shared
// by two chains is hoisted into a 16-register tuple instead of riding in the instruction.
// (layer 4 uses 0.5, -0.5 and -1.0: forward_wg.hpp, bias4)
__host__ __device__ constexpr int pbias(int slot) { return slot == 0 ? 0x3F800000 : slot == 1 ? 0x40000000 : 0x40800000; }
constexpr int PBIAS_TAIL = pbias(2);

// Diagnostic phase stamps (tools/probe.hip builds with -DMIB_STAMPS; compiled out otherwise).
#ifdef MIB_STAMPS
// g_stamps[8 w + i]: phase i cycles summed over wave w of every workgroup (w < 8);
// [64] s_memtime total, [65] s_memrealtime total, [66] flushers
__device__ unsigned long long g_stamps[72];
#define MIB_STAMP_INIT unsigned long long _st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}; \
  unsigned long long _st_t = __builtin_amdgcn_s_memtime(); \
  const unsigned long long _st_t0 = _st_t, _st_r0 = __builtin_amdgcn_s_memrealtime();
#define MIB_STAMP(i) { const unsigned long long _t = __builtin_amdgcn_s_memtime(); _st_acc[i] += _t - _st_t; _st_t = _t; }
#define MIB_STAMP_FLUSH(cond, slot) if (cond) { for (int _i = 0; _i < 8; _i++) atomicAdd(&g_stamps[8 * (slot) + _i], _st_acc[_i]); \
  atomicAdd(&g_stamps[64], __builtin_amdgcn_s_memtime() - _st_t0); atomicAdd(&g_stamps[65], __builtin_amdgcn_s_memrealtime() - _st_r0); \
  atomicAdd(&g_stamps[66], 1ull); }
#else
#define MIB_STAMP_INIT
#define MIB_STAMP(i)
#define MIB_STAMP_FLUSH(cond, slot)
#endif

// Diagnostic in-kernel clock (tools/clock_probe.hip builds with -DMIB_CLOCK; compiled out
// otherwise): one s_memtime / s_memrealtime pair around the trial loop per workgroup, summed
// per workgroup over launches into g_clk[2 wg], g_clk[2 wg + 1].  No stamp inside the loop, and
// nothing the kernel computes reads g_clk.  clock = d(memtime) / d(memrealtime) x 100 MHz.
#ifdef MIB_CLOCK
constexpr int CLK_SLOTS = 4096;
__device__ unsigned long long g_clk[2 * CLK_SLOTS];
#define MIB_CLOCK_INIT const unsigned long long _ck_t0 = __builtin_amdgcn_s_memtime(), \
  _ck_r0 = __builtin_amdgcn_s_memrealtime();
#define MIB_CLOCK_FLUSH if (threadIdx.x == 0 && blockIdx.x < CLK_SLOTS) { \
  const unsigned long long _t = __builtin_amdgcn_s_memtime(), _r = __builtin_amdgcn_s_memrealtime(); \
  atomicAdd(&g_clk[2 * blockIdx.x], _t - _ck_t0); atomicAdd(&g_clk[2 * blockIdx.x + 1], _r - _ck_r0); }
#else
#define MIB_CLOCK_INIT
#define MIB_CLOCK_FLUSH
#endif

__host__ __device__ constexpr int align16(int x) { return (x + 15) & ~15; }
__host__ __device__ constexpr int cmax(int a, int b) { return a > b ? a : b; }
__host__ __device__ constexpr int cmin(int a, int b) { return a < b ? a : b; }
// smallest multiple of 4 >= x whose dword count is odd (conflict-free strided dword reads)
__host__ __device__ constexpr int odd_dwords(int x) { return ((x + 3) / 4 % 2) ? (x + 3) / 4 * 4 : (x + 3) / 4 * 4 + 4; }

// Parameters read into LDS by every workgroup.
struct SmallParams {
  v4i l4_bfrag[64];       // layer-4 B operand per lane (block diagonal, see host)
  v4i l2_tpar[F2];        // layer-2 tail per filter: {PBIAS_TAIL + thr, off + 8 thr, bits of r, 0}
                          // (thr = -(net_l2_offset >> 3); off + 8 thr = net_l2_offset & 7);
                          // XR: {.., .., xdiv magic, shift word}
  int l4_thr[F2];         // -(net_l4_offset >> 3), clamped to the conv range (mibminet.hip)
  int l4_offm[F2];        // net_l4_offset + 8 thr
  union {
    float l4_r[F2];
    unsigned l4_m[F2];    // XR: xdiv magic
  };
  // plain (non-REORDER_BN) layer-2/4 branches: per-element BN with offset >> 3 and factor >> 3 in
  // the floor form (mibminet.hip, choose_floor_form): MFMA C-init = per-filter magic bits + offset,
  // reciprocal r and integer-valued c, so that fma(acc bits, r, c) = FMAGIC + floor(element).
  // XR: C-init = offset >> 3, xdiv magic and shift word; l2_xs / l4_xs are also the shift words of
  // the REORDER_BN builds' layer-2 / layer-4 requant (whose plain fields are unused)
  int l2n_ci[F2];
  union {
    float l2n_r[F2];
    unsigned l2n_m[F2];
  };
  union {
    float l2n_c[F2];
    int l2_xs[F2];
  };
  int l4n_ci[F2];
  union {
    float l4n_r[F2];
    unsigned l4n_m[F2];
  };
  union {
    float l4n_c[F2];
    int l4_xs[F2];
  };
  int l5_w[N_OUT][ND5_MAX];  // [k][v] with row stride T64_ALIGN, zero padded
  int l5_b[N_OUT];
  float l3_r;
  float l5_r;
  float l3_c;             // -(1.5 * 2^23) * l3_r (layer 3's magic C-init requant)
  int pad[1];
};

// Operand fragments and requantisation constants, built by the host from the net.h arrays.
struct DevParams {
  v4i l1_wfrag[2][64];      // layer-1 B operand per N-tile and lane
  int l1_cinit[2][16];      // offset + FMAGIC_I per N-tile column (XR: offset)
  union {
    float l1_r[2][16];      // reciprocal per N-tile column
    unsigned l1_m[2][16];   // XR: xdiv magic
  };
  union {
    float l1_c[2][16];      // -(1.5 * 2^23) * r, exact
    int l1_xs[2][16];       // XR: xdiv shift word
  };
  v4i l2_afrag[F2][3][64];  // layer-2 A operand (banded weights) per filter, K-step and lane
  int l2_thrb[F2];          // pbias(f & 1) + thr, thr = -(net_l2_offset >> 3) clamped: full-tile threshold
  int l2_offm[F2];          // net_l2_offset + 8 thr
  union {
    float l2_r[F2];
    unsigned l2_m[F2];      // XR: xdiv magic (shift word: sp.l2_xs)
  };
  // layer-3 A operands per filter pair (wave) and lane, MFMA 16x16x64 with a block-diagonal K
  // (forward_wg.hpp, layer3): tile 1 = 16 shifts x both filters' 32-slot bands, tile 2 = the same
  // with shift g on row 4g and the other rows zero
  v4i l3_a1[F2 / 2][64];
  v4i l3_a2[F2 / 2][64];
  // layer-2 tail A operand per filter pair (wave) and K-step: MFMA 16x16x64, 16 shifts x 192
  // K-slots = the two filters' 96-slot bands side by side (K block diagonal, see forward_wg.hpp)
  v4i l2t_afrag[F2 / 2][3][64];
  SmallParams sp;
  v4i l1_wfrag_ct[2][64];   // layer-1 B operand for the channel-major staging's K-slot order (stage_block)
};

// LO: lower clip bound, -128 (the C's __CLIP_R(x, 127), clip_balanced=False) or -127
// (golden_model.py clip_balanced=True, functional.py:89-91)
template <int LO = -128>
__device__ __forceinline__ int rq(int v, float r) {
  const int t = (int)((float)v * r);
  return min(max(t, LO), 127);
}

// int32 -> saturated int8 pairs (gfx950 v_ashr_pk_i8_i32, shift 0): a to byte 0, b to byte 1.
// The op_sel form writes bytes 2/3 and keeps bytes 0/1 (checked on hardware by
// tools/isa_probe.hip).
template <int LO = -128>
__device__ __forceinline__ unsigned sat8x2(int a, int b) {
  if constexpr (LO != -128) {  // the pack saturates at -128 only
    a = max(a, LO);
    b = max(b, LO);
  }
  unsigned r;
  asm("v_ashr_pk_i8_i32 %0, %1, %2, 0" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
template <int LO = -128>
__device__ __forceinline__ unsigned sat8x4(int a, int b, int c, int d) {
  if constexpr (LO != -128) {
    c = max(c, LO);
    d = max(d, LO);
  }
  unsigned r = sat8x2<LO>(a, b);
  asm("v_ashr_pk_i8_i32 %0, %1, %2, 0 op_sel:[0,0,0,1]" : "+v"(r) : "v"(c), "v"(d));
  return r;
}

// sat8x4 through the compiler builtin (no inline asm): the compiler sees the instructions and
// orders them against MFMAs still in flight (layer 3, whose tile 2 uses only part of its result);
// the high pair costs a shift and an OR instead of op_sel
template <int LO = -128>
__device__ __forceinline__ unsigned sat8x4_b(int a, int b, int c, int d) {
  if constexpr (LO != -128) {
    a = max(a, LO); b = max(b, LO); c = max(c, LO); d = max(d, LO);
  }
  const unsigned lo = __builtin_amdgcn_ashr_pk_i8_i32(a, b, 0), hi = __builtin_amdgcn_ashr_pk_i8_i32(c, d, 0);
  return (lo & 0xFFFFu) | (hi << 16);
}

// Layer-1 per-lane constants of one N-tile (kept as a scalarisable struct: arrays of these
// fields get merged into vector loads of a stack slot by LLVM and end up in scratch).
struct L1Tile {
  v4i wf;
  int ci;
  float rr, cc;      // float requant: reciprocal and magic constant
  unsigned xm;       // XR: the xdiv constant's low and high words, carried as integers
  int xs;
};

// Two requant fmas / multiplies on float bit patterns, issued as two v_fma_f32 / v_mul_f32: packed
// f32 VALU beside MFMAs costs more issue time than the two plain instructions (same-box A/B of
// the fused kernel: -0.5 %, 13 of 15 interleaved rounds).  PACKED: one v_pk_fma_f32 (layer 3, where
// no MFMA of the wave is in flight: -0.8 %).
template <bool PACKED = false>
__device__ __forceinline__ f2 fma2(int a, int b, float r, float c) {
  if constexpr (!PACKED)
    return (f2){__builtin_fmaf(__int_as_float(a), r, c), __builtin_fmaf(__int_as_float(b), r, c)};
  return __builtin_elementwise_fma((f2){__int_as_float(a), __int_as_float(b)}, (f2){r, r}, (f2){c, c});
}
__device__ __forceinline__ f2 mul2(float a, float b, float r) { return (f2){a * r, b * r}; }

// Exact C division trunc(e / d) for every int32 e and d != 0 (the reference's int32 division;
// INT_MIN / -1 is refused at load), for the exact-division builds (Cfg::XR).  (lo, hi) are the two
// halves of the double r = sign(d) RU(1 / |d|) (mibminet.hip, xdiv_consts): trunc(e r) in double
// (v_cvt_f64_i32, v_mul_f64, v_cvt_i32_f64) equals trunc(e / d).  For e, d > 0 with e / d = q + f:
// e r >= e / d, so the rounded product is >= q; e r - e / d <= e 2^-52 / d, and the distance from
// q + f to q + 1 is >= 1 / d > 1.5 (e / d) 2^-52 for |e| <= 2^31, more than the error plus half an
// ulp of the product, so it stays below q + 1.  The other signs are the mirror image.  Proof and
// host emulation: mibminet.hip, xdiv_consts / xdiv_host; every int32 dividend on the device for
// three divisors and every quotient step for many more: tests/test_gpu_xr.py.  (Round 5 used a
// 32 x 32 -> 64-bit integer multiply-shift, about twice the issue cycles.)
__device__ __forceinline__ int xdiv(int e, unsigned lo, int hi) {
  const double r = __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi << 32) | lo);
  return (int)((double)e * r);
}

// max(a, thr) - thr for a biased accumulator value acc = a + B and thrb = thr + B
__device__ __forceinline__ unsigned relu_b(int acc, int thrb) {
  return __builtin_elementwise_sub_sat((unsigned)acc, (unsigned)thrb);
}

// sum_{i<8} max(a[base + i], thr) + off = sum_{i<8} relu_b(acc[base + i], thrb) + offm, offm =
// off + 8 thr  (the REORDER_BN ReLU + sum-pool of layers 2 and 4; acc = a + B)
template <int BASE>
__device__ __forceinline__ int pool8b(const v16i& acc, int thrb, int offm) {
  unsigned m[8];
#pragma unroll
  for (int i = 0; i < 8; i++) m[i] = relu_b(acc[BASE + i], thrb);
  return (int)(((m[0] + m[1] + m[2]) + (m[3] + m[4]) + (m[5] + m[6])) + (m[7] + (unsigned)offm));
}

}  // namespace mib
