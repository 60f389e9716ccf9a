// forward.hpp — gfx950 (CDNA4) device code of the fused MI-BMInet int8 forward pass.
//
// One workgroup (4 wave64s) owns one trial at a time and walks a grid-strided list of trials
// (persistent).  Per trial:
//   stage   HBM -> LDS: the trial's [T][C] int8 block, 16 B per lane, nontemporal.
//   layer1  spatial 22->16 contraction on MFMA i32_16x16x64_i8.  A = time groups x 64-byte input
//           window (P = 2 samples of 22 channels per group), B = per-(filter, parity) weight
//           fragment, C-init = offset + float-magic, requantised in VALU with an exact float
//           reciprocal, packed 4 samples per lane (DPP pair exchange) into LDS rows [16][1184].
//           (reference: layer1.c:53-101, golden_model.py:192-196)
//   layer2  64-tap depthwise temporal xcorr as a banded-Toeplitz GEMM on MFMA i32_32x32x32_i8:
//           A = 32 output shifts x 96-tap band of the filter (rows permuted so that each lane owns
//           two whole pool-8 windows), B = 16-byte slices of the layer-1 row, 3 K-steps.  ReLU
//           (threshold -(off>>3)) + sum-pool 8 + requant in registers.
//           (reference: layer2.c:56-118, xcorr.c:44, golden_model.py:241-247)
//   layer3  16-tap depthwise conv: v_dot4_i32_i8 over byte-aligned windows (alignbyte).
//           (reference: layer3.c:49-79, conv.c:105-146)
//   layer4  16x16 pointwise + ReLU + pool 8 + requant: v_dot4_i32_i8 on the transposed layer-3
//           output (the reference's net_layer3_flip_inplace is free index math here).
//           (reference: layer4.c:51-149)
//   layer5  272 -> 4 linear + bias + requant: one wave, 16 lanes per class, DPP/shuffle reduce.
//           (reference: layer5.c:43-89)
//
// Requantisation y = clip(trunc((acc + off) / fac), -128, 127) is computed as
// clip(int(float(acc + off) * r)) with r chosen on the host (mibminet.hip: choose_reciprocal) and
// verified at every step boundary of the clipped output range, so it is bit-exact to C's integer
// division for every reachable accumulator.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mib {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

constexpr int F2 = 16;          // filters (F1 == F2, D == 1)
constexpr int NWAVES = 4;
constexpr int NTHREADS = 64 * NWAVES;
constexpr int N_OUT = 4;        // classes
constexpr int L2_TAPS = 64;
constexpr int L3_TAPS = 16;
constexpr int ND5_MAX = 96;     // dwords of the flattened layer-4 output (F2*T64 <= 384)
constexpr int FMAGIC_I = 0x4B400000;   // bit pattern of 1.5 * 2^23
constexpr float FMAGIC_F = 12582912.0f;

__host__ __device__ constexpr int align16(int x) { return (x + 15) & ~15; }
__host__ __device__ constexpr int cmax(int a, int b) { return a > b ? a : b; }

// Parameters read into LDS by every workgroup (small, re-read per trial).
struct SmallParams {
  int l3_w[F2][4];        // torch-order taps, 4 per dword (tap j multiplies window byte j)
  int l4_w[F2][4];        // W4[k][f], 4 per dword
  int l4_thr[F2];
  int l4_off[F2];
  float l4_r[F2];
  int l5_w[N_OUT][ND5_MAX];  // flattened [k][v] order, zero padded
  int l5_b[N_OUT];
  float l3_r;
  float l5_r;
  int pad[2];
};

// Operand fragments and requantisation constants, built by the host from the net.h arrays.
struct DevParams {
  v4i l1_wfrag[2][64];      // layer-1 B operand per N-tile and lane
  int l1_cinit[2][16];      // offset + FMAGIC_I per N-tile column
  float l1_r[2][16];        // reciprocal per N-tile column
  v4i l2_afrag[F2][3][64];  // layer-2 A operand (banded weights) per filter, K-step and lane
  int l2_thr[F2];
  int l2_off[F2];
  float l2_r[F2];
  SmallParams sp;
};

template <int C_, int T_>
struct Cfg {
  static constexpr int C = C_, T = T_;
  static constexpr int P = (C <= 32) ? 2 : 1;          // samples per 64-byte L1 window
  static constexpr int GS = P * C;                      // bytes per time group
  static constexpr int NB1 = (T + 16 * P - 1) / (16 * P);  // L1 blocks of 16 groups
  static constexpr int T8 = T / 8, T64 = T8 / 8;
  static constexpr int NB2 = (8 * T8 + 31) / 32;        // L2 column blocks of 32 outputs
  static constexpr int NT2 = (NB2 + 31) / 32;           // L2 N-tiles
  static constexpr int Y1ROW = align16(cmax(32 + 16 * P * NB1, 32 * (NB2 - 1) + 96));
  static constexpr int XTRIAL = align16(T * C);         // batched trial stride (bytes)
  static constexpr int XBYTES = align16(cmax((16 * NB1 - 1) * GS + 64, XTRIAL));
  static constexpr int Q4 = (T8 + 3) / 4;               // L3 tasks per filter (4 outputs each)
  static constexpr int Y2ROW = align16(4 * Q4 + 24);
  static constexpr int Y3ROWS = 4 * Q4;
  static constexpr int ND5 = (F2 * T64 + 3) / 4;
  static constexpr int Y4BYTES = align16(4 * ND5);
  // LDS carve: layer-2..4 outputs alias the input region once layer 1 has consumed it.
  static constexpr int OFF_X = 0;
  static constexpr int OFF_Y2 = 0;
  static constexpr int OFF_Y3 = OFF_Y2 + F2 * Y2ROW;
  static constexpr int OFF_Y4 = OFF_Y3 + Y3ROWS * F2;
  static constexpr int OFF_Y1 = XBYTES;
  static constexpr int OFF_SP = OFF_Y1 + F2 * Y1ROW;
  static constexpr int LDS = align16(OFF_SP + (int)sizeof(SmallParams));
  static_assert(C >= 1 && C <= 64, "C must be <= 64 (one 64-byte MFMA K window)");
  static_assert(GS % 4 == 0, "time-group stride must be dword aligned");
  static_assert(T64 >= 1, "T >= 64");
  static_assert(ND5 <= ND5_MAX, "layer-5 input too long");
  static_assert(OFF_Y4 + Y4BYTES <= XBYTES, "aliased outputs exceed the input region");
};

__device__ __forceinline__ int rq(int v, float r) {
  const int t = (int)((float)v * r);
  return min(max(t, -128), 127);
}

__device__ __forceinline__ unsigned pack4(int a, int b, int c, int d) {
  return (unsigned)(a & 255) | ((unsigned)(b & 255) << 8) | ((unsigned)(c & 255) << 16) |
         ((unsigned)d << 24);
}

// Per-lane register state that lives across the trial loop.
template <class K>
struct Regs {
  v4i wf[K::P];
  int ci[K::P];
  float rr[K::P];
  v4i af[4][3];
  int thr2[4], off2[4];
  float r2[4];
};

template <class K>
__device__ __forceinline__ void setup(const DevParams* __restrict__ prm, int8_t* smem, Regs<K>& R,
                                      int tid, int wave, int lane) {
#pragma unroll
  for (int t = 0; t < K::P; t++) {
    R.wf[t] = prm->l1_wfrag[t][lane];
    R.ci[t] = prm->l1_cinit[t][lane & 15];
    R.rr[t] = prm->l1_r[t][lane & 15];
  }
#pragma unroll
  for (int fi = 0; fi < 4; fi++) {
    const int f = wave * 4 + fi;
#pragma unroll
    for (int s = 0; s < 3; s++) R.af[fi][s] = prm->l2_afrag[f][s][lane];
    R.thr2[fi] = prm->l2_thr[f];
    R.off2[fi] = prm->l2_off[f];
    R.r2[fi] = prm->l2_r[f];
  }
  // small parameters -> LDS
  const v4i* src = (const v4i*)&prm->sp;
  v4i* dst = (v4i*)(smem + K::OFF_SP);
  for (int i = tid; i < (int)(sizeof(SmallParams) / 16); i += NTHREADS) dst[i] = src[i];
  // layer-1 rows: the zero pads (positions [0,32) and beyond the last L1 block) are never
  // rewritten, so clear the whole region once.
  v4i* y1 = (v4i*)(smem + K::OFF_Y1);
  for (int i = tid; i < F2 * K::Y1ROW / 16; i += NTHREADS) y1[i] = (v4i){0, 0, 0, 0};
}

// HBM -> LDS copy of one trial (XTRIAL bytes, 16 B per lane, nontemporal: read once).
template <class K>
__device__ __forceinline__ void stage_x(const int8_t* __restrict__ xg, int8_t* smem, int tid) {
  constexpr int NCH = K::XTRIAL / 16;
  constexpr int IT = (NCH + NTHREADS - 1) / NTHREADS;
  constexpr int BATCH = 8;
  const v4i* src = (const v4i*)xg;
  v4i* dst = (v4i*)(smem + K::OFF_X);
#pragma unroll
  for (int i0 = 0; i0 < IT; i0 += BATCH) {
    v4i tmp[BATCH];
#pragma unroll
    for (int i = 0; i < BATCH; i++) {
      const int c = tid + (i0 + i) * NTHREADS;
      if (i0 + i < IT && c < NCH) tmp[i] = __builtin_nontemporal_load(src + c);
    }
#pragma unroll
    for (int i = 0; i < BATCH; i++) {
      const int c = tid + (i0 + i) * NTHREADS;
      if (i0 + i < IT && c < NCH) dst[c] = tmp[i];
    }
  }
}

// Layer 1: x[T][C] (LDS) -> y1 rows (LDS, position 32 + t).
template <class K>
__device__ __forceinline__ void layer1(const int8_t* smem_x, int8_t* smem_y1, const Regs<K>& R,
                                       int wave, int lane) {
  const int j = lane & 15, g = lane >> 4;
  for (int blk = wave; blk < K::NB1; blk += NWAVES) {
    const int n = blk * 16 + j;  // A row of this lane = time group
    const int8_t* pa = smem_x + n * K::GS + 16 * g;
    v4i a;
    if constexpr (K::GS % 16 == 0) {
      a = *(const v4i*)pa;
    } else {
      const int* q = (const int*)pa;
      a = (v4i){q[0], q[1], q[2], q[3]};
    }
    const bool last = (blk == K::NB1 - 1);
#pragma unroll
    for (int t = 0; t < K::P; t++) {
      v4i acc = {R.ci[t], R.ci[t], R.ci[t], R.ci[t]};
      acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, R.wf[t], acc, 0, 0, 0);
      int y[4];
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const float q = (__int_as_float(acc[r]) - FMAGIC_F) * R.rr[t];
        y[r] = min(max((int)q, -128), 127);
      }
      if constexpr (K::P == 2) {
        // lane column j = (filter 8t + j/2, parity j&1); row 4g + r = time group
        const int p = j & 1, f = 8 * t + (j >> 1);
        const int tb = 32 * blk + 8 * g + p;  // sample of y[r] = tb + 2r
        if (last) {
#pragma unroll
          for (int r = 0; r < 4; r++)
            if (tb + 2 * r >= K::T) y[r] = 0;
        }
        const unsigned d = pack4(y[0], y[1], y[2], y[3]);
        const unsigned e = (unsigned)__builtin_amdgcn_mov_dpp((int)d, 0xB1, 0xF, 0xF, false);
        const unsigned o = __builtin_amdgcn_perm(e, d, p ? 0x03070206u : 0x05010400u);
        *(unsigned*)(smem_y1 + f * K::Y1ROW + 32 + 32 * blk + 8 * g + 4 * p) = o;
      } else {
        const int f = j;
        const int tb = 16 * blk + 4 * g;  // sample of y[r] = tb + r
        if (last) {
#pragma unroll
          for (int r = 0; r < 4; r++)
            if (tb + r >= K::T) y[r] = 0;
        }
        *(unsigned*)(smem_y1 + f * K::Y1ROW + 32 + tb) = pack4(y[0], y[1], y[2], y[3]);
      }
    }
  }
}

// Layer 2: y1 rows -> y2 rows (LDS, position 8 + u, zero pads around).
template <class K>
__device__ __forceinline__ void layer2(const int8_t* smem_y1, int8_t* smem_y2, const Regs<K>& R,
                                       int wave, int lane) {
  const int c = lane & 31, h = lane >> 5;
  constexpr int NPAD = 8 + (K::Y2ROW - 8 - K::T8);
#pragma unroll
  for (int fi = 0; fi < 4; fi++) {
    int8_t* row = smem_y2 + (wave * 4 + fi) * K::Y2ROW;
    for (int i = lane; i < NPAD; i += 64) row[i < 8 ? i : K::T8 + i] = 0;
  }
#pragma unroll
  for (int fi = 0; fi < 4; fi++) {
    const int f = wave * 4 + fi;
    const int8_t* row = smem_y1 + f * K::Y1ROW;
#pragma unroll
    for (int tile = 0; tile < K::NT2; tile++) {
      const int m = tile * 32 + c;
      const int mm = (m < K::NB2) ? m : 0;
      const int8_t* pb = row + 32 * mm + 16 * h;
      v16i acc = {};
#pragma unroll
      for (int s = 0; s < 3; s++) {
        const v4i b = *(const v4i*)(pb + 32 * s);
        acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(R.af[fi][s], b, acc, 0, 0, 0);
      }
      // reg i of this lane = shift 16h + i of block m -> pooled samples u0 (i<8), u0+1 (i>=8)
      int s0 = 0, s1 = 0;
#pragma unroll
      for (int i = 0; i < 8; i++) {
        s0 += max(acc[i], R.thr2[fi]);
        s1 += max(acc[i + 8], R.thr2[fi]);
      }
      const int y0 = rq(s0 + R.off2[fi], R.r2[fi]);
      const int y1 = rq(s1 + R.off2[fi], R.r2[fi]);
      const int u0 = 4 * m + 2 * h;
      int8_t* dst = smem_y2 + f * K::Y2ROW + 8 + u0;
      if (m < K::NB2) {
        if (u0 + 1 < K::T8)
          *(unsigned short*)dst = (unsigned short)((y0 & 255) | ((y1 & 255) << 8));
        else if (u0 < K::T8)
          dst[0] = (int8_t)y0;
      }
    }
  }
}

// Layer 3: y2 rows -> y3t[u][f] (LDS).
template <class K>
__device__ __forceinline__ void layer3(const int8_t* smem_y2, int8_t* smem_y3, const SmallParams* sp,
                                       int tid) {
  for (int idx = tid; idx < F2 * K::Q4; idx += NTHREADS) {
    const int f = idx / K::Q4, q = idx - f * K::Q4, u0 = 4 * q;
    const int* rowd = (const int*)(smem_y2 + f * K::Y2ROW + u0);
    int D[6];
#pragma unroll
    for (int i = 0; i < 6; i++) D[i] = rowd[i];
    const int w0 = sp->l3_w[f][0], w1 = sp->l3_w[f][1], w2 = sp->l3_w[f][2], w3 = sp->l3_w[f][3];
    const float r3 = sp->l3_r;
#pragma unroll
    for (int d = 0; d < 4; d++) {
      // window of output u0+d starts at row position u0 + 1 + d (pad 7 -> stored at +8)
      int win[4];
#pragma unroll
      for (int i = 0; i < 4; i++)
        win[i] = (d == 3) ? D[i + 1] : (int)__builtin_amdgcn_alignbyte(D[i + 1], D[i], 1 + d);
      int acc = __builtin_amdgcn_sdot4(win[0], w0, 0, false);
      acc = __builtin_amdgcn_sdot4(win[1], w1, acc, false);
      acc = __builtin_amdgcn_sdot4(win[2], w2, acc, false);
      acc = __builtin_amdgcn_sdot4(win[3], w3, acc, false);
      const int u = u0 + d;
      if (u < K::T8) smem_y3[u * F2 + f] = (int8_t)rq(acc, r3);
    }
  }
}

// Layer 4: y3t[u][f] -> y4 flat [k][v] (LDS).
template <class K>
__device__ __forceinline__ void layer4(const int8_t* smem_y3, int8_t* smem_y4, const SmallParams* sp,
                                       int tid) {
  for (int idx = tid; idx < F2 * K::T64; idx += NTHREADS) {
    const int k = idx / K::T64, v = idx - k * K::T64;
    const int w0 = sp->l4_w[k][0], w1 = sp->l4_w[k][1], w2 = sp->l4_w[k][2], w3 = sp->l4_w[k][3];
    const int thr = sp->l4_thr[k];
    int sum = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const v4i x = *(const v4i*)(smem_y3 + (8 * v + i) * F2);
      int b = __builtin_amdgcn_sdot4(x[0], w0, 0, false);
      b = __builtin_amdgcn_sdot4(x[1], w1, b, false);
      b = __builtin_amdgcn_sdot4(x[2], w2, b, false);
      b = __builtin_amdgcn_sdot4(x[3], w3, b, false);
      sum += max(b, thr);
    }
    smem_y4[idx] = (int8_t)rq(sum + sp->l4_off[k], sp->l4_r[k]);
  }
  if constexpr (4 * K::ND5 > F2 * K::T64) {
    if (tid < 4 * K::ND5 - F2 * K::T64) smem_y4[F2 * K::T64 + tid] = 0;
  }
}

// Layer 5 (one wave): y4 flat -> 4 logits written to global memory.
template <class K>
__device__ __forceinline__ void layer5(const int8_t* smem_y4, const SmallParams* sp, int lane,
                                       int8_t* __restrict__ outg) {
  const int n = lane >> 4, c = lane & 15;
  const int* xd = (const int*)smem_y4;
  int part = 0;
#pragma unroll
  for (int i = c; i < K::ND5; i += 16) part = __builtin_amdgcn_sdot4(xd[i], sp->l5_w[n][i], part, false);
  part += __shfl_xor(part, 8, 16);
  part += __shfl_xor(part, 4, 16);
  part += __shfl_xor(part, 2, 16);
  part += __shfl_xor(part, 1, 16);
  if (c == 0) outg[n] = (int8_t)rq(part + sp->l5_b[n], sp->l5_r);
}

// Fused forward over a batch (persistent, grid-strided over trials).
template <class K>
__global__ __launch_bounds__(NTHREADS) void k_forward(const DevParams* __restrict__ prm,
                                                       const int8_t* __restrict__ x,
                                                       int8_t* __restrict__ out, int B) {
  __shared__ __attribute__((aligned(16))) int8_t smem[K::LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  Regs<K> R;
  setup<K>(prm, smem, R, tid, wave, lane);
  const SmallParams* sp = (const SmallParams*)(smem + K::OFF_SP);
  for (int b = blockIdx.x; b < B; b += gridDim.x) {
    __syncthreads();  // previous trial's layer-5 reads of the aliased region are done
    stage_x<K>(x + (size_t)b * K::XTRIAL, smem, tid);
    __syncthreads();
    layer1<K>(smem + K::OFF_X, smem + K::OFF_Y1, R, wave, lane);
    __syncthreads();
    layer2<K>(smem + K::OFF_Y1, smem + K::OFF_Y2, R, wave, lane);
    __syncthreads();
    layer3<K>(smem + K::OFF_Y2, smem + K::OFF_Y3, sp, tid);
    __syncthreads();
    layer4<K>(smem + K::OFF_Y3, smem + K::OFF_Y4, sp, tid);
    __syncthreads();
    if (wave == 0) layer5<K>(smem + K::OFF_Y4, sp, lane, out + (size_t)b * N_OUT);
  }
}

// Single-trial, single-layer kernel for the reference's per-layer entry points (debug/parity):
// reads the layer input in its reference layout, runs the same device code as k_forward and
// writes the layer output in its reference layout (pads zero).
template <class K>
__global__ __launch_bounds__(NTHREADS) void k_layer(const DevParams* __restrict__ prm,
                                                     const int8_t* __restrict__ in,
                                                     int8_t* __restrict__ out, int stage) {
  __shared__ __attribute__((aligned(16))) int8_t smem[K::LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  Regs<K> R;
  setup<K>(prm, smem, R, tid, wave, lane);
  const SmallParams* sp = (const SmallParams*)(smem + K::OFF_SP);
  constexpr int T_AL = (K::T + 3) & ~3, T8_AL = (K::T8 + 3) & ~3, T64_AL = (K::T64 + 3) & ~3;
  int8_t* y1 = smem + K::OFF_Y1;
  int8_t* y2 = smem + K::OFF_Y2;
  int8_t* y3 = smem + K::OFF_Y3;
  int8_t* y4 = smem + K::OFF_Y4;
  __syncthreads();
  if (stage == 1) {  // [T][C] packed -> [F1][T_ALIGN]
    stage_x<K>(in, smem, tid);
    __syncthreads();
    layer1<K>(smem + K::OFF_X, y1, R, wave, lane);
    __syncthreads();
    for (int i = tid; i < F2 * T_AL; i += NTHREADS) {
      const int f = i / T_AL, t = i - f * T_AL;
      out[i] = t < K::T ? y1[f * K::Y1ROW + 32 + t] : 0;
    }
  } else if (stage == 2) {  // [F1][T_ALIGN] -> [F2][T8_ALIGN]
    for (int i = tid; i < F2 * K::T; i += NTHREADS) {
      const int f = i / K::T, t = i - f * K::T;
      y1[f * K::Y1ROW + 32 + t] = in[f * T_AL + t];
    }
    __syncthreads();
    layer2<K>(y1, y2, R, wave, lane);
    __syncthreads();
    for (int i = tid; i < F2 * T8_AL; i += NTHREADS) {
      const int f = i / T8_AL, u = i - f * T8_AL;
      out[i] = u < K::T8 ? y2[f * K::Y2ROW + 8 + u] : 0;
    }
  } else if (stage == 3) {  // [F2][T8_ALIGN] -> [F2][T8_ALIGN]
    for (int i = tid; i < F2 * K::Y2ROW; i += NTHREADS) {
      const int f = i / K::Y2ROW, pos = i - f * K::Y2ROW, u = pos - 8;
      y2[i] = (u >= 0 && u < K::T8) ? in[f * T8_AL + u] : 0;
    }
    __syncthreads();
    layer3<K>(y2, y3, sp, tid);
    __syncthreads();
    for (int i = tid; i < F2 * T8_AL; i += NTHREADS) {
      const int f = i / T8_AL, u = i - f * T8_AL;
      out[i] = u < K::T8 ? y3[u * F2 + f] : 0;
    }
  } else if (stage == 4) {  // [T8][F2] -> [F2][T64_ALIGN]
    for (int i = tid; i < K::T8 * F2; i += NTHREADS) y3[i] = in[i];
    __syncthreads();
    layer4<K>(y3, y4, sp, tid);
    __syncthreads();
    for (int i = tid; i < F2 * T64_AL; i += NTHREADS) {
      const int k = i / T64_AL, v = i - k * T64_AL;
      out[i] = v < K::T64 ? y4[k * K::T64 + v] : 0;
    }
  } else if (stage == 5) {  // [F2][T64_ALIGN] -> [N]
    for (int i = tid; i < 4 * K::ND5; i += NTHREADS) {
      const int k = i / K::T64, v = i - k * K::T64;
      y4[i] = (k < F2) ? in[k * T64_AL + v] : 0;
    }
    __syncthreads();
    if (wave == 0) layer5<K>(y4, sp, lane, out);
  } else if (stage == 6) {  // flip [F2][T8_ALIGN] -> [T8][F2] (net_layer3_flip_inplace)
    for (int i = tid; i < F2 * T8_AL; i += NTHREADS) smem[i] = in[i];
    __syncthreads();
    for (int i = tid; i < F2 * T8_AL; i += NTHREADS) {
      const int u = i / F2, f = i - u * F2;
      out[i] = u < K::T8 ? smem[f * T8_AL + u] : 0;
    }
  }
}

}  // namespace mib
