// forward_gen.hpp — gfx950 fused forward for every network geometry the reference's generator
// emits (edge-eegnet_wolf/data/gen_net_header.py:78-89): C <= 64 channels (channel-selected
// MI-BMInet inputs, QuantLab/.../PhysionetMMMI/edgeEEGNet/preprocess.py:86-87), 64 <= T <= 4096
// samples (every time window of the loaders: 480 and 960 in get_data.py:156-159, 1125 for
// BCI-IV-2a), 1 <= N <= 16 classes (the 2- and 3-class PhysioNet nets, get_data.py:73-82), with
// F1 = F2 = 16 and D = 1 as layer2.c:246 fixes them.
//
// The dimensions are kernel-uniform run-time values (GenParams), so one compiled kernel per input
// layout serves every geometry; the three geometries of the reference's own configurations keep
// their compile-time specialisations (forward_wg.hpp), which this file does not touch.
//
// One workgroup of NW = 8 wave64s owns one trial at a time (persistent, grid-strided), with two
// barriers per trial: waves 0-6 run layer 1 while wave 7 runs layers 4-5 of the previous trial
// and then the trial's last K7 layer-1 blocks.  Int8 trials arrive in LDS a trial ahead by
// LDS-DMA.  Every intermediate stays in LDS:
//   layer1  MFMA i32_16x16x64_i8: A = 16 samples x 64 channel slots, B = the 16 filters' weights
//           (zero past C), C-init = the offset.  Time-major trials: a lane's 16 bytes of sample
//           t are t C + 16 c .. +15 of the trial (chunk c = l1_chunk(g, C)), read as five aligned
//           dwords and realigned by v_alignbyte (one ds_read_b128 when every fragment is
//           16-byte aligned); channel-major trials (int8 or float32, quantised here) go through
//           the same LDS transpose as the specialised kernels (wg::stage_block, ds_read_b64_tr_b8).
//                                                               (reference: layer1.c:53-101)
//   layer2  the 64-tap depthwise xcorr as a banded-Toeplitz GEMM on MFMA i32_32x32x32_i8 (A = 32
//           output shifts x 96-tap band, rows permuted so that a lane holds two whole pool-8
//           windows; B = 16-byte slices of the layer-1 row), ReLU-pool and requant per lane.
//                                                               (reference: layer2.c:56-118, 139-210)
//   layer3  16-tap depthwise conv on MFMA i32_16x16x64_i8 with a block-diagonal K (the wave's two
//           filters), written transposed [u][f] (the reference's flip is index math).
//                                                               (reference: layer3.c:49-79)
//   layer4  16x16 pointwise on MFMA i32_32x32x32_i8 with a block-diagonal B (two 32-sample
//           blocks), ReLU-pool and requant per lane.               (reference: layer4.c:51-149)
//   layer5  N-class linear layer: four classes per pass, 16 lanes each, v_dot4 + a DPP prefix.
//                                                               (reference: layer5.c:43-89)
// Requantisation as in the compiled kernels: where the host proves the float form exact on every
// reachable value (mibminet.hip: choose_reciprocal, choose_floor_form) the XR = false build runs
// it; any requant without a proven float form sends the set to the XR = true build, exact
// division (xdiv, forward_common.hpp) at layers 1-4.  Layer 5 always divides exactly (its
// sums pass 2^24 at T = 4096).  CB: balanced clipping ([-127, 127], golden model clip_balanced).
#pragma once
#include "forward_wg.hpp"

namespace mib {
namespace gen {

constexpr int NW = 8;                  // waves per workgroup
constexpr int NT = 64 * NW;
constexpr int TMAX = 4096;             // samples per trial (16 s at 250 Hz)
constexpr int NMAX = 16;               // classes
constexpr int T64A_MAX = TMAX / 64;
constexpr int L5W = F2 * T64A_MAX;     // bytes of one class's layer-5 weight row

enum Layout { TM = 0, CT = 1, F32 = 2 };

// Per-filter constants read by layers 3 and 4 of every wave: copied into LDS once per workgroup.
struct SmallG {
  v4i l3_a[NW][64];       // layer 3: wave w's A fragment per lane (filters 2w, 2w + 1; layer3)
  v4i l4_b[64];           // layer 4: the block-diagonal B fragment per lane (layer4)
  int l4_thr[F2];         // REORDER_BN: -(offset >> 3); plain: unused
  int l4_off[F2];         // REORDER_BN: offset; plain: offset >> 3
  unsigned l4_m[F2];      // XR: xdiv magic of factor (plain: factor >> 3)
  int l4_xs[F2];
  float l4_r[F2];         // float form: reciprocal (REORDER_BN) / floor-form r (plain)
  float l4_c[F2];         // plain floor form: c
  int l4_ci[F2];          // plain floor form: magic bits + offset >> 3
  int zero16[4];          // 16 zero bytes (layer 3's off-diagonal K halves)
};
static_assert(sizeof(SmallG) % 16 == 0, "SmallG is copied in 16-byte pieces");

// Device parameter image of the general path (built on the host: mibminet.hip, build_genparams).
struct GenParams {
  int C, T, N, T8;
  int T64, T64A, NB1, MT;       // NB1: layer-1 blocks of 16 samples; MT: full layer-2 tiles of 1024 outputs
  int NTT;                      // layer-2 tail tiles of 256 outputs per filter past the MT full tiles
  int K7;                       // layer-1 blocks of the last wave (its layers 4-5 first), the trial's last ones
  int K7T1;                     // the same for time-major trials at one workgroup per CU
  int pad2;
  int rb, lo, xstride, xr;      // REORDER_BN branches; lower clip bound; time-major trial stride;
                                // exact division (no proven float form for some requant)
  unsigned l3_m;
  int l3_xs;
  unsigned l5_m;
  int l5_xs;
  float l3_r, l3_c;             // float form of layer 3: magic C-init, fma(acc bits, r, c)
  int pad1[2];
  v4i l1_b[64];                 // layer-1 B operand, time-major: lane (filter lane & 15, g) = W1[f] chunk
                                // l1_chunk(g, C) (zero in K groups 1 and 3 when C <= 32)
  v4i l1_bn[64];                // the same in natural order (channel-major, float32): chunk g
  int l1_off[F2];               // XR: offset (the MFMA C-init); float: offset + FMAGIC_I
  unsigned l1_m[F2];            // XR: xdiv magic
  int l1_xs[F2];
  float l1_r[F2], l1_c[F2];     // float form: fma(acc bits, r, c) = RN((dot + off) r)
  int l2_thr[F2];               // REORDER_BN: -(offset >> 3); plain float form: magic bits + offset >> 3
  int l2_off[F2];               // REORDER_BN: offset; plain: offset >> 3
  unsigned l2_m[F2];            // XR: xdiv magic of factor (plain: factor >> 3)
  int l2_xs[F2];
  float l2_r[F2], l2_c[F2];     // float form: reciprocal (REORDER_BN); floor-form r, c (plain)
  int l5_b[NMAX];
  SmallG sg;
  v4i l2_a[F2][3][64];          // layer-2 A operand (banded weights) per filter, K-step and lane
  v4i l2t_a[F2][2][64];         // layer-2 tail A operand (16 shifts x 128 K-slots) per filter, K-step, lane
  int8_t l5_w[NMAX][L5W];       // [n][k T64A + v], zero pads
};

constexpr int LDS_MAX = 160 * 1024;    // LDS per CU
constexpr int LDS_2WG = LDS_MAX / 2;    // two workgroups per CU at most this much each

// bytes of one layer-5 weight row in LDS: F2 T64A rounded up to 256 (64 dwords: the four reads
// per pass of layer5's sixteen lanes per class need no bound check; the pads are zero)
__host__ __device__ constexpr int w5_row(int T64A) { return (F2 * T64A + 255) / 256 * 256; }

// LDS carve of one workgroup (host and device compute it alike).  Int8 trials (time-major and
// channel-major) are staged whole in LDS ("raw", the trial a grid stride ahead arriving by LDS-DMA
// during layers 2-5) when that fits in LDS_MAX; otherwise, and for float32 trials, layer 1 loads
// its fragments from memory.
struct Carve {
  int y1s, y2s;                 // row strides of y1 (positions t + 32) and y2 (positions u + 8)
  int y2, y3, y4, sg, w5, stg, raw, chunks, bytes;  // raw < 0: not staged; chunks: 1 KB DMA pieces
};
__host__ __device__ inline Carve carve_of(int C, int T, int N, int T8, int T64A, int NB1, int MT, int NTT,
                                          int layout) {
  Carve c;
  // layer 2 reads positions < 1024 MT + 64 (full tiles) and < 1024 MT + 256 NTT + 112 (tail);
  // layer 1 writes positions < 32 + 16 NB1.  Stride = 16 (mod 256): the sixteen filters' layer-1
  // dword stores of a block fall on distinct banks
  const int need = cmax(cmax(32 + 16 * NB1, 1024 * MT + 64), NTT ? 1024 * MT + 256 * NTT + 112 : 0);
  c.y1s = (need + 239) / 256 * 256 + 16;
  c.y2s = align16(T8 + 32);     // 8 pad bytes, T8 outputs, zeros under layer 3's 20-byte windows
  c.y2 = 16 * c.y1s;
  c.y3 = c.y2 + 16 * c.y2s;
  c.y4 = c.y3 + align16(16 * (T8 + 3));       // rows < T8 (layer 3), zeros past them
  c.sg = c.y4 + w5_row(T64A);                 // y4 padded with zeros to whole 256-byte rows
  c.w5 = c.sg + (int)sizeof(SmallG);          // layer-5 weights [N][w5_row], then the N biases
  c.stg = c.w5 + N * w5_row(T64A) + align16(4 * N);  // channel-major transpose staging, 1 KB per wave
  // layout: 0 time-major, 1 channel-major, 2 float32 (gen::Layout); 3: the single-layer kernel
  const int base = c.stg + ((layout == 1 || layout == 2) ? NW * 1024 : 0);
  // the trial's bytes from its dword-aligned base (delta <= 3), in 1 KB pieces, plus the slack the
  // 20-byte fragment windows read past them (time-major: 16 NB1 samples of C bytes; channel-major:
  // row C - 1 read 16 NB1 samples in)
  const int bytes = C * T + 3;
  c.chunks = (bytes + 1023) / 1024;
  const int region = align16(cmax(cmax(1024 * c.chunks, 16 * NB1 * C + 96), C * T + 16 * NB1 + 96));
  c.raw = ((layout == 0 || layout == 1) && base + region <= LDS_MAX) ? base : -1;
  c.bytes = base + (c.raw >= 0 ? region : 0);
  return c;
}

__device__ __forceinline__ int clampq(int v, int lo) { return min(max(v, lo), 127); }
__device__ __forceinline__ unsigned pack4(int a, int b, int c, int d) {
  return (unsigned)(a & 255) | ((unsigned)(b & 255) << 8) | ((unsigned)(c & 255) << 16) | ((unsigned)d << 24);
}

typedef unsigned v4u __attribute__((ext_vector_type(4)));

// 16 bytes at byte offset o of the view, from five aligned dwords: each dword lies wholly inside
// or wholly outside num_records (which is a multiple of 4), so the range check zeroes no byte the
// trial holds.  v_alignbyte_b32(hi, lo, s) = bytes s .. s + 3 of hi:lo.
__device__ __forceinline__ v4i load16u(wg::Rsrc r, int o) {
  const int o4 = o & ~3;
  const unsigned s = (unsigned)(o & 3);
  const v4u a = __builtin_amdgcn_raw_buffer_load_b128(r, o4, 0, 0);
  const unsigned e = __builtin_amdgcn_raw_buffer_load_b32(r, o4 + 16, 0, 0);
  return (v4i){(int)__builtin_amdgcn_alignbyte(a[1], a[0], s), (int)__builtin_amdgcn_alignbyte(a[2], a[1], s),
               (int)__builtin_amdgcn_alignbyte(a[3], a[2], s), (int)__builtin_amdgcn_alignbyte(e, a[3], s)};
}

// The view of trial b: base = the trial's first byte rounded down to a dword, delta = the rest,
// num_records = the trial's bytes from base rounded up to a dword (a dword holding a trial byte is
// inside the page of that byte, so the rounding reads no unmapped memory).
struct View {
  wg::Rsrc r;
  int delta;
};
template <int L>
__device__ __forceinline__ View trial_view(const int8_t* x, long long b, int C, int T, int xstride) {
  const long long ct = (long long)C * T;
  const int8_t* p = L == TM ? x + b * xstride : L == CT ? x + b * ct : x + 4 * b * ct;
  const int delta = (int)((size_t)p & 3);
  const int bytes = (int)((L == F32 ? 4 : 1) * ct);
  View v;
  v.r = __builtin_amdgcn_make_buffer_rsrc((void*)(p - delta), (short)0, (delta + bytes + 3) & ~3, 0x00020000);
  v.delta = delta;
  return v;
}

// Time-major K groups: with C <= 32 channels 0..15 go to K group 0 and 16..31 to K group 2, and
// groups 1 and 3 (zero weights) re-read the same 16 bytes.  A ds_read_b32 serves lanes 0-31 and
// 32-63 in separate cycles, so each cycle then reads only 16 distinct windows, whose dwords
// (5.5 j apart at C = 22) fall on distinct banks; groups 0 and 1 together, 16 bytes apart, met
// 2-way conflicts (profiles/r06_lds_conflicts.txt).
__host__ __device__ inline int l1_chunk(int g, int C) { return C <= 32 ? g >> 1 : g; }

// The A fragment of layer-1 block blk (samples 16 blk .. +15), before staging: time-major, lane
// (j, g) holds channels 16 c .. +15 (c = l1_chunk(g, C)) of sample 16 blk + j; channel-major, lane c holds samples
// 16 blk .. +15 of channel c.  K-slots past C meet zero weights, so what those lanes read does not
// matter: the loads are unconditional (no per-lane branch between one block's loads and the next
// block's), and channel-major rows past C re-read row C - 1.
template <int L>
__device__ __forceinline__ v4i l1_fetch(const View& v, int blk, int C, int T, int lane, float qs, float qy) {
  if constexpr (L == TM) {
    const int j = lane & 15, g = lane >> 4;
    return load16u(v.r, v.delta + (16 * blk + j) * C + 16 * l1_chunk(g, C));
  } else if constexpr (L == CT) {
    return load16u(v.r, v.delta + min(lane, C - 1) * T + 16 * blk);
  } else {
    const int c = min(lane, C - 1);
    v4i w;
#pragma unroll
    for (int m = 0; m < 4; m++) {
      const v4u f = __builtin_amdgcn_raw_buffer_load_b128(v.r, 4 * (c * T + 16 * blk) + 16 * m, 0, 0);
      // the reference's input quantisation (gen_input_header.py:66-76), wg::quantize1_f; the
      // truncating convert lies in [-127, 127]
      int q[4];
#pragma unroll
      for (int i = 0; i < 4; i++) q[i] = (int)wg::quantize1_f(__uint_as_float(f[i]), qs, qy);
      w[m] = (int)pack4(q[0], q[1], q[2], q[3]);
    }
    return w;
  }
}

struct TrK {
  static constexpr bool TR16 = false;  // wg::stage_block's P == 1 transpose (ds_read_b64_tr_b8)
};

// 16 bytes at p + s of the staged trial (p 4-byte aligned, s < 4): five aligned dwords, realigned
// by v_alignbyte.  Not a ds_read_b128 at p: off its 16-byte alignment that one is replayed at 64
// LDS cycles per wave-instruction (MI355X_MICROARCH.md, LDS), which made layer 1 the LDS array's
// largest user (general kernels)
__device__ __forceinline__ v4i lds16u(const int8_t* p, unsigned s) {
  const unsigned* q = (const unsigned*)p;
  unsigned d[5];
#pragma unroll
  for (int i = 0; i < 5; i++) d[i] = q[i];
  return (v4i){(int)__builtin_amdgcn_alignbyte(d[1], d[0], s), (int)__builtin_amdgcn_alignbyte(d[2], d[1], s),
               (int)__builtin_amdgcn_alignbyte(d[3], d[2], s), (int)__builtin_amdgcn_alignbyte(d[4], d[3], s)};
}

// A lane's layer-1 fragments in the staged trial: block blk's 16 bytes start at lb + step blk, with
// lb = delta + j C + 16 l1_chunk(g, C) (time-major) or delta + c T (channel-major, c = min(lane,
// C - 1)) and
// step = 16 C or 16.  step is a multiple of 4, so the byte shift lb & 3 is the same for every block
// and each block costs one address add.  AL: every fragment 16-byte aligned (delta = 0 and the row
// length a multiple of 16), one ds_read_b128 each; otherwise lds16u (at C = 64 its five dwords per
// lane would also meet 8-way bank conflicts).
struct L1Src {
  const int8_t* p;  // sraw + (lb & ~3)
  int step;
  unsigned sh;      // lb & 3
};
template <int L>
__device__ __forceinline__ L1Src l1_src(const int8_t* raw, int delta, int C, int T, int lane) {
  const int lb = L == TM ? delta + (lane & 15) * C + 16 * l1_chunk(lane >> 4, C) : delta + min(lane, C - 1) * T;
  return L1Src{raw + (lb & ~3), L == TM ? 16 * C : 16, (unsigned)(lb & 3)};
}
template <bool AL>
__device__ __forceinline__ v4i l1_fetch_lds(const L1Src& q, int blk) {
  const int8_t* p = q.p + q.step * blk;
  if constexpr (AL) return *(const v4i*)p;
  else return lds16u(p, q.sh);
}

// LDS-DMA of trial view v into the raw area: 1 KB pieces i = wave, wave + NW, ... (lane L's 16
// bytes land at byte 16 L of its piece); pieces past num_records land as zeros.  wg::dma_b128 is
// inline asm, so no barrier waits for it: the wave waits vmcnt(0) before barrier B (k_forward).
__device__ __forceinline__ void stage_trial(const View& v, int8_t* raw, int chunks, int wave, int lane) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of the area have returned
  const unsigned base = wg::lds_addr(raw);
  for (int i = wave; i < chunks; i += NW) wg::dma_b128(v.r, 1024 * i + 16 * lane, 0, base + 1024 * i);
}

// Layer 1: the blocks first, first + nw, ... < end -> y1 rows (position 32 + t).  Loads of
// U blocks are issued before their MFMAs.
// Requant of one layer-1 output (acc = dot + offset, or its float-magic form): exact division
// (XR) or fma(acc bits, r, c) = RN((dot + off) r), truncated (the host proves it equals C's
// division on every reachable value).  Both clip to [LO, 127] (the upper bound and -128 by the
// saturating pack).
template <bool XR, bool CB>
__device__ __forceinline__ int rq1(int acc, unsigned m, int xs, float r, float c) {
  int y = XR ? xdiv(acc, m, xs) : (int)__builtin_fmaf(__int_as_float(acc), r, c);
  if (XR) y = min(y, 127);
  return CB ? max(y, -127) : XR ? max(y, -128) : y;
}
// four outputs in [-128, 127] (or to be saturated there) -> bytes 0..3
typedef unsigned short v2us __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned sat4(int a, int b, int c, int d) {
  // two saturating pairs joined as a 2 x 16-bit vector: one v_perm_b32, no masking
  const v2us t = {__builtin_amdgcn_ashr_pk_i8_i32(a, b, 0), __builtin_amdgcn_ashr_pk_i8_i32(c, d, 0)};
  return __builtin_bit_cast(unsigned, t);
}

struct L1C {  // a lane's layer-1 constants (filter lane & 15)
  v4i wf;
  int off, xs;
  unsigned m;
  float r, c;
};

// ST: the trial is staged in LDS (sraw).  The U blocks' loads are all issued before the first MFMA
// (slots past NB1 re-read the last block; their results are not stored).  U4: four blocks per
// group, else two (float32: always two).
template <int L, bool ST, bool XR, bool CB, bool U4 = true>
__device__ __forceinline__ void layer1(const GenParams* __restrict__ gp, const View& v, const int8_t* sraw, int8_t* y1,
                                       int y1s, int8_t* stg, const L1C& k, int first, int nw, int end, int lane,
                                       float qs, float qy) {
  const int C = gp->C, T = gp->T, NB1 = gp->NB1;
  const int j = lane & 15, g = lane >> 4;
  constexpr int U = L == F32 || !U4 ? 2 : 4;
  // staged fragments all 16-byte aligned (wave-uniform: a scalar branch per group of U blocks)
  const bool al = ST && v.delta == 0 && ((L == TM ? C : T) & 15) == 0;
  const L1Src src = l1_src<L>(sraw, v.delta, C, T, lane);
  for (int b0 = first; b0 < end; b0 += U * nw) {  // the blocks first, first + nw, ... < end
    v4i raw[U];
    if (al) {
#pragma unroll
      for (int u = 0; u < U; u++) raw[u] = l1_fetch_lds<true>(src, min(b0 + u * nw, end - 1));
    } else {
#pragma unroll
      for (int u = 0; u < U; u++) {
        const int blk = min(b0 + u * nw, end - 1);
        if constexpr (ST) raw[u] = l1_fetch_lds<false>(src, blk);
        else raw[u] = l1_fetch<L>(v, blk, C, T, lane, qs, qy);
      }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int blk = b0 + u * nw;
      if (blk < end) {  // wave-uniform
        const v4i a = L == TM ? raw[u] : wg::stage_block<TrK>(raw[u], stg, lane);
        const v4i acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, k.wf, (v4i){k.off, k.off, k.off, k.off}, 0, 0, 0);
        // lane column j = filter j, rows 4 g + r = samples 16 blk + 4 g + r
        const int t0 = 16 * blk + 4 * g;
        int y[4];
#pragma unroll
        for (int r = 0; r < 4; r++) y[r] = rq1<XR, CB>(acc[r], k.m, k.xs, k.r, k.c);
        if (blk == NB1 - 1) {  // the trial's last block: samples >= T are zero (the xcorr's pad)
#pragma unroll
          for (int r = 0; r < 4; r++) y[r] = t0 + r < T ? y[r] : 0;
        }
        *(unsigned*)(y1 + j * y1s + 32 + t0) = sat4(y[0], y[1], y[2], y[3]);
      }
    }
  }
}

// Layer 2 (layer2.c:56-118 REORDER_BN, :139-210 plain): the wave's filters 2 wave + fi.  Lane
// (n, h) of tile mt holds conv outputs 1024 mt + 32 n + 16 h + r (r < 16), i.e. the pool windows
// u0 = 128 mt + 4 n + 2 h and u0 + 1.
struct L2C {  // a wave's layer-2 constants (filters 2 wave, 2 wave + 1)
  v4i af[2][3];
  v4i at[2][2];   // tail bands
  int thr[2], off[2], xs[2];
  unsigned m[2];
  float r[2], c[2];
};

// floor form of one plain-branch element (mibminet.hip, choose_floor_form): acc holds the bits of
// float(M + x) (MFMA C-init M + offset), and bits(fmed3(fma(acc, r, c), K, K + emax)) - bits(K) =
// clamp(floor(x / fac), 0, emax) = the element after its clip and ReLU
template <int EMAX>
__device__ __forceinline__ int floor_el(int acc, float r, float c) {
  const float g = __builtin_fmaf(__int_as_float(acc), r, c);
  return __float_as_int(__builtin_amdgcn_fmed3f(g, FMAGIC_F, FMAGIC_F + (float)EMAX)) - FMAGIC_I;
}

template <bool RB, bool XR, bool CB>
__device__ __forceinline__ void layer2(const GenParams* __restrict__ gp, const int8_t* y1, int y1s, int8_t* y2, int y2s,
                                       const L2C& k, int wave, int lane) {
  constexpr int LO = CB ? -127 : -128;
  const int T8 = gp->T8, MT = gp->MT;
  constexpr bool rb = RB;  // the blob's REORDER_BN flag (gp->rb), an instantiation
  const int n = lane & 31, h = lane >> 5;
  for (int mt = 0; mt < MT; mt++) {
    // both filters' B slices first: the six LDS reads overlap instead of each MFMA waiting on one
    v4i bs[2][3];
#pragma unroll
    for (int fi = 0; fi < 2; fi++)
#pragma unroll
      for (int s = 0; s < 3; s++)
        bs[fi][s] = *(const v4i*)(y1 + (2 * wave + fi) * y1s + 1024 * mt + 32 * n + 16 * h + 32 * s);
#pragma unroll
    for (int fi = 0; fi < 2; fi++) {
      const int f = 2 * wave + fi;
      // plain float form: the chain starts from the floor form's magic (+ offset >> 3)
      const int ci = (!rb && !XR) ? k.thr[fi] : 0;
      v16i acc;
#pragma unroll
      for (int i = 0; i < 16; i++) acc[i] = ci;
#pragma unroll
      for (int s = 0; s < 3; s++) acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(k.af[fi][s], bs[fi][s], acc, 0, 0, 0);
      int q[2];
#pragma unroll
      for (int w = 0; w < 2; w++) {
        int sum = 0;
        if constexpr (rb) {
#pragma unroll
          for (int i = 0; i < 8; i++) sum += max(acc[8 * w + i], k.thr[fi]);
          sum += k.off[fi];
          q[w] = XR ? clampq(xdiv(sum, k.m[fi], k.xs[fi]), LO) : clampq((int)((float)sum * k.r[fi]), LO);
        } else {
          // func_xcorr_scale per element (clip to int8), ReLU, sum of 8 >> 3
#pragma unroll
          for (int i = 0; i < 8; i++)
            sum += XR ? min(max(xdiv(acc[8 * w + i] + k.off[fi], k.m[fi], k.xs[fi]), 0), 127)
                      : floor_el<127>(acc[8 * w + i], k.r[fi], k.c[fi]);
          q[w] = sum >> 3;  // in [0, 127]
        }
      }
      const int u0 = 128 * mt + 4 * n + 2 * h;
      int8_t* dst = y2 + f * y2s + 8 + u0;
      if (u0 + 1 < T8) *(unsigned short*)dst = (unsigned short)((q[0] & 255) | ((q[1] & 255) << 8));
      else if (u0 < T8) *dst = (int8_t)q[0];
    }
  }
  // Tail: the column blocks past the full tiles, when at most 16 per filter are left (gp->NTT
  // tiles): MFMA i32_16x16x64_i8, 16 output shifts x 16 columns of 16 outputs, K = the 128
  // window positions from the column's first output (the band reaches 79 of them).  Lane (col, g)
  // holds shifts 4 g .. 4 g + 3 of its column: half a pool window, whose other half sits in row
  // g ^ 1 and arrives by v_permlane16_swap.
  const int NTT = gp->NTT;
  const int col = lane & 15, g = lane >> 4;
  for (int tt = 0; tt < NTT; tt++) {
    const int p0 = 1024 * MT + 256 * tt + 16 * col;  // the column's first output (row position p0 + 32 - 32)
    v4i bt[2][2];
#pragma unroll
    for (int fi = 0; fi < 2; fi++)
#pragma unroll
      for (int s = 0; s < 2; s++) bt[fi][s] = *(const v4i*)(y1 + (2 * wave + fi) * y1s + p0 + 64 * s + 16 * g);
#pragma unroll
    for (int fi = 0; fi < 2; fi++) {
      const int ci = (!rb && !XR) ? k.thr[fi] : 0;
      v4i acc = (v4i){ci, ci, ci, ci};
#pragma unroll
      for (int s = 0; s < 2; s++) acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(k.at[fi][s], bt[fi][s], acc, 0, 0, 0);
      int part = 0;
      if constexpr (rb) {
#pragma unroll
        for (int i = 0; i < 4; i++) part += max(acc[i], k.thr[fi]);
      } else {
#pragma unroll
        for (int i = 0; i < 4; i++)
          part += XR ? min(max(xdiv(acc[i] + k.off[fi], k.m[fi], k.xs[fi]), 0), 127) : floor_el<127>(acc[i], k.r[fi], k.c[fi]);
      }
      const auto sw = __builtin_amdgcn_permlane16_swap((unsigned)part, (unsigned)part, false, false);
      const int tot = (int)(sw[0] + sw[1]);  // the whole window (rows g and g ^ 1 hold the same)
      int q;
      if constexpr (rb) q = XR ? clampq(xdiv(tot + k.off[fi], k.m[fi], k.xs[fi]), LO) : clampq((int)((float)(tot + k.off[fi]) * k.r[fi]), LO);
      else q = tot >> 3;
      const int u = (p0 >> 3) + (g >> 1);
      if (!(g & 1) && u < T8) y2[(2 * wave + fi) * y2s + 8 + u] = (int8_t)q;
    }
  }
}

// Layer 3 (layer3.c:49-79, conv.c:105): output u of filter f = sum_j y2p[u + j] W3t[j], y2p[i] at
// row byte i + 1, so a block of 16 outputs from u0 reads row bytes u0 + 1 .. u0 + 31.  One MFMA
// i32_16x16x64_i8 per 128 outputs of the wave's two filters, with a block-diagonal K as in the
// compiled kernels (forward_wg.hpp, layer3): columns 0..7 are filter 2w's blocks j = 0..7,
// columns 8..15 filter 2w+1's; K-slots 0..31 carry filter 2w's 32-byte windows and band
// (A[r][k] = W3t[k - r - 1], SmallG::l3_a), slots 32..63 filter 2w+1's; a lane whose K half
// belongs to the other filter reads 16 zero bytes.  D lane (col, g) holds outputs
// u0 + 4 g .. u0 + 4 g + 3 of its column's block, written to y3t[u][f] (net_layer3_flip_inplace as
// index math); windows past T8 read zero pads or other rows, and their outputs are not stored.
template <bool XR, bool CB>
__device__ __forceinline__ void layer3(const GenParams* __restrict__ gp, const SmallG* sg, const int8_t* y2, int y2s,
                                       int8_t* y3, int wave, int lane) {
  constexpr int LO = CB ? -127 : -128;
  const int T8 = gp->T8;
  const unsigned m = gp->l3_m;
  const int xs = gp->l3_xs;
  const float r = gp->l3_r, c = gp->l3_c;
  const int col = lane & 15, g = lane >> 4, fi = col >> 3, j = col & 7;
  const int f = 2 * wave + fi;
  asm volatile("" ::: "memory");  // the A fragment is read here, not kept in registers across the trial loop
  const v4i a = sg->l3_a[wave][lane];
  // this lane's 16 window bytes: its column's filter row when the K half is that filter's, else zeros
  const int8_t* src = (g >> 1) == fi ? y2 + f * y2s + 16 * j + 16 * (g & 1) : (const int8_t*)sg->zero16;
  const int step = (g >> 1) == fi ? 128 : 0;
  const int ci = XR ? 0 : FMAGIC_I;  // float form: |conv| < 2^22 rides on the magic (exact)
  for (int t = 0; 128 * t < T8; t++) {
    const v4i b = *(const v4i*)(src + step * t);
    const v4i acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, (v4i){ci, ci, ci, ci}, 0, 0, 0);
    const int u0 = 128 * t + 16 * j + 4 * g;
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int y = XR ? xdiv(acc[q], m, xs) : (int)__builtin_fmaf(__int_as_float(acc[q]), r, c);
      if (u0 + q < T8) y3[16 * (u0 + q) + f] = (int8_t)clampq(y, LO);
    }
  }
}

// Layer 4 (layer4.c:51-149, FLIP_LAYERS): b[k][u] = W4[k] . y3t[u], pooled over u = 8 v .. 8 v + 7;
// REORDER_BN: sum max(b, thr) + off, / fac; plain: sum max(tdiv(b + off >> 3, fac >> 3), 0) >> 3.
// One MFMA i32_32x32x32_i8 per part p of 64 samples, as the compiled kernels' layer 4: A row i of
// lane (i, h) = y3t[64 p + 32 h + n(i)] in K-slots 16 h .. 16 h + 15 (n(i) = 16 ((i >> 2) & 1) +
// 4 (i >> 3) + (i & 3)); B block-diagonal (SmallG::l4_b: column c < 16 = channel c on slots 0..15,
// column c >= 16 = channel c - 16 on slots 16..31).  Lane (c, h) register r then holds
// b[c & 15][64 p + 32 (c >> 4) + 16 h + r]: the two pool windows v = 8 p + 4 (c >> 4) + 2 h + {0, 1}.
// Parts p0, p0 + pstep, ...; samples past T8 read other LDS bytes and feed only windows v >= T64,
// which are not stored.
template <bool RB, bool XR, bool CB>
__device__ __forceinline__ void layer4(const GenParams* __restrict__ gp, const int8_t* y3, int8_t* y4,
                                       const SmallG* sg, int lane, int p0, int pstep) {
  constexpr int LO = CB ? -127 : -128;
  const int T64 = gp->T64, T64A = gp->T64A;
  constexpr bool rb = RB;  // the blob's REORDER_BN flag (gp->rb), an instantiation
  // the lane's addresses and constants are derived and read here, per call: hoisted out of the
  // trial loop they were held in registers (and spilled in the plain float builds)
  int ln;
  asm volatile("v_mov_b32 %0, %1" : "=v"(ln) : "v"(lane));
  const int c = ln & 31, h = ln >> 5, k = c & 15;
  const int i = c;  // A row of this lane
  const int n = 16 * ((i >> 2) & 1) + 4 * (i >> 3) + (i & 3);
  asm volatile("" ::: "memory");
  const v4i bw = sg->l4_b[ln];
  const int thr = sg->l4_thr[k], off = sg->l4_off[k], xs = sg->l4_xs[k];
  const unsigned m = sg->l4_m[k];
  const float r4 = sg->l4_r[k], c4 = sg->l4_c[k];
  const int ci = (!rb && !XR) ? sg->l4_ci[k] : 0;  // plain float form: the floor form's C-init
  const int NP = (T64 + 7) / 8;
  for (int p = p0; p < NP; p += pstep) {
    const v4i a = *(const v4i*)(y3 + 16 * (64 * p + 32 * h + n));
    const v16i acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, bw, (v16i){ci, ci, ci, ci, ci, ci, ci, ci, ci, ci, ci, ci, ci, ci, ci, ci}, 0, 0, 0);
    int q[2];
#pragma unroll
    for (int w = 0; w < 2; w++) {
      int sum = 0;
      if constexpr (rb) {
#pragma unroll
        for (int e = 0; e < 8; e++) sum += max(acc[8 * w + e], thr);
        q[w] = clampq(XR ? xdiv(sum + off, m, xs) : (int)((float)(sum + off) * r4), LO);
      } else {
        // plain: layer4.c:113-118 clips no element (the float form clamps at 1024, past which the
        // result saturates anyway)
#pragma unroll
        for (int e = 0; e < 8; e++) sum += XR ? max(xdiv(acc[8 * w + e] + off, m, xs), 0) : floor_el<1024>(acc[8 * w + e], r4, c4);
        q[w] = clampq(sum >> 3, LO);
      }
    }
    const int v = 8 * p + 4 * (c >> 4) + 2 * h;
    int8_t* dst = y4 + k * T64A + v;
    if (v + 1 < T64) *(unsigned short*)dst = (unsigned short)((q[0] & 255) | ((q[1] & 255) << 8));
    else if (v < T64) *dst = (int8_t)q[0];
  }
}

// Layer 5 (layer5.c:43-89, transform.c:47): z = W5[n] . y4 + b5[n], clip(z / fac) (pad columns
// meet zero weights).  Four classes per wave pass, sixteen lanes each: lane (n, c) sums dwords
// c, c + 16, ... of its class, a DPP row_shr prefix sum leaves the class total in the row's lane
// 15.  Class groups g0, g0 + gstep, ... of four classes.
template <bool CB>
__device__ __forceinline__ void layer5(const GenParams* __restrict__ gp, const int8_t* y4, const int8_t* w5,
                                       int8_t* out, int g0, int gstep, int lane) {
  constexpr int LO = CB ? -127 : -128;
  const int N = gp->N, rp = w5_row(gp->T64A) / 4;  // dwords of a padded y4 / weight row
  const int c = lane & 15;
  const int* b5 = (const int*)(w5 + N * 4 * rp);
  for (int n0 = 4 * g0; n0 < N; n0 += 4 * gstep) {
    const int n = n0 + (lane >> 4);
    const int* w = (const int*)(w5 + (n < N ? n : 0) * 4 * rp);
    int part = 0;
    for (int d = c; d < rp; d += 64) {  // rp is a multiple of 64: four independent reads per pass
#pragma unroll
      for (int q = 0; q < 4; q++)
        part = __builtin_amdgcn_sdot4(((const int*)y4)[d + 16 * q], w[d + 16 * q], part, false);
    }
    part += __builtin_amdgcn_update_dpp(0, part, 0x111, 0xF, 0xF, true);  // row_shr:1
    part += __builtin_amdgcn_update_dpp(0, part, 0x112, 0xF, 0xF, true);  // row_shr:2
    part += __builtin_amdgcn_update_dpp(0, part, 0x114, 0xF, 0xF, true);  // row_shr:4
    part += __builtin_amdgcn_update_dpp(0, part, 0x118, 0xF, 0xF, true);  // row_shr:8
    if (c == 15 && n < N) out[n] = (int8_t)clampq(xdiv(part + b5[n], gp->l5_m, gp->l5_xs), LO);
  }
}

// Per-lane constants and the LDS initialisation shared by both kernels.
__device__ __forceinline__ void setup(const GenParams* __restrict__ gp, int8_t* smem, const Carve& cv, L1C& k1,
                                      L2C& k2, int tid, int wave, int lane) {
  const int j = lane & 15;
  k1.wf = gp->l1_b[lane];
  k1.off = gp->l1_off[j];
  k1.m = gp->l1_m[j];
  k1.xs = gp->l1_xs[j];
  k1.r = gp->l1_r[j];
  k1.c = gp->l1_c[j];
#pragma unroll
  for (int fi = 0; fi < 2; fi++) {
    const int f = 2 * wave + fi;
#pragma unroll
    for (int s = 0; s < 3; s++) k2.af[fi][s] = gp->l2_a[f][s][lane];
#pragma unroll
    for (int s = 0; s < 2; s++) k2.at[fi][s] = gp->l2t_a[f][s][lane];
    k2.thr[fi] = gp->l2_thr[f];
    k2.off[fi] = gp->l2_off[f];
    k2.m[fi] = gp->l2_m[f];
    k2.xs[fi] = gp->l2_xs[f];
    k2.r[fi] = gp->l2_r[f];
    k2.c[fi] = gp->l2_c[f];
  }
  // zero pads of every row (positions past the data are never rewritten), then the small params
  v4i* z = (v4i*)smem;
  for (int i = tid; i < cv.sg / 16; i += NT) z[i] = (v4i){0, 0, 0, 0};
  const v4i* src = (const v4i*)&gp->sg;
  v4i* dst = (v4i*)(smem + cv.sg);
  for (int i = tid; i < (int)(sizeof(SmallG) / 16); i += NT) dst[i] = src[i];
  const int row5 = F2 * gp->T64A, rp = w5_row(gp->T64A) / 4;  // layer-5 weight rows, [N][rp dwords]
  int* w5 = (int*)(smem + cv.w5);
  for (int i = tid; i < gp->N * rp; i += NT) {
    const int n = i / rp, d = i - n * rp;
    w5[i] = 4 * d < row5 ? ((const int*)gp->l5_w[n])[d] : 0;
  }
  for (int n = tid; n < gp->N; n += NT) w5[gp->N * rp + n] = gp->l5_b[n];
}

// Fused forward over a batch of B trials (layout L), logits [B][N].
// ST: int8 trials staged in LDS (the carve's raw area fits; the host picks the instantiation)
template <int L, bool ST, bool RB, bool XR, bool CB>
// two workgroups per CU (4 waves per SIMD): at most 128 VGPRs
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_forward(
    const GenParams* __restrict__ gp, const int8_t* __restrict__ x,
                                                 int8_t* __restrict__ out, int B, float qs, float qy) {
  static_assert(!ST || L != F32, "float32 trials are not staged");
  extern __shared__ v4i smem_v[];
  int8_t* smem = (int8_t*)smem_v;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const Carve cv = carve_of(gp->C, gp->T, gp->N, gp->T8, gp->T64A, gp->NB1, gp->MT, gp->NTT, L);
  L1C k1;
  L2C k2;
  setup(gp, smem, cv, k1, k2, tid, wave, lane);
  if constexpr (L != TM) k1.wf = gp->l1_bn[lane];  // channel-major fragments keep the natural K order
  const SmallG* sg = (const SmallG*)(smem + cv.sg);
  int8_t* y1 = smem;
  int8_t* y2 = smem + cv.y2;
  int8_t* y3 = smem + cv.y3;
  int8_t* y4 = smem + cv.y4;
  int8_t* stg = smem + cv.stg + 1024 * wave;
  // layer-1 groups of two blocks when two workgroups share the CU (the other one's waves cover the
  // latency; a wave's ~10 blocks then leave no slot re-reading the last block), of four at one
  // workgroup per CU (general kernels)
  const bool two_wg = cv.bytes <= LDS_2WG;
  const int C = gp->C, T = gp->T, N = gp->N, xstride = gp->xstride, NB1 = gp->NB1;
  const int K7 = L == TM && !two_wg ? gp->K7T1 : gp->K7;
  // int8 trials staged in LDS (cv.raw >= 0, uniform): the first one now; after that each trial a
  // grid stride ahead, by LDS-DMA issued after barrier A (layer 1 has read the area) and waited for
  // before barrier B, so it lands during layers 2-3 and no wave waits on HBM in layer 1
  int8_t* sraw = ST ? smem + cv.raw : nullptr;
  if (ST && (int)blockIdx.x < B) {
    stage_trial(trial_view<L>(x, blockIdx.x, C, T, xstride), sraw, cv.chunks, wave, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  // (phase stamps in tools/ builds with -DMIB_STAMPS: 0 layer 1 / the last wave's layers 4-5,
  // 1 barrier A, 2 layer 2, 3 layer 3, 4 barrier B, 7 loop top)
  MIB_STAMP_INIT
  // Two barriers per trial.  Waves 0 .. NW-2 run layer 1 while the last wave runs layers 4 and 5
  // of the previous trial (its y3t and y4 are untouched until this trial's layer 3, after barrier
  // A), as the compiled kernels do (forward_wg.hpp); A: layer 2 reads every wave's layer-1 rows;
  // B: layer 4 reads every filter's layer-3 rows.  The next trial's LDS-DMA goes out after A (layer
  // 1 has read the area) and is waited for before B.
  int bprev = -1;
  for (int b = blockIdx.x; b < B; b += gridDim.x) {
    const View v = trial_view<L>(x, b, C, T, xstride);
    MIB_STAMP(7)
    // priorities as in the compiled kernels (wg::PRIO_*): the last wave's layers 4-5 are the longest
    // dependency chain of the interval and issue first; layer 1 ahead of the other workgroup's 2-3
    if (wave < NW - 1) {
      __builtin_amdgcn_s_setprio(wg::PRIO_L1);
      if (two_wg) layer1<L, ST, XR, CB, false>(gp, v, sraw, y1, cv.y1s, stg, k1, wave, NW - 1, NB1 - K7, lane, qs, qy);
      else layer1<L, ST, XR, CB>(gp, v, sraw, y1, cv.y1s, stg, k1, wave, NW - 1, NB1 - K7, lane, qs, qy);
    } else {
      if (bprev >= 0) {
        __builtin_amdgcn_s_setprio(wg::PRIO_L45);
        layer4<RB, XR, CB>(gp, y3, y4, sg, lane, 0, 1);
        wg::wave_sync_lds();
        layer5<CB>(gp, y4, smem + cv.w5, out + (size_t)bprev * N, 0, 1, lane);
      }
      // then the trial's last K7 layer-1 blocks (host-balanced against layers 4-5)
      if (K7 > 0) {
        __builtin_amdgcn_s_setprio(wg::PRIO_L1);
        if (two_wg) layer1<L, ST, XR, CB, false>(gp, v, sraw, y1, cv.y1s, stg, k1, NB1 - K7, 1, NB1, lane, qs, qy);
        else layer1<L, ST, XR, CB>(gp, v, sraw, y1, cv.y1s, stg, k1, NB1 - K7, 1, NB1, lane, qs, qy);
      }
    }
    __builtin_amdgcn_s_setprio(0);
    MIB_STAMP(0)
    __syncthreads();  // A
    const int bn = b + (int)gridDim.x;
    if (ST && bn < B) stage_trial(trial_view<L>(x, bn, C, T, xstride), sraw, cv.chunks, wave, lane);
    MIB_STAMP(1)
    layer2<RB, XR, CB>(gp, y1, cv.y1s, y2, cv.y2s, k2, wave, lane);
    wg::wave_sync_lds();  // layer 3 of filter f reads only y2 row f, written by this wave
    MIB_STAMP(2)
    __builtin_amdgcn_s_setprio(wg::PRIO_L3);
    layer3<XR, CB>(gp, sg, y2, cv.y2s, y3, wave, lane);
    __builtin_amdgcn_s_setprio(0);
    MIB_STAMP(3)
    if (ST) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's part of the next trial
    __syncthreads();  // B
    MIB_STAMP(4)
    bprev = b;
  }
  if (wave == NW - 1 && bprev >= 0) {  // the last trial's layers 4-5
    layer4<RB, XR, CB>(gp, y3, y4, sg, lane, 0, 1);
    wg::wave_sync_lds();
    layer5<CB>(gp, y4, smem + cv.w5, out + (size_t)bprev * N, 0, 1, lane);
  }
  MIB_STAMP_FLUSH(lane == 0, wave)
}

// Single-trial, single-layer kernel for the reference's per-layer entry points on the general
// path: stage 1..5 = net_layerN, 6 = net_layer3_flip_inplace; reference layouts in and out (pads
// zero).  Stage 1 takes the trial packed time-major [T][C] (the batched layout).
template <bool RB, bool XR, bool CB>
__global__ __launch_bounds__(NT) void k_layer(const GenParams* __restrict__ gp, const int8_t* __restrict__ in,
                                              int8_t* __restrict__ out, int stage) {
  extern __shared__ v4i smem_v[];
  int8_t* smem = (int8_t*)smem_v;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const Carve cv = carve_of(gp->C, gp->T, gp->N, gp->T8, gp->T64A, gp->NB1, gp->MT, gp->NTT, 3);
  L1C k1;
  L2C k2;
  setup(gp, smem, cv, k1, k2, tid, wave, lane);
  const SmallG* sg = (const SmallG*)(smem + cv.sg);
  int8_t* y1 = smem;
  int8_t* y2 = smem + cv.y2;
  int8_t* y3 = smem + cv.y3;
  int8_t* y4 = smem + cv.y4;
  const int C = gp->C, T = gp->T, T8 = gp->T8, T64 = gp->T64, T64A = gp->T64A;
  const int TA = (T + 3) & ~3, T8A = (T8 + 3) & ~3;
  __syncthreads();
  if (stage == 1) {  // [T][C] packed -> [F1][T_ALIGN]
    const View v = trial_view<TM>(in, 0, C, T, gp->xstride);
    layer1<TM, false, XR, CB>(gp, v, nullptr, y1, cv.y1s, nullptr, k1, wave, NW, gp->NB1, lane, 0.0f, 0.0f);
    __syncthreads();
    for (int i = tid; i < F2 * TA; i += NT) {
      const int f = i / TA, t = i - f * TA;
      out[i] = t < T ? y1[f * cv.y1s + 32 + t] : 0;
    }
  } else if (stage == 2) {  // [F1][T_ALIGN] -> [F2][T8_ALIGN]
    for (int i = tid; i < F2 * T; i += NT) {
      const int f = i / T, t = i - f * T;
      y1[f * cv.y1s + 32 + t] = in[f * TA + t];
    }
    __syncthreads();
    layer2<RB, XR, CB>(gp, y1, cv.y1s, y2, cv.y2s, k2, wave, lane);
    __syncthreads();
    for (int i = tid; i < F2 * T8A; i += NT) {
      const int f = i / T8A, u = i - f * T8A;
      out[i] = u < T8 ? y2[f * cv.y2s + 8 + u] : 0;
    }
  } else if (stage == 3) {  // [F2][T8_ALIGN] -> [F2][T8_ALIGN]
    for (int i = tid; i < F2 * T8; i += NT) {
      const int f = i / T8, u = i - f * T8;
      y2[f * cv.y2s + 8 + u] = in[f * T8A + u];
    }
    __syncthreads();
    layer3<XR, CB>(gp, sg, y2, cv.y2s, y3, wave, lane);
    __syncthreads();
    for (int i = tid; i < F2 * T8A; i += NT) {
      const int f = i / T8A, u = i - f * T8A;
      out[i] = u < T8 ? y3[16 * u + f] : 0;
    }
  } else if (stage == 4) {  // [T8][F2] -> [F2][T64_ALIGN]
    for (int i = tid; i < T8 * F2; i += NT) y3[i] = in[i];
    __syncthreads();
    layer4<RB, XR, CB>(gp, y3, y4, sg, lane, wave, NW);
    __syncthreads();
    for (int i = tid; i < F2 * T64A; i += NT) out[i] = y4[i];
  } else if (stage == 5) {  // [F2][T64_ALIGN] -> [N] (the pad columns read as zero)
    for (int i = tid; i < F2 * T64A; i += NT) y4[i] = (i % T64A) < T64 ? in[i] : 0;
    __syncthreads();
    layer5<CB>(gp, y4, smem + cv.w5, out, wave, NW, lane);  // class group w on wave w
  } else if (stage == 6) {  // flip [F2][T8_ALIGN] -> [T8][F2]
    for (int i = tid; i < F2 * T8A; i += NT) {
      const int u = i / F2, f = i - u * F2;
      out[i] = u < T8 ? in[f * T8A + u] : 0;
    }
  }
}

}  // namespace gen
}  // namespace mib
