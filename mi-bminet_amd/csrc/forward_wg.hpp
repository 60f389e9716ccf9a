// forward_wg.hpp — gfx950 fused forward kernel of the int8 MI-BMInet (edgeEEGNet) network.
//
// One workgroup of NWAVES = 8 wave64s owns one trial at a time and walks a grid-strided list of
// trials (persistent; two workgroups per CU, i.e. four waves per SIMD, so one workgroup's
// barriers are covered by the other's work).  Per trial:
//   layer1  spatial C->16 contraction on MFMA i32_16x16x64_i8.  A = 16 time groups x 64-byte
//           input window (P = 2 samples of C <= 32 channels per group, or 1 sample of up to 64)
//           read straight from HBM into registers (4-byte-aligned 16-B loads, prefetched one
//           trial ahead while the current trial runs layers 2-5); B = per-(filter, parity)
//           weight fragment; C-init = offset + float magic, so requant is one exact fma per
//           output, a truncating convert and a saturating pack (v_ashr_pk_i8_i32) per 2 outputs.
//                                                    (reference: layer1.c:53-101)
//   layer2  64-tap depthwise temporal xcorr as a banded-Toeplitz GEMM on MFMA i32_32x32x32_i8:
//           A = 32 output shifts x 96-tap band of the filter (held in registers; rows permuted so
//           that each lane owns two whole pool-8 windows), B = 16-byte slices of the layer-1 row
//           at immediate offsets.  32 column blocks per filter form its full tile; the chain starts
//           from a float inline constant so the ReLU-pool is one saturating v_sub_u32 per element
//           (biased pooling).  The TB blocks of 32 outputs left per filter (the tail) run on one
//           3-step MFMA i32_16x16x64_i8 chain per wave (16 shifts, A from LDS): columns of 16
//           outputs, the wave's two filters side by side with a block-diagonal K (a lane reads the
//           zero chunk in the other filter's slots); a lane holds half a pool window, the two
//           halves meet by v_permlane16_swap.    (reference: layer2.c:56-118, xcorr.c:44)
//   layer3  16-tap depthwise conv on MFMA i32_16x16x64_i8, both filters of a wave in one tile
//           (block-diagonal K): tile 1 = the first 128 outputs of each filter (16-output columns),
//           tile 2 = the outputs past 128, four per column in register 0; C-init = float magic;
//           written transposed [u][f] (the reference's flip is index math).
//                                                    (reference: layer3.c:49-79, conv.c:105)
//   layer4  16x16 pointwise on MFMA i32_32x32x32_i8 with a block-diagonal B (two 32-sample time
//           blocks per MFMA, all 64 lanes busy) + biased ReLU pooling + requant.
//                                                    (reference: layer4.c:51-149)
//   layer5  F2*T64 -> 4 linear + bias + requant: one wave, 16 lanes per class, DPP row
//           reduction, one dword store.              (reference: layer5.c:43-89)
// The plain (non-REORDER_BN) build requantises every layer-2/4 element in the floor form (l2n_out,
// relu_sum8); its 22-channel time-major layer-1 blocks past the VGPR prefetch arrive a trial ahead
// in LDS by LDS-DMA (Cfg::LDMA).  Parameter sets outside the float requant envelope run Cfg::XR,
// exact integer division (xdiv) at layers 1, 2 and 4.
// Channel-major input (Cfg::CT, net_model_compute_batch_ct): each layer-1 block is read as
// 16-sample row segments and transposed through LDS (22 channels: an LDS-DMA ring read back with
// ds_read_b64_tr_b16; 64 channels: whole rows exchanged through a shared phase image) into the
// MFMA A fragment; everything after that is the same code.
#pragma once
#include "forward_common.hpp"
#ifdef MIB_DIAG
#include "forward_diag.hpp"  // timing proxies (tools/ builds only; results wrong)
#endif

namespace mib {
namespace wg {

constexpr int NWAVES = 8;             // waves per workgroup (one trial per workgroup)
constexpr int FPW = F2 / NWAVES;      // layer-2 / layer-3 filters per wave
constexpr int NTHREADS = 64 * NWAVES;
constexpr int WPE = 4;                // waves per SIMD (two workgroups per CU)
constexpr int LDS_WG_MAX = 160 * 1024 / 2;  // LDS per workgroup at two workgroups per CU
constexpr int PF_MAX = 9;             // layer-1 blocks per wave prefetched one trial ahead
constexpr int PF_MAX_PLAIN = 3;       // plain BN: fewer, no spills (config B -5.4 %, C -13.6 %; 4, 5
                                      // measured slower with the LDS-DMA of the rest)
constexpr int PF_MAX_PLAIN_CT = 2;
static_assert(FPW == 2, "tail-tile and layer-3 mapping assume two filters per wave");
// Wave priorities (s_setprio): the last wave's layers 4-5 are the longest dependency chain of the
// layer-1 interval, so that wave issues first while on them; layer 1 (HBM fragments, next-trial
// prefetch) goes ahead of the other workgroup's layers 2-3.  Same-box A/B: -4 %.  Layer 3 (the end
// of the barrier-B interval) at 1 as well: -1.7 %.  About 20 other placements measured slower
// (DESIGN.md §8).
constexpr int PRIO_L1 = 1, PRIO_L3 = 1, PRIO_L45 = 3;

// Layer-1 work split.  The last wave also runs layers 4 and 5 (in the same barrier interval as
// the next trial's layer 1), so it takes fewer layer-1 blocks: waves 0 .. NWAVES-2 get cm blocks
// (the first rm of them one more), the last wave cl, with layers 4-5 counted as W45 blocks.
constexpr int W45 = 4;

#ifndef MIB_DIAG
// Timing-proxy switches (forward_diag.hpp): all off in the library.
constexpr bool DIAG_NOL2 = false, DIAG_NOTAIL = false, DIAG_NOL3 = false, DIAG_NOL45 = false;
constexpr int DIAG_L2_STEPS = 3;
#endif

template <bool V>
struct BoolC {
  static constexpr bool value = V;
};
template <int V>
struct IntC {
  static constexpr int value = V;
};

struct L1Split {
  int cm, rm, cl;
};
constexpr L1Split l1_split(int nb1) {
  constexpr int nm = NWAVES - 1;
  L1Split best{0, 0, 0};
  int bcost = 1 << 30;
  for (int cl = 0; cl <= nb1; cl++) {
    const int cm = (nb1 - cl) / nm, rm = (nb1 - cl) % nm;
    const int hi = cmax(cm + (rm ? 1 : 0), cl + W45);
    if (hi < bcost) {
      bcost = hi;
      best = L1Split{cm, rm, cl};
    }
  }
  return best;
}

template <int C_, int T_, bool RB_ = true, bool CB_ = false, bool CT_ = false, bool FQ_ = false, bool XR_ = false>
struct Cfg {
  static constexpr int C = C_, T = T_;
  static constexpr bool XR = XR_;                       // exact integer division at layers 1, 2, 4 (xdiv)
  static constexpr bool FQ = FQ_;                       // float32 channel-major trials, quantised in layer1
  static_assert(!FQ_ || CT_, "float input is channel-major");
  static constexpr bool RB = RB_;                       // -DREORDER_BN variant (canonical)
  static constexpr bool CB = CB_;                       // golden-model clip_balanced: clip to [-127, 127]
  static constexpr bool CT = CT_;                       // channel-major [C][T] trials, staged in LDS (layer1)
  static constexpr int LO = CB ? -127 : -128;           // lower clip bound of every requant
  static constexpr int P = (C <= 32) ? 2 : 1;          // samples per 64-byte L1 window
  static constexpr int GS = P * C;                      // bytes per time group
  static constexpr int NB1 = (T + 16 * P - 1) / (16 * P);  // L1 blocks of 16 groups
  static constexpr int T8 = T / 8, T64 = T8 / 8;
  static constexpr int NT4 = (8 * T64 + 63) / 64;       // L4 MFMAs of 64 time samples
  static constexpr L1Split SPL = l1_split(NB1);
  static constexpr int NBW = cmax(SPL.cm + (SPL.rm ? 1 : 0), SPL.cl);  // L1 blocks per wave (max)
  // of which prefetched a trial ahead (the plain-BN and 22-channel exact-division builds hold more
  // per-lane state; the rest of their blocks go by LDMA below)
  // (float input: the first block's four 16-byte pieces; the others load one block ahead)
  static constexpr int PF = FQ_ ? 4 : cmin(NBW, RB && !(XR_ && P == 2) ? PF_MAX : CT_ ? PF_MAX_PLAIN_CT : PF_MAX_PLAIN);
  // Channel-major int8, 22 channels, through LDS-DMA (layer1): each block's rows go from HBM straight
  // into an LDS ring with buffer_load_dwordx4 ... lds, a trial ahead, and the A fragments come back
  // with ds_read_b64_tr_b16: no VGPR round trip, no ds_write (RS ring slots, LDS carve below).  The
  // 64-channel shapes load whole rows instead (RX): 64 rows of 16 bytes per DMA instruction measured
  // +50 % on config C.
  static constexpr bool DMA = CT_ && !FQ_ && P == 2;
  static constexpr int NB2 = (8 * T8 + 31) / 32;        // L2 column blocks of 32 outputs
  // full L2 tiles per filter, then a tail of TB blocks on the 16x16x64 chain when the wave's two
  // filters' tail columns fit its 16 columns (FPW * TC <= 16); otherwise (short trials, e.g.
  // T = 480) the last tile is a partial 32x32 tile whose columns past NB2 are computed and dropped
  static constexpr int MT0 = NB2 / 32;
  static constexpr bool TAIL = NB2 > 32 * MT0 && FPW * 2 * (NB2 - 32 * MT0) <= 16;
  static constexpr int MT = (TAIL || NB2 == 32 * MT0) ? MT0 : MT0 + 1;
  static constexpr int TB = TAIL ? NB2 - 32 * MT0 : 0;  // tail blocks (of 32 outputs) per filter
  static constexpr int TC = 2 * TB;                     // tail columns (of 16 outputs) per filter
  // layer-1 rows hold positions pos = t + 32 (32 leading zeros = the xcorr pad of 31, aligned).
  // PSPLIT (P == 2): parity-split planes [pos & 1][pos >> 1]: each lane's 4 outputs (samples of one
  // parity) are contiguous and layer 2's K-window slices are 16-B aligned.  P == 1: natural order.
  // Channel-major P == 2 (TR16): the block image's rows are channels (32 bytes = 16 sample pairs),
  // read with ds_read_b64_tr_b16, so MFMA row j is the sample pair (2 j, 2 j + 1) as in the
  // time-major kernel, and the y1 rows and layer-2 fragments are the time-major ones (tr16_pos,
  // staged_tr).  Channel-major P == 1: ds_read_b64_tr_b8 (stg_pos, rx_frag).
  static constexpr bool TR16 = CT_ && P == 2;
  static constexpr bool PSPLIT = P == 2;
  static constexpr int PL = PSPLIT ? 2 : 1;             // y1 layout: planes per row
  static constexpr int NPOS = cmax(cmax(32 + 16 * P * NB1, 32 * (NB2 - 1) + 96), 1024 * MT + 64);
  static constexpr int PLANE = align16((NPOS + PL - 1) / PL);
  static constexpr int Y1ROW = PL * PLANE;
  // batched trial stride (bytes): time-major trials are padded to 16 bytes, channel-major ones
  // are the caller's contiguous [B][C][T]
  static constexpr int XTRIAL = FQ ? 4 * C * T : CT ? C * T : align16(T * C);
  // Channel-major int8, 64 channels, either BN branch (RX): whole-row loads.  Wave w loads channel rows
  // w + 8 h + 16 m (h < 2, m < 4) in 512-byte phases (2 rows x 512 bytes per load, lane-contiguous,
  // where single-block loads read 16 bytes from each of 64 rows), and the waves exchange them
  // through a 32 KB LDS image of one phase: [64 rows][512 bytes], read back with ds_read_b64_tr_b8
  // (rx_*, layer1).  Phase 0 of the next trial is stored before barrier B; each further phase
  // costs two barriers (the image consumed, the image complete).  Config C -19.6 %;
  // the plain-BN build since round 5: C -23.0 %, 64x480 -11.0 %.  The float-input 64-channel build
  // stages one block at a time (stage_block), double-buffered in two 1 KB areas per wave.
  static constexpr bool RX = CT_ && !FQ_ && P == 1 && C == 64 && SPL.cl == 0 && (C * T) % 4 == 0;
  static constexpr int NPH = RX ? (16 * NB1 + 511) / 512 : 0;  // image phases of 512 samples
  static constexpr int STG = RX ? 32768 / NWAVES : 2048;  // staging bytes per wave
  static constexpr int NB3 = (T8 + 15) / 16;            // layer-3 column blocks of 16 outputs
  // layer 3: tile 1 = the first L3C blocks of both filters side by side (one 16x16x64 MFMA),
  // tile 2 = the L3R outputs past 128, four per column in register 0 only (layer3)
  static constexpr int L3C = cmin(NB3, 8);
  static constexpr int L3R = T8 > 128 ? T8 - 128 : 0;
  static constexpr int L3RC = (L3R + 3) / 4;
  // y2 row: pad [0, 8), positions at 8 + u, zero pads after; the last 16 bytes are the zero chunk
  // that block-diagonal B operands read (tile 1 reads bytes < 16 L3C + 16, tile 2 < 128 + 4 L3RC + 28)
  static constexpr int Y2ROW = align16(cmax(cmax(T8 + 8, 16 * L3C + 16), L3RC ? 128 + 4 * L3RC + 28 : 0) + 16);
  static constexpr int Y3ROWS = cmax(64 * NT4, T8);
  // y3t row u (16 filters) starts at byte 16 u + 4 (u >> 4) (y3_off): layer 3's 2-byte stores
  // (one wave instruction covers rows 16 col + 4 g + i of 32 lanes) then hit 32 different banks;
  // layer 4 reads a row with one (4-byte aligned) ds_read_b128, 2-way at most (3 per trial)
  static constexpr int Y3S = 16;
  static constexpr int T64A = (T64 + 3) & ~3;           // y4 row stride (reference T64_ALIGN)
  static constexpr bool L4PIPE = P == 2 && RB;  // layer-4 MFMA/pooling overlap (registers)
  static constexpr int ND5 = F2 * T64A / 4;             // layer-5 input dwords
  static constexpr int N5L = (ND5 + 15) / 16;           // layer-5 dwords per lane
  // LDS carve
  static constexpr int OFF_Y1 = 0;
  static constexpr int OFF_Y2 = OFF_Y1 + F2 * Y1ROW;
  static constexpr int OFF_Y3 = OFF_Y2 + align16(F2 * Y2ROW);  // layer 3 reads only inside the wave's y2 rows
  static constexpr int OFF_Y4 = OFF_Y3 + align16(Y3ROWS * Y3S + 4 * (Y3ROWS >> 4));
  static constexpr int OFF_SP = OFF_Y4 + align16(64 * N5L);
  static constexpr int OFF_LT = align16(OFF_SP + (int)sizeof(SmallParams));   // per-lane offsets
  static constexpr int OFF_L45 = OFF_LT + 64 * 48;                            // layer-4/5 lane offsets
  static constexpr int OFF_L2T = OFF_L45 + 64 * 32;                           // tail band fragments
  // DMA: the tail band fragments live in VGPRs (12 per lane; the ring frees the 4 per prefetched
  // block), so that the ring fits two workgroups per CU
  static constexpr bool L2TV = DMA && TB > 0;
  static constexpr int OFF_STG = OFF_L2T + (TB > 0 && !L2TV ? NWAVES * 3 * 64 * 16 : 0);  // CT staging / ring
  // DMA ring: RS slots of 1 KB per wave (one block image each), every block of the wave
  static constexpr int RS = DMA ? cmin(NBW, (LDS_WG_MAX - OFF_STG) / (NWAVES * 1024)) : 0;
  static constexpr int PFV = DMA ? 0 : RX ? 4 * NPH : PF;  // loads prefetched into VGPRs
  // time-major plain BN and exact division, 22 channels (LDMA): the blocks past PF go a trial ahead
  // into an LDS slot per block by LDS-DMA, where they wait in no register (the VGPR prefetch of all
  // blocks spills; loading them at the start of their own layer 1 exposes the HBM latency).  XR
  // config B: 5 VGPR blocks spilled 40-44 bytes; 3 + 2 by DMA, 8 bytes: -17 % same box.
  static constexpr bool LDMA = !CT_ && (!RB_ || XR_) && P == 2 && NBW > PF;
  static constexpr int NLD = LDMA ? NBW - PF : 0;

  static constexpr int LDS = OFF_STG + (DMA ? NWAVES * RS * 1024 : CT ? NWAVES * STG : NWAVES * NLD * 1024);
  static_assert(!LDMA || LDS <= LDS_WG_MAX, "two workgroups per CU");
  static_assert(!DMA || RS == NBW, "the DMA ring holds every layer-1 block of a wave");
  static_assert(!DMA || LDS <= LDS_WG_MAX, "two workgroups per CU");
  static_assert(C >= 1 && C <= 64, "C must be <= 64 (one 64-byte MFMA K window)");
  static_assert(GS % 4 == 0, "time-group stride must be dword aligned");
  static_assert(T64 >= 1, "T >= 64");
  static_assert(16 * N5L <= ND5_MAX, "layer-5 input too long");
  static_assert(MT >= 1, "at least one full layer-2 tile");
  static_assert(FPW * TC <= 16, "tail columns of a wave fit one 16-column tile");
  static_assert(L3RC <= 8, "layer-3 tile 2 covers at most 32 outputs past 128");
  static_assert(Y3ROWS >= 16 * L3C, "layer-3 tile-1 rows fit y3t");
};

// byte offset of layer-1 output (filter f, sample t) inside the LDS rows
template <class K>
__device__ __forceinline__ int y1_index(int f, int t) {
  if constexpr (K::PSPLIT) return f * K::Y1ROW + (t & 1) * K::PLANE + ((t + 32) >> 1);
  else return f * K::Y1ROW + 32 + t;
}

// Per-lane LDS offsets of layers 2 and 3 (wave-independent parts), built once per workgroup by
// build_lane_tab and re-read every trial with two ds_read_b128: cheaper than recomputing them
// from the lane id, and registers are too scarce to keep them live across the trial loop.
struct LaneTab {
  int l2b;  // full tile, B slice (filter 0, tile 0, K-step 0): (32 / PL) c + l2_boff(0, h)
  int l2y;  // full tile, y2 store (filter 0, tile 0): 8 + 4 c + 2 h
  int tb[3];  // tail B chunk of K-step s (offset within the wave's filter pair; a zero chunk when
             // the K-step's slots of this lane belong to the other filter)
  int ty;   // tail y2 store: fi_c * Y2ROW + 8 + u, or -1 (lane stores nothing)
  int tp;   // tail: filter slot fi_c of this lane's column (0 or 1)
  int l3b;  // layer-3 tile-1 B chunk (16-byte aligned, relative to the wave's y2 rows): filter
            // fi = col >> 3, block col & 7: fi Y2ROW + 16 (col & 7) + 16 (g & 1) when lane group g
            // lies in the filter's K half (g >> 1 == fi), else the zero chunk
  int l3w;  // tile-1 store: y3_off(r0), r0 = 16 (col & 7) + 4 g + 2 fi (rows r0, r0 + 1), or -1
  int l3s;  // tile-1 v_perm selector pairing the lane's bytes with its partner's (col ^ 8)
  int l3b2; // tile-2 B chunk (4-byte aligned): fi Y2ROW + 128 + 4 (col & 7) + 16 (g & 1), or zero chunk
  int l3w2; // tile-2 store: y3_off(128 + 4 (col & 7) + g) + fi, or -1
};
static_assert(sizeof(LaneTab) == 48, "LaneTab is read as three 16-byte pieces");

static_assert(sizeof(SmallParams) % 16 == 0, "SmallParams is copied to LDS in 16-byte pieces");

// byte offset of y3t row u (see Cfg::Y3S)
template <class K>
__host__ __device__ constexpr int y3_off(int u) {
  return u * K::Y3S + 4 * (u >> 4);
}

// Per-lane offsets of layers 4 and 5 (the last wave), built once per workgroup like LaneTab: the
// wave re-reads them after barrier B instead of recomputing them from the lane id every trial.
struct L45Tab {
  int l4a;  // y3_off(32 h + n(i)): layer-4 A row of part 0 (part t adds y3_off(64 t))
  int l4w;  // k T64A + 4 (i >> 4) + 2 h: layer-4 store of part 0 (part t adds 8 t)
  int l4k;  // 4 k: byte offset of output channel k in the per-channel parameter arrays
  int l4m;  // bit t set when part t's store lies inside the row (v < T64A)
  int l5y;  // 4 c: layer-5 input dword of lane (n, c) (dword j adds 16 dwords)
  int l5w;  // 4 (n ND5_MAX + c): its weight
  int l5n;  // 4 n: class n's bias
  int pad;
};

template <class K>
__device__ __forceinline__ L45Tab build_l45_tab(int lane) {
  L45Tab L;
  const int i = lane & 31, h = lane >> 5, k = i & 15;
  const int n = 16 * ((i >> 2) & 1) + (i & 3) + 4 * (i >> 3);
  const int vl = 4 * (i >> 4) + 2 * h;
  L.l4a = y3_off<K>(32 * h + n);
  L.l4w = k * K::T64A + vl;
  L.l4k = 4 * k;
  L.l4m = 0;
  for (int t = 0; t < K::NT4; t++) L.l4m |= (8 * t + vl < K::T64A) << t;
  const int n5 = lane >> 4, c = lane & 15;
  L.l5y = 4 * c;
  L.l5w = 4 * (n5 * ND5_MAX + c);
  L.l5n = 4 * n5;
  L.pad = 0;
  return L;
}

// layer-2 B operand: byte offset (within a filter's rows, column block 0) of the 16-byte slice of
// lane half h, K-step s.  PSPLIT: half h reads parity plane h, plane bytes 16 s .. 16 s + 15 of the
// block's window (K-slot 32 s + 16 h + j <-> position 2 (16 s + j) + h); otherwise natural order.
// The band fragments built on the host use the same K order.
template <class K>
__device__ __forceinline__ int l2_boff(int s, int h) {
  if constexpr (K::PSPLIT) return h * K::PLANE + 16 * s;
  else return 32 * s + 16 * h;
}

// Layer-2 tail window chunks.  Column (fi, bq) of the tail covers outputs 1024 MT + 16 bq + m
// (m < 16), which read row positions p0 + q, p0 = 1024 MT + 16 bq, q = m + 1 + tap <= 79.  The
// window is cut into 16-byte chunks mq = 0..5 of the row: PSPLIT: plane mq & 1, plane bytes
// p0 / 2 + 16 (mq >> 1) .. +15 (positions q = 32 (mq >> 1) + 2 jj + (mq & 1)); natural: bytes
// p0 + 16 mq .. +15 (q = 16 mq + jj; chunk 5 is never needed and reads zeros).  The host builds
// the band fragments (l2t_afrag) with the same slot -> position map.
template <class K>
__device__ __host__ constexpr int tail_q(int mq, int jj) {
  return K::PSPLIT ? 32 * (mq >> 1) + 2 * jj + (mq & 1) : 16 * mq + jj;
}
template <class K>
__device__ __forceinline__ int tail_chunk_off(int fi, int bq, int mq) {
  if constexpr (K::PSPLIT) return fi * K::Y1ROW + (mq & 1) * K::PLANE + 512 * K::MT + 8 * bq + 16 * (mq >> 1);
  else return mq < 5 ? fi * K::Y1ROW + 1024 * K::MT + 16 * bq + 16 * mq : 0;
}

template <class K>
__device__ __forceinline__ LaneTab build_lane_tab(int lane) {
  LaneTab T;
  {
    const int c = lane & 31, h = lane >> 5;
    T.l2b = (32 / K::PL) * c + l2_boff<K>(0, h);
    T.l2y = 8 + 4 * c + 2 * h;
  }
  {
    const int col = lane & 15, g = lane >> 4;
    const int fi_c = K::TC > 0 ? col / cmax(K::TC, 1) : 0, bq = col - fi_c * K::TC;
    const bool cvalid = fi_c < FPW;
    const int fs = cvalid ? fi_c : 0;
#pragma unroll
    for (int st = 0; st < 3; st++) {
      const int kap = 4 * st + g, kf = kap / 6, mq = kap - 6 * kf;  // chunk kap = filter kf's chunk mq
      int off = 0;  // zero chunk: plane bytes 0..15 of the pair's first row (positions < 32 are pads)
      if (cvalid && kf == fi_c) off = tail_chunk_off<K>(fi_c, bq, mq);
      T.tb[st] = off;
    }
    const int u = 128 * K::MT + 2 * bq + (g >> 1);
    T.ty = (cvalid && !(g & 1) && u < K::T8) ? fs * K::Y2ROW + 8 + u : -1;
    T.tp = fs;
    // layer 3 (see layer3): lane (col, g), filter slot fi = col >> 3, column j = col & 7
    const int fi3 = col >> 3, j3 = col & 7;
    const int zero = K::Y2ROW - 16;
    T.l3b = ((g >> 1) == fi3 && j3 < K::L3C) ? fi3 * K::Y2ROW + 16 * j3 + 16 * (g & 1) : zero;
    const int u3 = 16 * j3 + 4 * g;
    T.l3w = (j3 < K::L3C && u3 < K::T8) ? y3_off<K>(u3 + 2 * fi3) : -1;
    T.l3s = fi3 == 0 ? 0x05010400 : 0x03070206;
    T.l3b2 = ((g >> 1) == fi3 && j3 < K::L3RC) ? fi3 * K::Y2ROW + 128 + 4 * j3 + 16 * (g & 1) : zero;
    const int v3 = 128 + 4 * j3 + g;
    T.l3w2 = (j3 < K::L3RC && v3 < K::T8) ? y3_off<K>(v3) + fi3 : -1;
  }
  return T;
}

// Per-lane register state that lives across the trial loop.
template <class K>
struct Regs {
  L1Tile t0, t1;
  __device__ __forceinline__ const L1Tile& tile(int t) const { return t == 0 ? t0 : t1; }
  __device__ __forceinline__ L1Tile& tile(int t) { return t == 0 ? t0 : t1; }
  v4i af[FPW][3];          // layer-2 band fragments of the wave's filters
  int thr2[FPW], off2[FPW];  // REORDER_BN: biased threshold, offset + 8 thr; plain: MFMA C-init, magic c bits
  float r2[FPW];             // reciprocal
  unsigned m2[FPW];          // XR: xdiv magic
  int xs2[FPW];              // XR: xdiv shift word
  v4i a31, a32;            // layer-3 tile-1 / tile-2 band fragments of the wave's filter pair
  float r3, c3;            // layer-3 requant constants (uniform)
  float qs, qy;            // float input's quantisation scale and RN(1 / scale) (K::FQ)
  v4i pf[K::PFV > 0 ? K::PFV : 1];  // layer-1 fragments prefetched one trial ahead (VGPRs)
  v4i l2t[K::L2TV ? 3 : 1];  // layer-2 tail band fragments of the wave's filter pair (K::L2TV)
  int xoff;                // lane_xoff(lane)
  int fq0;                 // float input: slot of the wave's first block in walking order (odd waves
                           // walk backwards, layer1)
};

// ---- layer-1 input ---------------------------------------------------------------------------
// Layer-1 blocks of a wave: a contiguous range (see l1_split).  Slots past the wave's count
// repeat its last block (the loads stay unconditional, the compute is skipped).
template <class K>
__device__ __forceinline__ int l1_count(int wave) {
  constexpr L1Split S = K::SPL;
  return wave < NWAVES - 1 ? S.cm + (wave < S.rm) : S.cl;
}

template <class K>
__device__ __forceinline__ int l1_start(int wave) {
  constexpr L1Split S = K::SPL;
  return wave * S.cm + min(wave, S.rm);
}

template <class K>
__device__ __forceinline__ int l1_blk(int wave, int i) {
  const int n = l1_count<K>(wave);
  const int b = l1_start<K>(wave) + (i < n ? i : n - 1);
  return b < 0 ? 0 : (b > K::NB1 - 1 ? K::NB1 - 1 : b);
}

// A fragment of block `blk` (16 time groups): lane (j, g) holds bytes
// [ (16 blk + j) * GS + 16 g, +16 ) of the trial.  The loads are raw buffer loads through a
// descriptor per (trial, wave): base = the wave's first block, num_records = the wave's own bytes
// (see trial_rsrc).  The hardware range check is per dword (tools/buf_probe.hip), so windows
// running past them read zeros instead of faulting or fetching, and there is no per-trial
// address arithmetic: the lane offset is loop-invariant and slot i adds 16 * GS * i (the
// instruction's immediate offset while it fits in 12 bits).  Samples >= T of the last block are
// masked to zero by l1_block.
typedef __amdgpu_buffer_rsrc_t Rsrc;

// The view ends where the wave's own bytes end: its last group's P * C bytes, or the trial's end.
// Window bytes past a group's own data meet zero weights, so reading them as zeros changes
// nothing, and no wave fetches the next trial's bytes (slots past its block count, windows past
// the trial's end) from memory.  trials_left <= 0: an empty view.
template <class K>
__device__ __forceinline__ Rsrc trial_rsrc(const int8_t* xt, int trials_left, int wave) {
  if constexpr (K::CT) {
    // channel-major: a wave's blocks lie in every channel row, so the view is the whole trial;
    // row segments running past T read the next row (samples >= T, whose outputs are masked).
    // Rows start at any byte, and the range check is per dword OF THE LOAD (tools/ct_probe.hip):
    // a dword straddling num_records reads as zeros.  So the view runs 3 bytes past the trial,
    // into the next trial's bytes, except for the batch's last trial, whose straddling dword is
    // completed by byte loads (ct_tail).
    // (float input: dword-aligned rows, so the view is exactly the trial)
    const int n = trials_left <= 0 ? 0 : (trials_left == 1 || K::FQ) ? K::XTRIAL : K::XTRIAL + 3;
    return __builtin_amdgcn_make_buffer_rsrc((void*)xt, (short)0, n, 0x00020000);
  }
  const int wb = l1_start<K>(wave) * 16 * K::GS;  // byte offset of the wave's first block
  const int own = min(l1_count<K>(wave) * 16 * K::GS, K::XTRIAL - wb);
  const int nrec = trials_left <= 0 ? 0 : max(own, 0);
  return __builtin_amdgcn_make_buffer_rsrc((void*)(xt + wb), (short)0, nrec, 0x00020000);
}

// Physical row of K-slot k in a channel-major block image (see stage_block); its own inverse.
__device__ __forceinline__ int stg_pos(int k) { return k ^ ((k >> 1) & 8); }
// K::TR16 image: 32-byte row slot of channel c; channels c and c + 8, which the two 16-lane groups
// of a 32-lane half read together, land in different bank halves (conflict-free, as stg_pos); its
// own inverse.  Lane L stores / DMA-loads half L & 1 of channel tr16_pos(L >> 1) at byte 16 L.
__device__ __forceinline__ int tr16_pos(int c) { return c ^ (((c >> 3) & 1) << 2); }

template <class K>
__device__ __forceinline__ int lane_xoff(int lane, int wave) {
  if constexpr (K::CT) {
    // channel-major: lane (c, h) (P == 2) or c (P == 1) reads 16 samples of channel row c; block
    // slot i adds 16 P i samples.  P == 2 (TR16, and the DMA ring: lane L's 16 bytes land in row L
    // of the block image): half L & 1 of channel tr16_pos(L >> 1).  Lanes past the rows (C = 22:
    // lanes of channels 22..31) read zeros without a fetch.
    const int c = K::TR16 ? tr16_pos(lane >> 1) : lane, h = K::P == 2 ? lane & 1 : 0;
    if (c >= K::C) return (int)0x80000000u;
    return (K::FQ ? 4 : 1) * (c * K::T + 16 * K::P * l1_start<K>(wave) + 16 * h);
  }
  // A lane whose 16-byte chunk lies wholly past the group's P * C bytes (C = 22: bytes 48..63)
  // only meets zero weights: it reads past num_records instead (offset >= 2^31 > any
  // num_records), so the hardware returns zeros without fetching and the MFMA multiplies zeros.
  if (16 * (lane >> 4) >= K::GS) return (int)0x80000000u;
  return (lane & 15) * K::GS + 16 * (lane >> 4);
}

// slot i of the wave (block l1_start + i); slots past the wave's count read data nobody uses
template <class K>
__device__ __forceinline__ v4i load_a(Rsrc r, int xoff, int i) {
  typedef unsigned v4u __attribute__((ext_vector_type(4)));
  // block stride: 16 time groups (time-major) or 16 P samples of a row (channel-major)
  // cache policy: nt (2) for the time-major stream; none for channel-major, whose 128-byte lines
  // are read by several block loads of a wave (nt: +40 %, tools/ab.py)
  constexpr int AUX = K::CT ? 0 : 2;
  const v4u v = __builtin_amdgcn_raw_buffer_load_b128(r, xoff + i * (K::CT ? 16 * K::P : 16 * K::GS), 0, AUX);
  return (v4i)v;
}

// The batch's last trial, channel-major: the one dword of the view that holds the trial's last
// byte(s) and straddles its end read as zeros (trial_rsrc); the lane holding it reloads those 1-3
// bytes one at a time (byte loads are range-checked per byte).  Once per launch.
template <class K>
__device__ __forceinline__ v4i ct_tail(v4i a, Rsrc r, int o) {
  constexpr int N = K::C * K::T;
  if (o < N && N < o + 16 && ((N - o) & 3)) {
    const int k0 = (N - o) & ~3;
    unsigned w = 0;
    for (int m = 0; o + k0 + m < N; m++)
      w |= (unsigned)__builtin_amdgcn_raw_buffer_load_b8(r, o + k0 + m, 0, 0) << (8 * m);
#pragma unroll
    for (int q = 0; q < 4; q++)
      if (4 * q == k0) a[q] = (int)w;
  }
  return a;
}

// Channel-major staging (K::CT).  The hardware executes a wave's LDS accesses in order, so an A
// read sees the stores before it and the next stores follow it; wave_sync_lds tells the compiler.
__device__ __forceinline__ void wave_sync_lds() {
  // orders this wave's LDS accesses across lanes for the compiler (no instruction is emitted):
  // without it, a lane that stores nothing may be given its previous read's value instead of a
  // new read (the other lanes' stores are invisible to the per-thread memory model)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Channel-major staging: the A operand of a layer-1 block through LDS, transposed by the hardware.
// A K-slot's row is 16 consecutive samples of one channel, which is what a lane loads: P == 2:
// lane L = (channel L >> 1, half h = L & 1) holds samples 32 blk + 16 h .. +15, and K-slot L is
// channel L >> 1 at sample 16 h + j of MFMA row j (rows pair samples j and j + 16); P == 1: lane c
// = channel c, samples 16 blk .. +15, K-slot c.  Each lane stores its row with one ds_write_b128,
// and two ds_read_b64_tr_b8 return the fragment: per 16-lane group g, an 8-row x 16-column byte
// block read column-wise, so lane (j, g) receives byte j of K-slots 16 g .. 16 g + 7, then
// 16 g + 8 .. 16 g + 15 (tools/tr8_probe.hip checks the form).  Physical row of K-slot
// k = 16 g + 8 r + q is stg_pos(k) = 16 g + 8 (r ^ (g & 1)) + q: the two groups of a 32-lane half
// then read different bank halves (conflict-free); stg_pos is its own inverse.
// (stg_pos is defined above lane_xoff, whose DMA offsets use it)

// byte offsets of lane (i, g)'s two transposed reads: lane i of a group supplies the address of
// row q = i >> 1, bytes 8 p .. 8 p + 7 (p = i & 1) of its 8-row block
__device__ __forceinline__ int stg_read_off(int lane, int r) {
  const int i = lane & 15, g = lane >> 4;
  return 16 * stg_pos(16 * g + 8 * r + (i >> 1)) + 8 * (i & 1);
}

// the A fragment of the block image at stg (two transposed reads).  K::TR16: lane (i, g)'s read r
// takes channels 8 g + 4 r .. +3 as rows; lane i supplies row i >> 2, bytes 8 (i & 3) .. +7
// (tools/tr16_probe.hip checks the map and the fragment on gfx950).
template <class K>
__device__ __forceinline__ v4i staged_tr(const int8_t* stg, int lane) {
  typedef int v2i __attribute__((ext_vector_type(2)));
  typedef __attribute__((address_space(3))) v2i lds_v2i;
  if constexpr (K::TR16) {
    typedef short v4s __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(3))) v4s lds_v4s;
    const int i = lane & 15, g = lane >> 4;
    const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(stg + 32 * tr16_pos(8 * g + (i >> 2)) + 8 * (i & 3)));
    const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(stg + 32 * tr16_pos(8 * g + 4 + (i >> 2)) + 8 * (i & 3)));
    const v2i a = __builtin_bit_cast(v2i, lo), b = __builtin_bit_cast(v2i, hi);
    return (v4i){a[0], a[1], b[0], b[1]};
  } else {
    const v2i lo = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_v2i*)(stg + stg_read_off(lane, 0)));
    const v2i hi = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_v2i*)(stg + stg_read_off(lane, 1)));
    return (v4i){lo[0], lo[1], hi[0], hi[1]};
  }
}

// K::TR16: the lane's row goes to row lane of the image (lane_xoff's map)
template <class K>
__device__ __forceinline__ v4i stage_block(v4i raw, int8_t* stg, int lane) {
  wave_sync_lds();  // the previous block's reads precede this store
  *(v4i*)(stg + 16 * (K::TR16 ? lane : stg_pos(lane))) = raw;
  wave_sync_lds();
  return staged_tr<K>(stg, lane);
}

// LDS-DMA (channel-major ring, K::DMA): buffer_load_dwordx4 ... lds writes lane L's 16 bytes from
// voff + soff of the buffer to LDS byte m0 + 16 L (lane-linear; byte-unaligned sources and a dword
// straddling num_records, which lands as zeros, were checked on gfx950 by tools/tr8_probe.hip).
// Inline asm, not __builtin_amdgcn_raw_ptr_buffer_load_lds: with the builtin the compiler makes
// every __syncthreads() wait for the DMA (s_waitcnt vmcnt(0) before s_barrier), which would drain
// the trial-ahead fill at barrier A.  So the waits are explicit: layer1 waits vmcnt(0) before it
// reads the ring, and the fill waits lgkmcnt(0) (the ring's reads done) before it is issued.  The
// compiler's own vmcnt counts stay safe: a wait for one of its loads only ever waits longer when
// DMA loads it does not know about are in flight (in-order completion).
__device__ __forceinline__ unsigned lds_addr(const int8_t* p) {
  return (unsigned)(size_t)(const __attribute__((address_space(3))) int8_t*)p;
}
__device__ __forceinline__ void dma_b128(Rsrc r, int voff, int soff, unsigned lds) {
  // m0 (the LDS base) goes in through an "{m0}" operand: the compiler writes it and knows the asm
  // reads it, so no value of its own can be kept in m0 across the load
  asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds"
               :: "v"(voff), "s"(r), "s"(soff), "{m0}"(__builtin_amdgcn_readfirstlane(lds)) : "memory");
}

// Whole-row exchange (K::RX).  Load (m, ph) of wave w: lane L = (h, k) = (L >> 5, L & 31) reads bytes
// 512 ph + 16 k of channel row c = w + 8 h + 16 m.  In the phase image, row c's 16-byte chunk k sits
// at 512 c + 16 (k ^ rx_swz(c)): the 16 channels a 32-lane half of a transposed read takes
// (c & 7 and bit 4 of c) then fall on 16 distinct chunk positions mod 256 bytes (conflict-free),
// and a store's 8-lane groups still write 128 contiguous bytes.
__device__ __forceinline__ int rx_swz(int c) { return (c & 7) | ((c >> 1) & 8); }
template <class K>
__device__ __forceinline__ int rx_lane_off(int lane, int wave) {
  return (wave + 8 * (lane >> 5)) * K::T + 16 * (lane & 31);
}
// phase ph of the wave's rows (R.pf[4 ph + m]) into the image
template <class K>
__device__ __forceinline__ void rx_store(const Regs<K>& R, int ph, int8_t* img, int lane, int wave) {
  asm volatile("" : "+v"(lane));  // addresses recomputed per store (registers across the loop spill)
  const int h = lane >> 5, k = lane & 31;
  wave_sync_lds();
#pragma unroll
  for (int m = 0; m < 4; m++) {
    const int c = wave + 8 * h + 16 * m;
    *(v4i*)(img + 512 * c + 16 * (k ^ rx_swz(c))) = R.pf[4 * ph + m];
  }
}
// the A fragment of local block bl (16 samples, chunk bl) of the phase image: lane (i, g)'s read r
// takes channels 16 g + 8 r + q (q = i >> 1), bytes 8 (i & 1) of the chunk
__device__ __forceinline__ v4i rx_frag(const int8_t* img, int lane, int bl) {
  typedef int v2i __attribute__((ext_vector_type(2)));
  typedef __attribute__((address_space(3))) v2i lds_v2i;
  const int i = lane & 15, g = lane >> 4;
  v2i v[2];
#pragma unroll
  for (int r = 0; r < 2; r++) {
    const int c = 16 * g + 8 * r + (i >> 1);
    v[r] = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_v2i*)(img + 512 * c + 16 * (bl ^ rx_swz(c)) + 8 * (i & 1)));
  }
  return (v4i){v[0][0], v[0][1], v[1][0], v[1][1]};
}

// Float input, HBM traffic (float input; pmc_traffic.json b22_f32).  Float rows are
// not 128-byte aligned, so a cache line at a border between two blocks holds bytes of both.  With
// every wave walking forward, the next wave's first block was requested a trial ahead while this
// wave's last block arrived at the end of layer 1, and each such line came from HBM twice (1.23x).
// So odd waves walk their blocks backwards (both sides of every wave border are read in the same
// phase of the trial: 1.231x -> 1.089x), and a wave requests its first block at the start of its
// own layer 1, with no trial-ahead request (1.022x, -8.1 % time in two same-box steps,
// tools/ab.py --f32, profiles/r04_ab.txt): the other waves cover the first block's latency, and
// the wave's registers stay free through layers 2-5.
// float input (K::FQ): 16-byte piece m of the lane's 64 bytes of block slot i
template <class K>
__device__ __forceinline__ v4i load_f(Rsrc r, int xoff, int i, int m) {
  return (v4i)__builtin_amdgcn_raw_buffer_load_b128(r, xoff + 64 * K::P * i + 16 * m, 0, 0);
}

// LDS slots of wave `wave` filled by LDS-DMA (K::DMA: the channel-major ring; K::LDMA: the plain
// build's blocks past PF)
template <class K>
__device__ __forceinline__ int8_t* ring_base(int8_t* smem, int wave) {
  return smem + K::OFF_STG + wave * (K::DMA ? K::RS : K::NLD) * 1024;
}

template <class K>
__device__ __forceinline__ void prefetch_l1(Rsrc r, Regs<K>& R, int lane = 0, int wave = 0,
                                            int8_t* smem = nullptr) {
  int8_t* ring = (K::DMA || K::LDMA) ? ring_base<K>(smem, wave) : nullptr;
  // laundered: otherwise xoff + 16 GS i is hoisted out of the trial loop into a register per slot
  // instead of riding in the loads' immediate offsets
  int xo = R.xoff;
  asm volatile("" : "+v"(xo));
  if constexpr (K::DMA) {
    // ring slots 0 .. RS - 1 by LDS-DMA (the first trial of a workgroup; layer1 refills each slot
    // for the next trial).  The wait keeps a DMA write from racing an LDS access still queued.
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const unsigned rb = lds_addr(ring);
    const int n = l1_count<K>(wave);  // slots past the wave's blocks stay unfilled (wave-uniform)
#pragma unroll
    for (int i = 0; i < K::RS; i++)
      if (i < n) dma_b128(r, xo, 16 * K::P * i, rb + 1024 * i);
    return;
  }
  if constexpr (K::FQ) {  // the first block's four pieces
#pragma unroll
    for (int m = 0; m < 4; m++) R.pf[m] = load_f<K>(r, xo, R.fq0, m);
    return;
  }
  if constexpr (K::RX) {
    int ln = lane;  // the row offset recomputed per trial (a register across the loop spills)
    asm volatile("" : "+v"(ln));
    const int xr = rx_lane_off<K>(ln, wave);
#pragma unroll
    for (int ph = 0; ph < K::NPH; ph++)
#pragma unroll
      for (int m = 0; m < 4; m++)
        R.pf[4 * ph + m] = (v4i)__builtin_amdgcn_raw_buffer_load_b128(r, xr, 16 * m * K::T + 512 * ph, 0);
    return;
  }
  if constexpr (K::LDMA) {
    // issued before the VGPR loads: the compiler's vmcnt waits for those then also cover these
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slots' reads of this trial have returned
    const unsigned rb = lds_addr(ring);
#pragma unroll
    for (int i = 0; i < K::NLD; i++) dma_b128(r, xo + (K::PF + i) * 16 * K::GS, 0, rb + 1024 * i);
  }
#pragma unroll
  for (int i = 0; i < K::PF; i++) R.pf[i] = load_a<K>(r, xo, i);
}

template <class K>
__device__ __forceinline__ void setup(const DevParams* __restrict__ prm, int8_t* smem, Regs<K>& R,
                                      int tid, int wave, int lane) {
#pragma unroll
  for (int t = 0; t < K::P; t++) {
    L1Tile& T = R.tile(t);
    R.xoff = lane_xoff<K>(lane, wave);
    T.wf = K::CT ? prm->l1_wfrag_ct[t][lane] : prm->l1_wfrag[t][lane];
    T.ci = prm->l1_cinit[t][lane & 15];
    if constexpr (K::XR) {
      T.xm = prm->l1_m[t][lane & 15];
      T.xs = prm->l1_xs[t][lane & 15];
    } else {
      T.rr = prm->l1_r[t][lane & 15];
      T.cc = prm->l1_c[t][lane & 15];
    }
  }
#pragma unroll
  for (int fi = 0; fi < FPW; fi++) {
    const int f = wave * FPW + fi;
#pragma unroll
    for (int s = 0; s < 3; s++) R.af[fi][s] = prm->l2_afrag[f][s][lane];
    if constexpr (K::RB) {
      R.thr2[fi] = prm->l2_thrb[f];
      R.off2[fi] = prm->l2_offm[f];
      if constexpr (K::XR) R.m2[fi] = prm->l2_m[f];
      else R.r2[fi] = prm->l2_r[f];
    } else {
      R.thr2[fi] = prm->sp.l2n_ci[f];
      R.off2[fi] = __float_as_int(prm->sp.l2n_c[f]);
      if constexpr (K::XR) R.m2[fi] = prm->sp.l2n_m[f];
      else R.r2[fi] = prm->sp.l2n_r[f];
    }
    if constexpr (K::XR) R.xs2[fi] = prm->sp.l2_xs[f];
  }
  R.fq0 = (wave & 1) ? l1_count<K>(wave) - 1 : 0;
  R.a31 = prm->l3_a1[wave][lane];
  R.a32 = prm->l3_a2[wave][lane];
  R.r3 = prm->sp.l3_r;
  R.c3 = prm->sp.l3_c;
  // small parameters -> LDS
  const v4i* src = (const v4i*)&prm->sp;
  v4i* dst = (v4i*)(smem + K::OFF_SP);
  for (int i = tid; i < (int)(sizeof(SmallParams) / 16); i += NTHREADS) dst[i] = src[i];
  if (tid < 64) ((LaneTab*)(smem + K::OFF_LT))[tid] = build_lane_tab<K>(tid);
  if (tid < 64) ((L45Tab*)(smem + K::OFF_L45))[tid] = build_l45_tab<K>(tid);
  if constexpr (K::L2TV) {
#pragma unroll
    for (int s = 0; s < 3; s++) R.l2t[s] = prm->l2t_afrag[wave][s][lane];
  } else if constexpr (K::TB > 0) {
    const v4i* t = &prm->l2t_afrag[0][0][0];
    v4i* d = (v4i*)(smem + K::OFF_L2T);
    for (int i = tid; i < NWAVES * 3 * 64; i += NTHREADS) d[i] = t[i];
  }
  // everything else zero: layer-1 pads (positions [0,32) and past the last block), layer-2 pads
  // ([0,8) and [8+T8, Y2ROW)) and the zero row are never rewritten
  v4i* z = (v4i*)smem;
  for (int i = tid; i < K::OFF_SP / 16; i += NTHREADS) z[i] = (v4i){0, 0, 0, 0};
  if constexpr (K::DMA) {
    // the wave's own ring slots (rows that no lane fills, C = 22: K-slots 44..63, stay zero either
    // way); the wave's first fill waits for these stores (prefetch_l1)
    v4i* rz = (v4i*)(smem + K::OFF_STG + wave * K::RS * 1024);
    for (int i = lane; i < K::RS * 64; i += 64) rz[i] = (v4i){0, 0, 0, 0};
  }
}

// ---- layer 1 ---------------------------------------------------------------------------------
// One layer-1 block: 16 time groups x 16 filters (P == 2: two N-tiles of 8 filters x 2 parities).
// MAYBE_LAST: the block may be the trial's last one (samples >= T are masked to zero).
template <class K, bool MAYBE_LAST>
__device__ __forceinline__ void l1_block(v4i a, int blk, int8_t* smem_y1, const Regs<K>& R, int lane) {
  const int j = lane & 15, g = lane >> 4;
  v4i accs[K::P];
#pragma unroll
  for (int t = 0; t < K::P; t++) {  // both N-tiles' MFMAs before either requant
    const L1Tile& T = R.tile(t);
    // XR: the inline constant 0, the offset added before the division (a register C-init tuple
    // per tile did not stay resident beside the division's double temporaries, and its rebuild
    // inside the loop is the pattern tools/cinit_scan.py forbids)
    const int ci = K::XR ? 0 : T.ci;
    accs[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, T.wf, (v4i){ci, ci, ci, ci}, 0, 0, 0);
  }
#pragma unroll
  for (int t = 0; t < K::P; t++) {
    const L1Tile& T = R.tile(t);
    const v4i acc = accs[t];
    // lane column j = (filter 8t + j/2, parity or half j&1) when P == 2, filter j when P == 1.
    // Row 4g + r: time-major, time group 16 blk + 4g + r (its sample p when P == 2: stride 2);
    // channel-major P == 2: sample 32 blk + 16 p + 4g + r (consecutive).
    const int p = (K::P == 2) ? (j & 1) : 0;
    const int f = (K::P == 2) ? 8 * t + (j >> 1) : j;
    const int t0 = K::PSPLIT ? 2 * (16 * blk + 4 * g) + p : K::P == 2 ? 32 * blk + 16 * p + 4 * g : 16 * blk + 4 * g;
    constexpr int SS = K::PL;  // sample stride of the lane's 4 outputs
    int y[4];
    if constexpr (K::XR) {  // acc = dot (C-init 0): exact division of dot + off
#pragma unroll
      for (int r = 0; r < 4; r++) y[r] = xdiv(acc[r] + T.ci, T.xm, T.xs);
    } else {
      // acc bits = 1.5*2^23 + (dot + off) as f32; fma(x, r, -1.5*2^23*r) == RN((dot+off)*r)
      const f2 q01 = fma2(acc[0], acc[1], T.rr, T.cc);
      const f2 q23 = fma2(acc[2], acc[3], T.rr, T.cc);
      y[0] = (int)q01[0]; y[1] = (int)q01[1]; y[2] = (int)q23[0]; y[3] = (int)q23[1];  // trunc toward zero
    }
    if constexpr (MAYBE_LAST) {
#pragma unroll
      for (int r = 0; r < 4; r++) y[r] = (t0 + SS * r < K::T) ? y[r] : 0;
    }
    *(unsigned*)(smem_y1 + y1_index<K>(f, t0)) = sat8x4<K::LO>(y[0], y[1], y[2], y[3]);
  }
}

// Layer 1: x[T][C] (HBM, via R.pf) -> y1 rows (LDS, position 32 + t).  Prefetches the next
// trial's fragments (rnext) into R.pf once the current ones are consumed.
// Float input (K::FQ): 4 float32 samples (raw bits) -> 4 int8 bytes, the reference's input
// quantisation (gen_input_header.py:66-76, functional.py:308-334: x / s, clip to [-1, 1], * 254 / 2,
// truncate; each step rounded in float32), the same function as quant::quantize_one<float>.  The
// correctly rounded quotient RN(x / s) comes from Markstein's correction instead of the division
// sequence: q0 = RN(x y) with y = RN(1 / s) (host), r = x - q0 s exactly (fma), RN(q0 + r y) =
// RN(x / s) (y within half an ulp of 1 / s and q0 within one ulp of x / s).  x is first clamped to
// [-s, s]: RN is monotone, so RN(x / s) then lies in [-1, 1] and the reference's clip has nothing
// left to do (|x| > s gives RN(x / s) beyond +-1 and clips to +-1; the clamped x = +-s gives exactly
// +-1).  NaN clamps to -s (fmaxf), as in the two-pass quantiser.  q * 127 is then within
// [-127, 127], so its truncation needs no saturation and goes straight into its byte of the packed
// word (SDWA byte destination).  Checked against the two-pass quantiser on every float32 bit
// pattern for several scales (tests/test_gpu_f32.py).
__device__ __forceinline__ float quantize1_f(float x, float s, float y) {
  x = fminf(fmaxf(x, -s), s);
  const float q0 = x * y;
  const float r = __builtin_fmaf(-q0, s, x);
  return __builtin_fmaf(r, y, q0) * 127.0f;
}

__device__ __forceinline__ unsigned quantize4(v4i f, float s, float y) {
  // v_cvt_i32_f32 truncates toward zero; the byte destination keeps the low 8 bits (the int8 value,
  // as |q * 127| <= 127) and leaves the word's other bytes as they are
  unsigned w;
  asm("v_cvt_i32_f32_sdwa %0, %1 dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD"
      : "=v"(w) : "v"(quantize1_f(__int_as_float(f[0]), s, y)));
  asm("v_cvt_i32_f32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD"
      : "+v"(w) : "v"(quantize1_f(__int_as_float(f[1]), s, y)));
  asm("v_cvt_i32_f32_sdwa %0, %1 dst_sel:BYTE_2 dst_unused:UNUSED_PRESERVE src0_sel:DWORD"
      : "+v"(w) : "v"(quantize1_f(__int_as_float(f[2]), s, y)));
  asm("v_cvt_i32_f32_sdwa %0, %1 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:DWORD"
      : "+v"(w) : "v"(quantize1_f(__int_as_float(f[3]), s, y)));
  return w;
}

// test hook (mibminet_test_quantize_f32): the in-kernel quantiser on a flat array, four elements
// at a time through quantize4, the instruction sequence the forward kernel runs (elements past n
// in the last group are quantised as 0.0f and not stored)
__global__ void k_quantize_flat(const float* __restrict__ x, int8_t* __restrict__ q, long long n, float s, float y) {
  for (long long i = 4 * ((long long)blockIdx.x * blockDim.x + threadIdx.x); i < n;
       i += 4 * (long long)gridDim.x * blockDim.x) {
    v4i f;
#pragma unroll
    for (int j = 0; j < 4; j++) f[j] = i + j < n ? __float_as_int(x[i + j]) : 0;
    const unsigned w = quantize4(f, s, y);
#pragma unroll
    for (int j = 0; j < 4; j++)
      if (i + j < n) q[i + j] = (int8_t)(w >> (8 * j));
  }
}

template <class K>
__device__ __forceinline__ void layer1(Rsrc rcur, Rsrc rnext, int8_t* smem_y1, Regs<K>& R, int wave, int lane,
                                       bool last_trial = false) {
  if constexpr (K::FQ) {
    // float32 rows: the lane's 16 samples of a block are 64 bytes (4 loads), quantised to the
    // 16 int8 bytes the channel-major staging takes.  Block 0 is requested here (R.pf); block
    // i + 1 is loaded while block i is quantised and computed.
    const int n = l1_count<K>(wave);
    int8_t* stg = smem_y1 - K::OFF_Y1 + K::OFF_STG + wave * K::STG;
    prefetch_l1<K>(rcur, R);  // no trial-ahead request: the first block now
    v4i cur[4] = {R.pf[0], R.pf[1], R.pf[2], R.pf[3]};
    // odd waves walk their blocks backwards (slot n - 1 first), so that both sides of every wave
    // border are read in the same phase of the trial (float input)
    const bool back = wave & 1;
    // (a branch-free copy for waves with all NBW blocks, as in the channel-major int8 paths,
    // measured +2.7 % here: not kept)
#pragma unroll
    for (int i = 0; i < K::NBW; i++) {
      if (i < n) {  // wave-uniform
        const int blk = l1_blk<K>(wave, back ? n - 1 - i : i);
        v4i nxt[4] = {cur[0], cur[1], cur[2], cur[3]};
        if (i + 1 < n)
#pragma unroll
          for (int m = 0; m < 4; m++) nxt[m] = load_f<K>(rcur, R.xoff, back ? n - 2 - i : i + 1, m);
        v4i raw;
#pragma unroll
        for (int m = 0; m < 4; m++) raw[m] = (int)quantize4(cur[m], R.qs, R.qy);
        const v4i a = stage_block<K>(raw, stg, lane);
        if (blk == K::NB1 - 1) {
          l1_block<K, true>(a, blk, smem_y1, R, lane);
        } else {
          l1_block<K, false>(a, blk, smem_y1, R, lane);
        }
#pragma unroll
        for (int m = 0; m < 4; m++) cur[m] = nxt[m];
      }
    }
    return;
  }
  if constexpr (K::DMA) {
    // Channel-major through the LDS-DMA ring: slots 0 .. RS - 1 hold blocks 0 .. RS - 1, filled a
    // trial ahead (the first trial by prefetch_l1; after that, slot i during the previous trial's
    // layer 1, right after block i's MFMAs).  Block i + 1's fragment is read before block i's MFMAs
    // and requant.
    const int n = l1_count<K>(wave);
    int8_t* ring = smem_y1 - K::OFF_Y1 + K::OFF_STG + wave * K::RS * 1024;
    // this trial's fill has landed.  Issued after it on the last wave: the previous trial's logits
    // store, which need not complete (a vmcnt(0) there waited for that store's write
    // acknowledgement on the critical last wave: +1,200 cycles per trial)
    static_assert(K::PFV == 0, "no VGPR loads behind the ring fill");
    if (wave == NWAVES - 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (last_trial) {
      // the batch's last trial: its view ends at its last byte, so the one dword straddling that
      // end landed as zeros; the lane holding it patches the 1-3 real bytes in (byte loads and
      // stores, once per launch)
      constexpr int N = K::C * K::T;
#pragma unroll
      for (int i = 0; i < K::RS; i++) {
        const int o = R.xoff + 16 * K::P * i;
        if (i < n && l1_blk<K>(wave, i) == K::NB1 - 1 && o < N && N < o + 16 && ((N - o) & 3)) {
          const int k0 = (N - o) & ~3;
          for (int m = 0; o + k0 + m < N; m++)
            ring[1024 * i + 16 * lane + k0 + m] = (int8_t)__builtin_amdgcn_raw_buffer_load_b8(rcur, o + k0 + m, 0, 0);
        }
      }
      wave_sync_lds();
    }
    // FULL: the wave has all NBW blocks (config B: waves 0-6), so the blocks run straight, with no
    // wave-uniform branches between them (only the last may be the trial's last block); at every
    // such branch the compiler drains the LDS counter (lgkmcnt(0)), exposing the reads' latency.
    // (Reading the fragments 2 or 3 blocks ahead measured slower: DESIGN.md §3.)
    auto blocks = [&](auto full) {
      constexpr bool F = decltype(full)::value;
      v4i fr;
      if (F || 0 < n) fr = staged_tr<K>(ring, lane);
#pragma unroll
      for (int i = 0; i < K::NBW; i++) {
        if (F || i < n) {  // wave-uniform
          const int blk = l1_blk<K>(wave, i);
          const v4i a = fr;
          if (F ? i + 1 < K::NBW : i + 1 < n) fr = staged_tr<K>(ring + 1024 * (i + 1), lane);
          if ((!F || i == K::NBW - 1) && blk == K::NB1 - 1) {  // a wave's blocks are contiguous
            l1_block<K, true>(a, blk, smem_y1, R, lane);
          } else {
            l1_block<K, false>(a, blk, smem_y1, R, lane);
          }
          // slot i's fragment is in registers (its MFMAs read it): refill the slot with the next
          // trial's block i now, while the TA is idle, instead of all five fills after barrier A,
          // where the waves' fills queue behind one another (same box: -2.5 %; before barrier B:
          // +8.0 %)
          int xo = R.xoff;
          asm volatile("" : "+v"(xo));
          dma_b128(rnext, xo, 16 * K::P * i, lds_addr(ring) + 1024 * i);
        }
      }
    };
    if (n == K::NBW) blocks(BoolC<true>{});
    else blocks(BoolC<false>{});
    return;
  }
  constexpr int NX = K::NBW - K::PF;  // blocks not prefetched: load now (or from the LDS slots), consumed last
  v4i xa[NX > 0 ? NX : 1];
  if constexpr (K::LDMA) {
    // the slots were filled before this trial's VGPR prefetch was issued: once all but the last PF
    // vector-memory operations are done, so are the fills (in-order completion)
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(K::PF) : "memory");
    const int8_t* ring = smem_y1 - K::OFF_Y1 + K::OFF_STG + wave * K::NLD * 1024;
#pragma unroll
    for (int i = 0; i < NX; i++) xa[i] = *(const v4i*)(ring + 1024 * i + 16 * lane);
  } else {
#pragma unroll
    for (int i = 0; i < NX; i++) xa[i] = load_a<K>(rcur, R.xoff, K::PF + i);
  }
  const int n = l1_count<K>(wave);
  int8_t* stg = smem_y1 - K::OFF_Y1 + K::OFF_STG + wave * K::STG;  // channel-major staging
  if constexpr (K::RX) {
    // whole-row exchange: phase 0 of this trial was stored before the previous trial's barrier B
    // (k_forward); each further phase: barrier (the image consumed), store, barrier (complete).
    // Waves 0-6 split each phase's blocks; the last wave (layers 4-5) has none.
    int8_t* img = smem_y1 - K::OFF_Y1 + K::OFF_STG;
    static_assert(K::NPH >= 1 && K::NPH <= 2, "one or two image phases (T <= 1024)");
    auto phase = [&](auto PH) {
      constexpr int ph = decltype(PH)::value;
      if constexpr (ph > 0) {
        __syncthreads();
        rx_store<K>(R, ph, img, lane, wave);
        __syncthreads();
      }
      constexpr int NBP = cmin(32, K::NB1 - 32 * ph), BASE = NBP / (NWAVES - 1), REM = NBP % (NWAVES - 1);
      constexpr int MAXP = BASE + (REM ? 1 : 0);
      const int cnt = wave < NWAVES - 1 ? BASE + (wave < REM) : 0;
      const int lo = wave * BASE + min(wave, REM);
      auto frag = [&](int j) {
        int ln = lane;  // read offsets recomputed per block (hoisted, they hold 2 MAXP registers)
        asm volatile("" : "+v"(ln));
        return rx_frag(img, ln, lo + j);
      };
      // FULL: waves with MAXP blocks in this phase run them without branches
      auto blocks = [&](auto full) {
        constexpr bool F = decltype(full)::value;
        v4i an = frag(0);
#pragma unroll
        for (int j = 0; j < MAXP; j++) {
          if (F || j < cnt) {  // wave-uniform
            const int blk = 32 * ph + lo + j;
            const v4i a = an;
            if (F ? j + 1 < MAXP : j + 1 < cnt) an = frag(j + 1);
            if ((!F || j == MAXP - 1) && blk == K::NB1 - 1) l1_block<K, true>(a, blk, smem_y1, R, lane);
            else l1_block<K, false>(a, blk, smem_y1, R, lane);
          }
        }
      };
      if (cnt > 0) {
        if (cnt == MAXP) blocks(BoolC<true>{});
        else blocks(BoolC<false>{});
      }
    };
    phase(IntC<0>{});
    if constexpr (K::NPH > 1) phase(IntC<1>{});
    // (issued after barrier A instead: C -0.3 %, 64x480 +1.9 %; the image store before barrier B
    // then waits on loads with less lead)
    prefetch_l1<K>(rnext, R, lane, wave);
    return;
  }
  if constexpr (K::CT) {
    // single-block staging (64 channels, plain BN): block i + 1 is staged (store + transposed
    // reads) before block i's MFMAs and requant, so the LDS round trip of the staging overlaps the
    // previous block's work (two staging areas)
    auto raw = [&](int i) -> v4i {
      v4i a = (i < K::PF) ? R.pf[i < K::PF ? i : 0] : xa[i >= K::PF ? i - K::PF : 0];
      if (last_trial && l1_blk<K>(wave, i) == K::NB1 - 1) a = ct_tail<K>(a, rcur, R.xoff + 16 * K::P * i);
      return a;
    };
    // FULL: waves with all NBW blocks run them without wave-uniform branches, as in the DMA path
    auto blocks = [&](auto full) {
      constexpr bool F = decltype(full)::value;
      v4i an = stage_block<K>(raw(0), stg, lane);
#pragma unroll
      for (int i = 0; i < K::NBW; i++) {
        if (F || i < n) {  // wave-uniform
          const int blk = l1_blk<K>(wave, i);
          const v4i a = an;
          if (F ? i + 1 < K::NBW : i + 1 < n) an = stage_block<K>(raw(i + 1), stg + 1024 * ((i + 1) & 1), lane);
          if ((!F || i == K::NBW - 1) && blk == K::NB1 - 1) {  // a wave's blocks are contiguous
            l1_block<K, true>(a, blk, smem_y1, R, lane);
          } else {
            l1_block<K, false>(a, blk, smem_y1, R, lane);
          }
        }
      }
    };
    if (n == K::NBW) blocks(BoolC<true>{});
    else blocks(BoolC<false>{});
    prefetch_l1<K>(rnext, R);
    return;
  }
#pragma unroll
  for (int i = 0; i < K::NBW; i++) {
    if (i < n) {  // wave-uniform
      const int blk = l1_blk<K>(wave, i);
      const v4i a = (i < K::PF) ? R.pf[i < K::PF ? i : 0] : xa[i >= K::PF ? i - K::PF : 0];
      if (blk == K::NB1 - 1) {  // the trial's last block: samples >= T are masked
        l1_block<K, true>(a, blk, smem_y1, R, lane);
      } else {
        l1_block<K, false>(a, blk, smem_y1, R, lane);
      }
    }
  }
  prefetch_l1<K>(rnext, R, lane, wave, smem_y1 - K::OFF_Y1);
}

// ---- layer 2 ---------------------------------------------------------------------------------
// Plain (non-REORDER_BN) branch, layer2.c:139-210: each element requantised and clipped
// (func_xcorr_scale -> transform.c:224), ReLU, sum of 8, >> 3.  Behind the ReLU, trunc equals
// floor, so each element is the floor form of mibminet.hip (choose_floor_form): acc holds the float
// bits of M + x (C-init = per-filter magic + offset) and fma(bits, r, c) = FMAGIC + floor(x / f) on
// every reachable x (host-verified); fmed3 to [FMAGIC, FMAGIC + 127] is the clip and the ReLU, and
// the bits of FMAGIC + e are FMAGIC_I + e, so a window's sum is its bits' integer sum minus
// 8 FMAGIC_I (mod 2^32).  No float->int convert per element.
template <int EMAX>
__device__ __forceinline__ f2 floor_form2(int a, int b, float r, float c) {
  const f2 q = __builtin_elementwise_fma((f2){__int_as_float(a), __int_as_float(b)}, (f2){r, r}, (f2){c, c});
  constexpr float HI = FMAGIC_F + (float)EMAX;
  return (f2){__builtin_amdgcn_fmed3f(q[0], FMAGIC_F, HI), __builtin_amdgcn_fmed3f(q[1], FMAGIC_F, HI)};
}

// sum of the eight floor-form elements acc[BASE .. BASE + 7] (e in [0, EMAX] each)
template <int BASE, int EMAX>
__device__ __forceinline__ unsigned floor_sum8(const v16i& acc, float r, float c) {
  unsigned e[8];
#pragma unroll
  for (int i = 0; i < 8; i += 2) {
    const f2 q = floor_form2<EMAX>(acc[BASE + i], acc[BASE + i + 1], r, c);
    e[i] = (unsigned)__float_as_int(q[0]);
    e[i + 1] = (unsigned)__float_as_int(q[1]);
  }
  return ((e[0] + e[1] + e[2]) + (e[3] + e[4]) + (e[5] + e[6])) + (e[7] - 8u * (unsigned)FMAGIC_I);
}

// Plain layer 4's elements have no clip in the reference, only the ReLU: e = max(q, 0) is one
// full-rate saturating subtract of the floor form's bits, bits(FMAGIC + q) - FMAGIC_I clamped at 0,
// where layer 2 needs the two-sided fmed3.  The host verifies the form exactly up to the step q = 1024;
// past it the form is monotone, so a larger element still reads >= 1024, and any element >= 1016
// already saturates the window's result (sum >> 3 >= 127).  Eight elements below 2^22 sum below 2^25.
template <int BASE>
__device__ __forceinline__ unsigned relu_sum8(const v16i& acc, float r, float c) {
  unsigned e[8];
#pragma unroll
  for (int i = 0; i < 8; i += 2) {
    const f2 q = __builtin_elementwise_fma((f2){__int_as_float(acc[BASE + i]), __int_as_float(acc[BASE + i + 1])},
                                           (f2){r, r}, (f2){c, c});
    e[i] = __builtin_elementwise_sub_sat(__float_as_uint(q[0]), (unsigned)FMAGIC_I);
    e[i + 1] = __builtin_elementwise_sub_sat(__float_as_uint(q[1]), (unsigned)FMAGIC_I);
  }
  return ((e[0] + e[1] + e[2]) + (e[3] + e[4])) + ((e[5] + e[6]) + e[7]);
}

__device__ __forceinline__ unsigned l2n_out(const v16i& acc, float r, float c) {
  const unsigned s0 = floor_sum8<0, 127>(acc, r, c), s1 = floor_sum8<8, 127>(acc, r, c);
  return (s0 >> 3) | ((s1 >> 3) << 8);
}

// XR: one plain-branch element, exactly: clamp(trunc(x / fac), 0, EMAX) (acc = x with C-init = the
// offset; the ReLU makes the lower clip bound 0)
template <int EMAX>
__device__ __forceinline__ int xelem(int x, unsigned m, int xs) {
  return min(max(xdiv(x, m, xs), 0), EMAX);
}
template <int BASE, int EMAX>
__device__ __forceinline__ int xelem_sum8(const v16i& acc, unsigned m, int xs) {
  int e[8];
#pragma unroll
  for (int i = 0; i < 8; i++) e[i] = xelem<EMAX>(acc[BASE + i], m, xs);
  return ((e[0] + e[1]) + (e[2] + e[3])) + ((e[4] + e[5]) + (e[6] + e[7]));
}

// Pooled + requantised pair of layer-2 outputs of one lane: bytes [y(u0), y(u0+1)].  rm: the
// reciprocal, or (XR) the xdiv magic.
template <int LO, bool XR>
__device__ __forceinline__ unsigned l2_out(const v16i& acc, int thr, int off, std::conditional_t<XR, unsigned, float> rm,
                                           int xs) {
  if constexpr (XR) {
    return sat8x2<LO>(xdiv(pool8b<0>(acc, thr, off), rm, xs), xdiv(pool8b<8>(acc, thr, off), rm, xs));
  } else {
    const float r = rm;
    const f2 q = mul2((float)pool8b<0>(acc, thr, off), (float)pool8b<8>(acc, thr, off), r);
    return sat8x2<LO>((int)q[0], (int)q[1]);
  }
}

// Layer-2 tail: outputs 1024 MT + 16 bq + m (m < 16) of the wave's two filters, one column of 16
// outputs per lane column col = TC fi + bq (filter fi).  One chain of three MFMA i32_16x16x64_i8
// with a block-diagonal K: K-slots 0..95 carry filter 0's window chunks and band, slots 96..191
// filter 1's (chunk kap = 4 s + g of K-step s and lane group g, see build_lane_tab), and a lane
// whose column belongs to the other filter reads a zero chunk there.  Every column so gets its own
// filter's sums and no MFMA work is thrown away.  D lane (col, g) holds shifts 4g .. 4g+3: half of
// pool window g >> 1; lanes g and g ^ 1 meet by v_permlane16_swap (layer2_tail_out).
template <class K>
__device__ __forceinline__ v4i layer2_tail_mfma(const int8_t* smem_y1, const SmallParams* sp, const LaneTab& T,
                                                const Regs<K>& R, int wave, int lane) {
  const v4i* tA = (const v4i*)(smem_y1 - K::OFF_Y1 + K::OFF_L2T) + wave * 3 * 64 + lane;
  const int8_t* pb = smem_y1 + wave * FPW * K::Y1ROW;
  v4i bv[3], a[3];
#pragma unroll
  for (int st = 0; st < 3; st++) {
    const long* q = (const long*)(pb + T.tb[st]);  // 8-byte aligned
    const long lo = q[0], hi = q[1];
    bv[st][0] = (int)lo; bv[st][1] = (int)(lo >> 32); bv[st][2] = (int)hi; bv[st][3] = (int)(hi >> 32);
    a[st] = K::L2TV ? R.l2t[st] : tA[st * 64];
  }
  const int c0 = K::RB ? PBIAS_TAIL : 0;
  v4i acc = {c0, c0, c0, c0};
#pragma unroll
  for (int st = 0; st < 3; st++) acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[st], bv[st], acc, 0, 0, 0);
  // Operands stay live until the result is ready (see DESIGN.md on the tail chains).
  asm volatile("" : "+v"(acc) : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(bv[0]), "v"(bv[1]), "v"(bv[2]));
  if constexpr (!K::RB) acc += sp->l2n_ci[wave * FPW + T.tp];  // plain branch: magic-offset C-init
  return acc;
}

template <class K>
__device__ __forceinline__ void layer2_tail_out(const v4i tacc, int8_t* smem_y2, const SmallParams* sp,
                                                const LaneTab& T, int wave) {
  const int fcol = wave * FPW + T.tp;
  const v4i tp = K::RB ? sp->l2_tpar[fcol] : (v4i){0, 0, 0, 0};  // {thr + PBIAS_TAIL, offm, r}
  int part;
  if constexpr (K::RB) {
    const int thrb = tp[0];
    part = (int)((relu_b(tacc[0], thrb) + relu_b(tacc[1], thrb)) + (relu_b(tacc[2], thrb) + relu_b(tacc[3], thrb)));
  } else if constexpr (K::XR) {  // exact elements (xelem)
    const unsigned m = sp->l2n_m[fcol];
    const int xs = sp->l2_xs[fcol];
    part = (xelem<127>(tacc[0], m, xs) + xelem<127>(tacc[1], m, xs)) + (xelem<127>(tacc[2], m, xs) + xelem<127>(tacc[3], m, xs));
  } else {
    const float r = sp->l2n_r[fcol], c = sp->l2n_c[fcol];  // floor form (l2n_out)
    const f2 q01 = floor_form2<127>(tacc[0], tacc[1], r, c), q23 = floor_form2<127>(tacc[2], tacc[3], r, c);
    part = (int)(((unsigned)__float_as_int(q01[0]) + (unsigned)__float_as_int(q01[1])) +
                 ((unsigned)__float_as_int(q23[0]) + (unsigned)__float_as_int(q23[1])) - 4u * (unsigned)FMAGIC_I);
  }
  const auto sw = __builtin_amdgcn_permlane16_swap((unsigned)part, (unsigned)part, false, false);
  const int tot = (int)sw[0] + (int)sw[1];  // whole window (rows 2k and 2k+1 hold the same)
  int y;
  if constexpr (K::RB && K::XR) y = min(max(xdiv(tot + tp[1], (unsigned)tp[2], tp[3]), K::LO), 127);
  else if constexpr (K::RB) y = rq<K::LO>(tot + tp[1], __int_as_float(tp[2]));
  else y = tot >> 3;
  if (T.ty >= 0) smem_y2[wave * FPW * K::Y2ROW + T.ty] = (int8_t)y;
}

// Layer 2: y1 rows -> y2 rows (LDS, position 8 + u).  Full tiles of the wave's filters, then the
// tail (layer2_tail).
template <class K>
__device__ __forceinline__ void layer2(const int8_t* smem_y1, int8_t* smem_y2, const SmallParams* sp,
                                       const Regs<K>& R, const LaneTab& T, int wave, int lane) {
  const int c = lane & 31, h = lane >> 5;
#pragma unroll
  for (int mt = 0; mt < K::MT; mt++)
#pragma unroll
    for (int fi = 0; fi < FPW; fi++) {
      const int f = wave * FPW + fi;
      const int8_t* pb = smem_y1 + f * K::Y1ROW + (32 / K::PL) * 32 * mt + T.l2b - l2_boff<K>(0, 0);
      v16i acc;
#pragma unroll
      for (int i = 0; i < 16; i++) acc[i] = K::RB ? pbias(fi) : R.thr2[fi];  // plain branch: C-init
#pragma unroll
      for (int s = 0; s < DIAG_L2_STEPS; s++)
        acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(R.af[fi][s], *(const v4i*)(pb + l2_boff<K>(s, 0)), acc, 0, 0, 0);
      // reg i of this lane = shift 16h + i of block m -> pooled samples u0 (i<8), u0+1 (i>=8)
      unsigned w;
      if constexpr (K::RB) {
        if constexpr (K::XR) w = l2_out<K::LO, true>(acc, R.thr2[fi], R.off2[fi], R.m2[fi], R.xs2[fi]);
        else w = l2_out<K::LO, false>(acc, R.thr2[fi], R.off2[fi], R.r2[fi], 0);
      } else if constexpr (K::XR) {
        const unsigned m = R.m2[fi];
        w = (unsigned)(xelem_sum8<0, 127>(acc, m, R.xs2[fi]) >> 3) | ((unsigned)(xelem_sum8<8, 127>(acc, m, R.xs2[fi]) >> 3) << 8);
      } else {
        w = l2n_out(acc, R.r2[fi], __int_as_float(R.off2[fi]));
        // 64-channel row exchange: both windows are summed on every path (sunk into the last
        // tile's byte-store branch, the second window's sum left accumulator registers unread on
        // the other path while the MFMA still wrote them, and the next layer 1's inline-asm pack
        // reused one: tools/mfma_lint.py, write-after-write; as in layer 4).  Not in the other
        // builds, where the lint finds no such reuse and the pinned order costs 4.4 % (config B).
        if constexpr (K::RX) asm volatile("" ::"v"(w));
      }
      int8_t* dst = smem_y2 + f * K::Y2ROW + 128 * mt + T.l2y;
      if (128 * (mt + 1) <= K::T8) {
        *(unsigned short*)dst = (unsigned short)w;
      } else {
        const int u0 = 4 * (32 * mt + c) + 2 * h;
        if (u0 + 1 < K::T8) *(unsigned short*)dst = (unsigned short)w;
        else if (u0 < K::T8) *dst = (int8_t)w;
      }
    }
  if constexpr (K::TB > 0 && !DIAG_NOTAIL) {
    const v4i tacc = layer2_tail_mfma<K>(smem_y1, sp, T, R, wave, lane);
    layer2_tail_out<K>(tacc, smem_y2, sp, T, wave);
  }
}

// ---- layer 3 ---------------------------------------------------------------------------------
// 16-tap depthwise conv (layer3.c:49-79, conv.c:105): output u of filter f reads y2 row bytes
// u+1 .. u+16 (pad 7, stored at +8), A[r][k] = tap[k - r - 1] over a 32-byte window.  The wave's
// two filters share MFMA i32_16x16x64_i8 tiles with a block-diagonal K (slots 0..31 filter 0's
// window and band, 32..63 filter 1's; a lane whose K half belongs to the other filter reads the
// zero chunk):
//   tile 1: columns 0..7 = filter 0's blocks of 16 outputs, 8..15 = filter 1's (the first 128
//           outputs of each; D lane (col, g) holds outputs 16 (col & 7) + 4g .. +3);
//   tile 2: the L3R outputs past 128 (T8 = 140: 12), four per column: A rows 4g carry shift g and
//           the other rows are zero, so only register 0 holds results and only it is requantised.
// The two filters' bytes of one output are adjacent in y3t[u][f]: after requant a lane trades its
// four bytes with the partner lane col ^ 8 (DPP row_ror:8) and stores two rows as 2-byte pairs.
template <class K>
__device__ __forceinline__ void layer3(const int8_t* smem_y2, int8_t* smem_y3, const SmallParams* sp,
                                       const Regs<K>& R, const LaneTab& T, int wave) {
  const float r3 = R.r3, c3 = R.c3;  // wave-uniform (SGPRs): no LDS read per trial
  const int8_t* y2w = smem_y2 + wave * FPW * K::Y2ROW;
  // C-init = float magic: acc bits = 1.5 * 2^23 + dot as f32, fma(bits, r, c) == RN(dot * r)
  const v4i magic = {FMAGIC_I, FMAGIC_I, FMAGIC_I, FMAGIC_I};
  const v4i acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(R.a31, *(const v4i*)(y2w + T.l3b), magic, 0, 0, 0);
  v4i acc2 = magic, b2 = magic;
  constexpr bool T2 = K::L3RC > 0;
  if constexpr (T2) {
    const int* p = (const int*)(y2w + T.l3b2);  // 4-byte aligned
    b2 = (v4i){p[0], p[1], p[2], p[3]};
    acc2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(R.a32, b2, magic, 0, 0, 0);
  }
  const f2 q01 = fma2<true>(acc[0], acc[1], r3, c3);
  const f2 q23 = fma2<true>(acc[2], acc[3], r3, c3);
  const unsigned w = sat8x4_b<K::LO>((int)q01[0], (int)q01[1], (int)q23[0], (int)q23[1]);
  const unsigned wp = (unsigned)__builtin_amdgcn_mov_dpp((int)w, 0x128, 0xF, 0xF, false);  // row_ror:8
  const unsigned pr = __builtin_amdgcn_perm(wp, w, (unsigned)T.l3s);  // (f0, f1) pairs of rows r0, r0+1
  // rows u .. u+3 (u = 16 col + 4 g) share the skew.  Tile 1 writes whole blocks of 16 rows, so
  // rows T8 .. 16 L3C - 1 are written too when T8 < 16 L3C (64 x 1000: 125..127, 64 x 480: 60..63):
  // layer 4 multiplies rows >= T8 only into its discarded outputs (v >= T64).  Tile 2 stores only
  // rows < T8 (LaneTab::l3w2).
  if (T.l3w >= 0) {
    int8_t* dst = smem_y3 + T.l3w + FPW * wave;
    *(unsigned short*)dst = (unsigned short)pr;
    *(unsigned short*)(dst + K::Y3S) = (unsigned short)(pr >> 16);
  }
  if constexpr (T2) {
    const int y = min(max((int)__builtin_fmaf(__int_as_float(acc2[0]), r3, c3), K::LO), 127);
    if (T.l3w2 >= 0) smem_y3[T.l3w2 + FPW * wave] = (int8_t)y;
  }
}

// ---- layer 4 ---------------------------------------------------------------------------------
// Part t (one wave, one MFMA) covers samples 64t .. 64t+63: A row i (lane (i, h)) = y3t[64t + 32h + n(i)] in
// K-slots 16h..16h+15; B is block diagonal (columns c < 16: channel c on slots 0..15, columns
// c >= 16: channel c-16 on slots 16..31), so column c of D = channel c & 15 of time block c >> 4.
// Rows n(i) permuted so lane (c, h) register r = time 16h + r of that block: two pool-8 windows.
// REORDER_BN: part t's MFMA starts from bias4(t) (biased relu pooling as in layer 2, a constant of
// its own per part so that none is hoisted into registers)
__host__ __device__ constexpr int bias4(int t) { return t == 0 ? (int)0x3F000000 : t == 1 ? (int)0xBF000000 : (int)0xBF800000; }

template <class K>
__device__ __forceinline__ unsigned l4_out(const v16i& acc, const SmallParams* sp, int kb, int bias) {
  // kb = 4 k (byte offset of channel k)
#define MIB_K4(arr, T) (*(const T*)((const char*)(arr) + kb))
  if constexpr (K::RB) {
    const int thrb = MIB_K4(sp->l4_thr, int) + bias, offm = MIB_K4(sp->l4_offm, int);
    if constexpr (K::XR) return l2_out<K::LO, true>(acc, thrb, offm, MIB_K4(sp->l4_m, unsigned), MIB_K4(sp->l4_xs, int));
    else return l2_out<K::LO, false>(acc, thrb, offm, MIB_K4(sp->l4_r, float), 0);
  } else if constexpr (K::XR) {
    const unsigned m = MIB_K4(sp->l4n_m, unsigned);
    const int xs = MIB_K4(sp->l4_xs, int);
    const int sm[2] = {min(xelem_sum8<0, 1024>(acc, m, xs) >> 3, 127), min(xelem_sum8<8, 1024>(acc, m, xs) >> 3, 127)};
    return (unsigned)sm[0] | ((unsigned)sm[1] << 8);
  } else {
    // layer4.c:113-130 without REORDER_BN: element = (dot + off) / factor (no clip), ReLU,
    // sum of 8, >> 3, clip.  Elements in the floor form (l2n_out) with the ReLU only (relu_sum8).
    const float rn = MIB_K4(sp->l4n_r, float), cn = MIB_K4(sp->l4n_c, float);
    const int sm[2] = {min((int)(relu_sum8<0>(acc, rn, cn) >> 3), 127), min((int)(relu_sum8<8>(acc, rn, cn) >> 3), 127)};
    return (unsigned)sm[0] | ((unsigned)sm[1] << 8);
  }
}

// Layer 4 on one wave.  MFMA t covers samples 64t .. 64t+63.  Output y4[k][v], row stride T64A;
// the pad columns v = T64 .. T64A-1 receive don't-care values (layer 5's weights there are zero).
// L4PIPE: software-pipelined by one part (the MFMA of part t+1 is issued before the pooling of
// part t, two accumulators live); otherwise one part at a time.
template <class K>
__device__ __forceinline__ void layer4(const int8_t* smem_y3, int8_t* smem_y4, const SmallParams* sp, const L45Tab& L,
                                       int lane) {
  const v4i bw = sp->l4_bfrag[lane];
  const int ci = K::RB ? 0 : *(const int*)((const char*)sp->l4n_ci + L.l4k);  // plain branch: C-init
  if constexpr (K::L4PIPE) {
    v4i a[K::NT4];
#pragma unroll
    for (int t = 0; t < K::NT4; t++) a[t] = *(const v4i*)(smem_y3 + L.l4a + y3_off<K>(64 * t));  // unaligned (4 B)
    v16i acc[2];
#pragma unroll
    for (int j = 0; j < 16; j++) acc[0][j] = K::RB ? bias4(0) : ci;
    acc[0] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[0], bw, acc[0], 0, 0, 0);
#pragma unroll
    for (int t = 0; t < K::NT4; t++) {
      if (t + 1 < K::NT4) {
#pragma unroll
        for (int j = 0; j < 16; j++) acc[(t + 1) & 1][j] = K::RB ? bias4(t + 1) : ci;
        acc[(t + 1) & 1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[t + 1 < K::NT4 ? t + 1 : 0], bw, acc[(t + 1) & 1], 0, 0, 0);
      }
      const unsigned w = l4_out<K>(acc[t & 1], sp, L.l4k, bias4(t));
      if ((L.l4m >> t) & 1) *(unsigned short*)(smem_y4 + L.l4w + 8 * t) = (unsigned short)w;
    }
  } else {
#pragma unroll
    for (int t = 0; t < K::NT4; t++) {
      const v4i a = *(const v4i*)(smem_y3 + L.l4a + y3_off<K>(64 * t));  // unaligned (4 B)
      v16i acc;
#pragma unroll
      for (int j = 0; j < 16; j++) acc[j] = K::RB ? bias4(t) : ci;
      acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, bw, acc, 0, 0, 0);
      const unsigned w = l4_out<K>(acc, sp, L.l4k, bias4(t));
      // the pooling reads the accumulator on every path: sunk into the store's branch, it left the
      // accumulator dead on the branch's execz path while the MFMA still wrote it, and a later
      // inline-asm pack could be given those registers (tools/mfma_lint.py, write-after-write)
      asm volatile("" ::"v"(w));
      if ((L.l4m >> t) & 1) *(unsigned short*)(smem_y4 + L.l4w + 8 * t) = (unsigned short)w;
    }
  }
}

// ---- layer 5 ---------------------------------------------------------------------------------
template <class K>
__device__ __forceinline__ unsigned layer5(const int8_t* smem_y4, const SmallParams* sp, const L45Tab& L) {
  int part = 0;
#pragma unroll
  for (int j = 0; j < K::N5L; j++) {  // dword c + 16 j of class n (pad columns and dwords past ND5 meet zero weights)
    part = __builtin_amdgcn_sdot4(*(const int*)(smem_y4 + L.l5y + 64 * j),
                                  *(const int*)((const char*)sp->l5_w + L.l5w + 64 * j), part, false);
  }
  // inclusive prefix sum within each 16-lane DPP row: lane 15 of the row holds the total
  part += __builtin_amdgcn_update_dpp(0, part, 0x111, 0xF, 0xF, true);  // row_shr:1
  part += __builtin_amdgcn_update_dpp(0, part, 0x112, 0xF, 0xF, true);  // row_shr:2
  part += __builtin_amdgcn_update_dpp(0, part, 0x114, 0xF, 0xF, true);  // row_shr:4
  part += __builtin_amdgcn_update_dpp(0, part, 0x118, 0xF, 0xF, true);  // row_shr:8
  const int z = rq<K::LO>(part + *(const int*)((const char*)sp->l5_b + L.l5n), sp->l5_r);
  const unsigned z0 = (unsigned)__builtin_amdgcn_readlane(z, 15) & 255u;
  const unsigned z1 = (unsigned)__builtin_amdgcn_readlane(z, 31) & 255u;
  const unsigned z2 = (unsigned)__builtin_amdgcn_readlane(z, 47) & 255u;
  const unsigned z3 = (unsigned)__builtin_amdgcn_readlane(z, 63);
  return z0 | (z1 << 8) | (z2 << 16) | (z3 << 24);
}

// Trial addressing.  Timing-proxy builds (tools/, -DMIB_DIAG: forward_diag.hpp) redefine these and
// the DIAG_* switches; the library builds the forms below.
#ifndef MIB_DIAG
#define MIB_LOOP_BARRIER() __syncthreads()
#define MIB_TRIAL_OFF(b) ((size_t)(b) * K::XTRIAL)
#define MIB_TRIALS_LEFT(b) (B - (int)(b))
#endif

// Fused forward over a batch (persistent, grid-strided over trials).
template <class K>
__global__ __launch_bounds__(NTHREADS) __attribute__((amdgpu_waves_per_eu(WPE, WPE))) void k_forward(
    const DevParams* __restrict__ prm, const int8_t* __restrict__ x, int8_t* __restrict__ out, int B, float qs,
    float qy) {
  __shared__ __attribute__((aligned(16))) int8_t smem[K::LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  Regs<K> R;
  setup<K>(prm, smem, R, tid, wave, lane);
  R.qs = qs;
  R.qy = qy;
  const SmallParams* sp = (const SmallParams*)(smem + K::OFF_SP);
  if ((int)blockIdx.x < B)
    prefetch_l1<K>(trial_rsrc<K>(x + MIB_TRIAL_OFF(blockIdx.x), MIB_TRIALS_LEFT(blockIdx.x), wave), R, lane, wave,
                   smem);
  // The first trial's fragments land before its layer 1 starts, as in k_layer (where loads still
  // in flight at layer 1 gave a rare wrong layer-1 row).  Once per workgroup.
  __builtin_amdgcn_s_waitcnt(0);
  if constexpr (K::RX) rx_store<K>(R, 0, smem + K::OFF_STG, lane, wave);  // the first trial's phase 0
  __syncthreads();
  MIB_STAMP_INIT
  MIB_CLOCK_INIT
  // Per trial two barriers: A after layer 1 (layer 2 of a filter reads all waves' layer-1
  // output), B after layer 3 (layer 4 reads all filters).  Layers 2 and 3 of a filter run on the
  // wave that owns it, with no barrier between.  After B the last wave runs layers 4 and 5 while
  // the others start the next trial's layer 1: the next trial's layers 1-2 touch neither y3t
  // nor y4, and its layer 3 comes after the next A, which the last wave reaches only when done.
  for (int b = blockIdx.x; b < B; b += gridDim.x) {
    const int bn = b + gridDim.x;
    const Rsrc rc = trial_rsrc<K>(x + MIB_TRIAL_OFF(b), MIB_TRIALS_LEFT(b), wave);
    const Rsrc rn = trial_rsrc<K>(x + MIB_TRIAL_OFF(bn), MIB_TRIALS_LEFT(bn), wave);  // bn >= B: empty
    // laundered lane id: per-lane addresses of layers 2-5 are recomputed every trial instead of
    // being hoisted out of the loop (they would be live across it and spill)
    int ln = lane;
    asm volatile("" : "+v"(ln));
    MIB_STAMP(7)
    __builtin_amdgcn_s_setprio(PRIO_L1);
    layer1<K>(rc, rn, smem + K::OFF_Y1, R, wave, lane, MIB_TRIALS_LEFT(b) == 1);
    __builtin_amdgcn_s_setprio(0);
    MIB_STAMP(0)
    // the lane table is read before barrier A, so its LDS latency hides in the barrier wait
    // instead of delaying layer 2's first loads (same-box A/B -1.8 %)
    const LaneTab T = ((const LaneTab*)(smem + K::OFF_LT))[ln];
    MIB_LOOP_BARRIER();  // A
    // DMA ring: the next trial's fill, off the layer-1 interval (-0.8 % same box); the ring's
    // reads all returned before the barrier
    MIB_STAMP(1)
    if constexpr (!DIAG_NOL2) layer2<K>(smem + K::OFF_Y1, smem + K::OFF_Y2, sp, R, T, wave, ln);
    // layer 3 of filter f reads only y2 row f, which this wave wrote
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    MIB_STAMP(2)
    // layer 3 ends the barrier-B interval: at priority 1 a wave's layer 3 wins the arbitration
    // against the other waves' layer 2 (same-box A/B -1.2 ... -1.6 %; 2: -1.0 %; from the layer-2
    // tail on: -0.2 %)
    __builtin_amdgcn_s_setprio(PRIO_L3);
    if constexpr (!DIAG_NOL3) layer3<K>(smem + K::OFF_Y2, smem + K::OFF_Y3, sp, R, T, wave);
    __builtin_amdgcn_s_setprio(0);
    // whole-row exchange: the next trial's phase 0 into the image (its previous contents were read
    // before barrier A), so that barrier B also completes it
    if constexpr (K::RX) rx_store<K>(R, 0, smem + K::OFF_STG, lane, wave);
    MIB_STAMP(3)
    MIB_LOOP_BARRIER();  // B
    MIB_STAMP(4)
    if (wave == NWAVES - 1) {
      __builtin_amdgcn_s_setprio(PRIO_L45);
      if constexpr (DIAG_NOL45) {
        if (ln == 0) *(unsigned*)(out + (size_t)b * N_OUT) = *(const unsigned*)(smem + K::OFF_Y3 + 4 * (b & 15));
      } else {
        const L45Tab L = ((const L45Tab*)(smem + K::OFF_L45))[ln];
        layer4<K>(smem + K::OFF_Y3, smem + K::OFF_Y4, sp, L, ln);
        MIB_STAMP(5)
        const unsigned z = layer5<K>(smem + K::OFF_Y4, sp, L);
        if (ln == 0) *(unsigned*)(out + (size_t)b * N_OUT) = z;
      }
      __builtin_amdgcn_s_setprio(0);
      MIB_STAMP(6)
    }
  }
  // the last fill (of an empty view past the batch) writes LDS: it lands before the wave ends
  // (the channel-major ring and the plain / exact-division LDMA slots alike)
  if constexpr (K::DMA || K::LDMA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  MIB_STAMP_FLUSH(lane == 0, wave)
  MIB_CLOCK_FLUSH
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
  if (stage == 1) {  // [T][C] packed (XTRIAL bytes) -> [F1][T_ALIGN]
    const Rsrc rin = trial_rsrc<K>(in, 1, wave);
    prefetch_l1<K>(rin, R, lane, wave, smem);
    // All fragment loads land before layer 1 starts.  With them still in flight, this single-
    // workgroup path gave a wrong layer-1 row in ~2 % of calls on gfx950 (tools/stress.py; the
    // batched kernel, whose fragments are loaded a whole trial ahead, showed none in 39 M trials).
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    layer1<K>(rin, rin, y1, R, wave, lane);
    __syncthreads();
    for (int i = tid; i < F2 * T_AL; i += NTHREADS) {
      const int f = i / T_AL, t = i - f * T_AL;
      out[i] = t < K::T ? y1[y1_index<K>(f, t)] : 0;
    }
  } else if (stage == 2) {  // [F1][T_ALIGN] -> [F2][T8_ALIGN]
    for (int i = tid; i < F2 * K::T; i += NTHREADS) {
      const int f = i / K::T, t = i - f * K::T;
      y1[y1_index<K>(f, t)] = in[f * T_AL + t];
    }
    __syncthreads();
    layer2<K>(y1, y2, sp, R, ((const LaneTab*)(smem + K::OFF_LT))[lane], wave, lane);
    __syncthreads();
    for (int i = tid; i < F2 * T8_AL; i += NTHREADS) {
      const int f = i / T8_AL, u = i - f * T8_AL;
      out[i] = u < K::T8 ? y2[f * K::Y2ROW + 8 + u] : 0;
    }
  } else if (stage == 3) {  // [F2][T8_ALIGN] -> [F2][T8_ALIGN]
    for (int i = tid; i < F2 * K::T8; i += NTHREADS) {
      const int f = i / K::T8, u = i - f * K::T8;
      y2[f * K::Y2ROW + 8 + u] = in[f * T8_AL + u];
    }
    __syncthreads();
    layer3<K>(y2, y3, sp, R, ((const LaneTab*)(smem + K::OFF_LT))[lane], wave);
    __syncthreads();
    for (int i = tid; i < F2 * T8_AL; i += NTHREADS) {
      const int f = i / T8_AL, u = i - f * T8_AL;
      out[i] = u < K::T8 ? y3[y3_off<K>(u) + f] : 0;
    }
  } else if (stage == 4) {  // [T8][F2] -> [F2][T64_ALIGN]
    for (int i = tid; i < K::Y3ROWS * F2; i += NTHREADS) y3[y3_off<K>(i / F2) + (i % F2)] = i < K::T8 * F2 ? in[i] : 0;
    __syncthreads();
    if (wave == 0)
      layer4<K>(y3, y4, sp, ((const L45Tab*)(smem + K::OFF_L45))[lane], lane);
    __syncthreads();
    for (int i = tid; i < F2 * T64_AL; i += NTHREADS) {
      const int k = i / T64_AL, v = i - k * T64_AL;
      out[i] = v < K::T64 ? y4[k * K::T64A + v] : 0;
    }
  } else if (stage == 5) {  // [F2][T64_ALIGN] -> [N]
    for (int i = tid; i < 64 * K::N5L; i += NTHREADS) {
      const int k = i / K::T64A, v = i - k * K::T64A;
      y4[i] = (k < F2 && v < K::T64) ? in[k * T64_AL + v] : 0;
    }
    __syncthreads();
    if (wave == 0) {
      const unsigned z = layer5<K>(y4, sp, ((const L45Tab*)(smem + K::OFF_L45))[lane]);
      if (lane == 0) *(unsigned*)out = z;
    }
  } else if (stage == 6) {  // flip [F2][T8_ALIGN] -> [T8][F2] (net_layer3_flip_inplace)
    for (int i = tid; i < F2 * T8_AL; i += NTHREADS) y1[i] = in[i];
    __syncthreads();
    for (int i = tid; i < F2 * T8_AL; i += NTHREADS) {
      const int u = i / F2, f = i - u * F2;
      out[i] = u < K::T8 ? y1[f * T8_AL + u] : 0;
    }
  }
}

}  // namespace wg
}  // namespace mib
