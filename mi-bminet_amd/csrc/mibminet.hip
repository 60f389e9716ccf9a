// mibminet.hip — host side of libmibminet.so: the C ABI declared in include/mibminet.h.
//
// * parses the parameter blob (mibminet/params.py, ParamSet.to_blob) holding the reference's
//   net.h arrays (edge-eegnet_wolf/data/gen_net_header.py:91-224),
// * builds the gfx950 operand fragments and exact requantisation reciprocals (DevParams),
// * uploads them lazily per device and dispatches the compiled (C, T) instantiations of the
//   kernel in forward_wg.hpp.
// There is no CPU compute path: without a usable HIP device every entry point returns an error.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <atomic>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/mibminet.h"
#include "../../include/mibminet_testing.h"
#include "forward_wg.hpp"
#include "forward_gen.hpp"
#include "quantize.hpp"
#include "classify.hpp"

using namespace mib;

// test hook (mibminet_test_xdiv_gpu): xdiv against C division in 64 bits over e0 .. e0 + count - 1;
// each thread writes its own mismatch count (plain stores, summed on the host)
__global__ void k_xdiv_check(int d, unsigned m, int xs, long long e0, long long count, unsigned long long* out) {
  const long long tid = (long long)blockIdx.x * blockDim.x + threadIdx.x, nt = (long long)gridDim.x * blockDim.x;
  unsigned long long bad = 0;
  for (long long i = tid; i < count; i += nt) {
    const int e = (int)(e0 + i);
    const long long want = (long long)e / (long long)d;
    bad += (long long)xdiv(e, m, xs) != (long long)(int)want;
  }
  out[tid] = bad;
}

namespace {

constexpr int MAX_DEVICES = 64;
constexpr int HEADER_SIZE = 64;
constexpr uint32_t FLAG_REORDER_BN = 1;
constexpr uint32_t FLAG_CLIP_BALANCED = 2;  // golden-model clip_balanced=True (functional.py:89-91)

struct Dims {
  int C = 0, T = 0, F1 = 0, F2 = 0, D = 0, N = 0, wbits = 8;
  int C_ALIGN() const { return (C + 3) & ~3; }
  int T_ALIGN() const { return (T + 3) & ~3; }
  int T8() const { return T / 8; }
  int T8_ALIGN() const { return (T8() + 3) & ~3; }
  int T64() const { return T8() / 8; }
  int T64_ALIGN() const { return (T64() + 3) & ~3; }
};

// Host copy of the net.h arrays (weights unpacked to int8).
struct HostParams {
  Dims d;
  std::vector<int32_t> l1_factor, l1_offset, l2_factor, l2_offset, l4_factor, l4_offset;
  std::vector<int8_t> l1_weight_align, l2_weight_reverse, l3_weight, l4_weight, l5_bias, l5_weight;
  int32_t l3_factor = 0, l5_factor = 0;
  bool reorder_bn = true;  // blob flag: -DREORDER_BN variant (canonical) or the plain BN branches
  bool clip_balanced = false;  // blob flag: clip to [-127, 127] (golden model's default; the C clips to -128)
  bool xr = false;             // set at load: exact integer division at layers 1, 2, 4 (Cfg::XR)
  int xr_layer = 0, xr_filter = -1;  // the first requant without a proven float form (xr = true)
  bool general = false;        // set at load: the run-time-dimension kernels (forward_gen.hpp)
  int folded = 0;              // set at load: constant filters folded (fold_constant_filters)
};

// test hook (mibminet_test_force_general): load every later set on the general path
std::atomic<int> g_force_general{0};

// ---- exact requantisation ------------------------------------------------------------------
// y = clip(trunc(v / fac), -128, 127) is computed on the GPU as clip((int)((float)v * r)).
// (float)v is exact for |v| < 2^24 and (int) truncates toward zero.  q(v) = (int)RN(v * r) is
// monotone in v, so it equals trunc(v / fac) on a whole constant interval of trunc(v / fac) iff it
// does at both ends.  verify() checks both ends of the intervals for k = -129 .. 128 that hold a
// reachable v (|v| <= vmax, the layer's accumulator bound), which pins the clipped result for
// every reachable v.  choose_reciprocal() starts two floats below RN(1/|fac|) and nudges upward
// until verify() passes: for large factors the admissible window is only a few floats wide
// (about 1 / (|fac| * 129) relative), so it must not be stepped over.

inline int64_t trunc_div(int64_t a, int64_t b) { return a / b; }  // C semantics

inline int64_t qf(int64_t v, float r) { return (int64_t)(int32_t)((float)v * r); }

// kmax: largest output step that must be exact (128 for int8 clipping; the non-REORDER_BN
// layer 4 clamps its unclipped elements at 1024 instead).  vmax: largest reachable |v|;
// intervals beyond it are not checked.
bool verify_reciprocal(int32_t fac, float r, int64_t kmax = 128, int64_t vmax = (1 << 24) - 1) {
  const int64_t F = fac < 0 ? -(int64_t)fac : (int64_t)fac;
  for (int64_t k = -129; k <= kmax; k++) {
    // interval of v (for |fac|) with trunc(v / F) == k
    int64_t lo, hi;
    if (k > 0) { lo = k * F; hi = k * F + F - 1; }
    else if (k == 0) { lo = -(F - 1); hi = F - 1; }
    else { lo = k * F - (F - 1); hi = k * F; }
    if (fac < 0) {  // trunc(v / fac) = trunc(-v / F): result k on the mirrored interval -[lo, hi]
      const int64_t a = -hi, b = -lo;
      lo = a; hi = b;
    }
    const int64_t want = k;
    if (lo > vmax || hi < -vmax) continue;  // unreachable
    lo = std::max(lo, -vmax);
    hi = std::min(hi, vmax);
    if (std::llabs(lo) >= (1 << 24) || std::llabs(hi) >= (1 << 24)) return false;
    if (qf(lo, r) != want || qf(hi, r) != want) return false;
    if (trunc_div(lo, fac) != want || trunc_div(hi, fac) != want) return false;  // self-check
  }
  return true;
}

bool choose_reciprocal(int32_t fac, float* out, float* magic_c = nullptr, int64_t kmax = 128,
                       int64_t vmax = (1 << 24) - 1) {
  // magic_c != nullptr: additionally require c = -(1.5 * 2^23) * r to be exact in f32, so that
  // fma(bits_as_float(v + 0x4B400000), r, c) == RN(v * r) (layer 1's one-instruction requant).
  if (fac == 0) return false;
  const double F = std::fabs((double)fac);
  float r = std::nextafterf(std::nextafterf((float)(1.0 / F), 0.0f), 0.0f);
  for (int tries = 0; tries < 4096; tries++) {
    const float rs = fac < 0 ? -r : r;
    bool ok = true;
    if (magic_c) {
      const double cd = -12582912.0 * (double)rs;
      const float cf = (float)cd;
      ok = ((double)cf == cd);
      if (ok) *magic_c = cf;
    }
    if (ok && verify_reciprocal(fac, rs, kmax, vmax)) { *out = rs; return true; }
    r = std::nextafterf(r, INFINITY);
  }
  return false;
}

// ---- floor-form element requant (plain-BN branches) ----------------------------------------
// The plain branches requantise every conv element and apply the ReLU right after:
// e = max(clip(trunc(x / fac)), 0) (layer2.c:139-210, layer4.c:113-130).  Behind the ReLU, trunc and
// floor agree (they differ only for negative quotients, which both clamp to 0), so
// e = clamp(floor(x / fac), 0, emax).  The GPU computes it without a float->int convert:
//   g(x) = fma(bits_as_float(Mbits + x), r, c)        (one rounding, round-to-nearest-even)
//   e    = bits(fmed3(g, K, K + emax)) - bits(K),       K = 1.5 * 2^23 (FMAGIC)
// The MFMA C-init carries Mbits + offset, so the accumulator's bits are exactly float(M + x).  The
// exact value of the fma is K + delta + x r with delta = M r + c - K; c is an integer-valued float
// that f32 holds exactly, so delta = M r - n for the integer n = K - c, and M is searched so that delta
// sits just below -1/2: then RN(K + delta + x r) = K + floor(x / fac) at every step boundary.  g is
// monotone in x, so checking both ends of every step interval k = -1 .. emax of the reachable range
// |x| <= vmax (with std::fmaf, the same correctly rounded fma) proves it for every reachable x.
float floor_form(int32_t mbits, int64_t x, float r, float c) {
  float m;
  const int32_t b = mbits + (int32_t)x;
  std::memcpy(&m, &b, 4);
  return std::fmaf(m, r, c);
}

bool verify_floor_form(int32_t fac, int32_t mbits, float r, float c, int64_t emax, int64_t vmax) {
  const int64_t F = fac < 0 ? -(int64_t)fac : (int64_t)fac;
  const float K = 12582912.0f;
  for (int64_t k = -1; k <= emax; k++) {
    // x with floor(x / fac) == k: fac > 0: [k F, k F + F - 1]; fac < 0: [-(k + 1) F + 1, -k F]
    int64_t lo = fac > 0 ? k * F : -(k + 1) * F + 1;
    int64_t hi = fac > 0 ? k * F + F - 1 : -k * F;
    if (lo > vmax || hi < -vmax) continue;
    lo = std::max(lo, -vmax);
    hi = std::min(hi, vmax);
    const int64_t want = std::min(std::max(k, (int64_t)0), emax);
    for (const int64_t x : {lo, hi}) {
      const float g = floor_form(mbits, x, r, c);
      const double e = std::min(std::max((double)g, (double)K), (double)K + (double)emax) - (double)K;
      if (e != (double)want) return false;
    }
  }
  return true;
}

bool choose_floor_form(int32_t fac, int64_t emax, int64_t vmax, int32_t* mbits, float* r_out, float* c_out) {
  if (fac == 0 || vmax >= (1 << 22) || emax > 1024) return false;
  const double F = std::fabs((double)fac);
  const double K = 12582912.0;
  const int64_t mlo = (1 << 23) + vmax, mhi = (1 << 24) - 1 - vmax;  // M + x stays in [2^23, 2^24)
  // target delta: -1/2 + 1/(2F), the middle of the window that maps each step to its floor
  const double target = -0.5 + 0.5 / F;
  float r = std::nextafterf(std::nextafterf((float)(1.0 / F), 0.0f), 0.0f);
  for (int tries = 0; tries < 16; tries++, r = std::nextafterf(r, INFINITY)) {
    const double rs = fac < 0 ? -(double)r : (double)r;
    // for each integer n, M = round((n + target) / rs) puts delta = M rs - n within rs / 2 of the
    // target; successive n give different residues, and the check below decides
    const double t0 = std::min((double)mlo * rs, (double)mhi * rs);
    const int64_t n0 = (int64_t)std::ceil(t0 - target) + 1;
    for (int64_t i = 0; i < 512 + 128; i++) {
      int64_t n, M;
      if (i < 512) {
        n = n0 + i;
        M = std::llround(((double)n + target) / rs);
      } else {
        // |fac| so large that M r moves by less than 1 over the whole magic range (every reachable
        // output is 0 or 1): the first magics with n on either side of M r
        M = mlo + (i - 512) / 2;
        n = (int64_t)((i & 1) ? std::ceil((double)M * rs) : std::floor((double)M * rs));
      }
      if (M < mlo || M > mhi) continue;
      const double c = K - (double)n;  // integer-valued (exact in f32 below 2^24, and when even below 2^25)
      if ((double)(float)c != c) continue;
      const float Mf = (float)M;
      int32_t mb;
      std::memcpy(&mb, &Mf, 4);
      if (verify_floor_form(fac, mb, (float)rs, (float)c, emax, vmax)) {
        *mbits = mb;
        *r_out = (float)rs;
        *c_out = (float)c;
        return true;
      }
    }
  }
  return false;
}

// ---- exact integer division (XR builds) ------------------------------------------------------
// Parameter sets outside the float envelope above (large folded BN offsets, or factors whose
// reciprocal window the check cannot prove) run the Cfg::XR kernels, which divide exactly
// (forward_common.hpp, xdiv): trunc(e r) in IEEE double with r = sign(d) RU(1 / |d|) equals C's
// trunc(e / d) for every int32 e.  For e, d > 0 with e / d = q + f (f a multiple of 1 / d,
// f <= 1 - 1 / d): 0 <= e r - e / d <= e 2^-52 / d, so the exact product lies in
// [q + f, q + f + e 2^-52 / d]; rounding it cannot go below q (q is a double), and its distance
// from q + 1 is at least (1 - e 2^-52) / d, more than half an ulp of the product ((e / d) 2^-53)
// for every e <= 2^31.  Negative e or d mirror it (the product changes sign only).  Round 5's
// integer form (m = ceil(2^(31 + l) / |d|), a 32 x 32 -> 64 product and a shift) took about
// twice the issue cycles.
// Exact division constants (forward_common.hpp, xdiv): the double r = sign(d) RU(1 / |d|), split
// into its low word (m) and high word (xs).  RU: 1 / |d| rounded to nearest, then one ulp up when
// that fell below (the fma residual r |d| - 1 is exact in sign).  Powers of two are exact.
struct XDiv {
  uint32_t m;
  int32_t xs;
};

XDiv xdiv_consts(int32_t d) {
  const double D = std::fabs((double)d);
  double r = 1.0 / D;
  if (std::fma(r, D, -1.0) < 0.0) r = std::nextafter(r, INFINITY);
  if (d < 0) r = -r;
  uint64_t bits;
  std::memcpy(&bits, &r, 8);
  return XDiv{(uint32_t)bits, (int32_t)(uint32_t)(bits >> 32)};
}

// the device sequence of xdiv on the host (mibminet_test_xdiv): IEEE double product, truncation
int32_t xdiv_host(int32_t e, XDiv c) {
  const uint64_t bits = ((uint64_t)(uint32_t)c.xs << 32) | c.m;
  double r;
  std::memcpy(&r, &bits, 8);
  return (int32_t)((double)e * r);
}

// Reachable range of an int8 dot product sum_i w[i] x[i] over inputs x in [-128, 127] (every
// layer entry point takes arbitrary int8 input, and the zero pads lie inside the range).
struct Range {
  int64_t lo = 0, hi = 0;
  int64_t amax() const { return std::max(std::llabs(lo), std::llabs(hi)); }
};
Range dot_range(const int8_t* w, int n) {
  Range r;
  for (int i = 0; i < n; i++) {
    r.lo += std::min(-128 * (int64_t)w[i], 127 * (int64_t)w[i]);
    r.hi += std::max(-128 * (int64_t)w[i], 127 * (int64_t)w[i]);
  }
  return r;
}
inline bool fits_i32(int64_t v) { return v >= INT32_MIN && v <= INT32_MAX; }
// the reference's int32 division v / d over v in [lo, hi] is defined (no zero divisor, no
// INT_MIN / -1) and its operands fit
inline bool div_ok(Range v, int64_t d) {
  return d != 0 && fits_i32(v.lo) && fits_i32(v.hi) && !(d == -1 && v.lo == INT32_MIN);
}
// REORDER_BN pooled sum of 8: sum_i max(v_i, thr) + off, accumulated in int32 (layer2.c:97-111,
// layer4.c:99-130): every partial sum and the total must fit
inline bool pooled_range(Range v, int32_t off, Range* s) {
  const int64_t thr = -((int64_t)off >> 3);
  const int64_t mlo = std::max(v.lo, thr), mhi = std::max(v.hi, thr);
  if (!fits_i32(8 * mlo) || !fits_i32(8 * mhi)) return false;
  s->lo = 8 * mlo + off;
  s->hi = 8 * mhi + off;
  return fits_i32(s->lo) && fits_i32(s->hi);
}

// REORDER_BN pooling constants (build_devparams, requant): the threshold clamped to [-V, V] and the
// offset term off + 8 max(thr, -V), thr = -(off >> 3).
void pool_consts(int32_t off, int64_t V, int32_t* thr_c, int32_t* offm) {
  const int64_t thr = -((int64_t)off >> 3);
  *thr_c = (int32_t)std::min(std::max(thr, -V), V);
  *offm = (int32_t)(uint32_t)((int64_t)off + 8 * std::max(thr, -V));  // the pooled sums wrap mod 2^32
}

// ---- blob parsing ------------------------------------------------------------------------
struct Reader {
  const uint8_t* p;
  size_t n, pos;
  bool ok = true;
  const uint8_t* take(size_t bytes) {
    if (!ok || pos + bytes > n) { ok = false; return nullptr; }
    const uint8_t* r = p + pos;
    pos += bytes + ((4 - bytes % 4) % 4);
    if (pos > n) { ok = false; return nullptr; }
    return r;
  }
  std::vector<int32_t> i32(size_t count) {
    std::vector<int32_t> v(count);
    const uint8_t* s = take(4 * count);
    if (s) std::memcpy(v.data(), s, 4 * count);
    return v;
  }
  std::vector<int8_t> w(size_t count, int wbits) {
    std::vector<int8_t> v(count);
    if (wbits == 8) {
      const uint8_t* s = take(count);
      if (s) std::memcpy(v.data(), s, count);
    } else {
      const uint8_t* s = take((count + 1) / 2);
      if (s)
        for (size_t i = 0; i < count; i++) {
          int nib = (s[i / 2] >> (4 * (i & 1))) & 0xF;
          v[i] = (int8_t)(nib >= 8 ? nib - 16 : nib);
        }
    }
    return v;
  }
  std::vector<int8_t> i8(size_t count) {
    std::vector<int8_t> v(count);
    const uint8_t* s = take(count);
    if (s) std::memcpy(v.data(), s, count);
    return v;
  }
};

// The reference multiplies the weight pads too (func_dotp over all C_ALIGN / F2 * T64_ALIGN bytes,
// layer1.c:90, layer5.c:81) and gen_net_header.py writes them as zeros; the GPU skips them, so a
// set with non-zero pads is rejected (NET_ERR_BLOB), as ParamSet.validate does.
int check_pads(const HostParams& hp) {
  const Dims& d = hp.d;
  const int F2 = d.F2;
  for (int f = 0; f < F2; f++)
    for (int c = d.C; c < d.C_ALIGN(); c++)
      if (hp.l1_weight_align[(size_t)f * d.C_ALIGN() + c] != 0) return NET_ERR_BLOB;
  for (int n = 0; n < d.N; n++)
    for (int k = 0; k < F2; k++)
      for (int v = d.T64(); v < d.T64_ALIGN(); v++)
        if (hp.l5_weight[((size_t)n * F2 + k) * d.T64_ALIGN() + v] != 0) return NET_ERR_BLOB;
  return NET_OK;
}

int parse_blob(const void* blob, size_t len, HostParams& hp) {
  if (!blob || len < (size_t)HEADER_SIZE) return NET_ERR_BLOB;
  const uint8_t* b = (const uint8_t*)blob;
  if (std::memcmp(b, "MIBMINET", 8) != 0) return NET_ERR_BLOB;
  uint32_t h[11];
  std::memcpy(h, b + 8, sizeof(h));
  const uint32_t version = h[0];
  Dims d;
  d.C = (int)h[1]; d.T = (int)h[2]; d.F1 = (int)h[3]; d.F2 = (int)h[4]; d.D = (int)h[5];
  d.N = (int)h[6]; d.wbits = (int)h[7];
  const uint32_t l2t = h[8], l3t = h[9], flags = h[10];
  if (version != 1 || l2t != 64 || l3t != 16) return NET_ERR_BLOB;
  if (flags & ~(FLAG_REORDER_BN | FLAG_CLIP_BALANCED)) return NET_ERR_BLOB;
  hp.reorder_bn = (flags & FLAG_REORDER_BN) != 0;
  hp.clip_balanced = (flags & FLAG_CLIP_BALANCED) != 0;
  if (d.wbits != 8 && d.wbits != 4) return NET_ERR_BLOB;
  if (d.C <= 0 || d.T < 64 || d.F1 <= 0 || d.N <= 0 || d.F2 != d.F1 * d.D) return NET_ERR_BLOB;
  Reader r{b, len, (size_t)HEADER_SIZE};
  const int F2 = d.F2;
  hp.d = d;
  hp.l1_factor = r.i32(F2); hp.l1_offset = r.i32(F2);
  hp.l1_weight_align = r.w((size_t)F2 * d.C_ALIGN(), d.wbits);
  hp.l2_factor = r.i32(F2); hp.l2_offset = r.i32(F2);
  hp.l2_weight_reverse = r.w((size_t)F2 * 64, d.wbits);
  hp.l3_factor = r.i32(1)[0];
  hp.l3_weight = r.w((size_t)F2 * 16, d.wbits);
  hp.l4_factor = r.i32(F2); hp.l4_offset = r.i32(F2);
  hp.l4_weight = r.w((size_t)F2 * F2, d.wbits);
  hp.l5_factor = r.i32(1)[0];
  hp.l5_bias = r.i8(d.N);
  hp.l5_weight = r.w((size_t)d.N * F2 * d.T64_ALIGN(), d.wbits);
  if (!r.ok || r.pos != len) return NET_ERR_BLOB;
  return check_pads(hp);
}

// ---- device parameter image --------------------------------------------------------------
// Three outcomes per parameter set:
//  * NET_ERR_RANGE where the reference's own int32 arithmetic is undefined for some input: a zero
//    divisor (factor, or factor >> 3 in the plain branches), INT_MIN / -1, or an overflowing sum
//    (acc + off of layer1.c:90-91, the pooled partial sums and sum + off of layer2.c:97-111 /
//    layer4.c:99-130, the plain layer 4's sum of eight unclipped elements, layer4.c:113-130);
//  * the float requant kernels (hp.xr = false) when every layer-1, -2 and -4 requant has a proven
//    float form (choose_reciprocal / choose_floor_form above);
//  * otherwise the exact-division kernels (hp.xr = true, Cfg::XR: xdiv at layers 1, 2 and 4).
// Layers 3 and 5 always use the float form (|acc| <= 16 * 128^2 and F2 * T64 * 128^2 + 128, every
// int32 factor proven: tests/test_requant_exact.py).
// Reachable ranges of the layer-1, -2 and -4 requant numerators, and NET_ERR_RANGE where the
// reference's int32 arithmetic is undefined for some int8 input (both kernel families).
struct Ranges {
  Range e1[F2], s2[F2], s4[F2];
};
int check_ranges(const HostParams& hp, Ranges& rg) {
  const Dims& d = hp.d;
  const int C = d.C, CA = d.C_ALIGN();
  Range* e1 = rg.e1;
  Range* s2 = rg.s2;
  Range* s4 = rg.s4;
  // reachable ranges: e1 = dot + off1 (layer 1); RB: the pooled sums + offset of layers 2 and 4;
  // plain: the per-element numerators conv + (off >> 3)
  for (int f = 0; f < F2; f++) {
    const Range r1 = dot_range(&hp.l1_weight_align[(size_t)f * CA], C);
    const Range r2 = dot_range(&hp.l2_weight_reverse[(size_t)f * 64], 64);
    const Range r4 = dot_range(&hp.l4_weight[(size_t)f * F2], F2);
    e1[f].lo = r1.lo + hp.l1_offset[f];
    e1[f].hi = r1.hi + hp.l1_offset[f];
    if (!div_ok(e1[f], hp.l1_factor[f])) return NET_ERR_RANGE;
    if (hp.reorder_bn) {
      if (!pooled_range(r2, hp.l2_offset[f], &s2[f]) || !div_ok(s2[f], hp.l2_factor[f])) return NET_ERR_RANGE;
      if (!pooled_range(r4, hp.l4_offset[f], &s4[f]) || !div_ok(s4[f], hp.l4_factor[f])) return NET_ERR_RANGE;
    } else {
      const int32_t f2 = hp.l2_factor[f] >> 3, o2 = hp.l2_offset[f] >> 3;
      const int32_t f4 = hp.l4_factor[f] >> 3, o4 = hp.l4_offset[f] >> 3;
      s2[f].lo = r2.lo + o2; s2[f].hi = r2.hi + o2;
      s4[f].lo = r4.lo + o4; s4[f].hi = r4.hi + o4;
      if (!div_ok(s2[f], f2) || !div_ok(s4[f], f4)) return NET_ERR_RANGE;
      // the eight elements max((v + off) / fac, 0) are summed unclipped: trunc is monotone in v
      const int64_t q4 = std::max({(int64_t)0, s4[f].lo / f4, s4[f].hi / f4});
      if (!fits_i32(8 * q4)) return NET_ERR_RANGE;
    }
  }
  if (hp.l3_factor == 0 || hp.l5_factor == 0) return NET_ERR_RANGE;
  return NET_OK;
}

// Per-filter classification ahead of the float / exact choice.  A layer-1, -2 or -4 filter whose
// output is one value y over its whole reachable numerator range
// (a rail: an offset far past anything the weights reach, a factor that sends every sum to zero, a
// REORDER_BN threshold above every conv value) is folded into zero weights with offset y and
// factor 1, or offset -y and factor -1 when y < 0 (a pooled sum of zeros with offset |y| and
// threshold -(|y| >> 3) <= 0 is |y|).  The kernels then produce the same y for every input with
// either requant form, and the filter no longer takes the set off the float kernels.  trunc(v /
// fac) and the clip are monotone in v, so the output is constant iff it is equal at both ends of
// the range.  Returns the count.
int fold_constant_filters(HostParams& h, const Ranges& rg) {
  const Dims& d = h.d;
  const int64_t lo = h.clip_balanced ? -127 : -128;
  auto q = [&](int64_t v, int64_t fac) { return std::min<int64_t>(127, std::max<int64_t>(lo, v / fac)); };
  auto constant = [&](const Range& r, int32_t fac, int32_t* y) {
    const int64_t a = q(r.lo, fac), b = q(r.hi, fac);
    *y = (int32_t)a;
    return a == b;
  };
  int n = 0;
  const int CA = d.C_ALIGN();
  for (int f = 0; f < d.F2; f++) {
    int32_t y;
    if (constant(rg.e1[f], h.l1_factor[f], &y)) {
      std::fill_n(&h.l1_weight_align[(size_t)f * CA], CA, (int8_t)0);
      h.l1_offset[f] = y;
      h.l1_factor[f] = 1;
      n++;
    }
    if (!h.reorder_bn) {
      // plain branches: the elements e = trunc((conv + (off >> 3)) / (fac >> 3)) (clipped in layer
      // 2, not in the C's layer 4) go through max(e, 0), a sum of 8 and // 8 (and the final clip in
      // layer 4): the output is 0 when every e <= 0, 127 when every e >= 127, e when e is
      // constant.  Folded: factor 8 and offset 8 y, so every element is y (in [0, 127]).
      auto plain = [&](const Range& r, int32_t fac, int32_t* yp) {
        const int64_t a = r.lo / (int64_t)(fac >> 3), b = r.hi / (int64_t)(fac >> 3);
        const int64_t emin = std::min(a, b), emax = std::max(a, b);
        if (emax > 0 && emin < 127 && emin != emax) return false;
        *yp = (int32_t)std::min<int64_t>(127, std::max<int64_t>(0, emin));
        return true;
      };
      if (plain(rg.s2[f], h.l2_factor[f], &y)) {
        std::fill_n(&h.l2_weight_reverse[(size_t)f * 64], 64, (int8_t)0);
        h.l2_offset[f] = 8 * y;
        h.l2_factor[f] = 8;
        n++;
      }
      if (plain(rg.s4[f], h.l4_factor[f], &y)) {
        std::fill_n(&h.l4_weight[(size_t)f * d.F2], d.F2, (int8_t)0);
        h.l4_offset[f] = 8 * y;
        h.l4_factor[f] = 8;
        n++;
      }
      continue;
    }
    if (constant(rg.s2[f], h.l2_factor[f], &y)) {
      std::fill_n(&h.l2_weight_reverse[(size_t)f * 64], 64, (int8_t)0);
      h.l2_offset[f] = y < 0 ? -y : y;
      h.l2_factor[f] = y < 0 ? -1 : 1;
      n++;
    }
    if (constant(rg.s4[f], h.l4_factor[f], &y)) {
      std::fill_n(&h.l4_weight[(size_t)f * d.F2], d.F2, (int8_t)0);
      h.l4_offset[f] = y < 0 ? -y : y;
      h.l4_factor[f] = y < 0 ? -1 : 1;
      n++;
    }
  }
  return n;
}

// Layer-2 A operand = banded weights (wg::layer2 and gen::layer2): row i <-> shift n(i) so that
// lane (c, h) register r holds output shift 16h + r (two complete pool-8 windows per lane).  PL:
// layer-1 row layout, 2 = parity-split planes (the specialised C <= 32 kernels), 1 = natural order.
void l2_bands(const HostParams& hp, int PL, v4i (*afrag)[3][64]) {
  for (int f = 0; f < F2; f++)
    for (int s = 0; s < 3; s++)
      for (int lane = 0; lane < 64; lane++) {
        const int i = lane & 31, hh = lane >> 5;
        const int n = 16 * ((i >> 2) & 1) + (i & 3) + 4 * (i >> 3);
        int8_t bytes[16];
        for (int jj = 0; jj < 16; jj++) {
          const int kq = 32 * s + 16 * hh + jj;  // K-slot
          // position in the 96-byte row window.  PL == 2: lane half hh reads
          // parity plane hh, bytes 16s .. 16s+15 of the block's window; PL == 1: natural order.
          const int kp = PL == 2 ? 2 * (16 * s + jj) + hh : kq;
          const int idx = kp - n - 1;            // tap (torch order)
          bytes[jj] = (int8_t)((idx >= 0 && idx < 64) ? hp.l2_weight_reverse[(size_t)f * 64 + idx] : 0);
        }
        std::memcpy(&afrag[f][s][lane], bytes, 16);
      }
}

int build_devparams(HostParams& hp, DevParams& dp) {
  const Dims& d = hp.d;
  if (d.F1 != F2 || d.F2 != F2 || d.N != N_OUT) return NET_ERR_UNSUPPORTED;
  if (d.C > 64) return NET_ERR_UNSUPPORTED;
  const int P = d.C <= 32 ? 2 : 1;
  const int C = d.C, CA = d.C_ALIGN();
  std::memset(&dp, 0, sizeof(dp));
  auto w1 = [&](int f, int c) -> int { return hp.l1_weight_align[(size_t)f * CA + c]; };
  const int64_t A = 128 * 128;
  Ranges rg;
  if (const int rc = check_ranges(hp, rg)) return rc;
  const Range* e1 = rg.e1;
  const Range* s2 = rg.s2;
  const Range* s4 = rg.s4;
  // Requant constants of layers 1, 2 and 4.  Float forms (xr = false) fail when a range leaves
  // the float window (|v| < 2^22 for a magic-offset C-init, 2^24 for a converted pooled sum) or a
  // reciprocal / floor form is not proven; the exact forms (xr = true) always succeed.  The first
  // failing requant (layer, filter) is kept for net_params_info.
  auto fail = [&](int layer, int f) {
    hp.xr_layer = layer;
    hp.xr_filter = f;
    return false;
  };
  auto requant = [&](bool xr) -> bool {
    SmallParams& sp = dp.sp;
    for (int t = 0; t < P; t++)
      for (int j = 0; j < 16; j++) {  // N-tile column j: filter 8t + j/2 (P == 2) or j (P == 1)
        const int f = P == 2 ? 8 * t + (j >> 1) : j;
        if (xr) {
          const XDiv x1 = xdiv_consts(hp.l1_factor[f]);
          dp.l1_cinit[t][j] = hp.l1_offset[f];
          dp.l1_m[t][j] = x1.m;
          dp.l1_xs[t][j] = x1.xs;
        } else {
          dp.l1_cinit[t][j] = hp.l1_offset[f] + FMAGIC_I;
          if (e1[f].amax() >= (1 << 22) ||
              !choose_reciprocal(hp.l1_factor[f], &dp.l1_r[t][j], &dp.l1_c[t][j], 128, e1[f].amax()))
            return fail(1, f);
        }
      }
    for (int f = 0; f < F2; f++) {
      if (hp.reorder_bn) {
        // biased relu pooling (forward_common.hpp, pool8b): sum_8 max(v, thr) + off =
        // sum_8 max(v - thr, 0) + (off + 8 thr), thr = -(off >> 3) (layer2.c:97-111), with thr
        // clamped to the conv range [-V, V] (V = 64 * 128^2 = 2^20 in layer 2, 16 * 128^2 = 2^18 in
        // layer 4) so that the biased values cannot wrap.  Past the upper end every max(v, thr) is
        // thr: the relu terms are 0 either way and the offset term keeps the true thr.  Past the
        // lower end every max(v, thr) is v: with thr' = -V the relu terms are v + V, so the offset
        // term is off - 8 V.  Hence offm = off + 8 max(thr, -V).
        int32_t t2, t4;
        pool_consts(hp.l2_offset[f], 1 << 20, &t2, &dp.l2_offm[f]);
        pool_consts(hp.l4_offset[f], 1 << 18, &t4, &sp.l4_offm[f]);
        dp.l2_thrb[f] = pbias(f & 1) + t2;  // the wave's filter slot f & 1 (forward_wg.hpp, layer2)
        sp.l4_thr[f] = t4;
        int32_t rbits = 0, xs2 = 0;
        if (xr) {
          const XDiv x2 = xdiv_consts(hp.l2_factor[f]), x4 = xdiv_consts(hp.l4_factor[f]);
          dp.l2_m[f] = x2.m;
          sp.l2_xs[f] = x2.xs;
          sp.l4_m[f] = x4.m;
          sp.l4_xs[f] = x4.xs;
          rbits = (int32_t)x2.m;
          xs2 = x2.xs;
        } else {
          if (s2[f].amax() >= (1 << 24) || !choose_reciprocal(hp.l2_factor[f], &dp.l2_r[f], nullptr, 128, s2[f].amax()))
            return fail(2, f);
          if (s4[f].amax() >= (1 << 24) || !choose_reciprocal(hp.l4_factor[f], &sp.l4_r[f], nullptr, 128, s4[f].amax()))
            return fail(4, f);
          std::memcpy(&rbits, &dp.l2_r[f], 4);
        }
        sp.l2_tpar[f] = (v4i){PBIAS_TAIL + t2, dp.l2_offm[f], rbits, xs2};
      } else {
        // plain branches: per-element BN with offset >> 3 and factor >> 3, ReLU right after.  Float:
        // the floor form (choose_floor_form), MFMA C-init = per-filter magic plus the offset
        // (|x| < 2^22); layer 2's elements clamp to [0, 127], layer 4's to [0, 1024] (anything
        // above saturates the result).  Exact: C-init = the offset, each element xdiv and a clamp.
        const int32_t f2 = hp.l2_factor[f] >> 3, o2 = hp.l2_offset[f] >> 3;
        const int32_t f4 = hp.l4_factor[f] >> 3, o4 = hp.l4_offset[f] >> 3;
        if (xr) {
          const XDiv x2 = xdiv_consts(f2), x4 = xdiv_consts(f4);
          sp.l2n_ci[f] = o2;
          sp.l2n_m[f] = x2.m;
          sp.l2_xs[f] = x2.xs;
          sp.l4n_ci[f] = o4;
          sp.l4n_m[f] = x4.m;
          sp.l4_xs[f] = x4.xs;
        } else {
          int32_t m2, m4;
          if (s2[f].amax() >= (1 << 22) || !choose_floor_form(f2, 127, s2[f].amax(), &m2, &sp.l2n_r[f], &sp.l2n_c[f]))
            return fail(2, f);
          if (s4[f].amax() >= (1 << 22) || !choose_floor_form(f4, 1024, s4[f].amax(), &m4, &sp.l4n_r[f], &sp.l4n_c[f]))
            return fail(4, f);
          sp.l2n_ci[f] = m2 + o2;
          sp.l4n_ci[f] = m4 + o4;
        }
      }
    }
    return true;
  };
  hp.xr = !requant(false);
  if (hp.xr) {
    std::memset(&dp, 0, sizeof(dp));
    (void)requant(true);
  }
  // layer 1: B operand (column j of N-tile t: filter 8t + j/2, parity j&1 when P == 2)
  for (int t = 0; t < P; t++) {
    for (int lane = 0; lane < 64; lane++) {
      const int j = lane & 15, g = lane >> 4;
      const int f = P == 2 ? 8 * t + (j >> 1) : j;
      const int p = P == 2 ? (j & 1) : 0;
      int8_t bytes[16];
      for (int jj = 0; jj < 16; jj++) {
        const int k = 16 * g + jj;  // byte of the 64-byte window
        const int c = k - C * p;    // channel of sample p in the window
        bytes[jj] = (int8_t)((c >= 0 && c < C) ? w1(f, c) : 0);
      }
      std::memcpy(&dp.l1_wfrag[t][lane], bytes, 16);
      // channel-major staging (forward_wg.hpp, stage_block): P == 2 K-slot 2c + p holds channel
      // c at sample 16 p + j of MFMA row j (column parity p selects it); P == 1 is the same slot
      // order as above
      for (int jj = 0; jj < 16; jj++) {
        const int k = 16 * g + jj;
        const int c = P == 2 ? k >> 1 : k, pk = P == 2 ? k & 1 : 0;
        bytes[jj] = (int8_t)((c < C && pk == p) ? w1(f, c) : 0);
      }
      std::memcpy(&dp.l1_wfrag_ct[t][lane], bytes, 16);
    }
  }
  // layer-2 tail bands (forward_wg.hpp, layer2_tail_mfma): filter pair w = filters 2w, 2w+1;
  // lane (m, g) of K-step s holds K-slots 64 s + 16 g + jj = chunk kap = 4 s + g, byte jj, which
  // is chunk mq = kap - 6 kf of filter kf = kap / 6; its window position q (tail_q) meets tap
  // q - m - 1 of the output shift m.
  auto l2_tail_bands = [&](int PL, v4i (*tfrag)[3][64]) {
    for (int w = 0; w < F2 / 2; w++)
      for (int s = 0; s < 3; s++)
        for (int lane = 0; lane < 64; lane++) {
          const int m = lane & 15, g = lane >> 4, kap = 4 * s + g, kf = kap / 6, mq = kap - 6 * kf;
          const int f = 2 * w + kf;
          int8_t bytes[16];
          for (int jj = 0; jj < 16; jj++) {
            const int q = PL == 2 ? 32 * (mq >> 1) + 2 * jj + (mq & 1) : 16 * mq + jj;
            const int idx = q - m - 1;
            bytes[jj] = (int8_t)((idx >= 0 && idx < 64 && (PL == 2 || mq < 5)) ? hp.l2_weight_reverse[(size_t)f * 64 + idx] : 0);
          }
          std::memcpy(&tfrag[w][s][lane], bytes, 16);
        }
  };
  l2_bands(hp, P, dp.l2_afrag);
  l2_tail_bands(P, dp.l2t_afrag);
  SmallParams& sp = dp.sp;
  // layer 3: net_l3_weight is stored flipped (true convolution); torch order = reversed.  A
  // operand of MFMA i32_16x16x64_i8 (forward_wg.hpp, layer3): row r, K-slot k of filter f's half
  // (byte 16 col + k of its layer-2 row window, which holds position k - 8 + 16 col): output
  // 16 col + r uses bytes +1 .. +16, so A[r][k] = tap[k - r - 1].  Lane l holds row l & 15,
  // K-slots 16 (l >> 4) .. +15: groups 0-1 filter 2w, groups 2-3 filter 2w + 1.  Tile 2 carries
  // shift g on row 4g only.
  for (int w = 0; w < F2 / 2; w++)
    for (int lane = 0; lane < 64; lane++) {
      const int r = lane & 15, kg = lane >> 4, f = 2 * w + (kg >> 1);
      int8_t taps[16];
      for (int j = 0; j < 16; j++) taps[j] = hp.l3_weight[(size_t)f * 16 + 15 - j];
      int8_t b1[16], b2[16];
      for (int jj = 0; jj < 16; jj++) {
        const int k = 16 * (kg & 1) + jj;
        const int t1 = k - r - 1, t2 = k - r / 4 - 1;
        b1[jj] = (t1 >= 0 && t1 < 16) ? taps[t1] : 0;
        b2[jj] = ((r & 3) == 0 && t2 >= 0 && t2 < 16) ? taps[t2] : 0;
      }
      std::memcpy(&dp.l3_a1[w][lane], b1, 16);
      std::memcpy(&dp.l3_a2[w][lane], b2, 16);
    }
  // |layer-3 accumulator| <= 16 * 128 * 128 < 2^22: magic C-init form
  if (!choose_reciprocal(hp.l3_factor, &sp.l3_r, &sp.l3_c, 128, 16LL * A)) return NET_ERR_RANGE;
  // layer 4: B operand of MFMA 32x32x32 = W4^T, block diagonal: lane (column k, half h) holds
  // K-slots 16h..16h+15; columns 0..15 carry output channels 0..15 on slots 0..15 and columns
  // 16..31 repeat them on slots 16..31 (a second 32-sample time block rides in the other K half).
  for (int lane = 0; lane < 64; lane++) {
    const int k = lane & 31, hh = lane >> 5;
    int8_t bytes[16] = {0};
    if ((k >> 4) == hh) std::memcpy(bytes, &hp.l4_weight[(size_t)(k & 15) * F2], 16);
    std::memcpy(&dp.sp.l4_bfrag[lane], bytes, 16);
  }
  const int T64 = d.T64(), T64A = d.T64_ALIGN();
  if (F2 * T64A / 4 > ND5_MAX) return NET_ERR_UNSUPPORTED;
  for (int n = 0; n < N_OUT; n++) {
    int8_t* dst = (int8_t*)sp.l5_w[n];
    for (int k = 0; k < F2; k++)
      for (int v = 0; v < T64; v++) dst[k * T64A + v] = hp.l5_weight[(size_t)n * F2 * T64A + k * T64A + v];
    sp.l5_b[n] = hp.l5_bias[n];
  }
  if (!choose_reciprocal(hp.l5_factor, &sp.l5_r, nullptr, 128, (int64_t)F2 * T64 * A + 128)) return NET_ERR_RANGE;
  return NET_OK;
}

// ---- general-geometry parameter image (forward_gen.hpp) ------------------------------------
// Every network gen_net_header.py emits with F1 = F2 = 16: C <= 64, 64 <= T <= gen::TMAX,
// 1 <= N <= gen::NMAX.  The same range checks as the specialised image decide NET_ERR_RANGE.
// Requant: the float forms of the compiled kernels where every layer-1..4 requant has one proven
// exact (gp.xr = 0), exact integer division (xdiv) at layers 1-4 otherwise (gp.xr = 1); layer 5
// always divides exactly.
int build_genparams(HostParams& hp, gen::GenParams& gp) {
  const Dims& d = hp.d;
  if (d.F1 != F2 || d.F2 != F2 || d.D != 1) return NET_ERR_UNSUPPORTED;
  if (d.C < 1 || d.C > 64 || d.T < 64 || d.T > gen::TMAX || d.N < 1 || d.N > gen::NMAX) return NET_ERR_UNSUPPORTED;
  Ranges rg;
  if (const int rc = check_ranges(hp, rg)) return rc;
  std::memset(&gp, 0, sizeof(gp));
  const int C = d.C, CA = d.C_ALIGN(), T8 = d.T8(), T64 = d.T64(), T64A = d.T64_ALIGN();
  gp.C = C;
  gp.T = d.T;
  gp.N = d.N;
  gp.T8 = T8;
  gp.T64 = T64;
  gp.T64A = T64A;
  gp.NB1 = (d.T + 15) / 16;
  const int NB2 = (8 * T8 + 31) / 32;  // layer-2 column blocks of 32 outputs
  // full 32x32 tiles of 32 blocks; at most 16 blocks left go to 16x16x64 tail tiles (16 columns of
  // 16 outputs each), more to one more full tile
  const int rest = NB2 % 32;
  gp.MT = NB2 / 32 + (rest > 16 ? 1 : 0);
  gp.NTT = (rest > 0 && rest <= 16) ? (2 * rest + 15) / 16 : 0;
  // the last wave runs layers 4-5 (about two layer-1 blocks' time per 64 samples of layer 4, on
  // the phase stamps) and then the trial's last K7 layer-1 blocks; the other seven share the rest:
  // (NB1 - K7) / 7 = 2 NP + K7, NP = layer-4 parts
  const int NP = (T64 + 7) / 8;
  gp.K7 = std::max(0, (gp.NB1 - 14 * NP) / 8);
  // time-major at one workgroup per CU: two fewer (same box: -0.9 ... -2.6 %; channel-major
  // measured +1.5 % and keeps K7, profiles/r06_ab_k7.txt)
  gp.K7T1 = std::max(0, gp.K7 - 2);
  gp.rb = hp.reorder_bn ? 1 : 0;
  gp.lo = hp.clip_balanced ? -127 : -128;
  gp.xstride = (int)(((size_t)C * d.T + 15) / 16 * 16);
  // layer 1: lane (filter j, K group g) holds channels 16 c .. 16 c + 15 (zero past C) of chunk c:
  // time-major c = gen::l1_chunk(g, C), zero in K groups 1 and 3 when C <= 32 (their lanes re-read
  // the previous group's bytes); natural order (channel-major, float32) c = g
  for (int lane = 0; lane < 64; lane++) {
    const int j = lane & 15, g = lane >> 4;
    int8_t bytes[16], nat[16];
    for (int i = 0; i < 16; i++) {
      const int c = 16 * gen::l1_chunk(g, C) + i, cn = 16 * g + i;
      bytes[i] = (c < C && !(C <= 32 && (g & 1))) ? hp.l1_weight_align[(size_t)j * CA + c] : 0;
      nat[i] = cn < C ? hp.l1_weight_align[(size_t)j * CA + cn] : 0;
    }
    std::memcpy(&gp.l1_b[lane], bytes, 16);
    std::memcpy(&gp.l1_bn[lane], nat, 16);
  }

  for (int f = 0; f < F2; f++) {
    const XDiv x1 = xdiv_consts(hp.l1_factor[f]);
    gp.l1_off[f] = hp.l1_offset[f];
    gp.l1_m[f] = x1.m;
    gp.l1_xs[f] = x1.xs;
    // layers 2 and 4: REORDER_BN pools max(v, -(off >> 3)) and divides by factor; the plain
    // branches divide each element by factor >> 3 after adding offset >> 3
    const bool rb = hp.reorder_bn;
    const XDiv x2 = xdiv_consts(rb ? hp.l2_factor[f] : hp.l2_factor[f] >> 3);
    gp.l2_thr[f] = -(hp.l2_offset[f] >> 3);
    gp.l2_off[f] = rb ? hp.l2_offset[f] : hp.l2_offset[f] >> 3;
    gp.l2_m[f] = x2.m;
    gp.l2_xs[f] = x2.xs;
    const XDiv x4 = xdiv_consts(rb ? hp.l4_factor[f] : hp.l4_factor[f] >> 3);
    gp.sg.l4_thr[f] = -(hp.l4_offset[f] >> 3);
    gp.sg.l4_off[f] = rb ? hp.l4_offset[f] : hp.l4_offset[f] >> 3;
    gp.sg.l4_m[f] = x4.m;
    gp.sg.l4_xs[f] = x4.xs;
  }
  // layer 4 (gen::layer4): lane (column c = lane & 31, K half h = lane >> 5) holds B[16 h .. +15][c]
  // = W4[c & 15][0 .. 15] when h == c >> 4, else zeros
  for (int lane = 0; lane < 64; lane++) {
    const int c = lane & 31, h = lane >> 5;
    int8_t bytes[16] = {0};
    if (h == (c >> 4)) std::memcpy(bytes, &hp.l4_weight[(size_t)(c & 15) * F2], 16);
    std::memcpy(&gp.sg.l4_b[lane], bytes, 16);
  }
  // layer 3 (gen::layer3): torch-order taps W3t[t] = net_l3_weight[f][15 - t] (stored flipped).  Wave
  // w's A fragment, lane (row r = lane & 15, K group kg = lane >> 4): K-slots 16 (kg & 1) .. +15 of
  // filter 2w + (kg >> 1)'s 32-byte window, A[r][k] = W3t[k - r - 1]
  for (int w = 0; w < gen::NW; w++)
    for (int lane = 0; lane < 64; lane++) {
      const int r = lane & 15, kg = lane >> 4, f = 2 * w + (kg >> 1);
      int8_t bytes[16];
      for (int jj = 0; jj < 16; jj++) {
        const int t = 16 * (kg & 1) + jj - r - 1;
        bytes[jj] = (t >= 0 && t < 16) ? hp.l3_weight[(size_t)f * 16 + 15 - t] : 0;
      }
      std::memcpy(&gp.sg.l3_a[w][lane], bytes, 16);
    }
  l2_bands(hp, 1, gp.l2_a);
  // tail bands (gen::layer2): lane (shift m = lane & 15, g) of K-step s holds K-slots
  // 64 s + 16 g .. +15, window position k of the column meets tap k - m - 1
  for (int f = 0; f < F2; f++)
    for (int s = 0; s < 2; s++)
      for (int lane = 0; lane < 64; lane++) {
        const int m = lane & 15, g = lane >> 4;
        int8_t bytes[16];
        for (int jj = 0; jj < 16; jj++) {
          const int idx = 64 * s + 16 * g + jj - m - 1;
          bytes[jj] = (idx >= 0 && idx < 64) ? hp.l2_weight_reverse[(size_t)f * 64 + idx] : 0;
        }
        std::memcpy(&gp.l2t_a[f][s][lane], bytes, 16);
      }
  // float forms (the proofs of build_devparams): xr stays 0 only if every one is proven
  auto floats = [&]() -> bool {
    const int64_t A = 128 * 128;
    if (!choose_reciprocal(hp.l3_factor, &gp.l3_r, &gp.l3_c, 128, 16 * A)) return false;
    for (int f = 0; f < F2; f++) {
      const Range e1 = rg.e1[f], s2 = rg.s2[f], s4 = rg.s4[f];
      if (e1.amax() >= (1 << 22) || !choose_reciprocal(hp.l1_factor[f], &gp.l1_r[f], &gp.l1_c[f], 128, e1.amax()))
        return false;
      if (hp.reorder_bn) {
        if (s2.amax() >= (1 << 24) || !choose_reciprocal(hp.l2_factor[f], &gp.l2_r[f], nullptr, 128, s2.amax()))
          return false;
        if (s4.amax() >= (1 << 24) || !choose_reciprocal(hp.l4_factor[f], &gp.sg.l4_r[f], nullptr, 128, s4.amax()))
          return false;
      } else {
        int32_t m2, m4;
        if (s2.amax() >= (1 << 22) ||
            !choose_floor_form(hp.l2_factor[f] >> 3, 127, s2.amax(), &m2, &gp.l2_r[f], &gp.l2_c[f]))
          return false;
        if (s4.amax() >= (1 << 22) ||
            !choose_floor_form(hp.l4_factor[f] >> 3, 1024, s4.amax(), &m4, &gp.sg.l4_r[f], &gp.sg.l4_c[f]))
          return false;
        gp.l2_thr[f] = m2 + (hp.l2_offset[f] >> 3);  // the layer-2 MFMA C-init
        gp.sg.l4_ci[f] = m4 + (hp.l4_offset[f] >> 3);
      }
    }
    for (int f = 0; f < F2; f++) gp.l1_off[f] = hp.l1_offset[f] + FMAGIC_I;
    return true;
  };
  gp.xr = floats() ? 0 : 1;
  if (gp.xr) {  // the half-built float constants are unused by the XR kernels; the C-inits revert
    for (int f = 0; f < F2; f++) {
      gp.l1_off[f] = hp.l1_offset[f];
      gp.l2_thr[f] = -(hp.l2_offset[f] >> 3);
    }
  }
  hp.xr = gp.xr != 0;
  const XDiv x3 = xdiv_consts(hp.l3_factor), x5 = xdiv_consts(hp.l5_factor);
  gp.l3_m = x3.m;
  gp.l3_xs = x3.xs;
  gp.l5_m = x5.m;
  gp.l5_xs = x5.xs;
  for (int n = 0; n < d.N; n++) {
    gp.l5_b[n] = hp.l5_bias[n];
    for (int k = 0; k < F2; k++)
      for (int v = 0; v < T64; v++) gp.l5_w[n][k * T64A + v] = hp.l5_weight[((size_t)n * F2 + k) * T64A + v];
  }
  return NET_OK;
}

// ---- compiled configurations --------------------------------------------------------------
// Three shapes: 22 x 1125 (BCI-IV-2a: configs A, B, D, E), 64 x 1000 (config C) and 64 x 480 (the
// reference's PhysioNet MMMI edgeEEGNet, QuantLab/PhysionetMMMI/config_INQ.json), each compiled
// with and without -DREORDER_BN, with both clip modes and with float or exact requant:
// wg::Cfg<C, T, RB, CB, CT, FQ, XR>.  Every other geometry (and N != 4) runs the general kernels
// (gen::k_forward<Layout>, run-time dimensions).
struct Variant {
  int shape = -1;  // 0: 22 x 1125, 1: 64 x 1000, 2: 64 x 480, 3: general, -1: unsupported
  bool rb = true;  // -DREORDER_BN branches (canonical)
  bool cb = false; // golden-model clip_balanced (clip to [-127, 127])
  bool xr = false; // exact integer division (parameters outside the float requant envelope)
  bool ok() const { return shape >= 0; }
  bool general() const { return shape == 3; }
};

// the compiled geometry of (C, T, N), or -1
int compiled_shape(const Dims& d) {
  if (d.F1 != F2 || d.F2 != F2 || d.N != N_OUT) return -1;
  if (d.C == 22 && d.T == 1125) return 0;
  if (d.C == 64 && d.T == 1000) return 1;
  if (d.C == 64 && d.T == 480) return 2;
  return -1;
}

Variant variant_of(const HostParams& hp) {
  Variant v;
  v.shape = hp.general ? 3 : compiled_shape(hp.d);
  v.rb = hp.reorder_bn;
  v.cb = hp.clip_balanced;
  v.xr = hp.xr;
  return v;
}

template <int C, int T, bool CT, bool FQ, bool XR, class F>
int with_variant_x(const Variant& v, F&& f) {
  if (v.rb) return v.cb ? f(wg::Cfg<C, T, true, true, CT, FQ, XR>{}) : f(wg::Cfg<C, T, true, false, CT, FQ, XR>{});
  return v.cb ? f(wg::Cfg<C, T, false, true, CT, FQ, XR>{}) : f(wg::Cfg<C, T, false, false, CT, FQ, XR>{});
}

template <int C, int T, bool CT, bool FQ, class F>
int with_variant(const Variant& v, F&& f) {
  return v.xr ? with_variant_x<C, T, CT, FQ, true>(v, f) : with_variant_x<C, T, CT, FQ, false>(v, f);
}

// Calls f(K{}) with the kernel configuration K of the variant (CT: channel-major input trials;
// FQ: float32 channel-major trials quantised in the kernel).
template <bool CT = false, bool FQ = false, class F>
int dispatch(const Variant& v, F&& f) {
  switch (v.shape) {
    case 0: return with_variant<22, 1125, CT, FQ>(v, f);
    case 1: return with_variant<64, 1000, CT, FQ>(v, f);
    case 2: return with_variant<64, 480, CT, FQ>(v, f);
    default: return NET_ERR_UNSUPPORTED;
  }
}

size_t trial_stride(const Dims& d) { return ((size_t)d.C * d.T + 15) / 16 * 16; }

// ---- global state --------------------------------------------------------------------------
// One device copy of the parameter image per loaded generation: a load never overwrites a copy
// that a kernel may still read, so launches in flight and launches captured into a HIP graph keep
// the image (and with it the compiled variant) they were enqueued with.  A reload of a
// byte-identical image reuses its copy.  When a new image would make more than MAX_IMAGES copies,
// only copies that no launch can still read are freed, least recently used first: every batched
// launch records an event per (copy, stream), and a copy is free once all its events have
// completed.  A copy used by a launch under stream capture (a HIP graph may replay it at any
// time) or on more than MAX_STREAMS streams is kept until net_params_unload.  Nothing here waits
// for the device, so a load never stalls or breaks a caller's capture; if no copy can be freed
// the device simply keeps more than MAX_IMAGES.  net_params_unload synchronises each device and
// frees every copy (graphs that captured a launch must not be replayed after it).
constexpr size_t MAX_IMAGES = 8;
constexpr size_t MAX_STREAMS = 16;

// A parameter image as uploaded: a wg DevParams (compiled geometries) or a gen::GenParams.
struct Image {
  std::shared_ptr<const void> data;
  size_t bytes = 0;
  bool same(const Image& o) const {
    return data == o.data || (bytes == o.bytes && std::memcmp(data.get(), o.data.get(), bytes) == 0);
  }
};
template <class P>
Image make_image(std::shared_ptr<P> p) {
  Image im;
  im.bytes = sizeof(P);
  im.data = std::move(p);
  return im;
}

struct DevImage {
  Image host;                             // what was uploaded
  void* dev = nullptr;
  uint64_t used = 0;                      // DeviceState::tick at the last selection
  bool pinned = false;                    // captured into a graph (or too many streams): kept
  std::vector<std::pair<hipStream_t, hipEvent_t>> last;  // the last launch per stream
};

struct DeviceState {
  std::mutex mu;
  uint64_t gen = 0;             // params generation of `cur`
  void* cur = nullptr;          // device copy of that generation (DevParams or gen::GenParams)
  std::vector<DevImage> images; // the copies uploaded to this device
  uint64_t tick = 0;
  int8_t* d_in = nullptr;       // single-trial scratch
  int8_t* d_out = nullptr;
  int8_t* h_in = nullptr;       // pinned host staging of the single-trial copies
  int8_t* h_out = nullptr;
  hipStream_t st = nullptr;     // the single-trial path's own non-blocking stream
  size_t scratch = 0;
  int cus = 0;
};

std::mutex g_mu;
std::shared_ptr<const HostParams> g_host;
Image g_img;
uint64_t g_gen = 0;
DeviceState g_devs[MAX_DEVICES];
std::atomic<int> g_single_device{0};  // net_set_device (read by every single-trial call)
std::atomic<int> g_device_count{-1};
thread_local int t_last_error = NET_OK;
// test counters (mibminet_test_upload_stats): parameter uploads, and those made while
// batch_multi was enqueueing shards (must stay 0: every device is prepared first)
std::atomic<long> g_uploads{0}, g_uploads_enqueue{0};
thread_local bool t_enqueueing = false;

inline int hip_err(hipError_t e) { return e == hipSuccess ? NET_OK : NET_ERR_HIP - (int)e; }

// NET_OK if `device` names a visible HIP device, NET_ERR_INVALID otherwise (or the HIP error).
int check_device(int device) {
  int n = g_device_count.load();
  if (n < 0) {
    const hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) return hip_err(e);
    g_device_count.store(n);
  }
  return (device >= 0 && device < n && device < MAX_DEVICES) ? NET_OK : NET_ERR_INVALID;
}

struct DeviceGuard {  // makes `dev` current and restores the caller's device; err: hipSetDevice's status
  int old = -1;
  hipError_t err = hipSuccess;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&old) != hipSuccess) old = -1;
    err = hipSetDevice(dev);
  }
  ~DeviceGuard() { if (old >= 0) (void)hipSetDevice(old); }
};

struct Snapshot {
  std::shared_ptr<const HostParams> host;
  Image img;
  uint64_t gen;
};

Snapshot snapshot() {
  std::lock_guard<std::mutex> lk(g_mu);
  return Snapshot{g_host, g_img, g_gen};
}

void free_image(DevImage& im) {
  for (auto& se : im.last) (void)hipEventDestroy(se.second);
  im.last.clear();
  (void)hipFree(im.dev);
  im.dev = nullptr;
}

// no launch recorded on the copy can still be running (graph-captured copies never qualify)
bool image_idle(const DevImage& im) {
  if (im.pinned) return false;
  for (const auto& se : im.last)
    if (hipEventQuery(se.second) != hipSuccess) return false;
  return true;
}

// Frees least-recently-used idle copies (never ds.cur) until fewer than MAX_IMAGES remain or none
// is idle.  No device synchronisation.
void evict_idle(DeviceState& ds) {
  while (ds.images.size() >= MAX_IMAGES) {
    int victim = -1;
    for (int i = 0; i < (int)ds.images.size(); i++) {
      const DevImage& im = ds.images[i];
      if (im.dev == ds.cur || !image_idle(im)) continue;
      if (victim < 0 || im.used < ds.images[victim].used) victim = i;
    }
    if (victim < 0) return;
    free_image(ds.images[victim]);
    ds.images.erase(ds.images.begin() + victim);
  }
}

// After a batched launch with ds.cur on `st` (ds.mu held, device current): remember it, so that
// the copy is freed only once the launch has finished.  Under stream capture the copy is pinned.
void note_launch(DeviceState& ds, hipStream_t st) {
  for (DevImage& im : ds.images) {
    if (im.dev != ds.cur) continue;
    if (im.pinned) return;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) {
      im.pinned = true;  // a graph may replay this launch at any time
      return;
    }
    for (auto& se : im.last)
      if (se.first == st) {
        if (hipEventRecord(se.second, st) != hipSuccess) im.pinned = true;
        return;
      }
    hipEvent_t ev = nullptr;
    if (im.last.size() >= MAX_STREAMS || hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
      im.pinned = true;
      return;
    }
    if (hipEventRecord(ev, st) != hipSuccess) {
      (void)hipEventDestroy(ev);
      im.pinned = true;
      return;
    }
    im.last.emplace_back(st, ev);
    return;
  }
}

// Ensure `dev` holds the parameters of snapshot s (ds.cur); called with ds.mu held and the device
// current.
int ensure_device(DeviceState& ds, int dev, const Snapshot& s) {
  if (!s.host) return NET_ERR_NO_PARAMS;
  if (ds.cus == 0) {
    int cus = 0;
    hipError_t e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return hip_err(e);
    ds.cus = cus;
  }
  if (ds.gen != s.gen || !ds.cur) {
    for (DevImage& im : ds.images)  // a set loaded before: its copy is still there, unchanged
      if (im.host.same(s.img)) {
        ds.cur = im.dev;
        ds.gen = s.gen;
        im.used = ++ds.tick;
        return NET_OK;
      }
    evict_idle(ds);
    DevImage im;
    im.host = s.img;
    im.used = ++ds.tick;
    hipError_t e = hipMalloc(&im.dev, s.img.bytes);
    if (e != hipSuccess) return hip_err(e);
    e = hipMemcpy(im.dev, s.img.data.get(), s.img.bytes, hipMemcpyHostToDevice);
    g_uploads++;
    if (t_enqueueing) g_uploads_enqueue++;
    if (e != hipSuccess) {
      (void)hipFree(im.dev);
      return hip_err(e);
    }
    ds.images.push_back(std::move(im));
    ds.cur = ds.images.back().dev;
    ds.gen = s.gen;
  }
  return NET_OK;
}

// Single-trial scratch: device buffers, pinned host staging (the copies run as DMA without the
// runtime's pageable bounce) and a non-blocking stream (no implicit sync with the null stream).
int ensure_scratch(DeviceState& ds, size_t bytes) {
  if (!ds.st) {
    hipError_t e = hipStreamCreateWithFlags(&ds.st, hipStreamNonBlocking);
    if (e != hipSuccess) {
      ds.st = nullptr;
      return hip_err(e);
    }
  }
  if (ds.scratch >= bytes) return NET_OK;
  if (ds.d_in) (void)hipFree(ds.d_in);
  if (ds.d_out) (void)hipFree(ds.d_out);
  if (ds.h_in) (void)hipHostFree(ds.h_in);
  if (ds.h_out) (void)hipHostFree(ds.h_out);
  ds.d_in = ds.d_out = ds.h_in = ds.h_out = nullptr;
  ds.scratch = 0;
  hipError_t e = hipMalloc((void**)&ds.d_in, bytes);
  if (e == hipSuccess) e = hipMalloc((void**)&ds.d_out, bytes);
  if (e == hipSuccess) e = hipHostMalloc((void**)&ds.h_in, bytes, hipHostMallocMapped | hipHostMallocCoherent);
  if (e == hipSuccess) e = hipHostMalloc((void**)&ds.h_out, bytes, hipHostMallocMapped | hipHostMallocCoherent);
  if (e != hipSuccess) return hip_err(e);
  ds.scratch = bytes;
  return NET_OK;
}

// Persistent grid: as many resident workgroups as the occupancy allows (two per CU).
template <class K>
int launch_forward_t(DeviceState& ds, const DevParams* p, const int8_t* x, int8_t* y, size_t B,
                     hipStream_t st, int32_t* info, float qs = 0.0f) {
  static std::atomic<int> bpc{0};  // per kernel instantiation (LDS and registers differ)
  int blocks_per_cu = bpc.load();
  if (blocks_per_cu == 0) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks_per_cu, wg::k_forward<K>, wg::NTHREADS, 0) != hipSuccess ||
        blocks_per_cu < 1)
      blocks_per_cu = 1;
    bpc.store(blocks_per_cu);
  }
  const size_t cap = (size_t)ds.cus * (size_t)blocks_per_cu;
  const int grid = (int)(B < cap ? B : cap);
  if (info) { info[0] = grid; info[1] = wg::NTHREADS; info[2] = K::LDS; return NET_OK; }
  if (B == 0) return NET_OK;
  const float qy = qs > 0.0f ? 1.0f / qs : 0.0f;  // RN(1 / scale): IEEE division on the host
  hipLaunchKernelGGL(wg::k_forward<K>, dim3(grid), dim3(wg::NTHREADS), 0, st, p, x, y, (int)B, qs, qy);
  return hip_err(hipGetLastError());
}

// General path: dynamic LDS from the run-time dimensions (gen::carve_of); the occupancy of each
// (kernel, LDS size) is queried once, and each kernel may take more than the default 64 KB of
// dynamic LDS.  Keyed by the kernel's address: every instantiation has the same function type.
int gen_blocks_per_cu(const void* k, int lds) {
  static std::mutex mu;
  static std::vector<std::pair<const void*, int>> attr;          // kernels with the LDS attribute set
  static std::vector<std::pair<std::pair<const void*, int>, int>> cache;  // ((kernel, lds), blocks per CU)
  std::lock_guard<std::mutex> lk(mu);
  bool seen = false;
  for (const auto& a : attr) seen = seen || a.first == k;
  if (!seen) {
    (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr.emplace_back(k, 1);
  }
  for (const auto& c : cache)
    if (c.first.first == k && c.first.second == lds) return c.second;
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k, gen::NT, (size_t)lds) != hipSuccess || n < 1) n = 1;
  cache.push_back({{k, lds}, n});
  return n;
}

template <int L, bool ST, bool RB, bool XR, bool CB>
int launch_gen_q(DeviceState& ds, const gen::GenParams& hg, const void* p, const int8_t* x, int8_t* y, size_t B,
                 hipStream_t st, int32_t* info, float qs) {
  const int lds = gen::carve_of(hg.C, hg.T, hg.N, hg.T8, hg.T64A, hg.NB1, hg.MT, hg.NTT, L).bytes;
  const void* kern = (const void*)gen::k_forward<L, ST, RB, XR, CB>;
  const size_t cap = (size_t)ds.cus * (size_t)gen_blocks_per_cu(kern, lds);
  const int grid = (int)(B < cap ? B : cap);
  if (info) { info[0] = grid; info[1] = gen::NT; info[2] = lds; return NET_OK; }
  if (B == 0) return NET_OK;
  const float qy = qs > 0.0f ? 1.0f / qs : 0.0f;  // RN(1 / scale), as the specialised float kernels
  hipLaunchKernelGGL((gen::k_forward<L, ST, RB, XR, CB>), dim3(grid), dim3(gen::NT), (size_t)lds, st,
                     (const gen::GenParams*)p, x, y, (int)B, qs, qy);
  return hip_err(hipGetLastError());
}

// the blob's flags as instantiations: REORDER_BN, exact division, balanced clip
template <int L, bool ST>
int launch_gen_s(DeviceState& ds, const gen::GenParams& hg, const void* p, const int8_t* x, int8_t* y, size_t B,
                 hipStream_t st, int32_t* info, float qs) {
  const int sel = (hg.rb ? 4 : 0) | (hg.xr ? 2 : 0) | (hg.lo == -127 ? 1 : 0);
  switch (sel) {
    case 0: return launch_gen_q<L, ST, false, false, false>(ds, hg, p, x, y, B, st, info, qs);
    case 1: return launch_gen_q<L, ST, false, false, true>(ds, hg, p, x, y, B, st, info, qs);
    case 2: return launch_gen_q<L, ST, false, true, false>(ds, hg, p, x, y, B, st, info, qs);
    case 3: return launch_gen_q<L, ST, false, true, true>(ds, hg, p, x, y, B, st, info, qs);
    case 4: return launch_gen_q<L, ST, true, false, false>(ds, hg, p, x, y, B, st, info, qs);
    case 5: return launch_gen_q<L, ST, true, false, true>(ds, hg, p, x, y, B, st, info, qs);
    case 6: return launch_gen_q<L, ST, true, true, false>(ds, hg, p, x, y, B, st, info, qs);
    default: return launch_gen_q<L, ST, true, true, true>(ds, hg, p, x, y, B, st, info, qs);
  }
}

// int8 trials that fit in LDS run the staged instantiation (gen::carve_of)
template <int L>
int launch_gen_t(DeviceState& ds, const gen::GenParams& hg, const void* p, const int8_t* x, int8_t* y, size_t B,
                 hipStream_t st, int32_t* info, float qs) {
  if constexpr (L != gen::F32) {
    if (gen::carve_of(hg.C, hg.T, hg.N, hg.T8, hg.T64A, hg.NB1, hg.MT, hg.NTT, L).raw >= 0)
      return launch_gen_s<L, true>(ds, hg, p, x, y, B, st, info, qs);
  }
  return launch_gen_s<L, false>(ds, hg, p, x, y, B, st, info, qs);
}

// layout: 0 time-major int8, 1 channel-major int8, 2 channel-major float32 (scale qs).  himg: the
// host copy of the image p points to (the general path reads its dimensions).
int launch_forward(const Variant& v, const void* himg, DeviceState& ds, const void* p, const int8_t* x, int8_t* y,
                   size_t B, hipStream_t st, int32_t* info = nullptr, int layout = 0, float qs = 0.0f) {
  if (v.general()) {
    const gen::GenParams& hg = *(const gen::GenParams*)himg;
    if (layout == 2) return launch_gen_t<gen::F32>(ds, hg, p, x, y, B, st, info, qs);
    if (layout == 1) return launch_gen_t<gen::CT>(ds, hg, p, x, y, B, st, info, qs);
    return launch_gen_t<gen::TM>(ds, hg, p, x, y, B, st, info, qs);
  }
  const DevParams* dp = (const DevParams*)p;
  auto f = [&](auto k) { return launch_forward_t<decltype(k)>(ds, dp, x, y, B, st, info, qs); };
  if (layout == 2) return dispatch<true, true>(v, f);
  return layout == 1 ? dispatch<true, false>(v, f) : dispatch<false, false>(v, f);
}

int launch_layer(const Variant& v, const void* himg, const void* p, const int8_t* in, int8_t* out, int stage,
                 hipStream_t st) {
  if (v.general()) {
    const gen::GenParams& hg = *(const gen::GenParams*)himg;
    const int lds = gen::carve_of(hg.C, hg.T, hg.N, hg.T8, hg.T64A, hg.NB1, hg.MT, hg.NTT, 3).bytes;
    auto go = [&](auto kern) {
      (void)gen_blocks_per_cu((const void*)kern, lds);  // the LDS attribute
      hipLaunchKernelGGL(kern, dim3(1), dim3(gen::NT), (size_t)lds, st, (const gen::GenParams*)p, in, out, stage);
      return hip_err(hipGetLastError());
    };
    const int sel = (hg.rb ? 4 : 0) | (hg.xr ? 2 : 0) | (hg.lo == -127 ? 1 : 0);
    switch (sel) {
      case 0: return go(gen::k_layer<false, false, false>);
      case 1: return go(gen::k_layer<false, false, true>);
      case 2: return go(gen::k_layer<false, true, false>);
      case 3: return go(gen::k_layer<false, true, true>);
      case 4: return go(gen::k_layer<true, false, false>);
      case 5: return go(gen::k_layer<true, false, true>);
      case 6: return go(gen::k_layer<true, true, false>);
      default: return go(gen::k_layer<true, true, true>);
    }
  }
  return dispatch(v, [&](auto k) {
    hipLaunchKernelGGL(wg::k_layer<decltype(k)>, dim3(1), dim3(wg::NTHREADS), 0, st, (const DevParams*)p, in, out, stage);
    return hip_err(hipGetLastError());
  });
}

// Runs one reference-layout single-trial stage on the single-trial device.
// stage 0 = whole model (input [T][C_ALIGN]); 1..5 = net_layerN; 6 = flip.
int run_single(int stage, const int8_t* in, int8_t* out) {
  if (!in || !out) return NET_ERR_INVALID;
  Snapshot s = snapshot();
  if (!s.host) return NET_ERR_NO_PARAMS;
  const Dims& d = s.host->d;
  const Variant v = variant_of(*s.host);
  if (!v.ok()) return NET_ERR_UNSUPPORTED;
  const int dev = g_single_device.load();
  DeviceState& ds = g_devs[dev];
  std::lock_guard<std::mutex> lk(ds.mu);
  DeviceGuard guard(dev);
  if (guard.err != hipSuccess) return hip_err(guard.err);
  int rc = ensure_device(ds, dev, s);
  if (rc) return rc;
  const size_t xs = trial_stride(d);
  rc = ensure_scratch(ds, xs > (size_t)d.F1 * d.T_ALIGN() ? xs + 64 : (size_t)d.F1 * d.T_ALIGN() + 64);
  if (rc) return rc;
  size_t in_bytes, out_bytes;
  switch (stage) {
    case 0:
    case 1: {  // reference input [T][C_ALIGN] -> packed [T][C], straight into the pinned staging
      for (int t = 0; t < d.T; t++) std::memcpy(ds.h_in + (size_t)t * d.C, in + (size_t)t * d.C_ALIGN(), d.C);
      std::memset(ds.h_in + (size_t)d.T * d.C, 0, xs - (size_t)d.T * d.C);
      in_bytes = xs;
      out_bytes = stage == 0 ? (size_t)d.N : (size_t)d.F1 * d.T_ALIGN();
      break;
    }
    case 2: in_bytes = (size_t)d.F1 * d.T_ALIGN(); out_bytes = (size_t)d.F2 * d.T8_ALIGN(); break;
    case 3: in_bytes = out_bytes = (size_t)d.F2 * d.T8_ALIGN(); break;
    case 4: in_bytes = (size_t)d.T8() * d.F2; out_bytes = (size_t)d.F2 * d.T64_ALIGN(); break;
    case 5: in_bytes = (size_t)d.F2 * d.T64_ALIGN(); out_bytes = (size_t)d.N; break;
    case 6: in_bytes = out_bytes = (size_t)d.F2 * d.T8_ALIGN(); break;
    default: return NET_ERR_INVALID;
  }
  if (stage > 1) std::memcpy(ds.h_in, in, in_bytes);
  hipError_t e;
#ifdef MIB_SINGLE_COPIES
  e = hipMemcpyAsync(ds.d_in, ds.h_in, in_bytes, hipMemcpyHostToDevice, ds.st);
  if (e != hipSuccess) return hip_err(e);
  int8_t* kin = ds.d_in;
  int8_t* kout = ds.d_out;
#else
  // zero copy: the kernel reads the trial from the pinned staging and writes its result there
  // (one launch per call instead of copy + launch + copy)
  int8_t* kin = nullptr;
  int8_t* kout = nullptr;
  e = hipHostGetDevicePointer((void**)&kin, ds.h_in, 0);
  if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&kout, ds.h_out, 0);
  if (e != hipSuccess) return hip_err(e);
#endif
  if (stage == 0)
    rc = launch_forward(v, s.img.data.get(), ds, ds.cur, kin, kout, 1, ds.st);
  else
    rc = launch_layer(v, s.img.data.get(), ds.cur, kin, kout, stage, ds.st);
  if (rc) {
    (void)hipStreamSynchronize(ds.st);  // a copy may still read the staging
    return rc;
  }
#ifdef MIB_SINGLE_COPIES
  e = hipMemcpyAsync(ds.h_out, ds.d_out, out_bytes, hipMemcpyDeviceToHost, ds.st);
  if (e != hipSuccess) {
    (void)hipStreamSynchronize(ds.st);
    return hip_err(e);
  }
#endif
  e = hipStreamSynchronize(ds.st);
  if (e != hipSuccess) return hip_err(e);
  std::memcpy(out, ds.h_out, out_bytes);
  return NET_OK;
}

template <class F>
int quantize_input(const F* x, int8_t* y, size_t B, int C, int T, F scale, int device, void* stream) {
  if ((!x || !y) && B) return NET_ERR_INVALID;
  if (C < 1 || C > quant::CMAX || T < 1 || device < 0 || device >= MAX_DEVICES) return NET_ERR_INVALID;
  // trial indices are int in the kernel: b + gridDim.y (<= B + YMAX) must not wrap
  if (B > (size_t)INT32_MAX - quant::YMAX || !(scale > 0)) return NET_ERR_INVALID;
  // one trial's input bytes form one buffer view (32-bit range); the tiles leave as 16-byte stores
  if ((size_t)C * T * sizeof(F) >= (size_t)1 << 31 || ((uintptr_t)y & 15)) return NET_ERR_INVALID;
  if (B == 0) return NET_OK;
  if (const int rc = check_device(device)) return rc;
  const int stride = (int)(((size_t)C * T + 15) / 16 * 16);
  DeviceGuard guard(device);
  if (guard.err != hipSuccess) return hip_err(guard.err);
  // each workgroup walks a few trials, loading one trial ahead
  constexpr size_t per = quant::qtrials<F>();
  const size_t rows = std::min((B + per - 1) / per, (size_t)quant::YMAX);
  dim3 grid((T + quant::TT - 1) / quant::TT, (unsigned)rows);
  hipLaunchKernelGGL(quant::k_quantize<F>, grid, dim3(quant::QTHREADS), 0, (hipStream_t)stream, x, y, C, T, stride, scale,
                     (int)B);
  return hip_err(hipGetLastError());
}

int argmax_batch(const int8_t* logits, int32_t* out, size_t B, int N, int device, void* stream) {
  if ((!logits || !out) && B) return NET_ERR_INVALID;
  // trial indices are int in the kernels: 4 q + 3 and blockIdx.x * CTHREADS + threadIdx.x reach
  // at most B + 4 CTHREADS, which must not wrap
  if (N < 1 || N > cls::NMAX || device < 0 || device >= MAX_DEVICES || B > (size_t)INT32_MAX - 4 * cls::CTHREADS)
    return NET_ERR_INVALID;
  if (B == 0) return NET_OK;
  if (const int rc = check_device(device)) return rc;
  DeviceGuard guard(device);
  if (guard.err != hipSuccess) return hip_err(guard.err);
  if (N == 4 && ((uintptr_t)logits & 15) == 0 && ((uintptr_t)out & 15) == 0) {
    const unsigned grid = (unsigned)((B + 4 * cls::CTHREADS - 1) / (4 * cls::CTHREADS));
    hipLaunchKernelGGL(cls::k_argmax4, dim3(grid), dim3(cls::CTHREADS), 0, (hipStream_t)stream,
                       (const unsigned*)logits, out, (int)B);
    return hip_err(hipGetLastError());
  }
  const unsigned grid = (unsigned)((B + cls::CTHREADS - 1) / cls::CTHREADS);
  hipLaunchKernelGGL(cls::k_argmax, dim3(grid), dim3(cls::CTHREADS), 0, (hipStream_t)stream, logits, out, (int)B, N);
  return hip_err(hipGetLastError());
}

}  // namespace

// ================================ C ABI ======================================================
extern "C" {

int net_version(void) { return MIBMINET_VERSION; }

const char* net_error_string(int code) {
  switch (code) {
    case NET_OK: return "ok";
    case NET_ERR_INVALID: return "invalid argument";
    case NET_ERR_NO_PARAMS: return "no parameters loaded";
    case NET_ERR_UNSUPPORTED: return "unsupported network configuration";
    case NET_ERR_BLOB: return "malformed parameter blob";
    case NET_ERR_RANGE: return "value outside the defined range (the reference's int32 arithmetic overflows or divides by zero on these parameters, or a float-input scale outside [2^-60, 2^60])";
    default:
      if (code <= NET_ERR_HIP) return hipGetErrorString((hipError_t)(NET_ERR_HIP - code));
      return "unknown error";
  }
}

namespace {
// Builds the device image of a parsed set and makes it current: the compiled kernels when its
// geometry has them, the general kernels otherwise.
int install(std::shared_ptr<HostParams> hp) {
  hp->general = g_force_general.load() != 0 || compiled_shape(hp->d) < 0;
  auto build = [&](HostParams& h, Image* img) -> int {
    if (h.general) {
      auto gp = std::make_shared<gen::GenParams>();
      if (const int rc = build_genparams(h, *gp)) return rc;
      *img = make_image(gp);
    } else {
      auto dp = std::make_shared<DevParams>();
      if (const int rc = build_devparams(h, *dp)) return rc;
      *img = make_image(dp);
    }
    return NET_OK;
  };
  Image img;
  if (const int rc = build(*hp, &img)) return rc;
  if (hp->xr) {
    // off the float envelope: fold the constant filters into an equivalent copy (the reference
    // ranges, NET_ERR_RANGE included, were checked on the set as given) and keep that image, float
    // if every remaining requant is proven, exact otherwise (xr_layer / xr_filter then name a
    // filter that really varies)
    HostParams fh = *hp;
    Ranges rg;
    if (check_ranges(fh, rg) == NET_OK && (fh.folded = fold_constant_filters(fh, rg)) > 0) {
      Image fimg;
      if (build(fh, &fimg) == NET_OK) {
        img = fimg;
        hp->xr = fh.xr;
        hp->xr_layer = fh.xr_layer;
        hp->xr_filter = fh.xr_filter;
        hp->folded = fh.folded;
      }
    }
  }
  std::lock_guard<std::mutex> lk(g_mu);
  g_host = hp;
  g_img = img;
  g_gen++;
  return NET_OK;
}
}  // namespace

int net_params_load(const void* blob, size_t len) {
  auto hp = std::make_shared<HostParams>();
  const int rc = parse_blob(blob, len, *hp);
  if (rc) return rc;
  return install(hp);
}

int net_params_load_arrays(const net_arrays_t* a) {
  if (!a) return NET_ERR_INVALID;
  if (a->flags & ~(FLAG_REORDER_BN | FLAG_CLIP_BALANCED)) return NET_ERR_BLOB;
  Dims d;
  d.C = a->C; d.T = a->T; d.F1 = a->F1; d.F2 = a->F2; d.D = a->D; d.N = a->N; d.wbits = 8;
  // the blob header's checks (parse_blob), then the arrays it would carry
  if (d.C <= 0 || d.T < 64 || d.F1 <= 0 || d.N <= 0 || d.F2 != d.F1 * d.D) return NET_ERR_BLOB;
  if ((size_t)d.C * d.T > ((size_t)1 << 30) || d.N > 4096 || d.F2 > 4096) return NET_ERR_UNSUPPORTED;
  if (!a->l1_factor || !a->l1_offset || !a->l1_weight_align || !a->l2_factor || !a->l2_offset ||
      !a->l2_weight_reverse || !a->l3_weight || !a->l4_factor || !a->l4_offset || !a->l4_weight || !a->l5_bias ||
      !a->l5_weight)
    return NET_ERR_INVALID;
  auto hp = std::make_shared<HostParams>();
  hp->d = d;
  hp->reorder_bn = (a->flags & FLAG_REORDER_BN) != 0;
  hp->clip_balanced = (a->flags & FLAG_CLIP_BALANCED) != 0;
  const size_t F2 = (size_t)d.F2;
  auto i32 = [](const int32_t* p, size_t n) { return std::vector<int32_t>(p, p + n); };
  auto i8 = [](const int8_t* p, size_t n) { return std::vector<int8_t>(p, p + n); };
  hp->l1_factor = i32(a->l1_factor, F2);
  hp->l1_offset = i32(a->l1_offset, F2);
  hp->l1_weight_align = i8(a->l1_weight_align, F2 * d.C_ALIGN());
  hp->l2_factor = i32(a->l2_factor, F2);
  hp->l2_offset = i32(a->l2_offset, F2);
  hp->l2_weight_reverse = i8(a->l2_weight_reverse, F2 * 64);
  hp->l3_factor = a->l3_factor;
  hp->l3_weight = i8(a->l3_weight, F2 * 16);
  hp->l4_factor = i32(a->l4_factor, F2);
  hp->l4_offset = i32(a->l4_offset, F2);
  hp->l4_weight = i8(a->l4_weight, F2 * F2);
  hp->l5_factor = a->l5_factor;
  hp->l5_bias = i8(a->l5_bias, (size_t)d.N);
  hp->l5_weight = i8(a->l5_weight, (size_t)d.N * F2 * d.T64_ALIGN());
  if (const int rc = check_pads(*hp)) return rc;
  return install(hp);
}

int net_params_info(int32_t* info) {
  if (!info) return NET_ERR_INVALID;
  Snapshot s = snapshot();
  for (int i = 0; i < 5; i++) info[i] = 0;
  if (!s.host) return NET_ERR_NO_PARAMS;
  const HostParams& hp = *s.host;
  info[0] = hp.general ? NET_PATH_GENERAL : hp.xr ? NET_PATH_EXACT : NET_PATH_FLOAT;
  info[1] = hp.general || !hp.xr ? 0 : hp.xr_layer;
  info[2] = hp.general || !hp.xr ? -1 : hp.xr_filter;
  info[3] = hp.general ? -1 : compiled_shape(hp.d);
  info[4] = hp.xr ? 1 : 0;
  return NET_OK;
}

void net_params_unload(void) {
  {
    std::lock_guard<std::mutex> lk(g_mu);
    g_host.reset();
    g_img = Image();
    g_gen++;
  }
  // free every device copy once the launches that may read it have finished
  for (int d = 0; d < MAX_DEVICES; d++) {
    DeviceState& ds = g_devs[d];
    std::lock_guard<std::mutex> lk(ds.mu);
    if (ds.images.empty()) continue;
    DeviceGuard guard(d);
    if (guard.err != hipSuccess || hipDeviceSynchronize() != hipSuccess) continue;  // keep them
    for (DevImage& im : ds.images) free_image(im);
    ds.images.clear();
    ds.cur = nullptr;
  }
}

int net_params_dims(int32_t* dims) {
  if (!dims) return NET_ERR_INVALID;
  Snapshot s = snapshot();
  if (!s.host) {
    for (int i = 0; i < 7; i++) dims[i] = 0;
    return NET_ERR_NO_PARAMS;
  }
  const Dims& d = s.host->d;
  dims[0] = d.C; dims[1] = d.T; dims[2] = d.F1; dims[3] = d.F2; dims[4] = d.N; dims[5] = d.wbits; dims[6] = 1;
  return NET_OK;
}

size_t net_trial_stride(void) {
  Snapshot s = snapshot();
  return s.host ? trial_stride(s.host->d) : 0;
}

int net_set_device(int device) {
  if (const int rc = check_device(device)) return rc;
  g_single_device.store(device);
  return NET_OK;
}

namespace {
// Makes sure `device` holds the parameter image of snapshot s (uploaded on first use).
int prepare_device(int device, const Snapshot& s) {
  if (const int rc = check_device(device)) return rc;
  DeviceState& ds = g_devs[device];
  std::lock_guard<std::mutex> lk(ds.mu);
  DeviceGuard guard(device);
  if (guard.err != hipSuccess) return hip_err(guard.err);
  return ensure_device(ds, device, s);
}

// ct: channel-major trials [B][C][T] (any alignment, trial stride C T bytes); otherwise the
// time-major batched layout (16-byte aligned, stride net_trial_stride())
// layout: 0 time-major int8, 1 channel-major int8, 2 channel-major float32 (scale qs)
int batch_async_s(const Snapshot& s, const int8_t* x, int8_t* y, size_t B, int device, void* stream, int layout,
                  float qs = 0.0f) {
  if ((!x || !y) && B) return NET_ERR_INVALID;
  const uintptr_t xa = layout == 0 ? 15 : layout == 2 ? 3 : 0;
  if (((uintptr_t)x & xa) != 0 || ((uintptr_t)y & 3) != 0) return NET_ERR_INVALID;
  if (layout == 2 && !(qs > 0.0f && qs <= 3.4e38f)) return NET_ERR_INVALID;
  // the in-kernel quotient correction stays exact while its products are normal floats: scales in
  // [2^-60, 2^60] (checked on every float32 input, tests/test_gpu_f32.py); others: the two-pass
  // quantiser (net_quantize_input_f32), which divides
  if (layout == 2 && !(qs >= 0x1p-60f && qs <= 0x1p60f)) return NET_ERR_RANGE;
  // trial indices are int in the kernel: b + gridDim.x (grid <= 2 per CU) must not wrap
  if (device < 0 || device >= MAX_DEVICES || B > (size_t)INT32_MAX - 65536) return NET_ERR_INVALID;
  if (!s.host) return NET_ERR_NO_PARAMS;
  const Variant v = variant_of(*s.host);
  if (!v.ok()) return NET_ERR_UNSUPPORTED;
  if (const int rc = check_device(device)) return rc;
  DeviceState& ds = g_devs[device];
  std::lock_guard<std::mutex> lk(ds.mu);
  DeviceGuard guard(device);
  if (guard.err != hipSuccess) return hip_err(guard.err);
  int rc = ensure_device(ds, device, s);
  if (rc) return rc;
  rc = launch_forward(v, s.img.data.get(), ds, ds.cur, x, y, B, (hipStream_t)stream, nullptr, layout, qs);
  if (rc == NET_OK && B) note_launch(ds, (hipStream_t)stream);
  return rc;
}

int batch_async(const int8_t* x, int8_t* y, size_t B, int device, void* stream, int layout, float qs = 0.0f) {
  return batch_async_s(snapshot(), x, y, B, device, stream, layout, qs);
}

// The multi-device driver: (1) every listed device gets the parameter image before any shard is
// enqueued, so a first call uploads to all devices up front instead of starting them one after
// another; (2) every shard is enqueued (asynchronous launches), then (3) waited for.  On an
// enqueue error the shards already enqueued are waited for before returning.
extern "C++" {
template <class Prep, class Enq, class Wait>
int multi_driver(int ndev, const int* devices, bool wait_all, Prep&& prep, Enq&& enq, Wait&& wait) {
  for (int i = 0; i < ndev; i++) {
    bool seen = false;
    for (int j = 0; j < i; j++) seen = seen || devices[j] == devices[i];
    if (seen) continue;
    if (const int rc = prep(devices[i])) return rc;
  }
  for (int i = 0; i < ndev; i++) {
    if (const int rc = enq(i)) {
      (void)wait(i);
      return rc;
    }
  }
  return wait_all ? wait(ndev) : NET_OK;
}
}  // extern "C++"
}  // namespace

int net_model_compute_batch_async(const int8_t* x, int8_t* y, size_t B, int device, void* stream) {
  return batch_async(x, y, B, device, stream, 0);
}

int net_model_compute_batch_ct(const int8_t* x, int8_t* y, size_t B, int device, void* stream) {
  return batch_async(x, y, B, device, stream, 1);
}

int net_model_compute_batch_f32(const float* x, int8_t* y, size_t B, float scale, int device, void* stream) {
  return batch_async((const int8_t*)x, y, B, device, stream, 2, scale);
}

int net_quantize_input_f32(const float* x, int8_t* y, size_t B, int C, int T, float scale, int device, void* stream) {
  return quantize_input<float>(x, y, B, C, T, scale, device, stream);
}

int net_quantize_input_f64(const double* x, int8_t* y, size_t B, int C, int T, double scale, int device, void* stream) {
  return quantize_input<double>(x, y, B, C, T, scale, device, stream);
}

int net_pack_trials_i8(const int8_t* x, int8_t* y, size_t B, int C, int T, int device, void* stream) {
  return quantize_input<int8_t>(x, y, B, C, T, (int8_t)1, device, stream);
}

int mibminet_test_reciprocal(int32_t fac, int64_t vmax, int32_t kmax, int32_t magic, float* r, float* c) {
  if (!r || (magic && !c) || vmax < 0 || vmax >= (1 << 24)) return NET_ERR_INVALID;
  return choose_reciprocal(fac, r, magic ? c : nullptr, kmax, vmax) ? NET_OK : NET_ERR_RANGE;
}

int mibminet_test_quantize_f32(const float* x, int8_t* q, size_t n, float scale, int device, void* stream) {
  if ((!x || !q) && n) return NET_ERR_INVALID;
  if (!(scale > 0.0f && scale <= 3.4e38f)) return NET_ERR_INVALID;
  if (!(scale >= 0x1p-60f && scale <= 0x1p60f)) return NET_ERR_RANGE;
  if (const int rc = check_device(device)) return rc;
  if (n == 0) return NET_OK;
  DeviceGuard guard(device);
  if (guard.err != hipSuccess) return hip_err(guard.err);
  hipLaunchKernelGGL(wg::k_quantize_flat, dim3(4096), dim3(256), 0, (hipStream_t)stream, x, q, (long long)n, scale,
                     1.0f / scale);
  return hip_err(hipGetLastError());
}

int mibminet_test_floor_form(int32_t fac, int64_t emax, int64_t vmax, int32_t* mbits, float* r, float* c) {
  if (!mbits || !r || !c || vmax < 0 || emax < 0) return NET_ERR_INVALID;
  return choose_floor_form(fac, emax, vmax, mbits, r, c) ? NET_OK : NET_ERR_RANGE;
}

int mibminet_test_multi_order(int ndev, const int* devices, int fail_at, char* log, size_t len) {
  if (!log || !len || ndev < 1 || ndev > MAX_DEVICES || !devices) return NET_ERR_INVALID;
  std::string out;
  auto prep = [&](int d) { out += "P" + std::to_string(d) + " "; return NET_OK; };
  auto enq = [&](int i) {
    out += "E" + std::to_string(i) + " ";
    return i == fail_at ? NET_ERR_INVALID : NET_OK;
  };
  auto wait = [&](int n) { out += "W" + std::to_string(n) + " "; return NET_OK; };
  const int rc = multi_driver(ndev, devices, true, prep, enq, wait);
  std::snprintf(log, len, "%s", out.c_str());
  return rc;
}

int mibminet_test_upload_stats(int64_t* uploads, int64_t* uploads_while_enqueueing) {
  if (!uploads || !uploads_while_enqueueing) return NET_ERR_INVALID;
  *uploads = g_uploads.load();
  *uploads_while_enqueueing = g_uploads_enqueue.load();
  return NET_OK;
}

int mibminet_test_xdiv_host(const int32_t* e, size_t n, int32_t d, int32_t* q) {
  if ((!e || !q) && n) return NET_ERR_INVALID;
  if (d == 0) return NET_ERR_INVALID;
  const XDiv c = xdiv_consts(d);
  for (size_t i = 0; i < n; i++) q[i] = xdiv_host(e[i], c);
  return NET_OK;
}

int mibminet_test_xdiv_gpu(int32_t d, int64_t e0, int64_t count, int64_t* mismatches, int device) {
  if (!mismatches || d == 0 || count < 0 || e0 < INT32_MIN || e0 + count - 1 > INT32_MAX) return NET_ERR_INVALID;
  if (const int rc = check_device(device)) return rc;
  DeviceGuard guard(device);
  if (guard.err != hipSuccess) return hip_err(guard.err);
  constexpr int GRID = 2048, THREADS = 256;
  unsigned long long* dn = nullptr;
  hipError_t e = hipMalloc((void**)&dn, sizeof(unsigned long long) * GRID * THREADS);
  if (e != hipSuccess) return hip_err(e);
  const XDiv c = xdiv_consts(d);
  hipLaunchKernelGGL(k_xdiv_check, dim3(GRID), dim3(THREADS), 0, nullptr, d, c.m, c.xs, (long long)e0, (long long)count, dn);
  e = hipGetLastError();
  std::vector<unsigned long long> h((size_t)GRID * THREADS);
  if (e == hipSuccess) e = hipMemcpy(h.data(), dn, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost);
  (void)hipFree(dn);
  if (e != hipSuccess) return hip_err(e);
  int64_t n = 0;
  for (unsigned long long v : h) n += (int64_t)v;
  *mismatches = n;
  return NET_OK;
}

int mibminet_test_pool_consts(int32_t off, int32_t layer, int32_t* thr, int32_t* offm) {
  if (!thr || !offm || (layer != 2 && layer != 4)) return NET_ERR_INVALID;
  pool_consts(off, layer == 2 ? (1 << 20) : (1 << 18), thr, offm);
  return NET_OK;
}

int mibminet_test_image_digest(uint64_t* digest) {
  if (!digest) return NET_ERR_INVALID;
  Snapshot s = snapshot();
  if (!s.host) return NET_ERR_NO_PARAMS;
  uint64_t h = 1469598103934665603ull;  // FNV-1a over the image bytes
  const uint8_t* p = (const uint8_t*)s.img.data.get();
  for (size_t i = 0; i < s.img.bytes; i++) h = (h ^ p[i]) * 1099511628211ull;
  *digest = h;
  return NET_OK;
}

int mibminet_test_folded_filters(int32_t* count) {
  if (!count) return NET_ERR_INVALID;
  Snapshot s = snapshot();
  if (!s.host) return NET_ERR_NO_PARAMS;
  *count = s.host->folded;
  return NET_OK;
}

int mibminet_test_force_general(int on) {
  g_force_general.store(on ? 1 : 0);
  return NET_OK;
}

int mibminet_test_params_xr(void) {
  Snapshot s = snapshot();
  if (!s.host) return NET_ERR_NO_PARAMS;
  return s.host->xr ? 1 : 0;
}

int mibminet_test_device_images(int device) {
  if (device < 0 || device >= MAX_DEVICES) return NET_ERR_INVALID;
  DeviceState& ds = g_devs[device];
  std::lock_guard<std::mutex> lk(ds.mu);
  return (int)ds.images.size();
}

int net_argmax_batch(const int8_t* logits, int32_t* cls, size_t B, int N, int device, void* stream) {
  return argmax_batch(logits, cls, B, N, device, stream);
}

namespace {
int batch_multi(int ndev, const int* devices, const int8_t* const* x, int8_t* const* y, const size_t* B,
                void* const* streams, bool ct) {
  if (ndev < 1 || ndev > MAX_DEVICES || !devices || !x || !y || !B) return NET_ERR_INVALID;
  // one parameter snapshot for every shard (a concurrent net_params_load cannot split the batch)
  const Snapshot s = snapshot();
  if (!s.host) return NET_ERR_NO_PARAMS;
  auto wait = [&](int n) -> int {
    int first = NET_OK;
    for (int i = 0; i < n; i++) {
      DeviceGuard guard(devices[i]);
      hipError_t e = guard.err;
      if (e == hipSuccess) e = hipStreamSynchronize(streams ? (hipStream_t)streams[i] : nullptr);
      if (e != hipSuccess && first == NET_OK) first = hip_err(e);
    }
    return first;
  };
  auto enq = [&](int i) -> int {
    t_enqueueing = true;
    const int rc = batch_async_s(s, x[i], y[i], B[i], devices[i], streams ? streams[i] : nullptr, ct ? 1 : 0);
    t_enqueueing = false;
    return rc;
  };
  return multi_driver(ndev, devices, !streams, [&](int d) { return prepare_device(d, s); }, enq, wait);
}
}  // namespace

int net_model_compute_batch_multi(int ndev, const int* devices, const int8_t* const* x, int8_t* const* y,
                                  const size_t* B, void* const* streams) {
  return batch_multi(ndev, devices, x, y, B, streams, false);
}

int net_model_compute_batch_multi_ct(int ndev, const int* devices, const int8_t* const* x, int8_t* const* y,
                                     const size_t* B, void* const* streams) {
  return batch_multi(ndev, devices, x, y, B, streams, true);
}

int net_model_compute_batch(const int8_t* x, int8_t* y, size_t B, int device) {
  int rc = net_model_compute_batch_async(x, y, B, device, nullptr);
  if (rc) return rc;
  DeviceGuard guard(device);
  if (guard.err != hipSuccess) return hip_err(guard.err);
  return hip_err(hipStreamSynchronize(nullptr));
}

int net_model_compute_batch_ct_sync(const int8_t* x, int8_t* y, size_t B, int device) {
  int rc = net_model_compute_batch_ct(x, y, B, device, nullptr);
  if (rc) return rc;
  DeviceGuard guard(device);
  if (guard.err != hipSuccess) return hip_err(guard.err);
  return hip_err(hipStreamSynchronize(nullptr));
}

namespace {
int launch_info(size_t B, int device, int32_t* out, bool ct) {
  if (!out || device < 0 || device >= MAX_DEVICES) return NET_ERR_INVALID;
  Snapshot s = snapshot();
  if (!s.host) return NET_ERR_NO_PARAMS;
  const Variant v = variant_of(*s.host);
  if (const int rc = check_device(device)) return rc;
  DeviceState& ds = g_devs[device];
  std::lock_guard<std::mutex> lk(ds.mu);
  DeviceGuard guard(device);
  if (guard.err != hipSuccess) return hip_err(guard.err);
  int rc = ensure_device(ds, device, s);
  if (rc) return rc;
  return launch_forward(v, s.img.data.get(), ds, nullptr, nullptr, nullptr, B, nullptr, out, ct);
}
}  // namespace

int net_launch_info(size_t B, int device, int32_t* out) { return launch_info(B, device, out, false); }

int net_launch_info_ct(size_t B, int device, int32_t* out) { return launch_info(B, device, out, true); }

int net_forward(const int8_t* p_data, int8_t* p_output) { return run_single(0, p_data, p_output); }

void net_model_compute(const int8_t* p_data, int8_t* p_output) { t_last_error = run_single(0, p_data, p_output); }
void net_layer1(const int8_t* p_data, int8_t* p_result) { t_last_error = run_single(1, p_data, p_result); }
void net_layer2(const int8_t* p_data, int8_t* p_result) { t_last_error = run_single(2, p_data, p_result); }
void net_layer3(const int8_t* p_data, int8_t* p_result) { t_last_error = run_single(3, p_data, p_result); }
void net_layer3_flip_inplace(int8_t* p_data) { t_last_error = run_single(6, p_data, p_data); }
void net_layer4(const int8_t* p_data, int8_t* p_result) { t_last_error = run_single(4, p_data, p_result); }
void net_layer5(const int8_t* p_data, int8_t* p_result) { t_last_error = run_single(5, p_data, p_result); }

int net_last_error(void) { return t_last_error; }

}  // extern "C"
