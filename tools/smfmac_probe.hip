// ISA probe (diagnostic, not part of the product): the operand layout of the gfx950 2:4 sparse
// i8 MFMA, v_smfmac_i32_32x32x64_i8 D(32x32) += A(32x64, 2:4 sparse) * B(64x32), groundwork for a
// sparse layer-2 band.  Random compressed A values, random valid index
// pairs and random B go through one instruction per wave; the host model below (the hypothesis)
// is compared element by element:
//   A: lane l holds row l % 32, compressed bytes 16 (l / 32) .. +16 -> logical K groups
//      8 (l / 32) .. +8, two values per group of 4 (byte 2q + s is value s of group q)
//   idx (one VGPR per lane, cbsz = abid = 0): 2 bits per value, value s of group q at bits
//      4 q + 2 s .. +2, the position (0..3) of that value inside its group of 4 logical K
//   B: lane l holds column l % 32; its bytes 0-15 are logical K 16 (l / 32) .. +16 and bytes
//      16-31 are K 32 + 16 (l / 32) .. +16 (measured: model 2 below, 0 of 20,480 outputs differ;
//      K 32 (l / 32) .. +32 contiguous, model 0, differs everywhere)
//   D: lane l, register r: row 8 (r / 4) + 4 (l / 32) + r % 4, column l % 32 (as the dense
//      32x32 shapes)
// usage: smfmac_probe [trials]   prints the mismatch count of each model variant
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v8i __attribute__((ext_vector_type(8)));
typedef int v16i __attribute__((ext_vector_type(16)));

__global__ void k_probe(const v4i* a, const v8i* b, const int* idx, v16i* d) {
  const int l = threadIdx.x;
  v16i c = {};
  d[l] = __builtin_amdgcn_smfmac_i32_32x32x64_i8(a[l], b[l], c, idx[l], 0, 0);
}

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      std::printf("%s: %s\n", #x, hipGetErrorString(e_));                     \
      std::exit(1);                                                           \
    }                                                                         \
  } while (0)

int main(int argc, char** argv) {
  const int trials = argc > 1 ? std::atoi(argv[1]) : 20;
  std::mt19937 rng(7);
  int8_t *da, *db;
  int *di, *dd;
  CHECK(hipMalloc(&da, 64 * 16));
  CHECK(hipMalloc(&db, 64 * 32));
  CHECK(hipMalloc(&di, 64 * 4));
  CHECK(hipMalloc(&dd, 64 * 64));
  // model variants: bit 0 = value order inside a group's index nibble swapped, bit 1 = B lane halves
  // interleaved (lane half h holds logical K 16 h + 32 j .. for j = 0, 1) instead of contiguous
  long bad[4] = {0, 0, 0, 0};
  for (int t = 0; t < trials; t++) {
    std::vector<int8_t> a(64 * 16), b(64 * 32);
    std::vector<int> idx(64), d(64 * 16);
    for (auto& v : a) v = (int8_t)(rng() % 256 - 128);
    for (auto& v : b) v = (int8_t)(rng() % 256 - 128);
    for (int l = 0; l < 64; l++) {
      unsigned w = 0;
      for (int q = 0; q < 8; q++) {
        int p0 = rng() % 4, p1 = rng() % 3;
        if (p1 >= p0) p1++;
        if (p0 > p1) std::swap(p0, p1);  // ascending positions in a group
        w |= (unsigned)(p0 | (p1 << 2)) << (4 * q);
      }
      idx[l] = (int)w;
    }
    CHECK(hipMemcpy(da, a.data(), a.size(), hipMemcpyHostToDevice));
    CHECK(hipMemcpy(db, b.data(), b.size(), hipMemcpyHostToDevice));
    CHECK(hipMemcpy(di, idx.data(), 64 * 4, hipMemcpyHostToDevice));
    k_probe<<<1, 64>>>((const v4i*)da, (const v8i*)db, di, (v16i*)dd);
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemcpy(d.data(), dd, 64 * 64, hipMemcpyDeviceToHost));
    for (int var = 0; var < 4; var++) {
      // logical dense A (32 x 64) and B (64 x 32) under this variant
      static int A[32][64], Bm[64][32];
      for (int i = 0; i < 32; i++)
        for (int k = 0; k < 64; k++) A[i][k] = 0;
      for (int l = 0; l < 64; l++) {
        const int row = l % 32, h = l / 32;
        for (int q = 0; q < 8; q++)
          for (int s = 0; s < 2; s++) {
            const int ss = (var & 1) ? 1 - s : s;
            const int pos = (idx[l] >> (4 * q + 2 * ss)) & 3;
            A[row][32 * h + 4 * q + pos] += a[16 * l + 2 * q + s];
          }
        for (int kk = 0; kk < 32; kk++) {
          const int k = (var & 2) ? 16 * h + 32 * (kk / 16) + kk % 16 : 32 * h + kk;
          Bm[k][l % 32] = b[32 * l + kk];
        }
      }
      for (int l = 0; l < 64; l++)
        for (int r = 0; r < 16; r++) {
          const int i = 8 * (r / 4) + 4 * (l / 32) + r % 4, j = l % 32;
          long s = 0;
          for (int k = 0; k < 64; k++) s += (long)A[i][k] * Bm[k][j];
          if (s != d[16 * l + r]) bad[var]++;
        }
    }
  }
  for (int var = 0; var < 4; var++)
    std::printf("model %d (index order %s, B halves %s): %ld of %d outputs differ\n", var,
                (var & 1) ? "swapped" : "as documented", (var & 2) ? "interleaved" : "contiguous", bad[var],
                trials * 64 * 16);
  return 0;
}
