// gfx950 probe (diagnostic, not part of the product) for a parity-split channel-major staging:
//  1. ds_read_b64_tr_b16: which 16-bit LDS elements each lane receives for per-lane addresses
//     8 * lane (prints, per 16-lane group, the row/column map the hardware applies);
//  2. the staging form: block image rows = channels (32 bytes = 16 sample pairs each), and two
//     transposed reads per lane must return the layer-1 A fragment with MFMA row j = sample pair j
//     and K-slot 2 c + p = (channel c, parity p): A[j][16 g + kk] = x[c][2 j + p], c = 8 g + kk / 2
//     (checked for every lane and byte, for each candidate lane -> (row, piece) map).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef short v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

__global__ void k_map(unsigned short* out) {
  __shared__ __attribute__((aligned(16))) unsigned short s[512];
  const int l = threadIdx.x;
  for (int i = l; i < 512; i += 64) s[i] = (unsigned short)i;
  __syncthreads();
  const v4s v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(s + 4 * l));
  for (int k = 0; k < 4; k++) out[4 * l + k] = (unsigned short)v[k];
}

// image: row r (32 bytes) at byte 32 pos(r); pos = swizzled row slot
__device__ __host__ inline int pos(int r, int sw) { return sw ? r ^ (((r >> 3) & 1) << 2) : r; }

__global__ void k_stage(const unsigned char* img_rows, unsigned* out, int qsel, int sw) {
  __shared__ __attribute__((aligned(16))) unsigned char s[1024];
  const int l = threadIdx.x;
  // lane l stores 16 bytes: row l >> 1, half l & 1
  const int r = l >> 1, h = l & 1;
  for (int b = 0; b < 16; b++) s[32 * pos(r, sw) + 16 * h + b] = img_rows[32 * r + 16 * h + b];
  __syncthreads();
  const int i = l & 15, g = l >> 4;
  unsigned w[4];
  for (int rr = 0; rr < 2; rr++) {
    // lane i supplies (row q, piece p) of its 4-row block: qsel 0: q = i >> 2, p = i & 3; 1: q = i & 3, p = i >> 2
    const int q = qsel ? (i & 3) : (i >> 2), p = qsel ? (i >> 2) : (i & 3);
    const int row = 8 * g + 4 * rr + q;
    const v4s v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(s + 32 * pos(row, sw) + 8 * p));
    w[2 * rr] = (unsigned short)v[0] | ((unsigned)(unsigned short)v[1] << 16);
    w[2 * rr + 1] = (unsigned short)v[2] | ((unsigned)(unsigned short)v[3] << 16);
  }
  for (int k = 0; k < 4; k++) out[4 * l + k] = w[k];
}

int main() {
  unsigned short* d;
  (void)hipMalloc(&d, 64 * 4 * 2);
  std::vector<unsigned short> m(256);
  hipLaunchKernelGGL(k_map, 1, 64, 0, 0, d);
  (void)hipMemcpy(m.data(), d, 512, hipMemcpyDeviceToHost);
  printf("1. ds_read_b64_tr_b16 with address 8 * lane: 16-bit element indices received\n");
  for (int l = 0; l < 64; l++) printf("  lane %2d: %4d %4d %4d %4d\n", l, m[4 * l], m[4 * l + 1], m[4 * l + 2], m[4 * l + 3]);
  // 2. staging form: 32 rows (channels) x 32 bytes
  std::vector<unsigned char> rows(1024);
  for (int i = 0; i < 1024; i++) rows[i] = (unsigned char)(i * 7 + 3);
  unsigned char* dr;
  unsigned* dout;
  (void)hipMalloc(&dr, 1024);
  (void)hipMalloc(&dout, 64 * 16);
  (void)hipMemcpy(dr, rows.data(), 1024, hipMemcpyHostToDevice);
  for (int sw = 0; sw < 2; sw++)
    for (int qsel = 0; qsel < 2; qsel++) {
      std::vector<unsigned> o(256);
      hipLaunchKernelGGL(k_stage, 1, 64, 0, 0, dr, dout, qsel, sw);
      (void)hipMemcpy(o.data(), dout, 1024, hipMemcpyDeviceToHost);
      int bad = 0;
      for (int l = 0; l < 64; l++) {
        const int j = l & 15, g = l >> 4;
        for (int kk = 0; kk < 16; kk++) {
          const int c = 8 * g + kk / 2, p = kk & 1;
          const unsigned char want = rows[32 * c + 2 * j + p];
          const unsigned char got = (unsigned char)(o[4 * l + kk / 4] >> (8 * (kk % 4)));
          bad += want != got;
        }
      }
      printf("2. staging form, swizzle %d, map %s: %d of 1024 bytes wrong\n", sw, qsel ? "q = i & 3, p = i >> 2" : "q = i >> 2, p = i & 3", bad);
    }
  return 0;
}
