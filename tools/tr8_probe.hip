// gfx950 probe (diagnostic, not part of the product) for the channel-major staging:
//  1. ds_read_b64_tr_b8: which LDS bytes each lane receives, for per-lane addresses 8 * lane
//     (prints, per 16-lane group, the row/column map the hardware applies);
//  2. the staging form forward_wg.hpp uses: lane L stores 16 bytes (a row of 16 samples) at
//     16 pos(L), and two transposed reads per lane must return the MFMA A fragment
//     A[j][16 g + jj] = row (16 g + jj) byte j  (checked for every lane and byte);
//  3. LDS-DMA (buffer_load_dwordx4 ... lds, __builtin_amdgcn_raw_ptr_buffer_load_lds) from
//     byte-unaligned source offsets and from lanes past num_records: what lands in LDS.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef int v2i __attribute__((ext_vector_type(2)));
typedef int v4i __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v2i lds_v2i;

__global__ void k_map(unsigned* out, int hi) {
  __shared__ __attribute__((aligned(16))) unsigned char s[1024];
  const int l = threadIdx.x;
  for (int i = l; i < 1024; i += 64) s[i] = hi ? (unsigned char)(i >> 8) : (unsigned char)i;
  __syncthreads();
  const v2i v = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_v2i*)(s + 8 * l));
  out[2 * l] = v[0];
  out[2 * l + 1] = v[1];
}

// staging form: row k (16 bytes) = logical K-slot k; physical row pos(k) = 16 g + 8 (r ^ (g & 1)) + q
__device__ __host__ inline int pos(int k) {
  const int g = k >> 4, r = (k >> 3) & 1, q = k & 7;
  return 16 * g + 8 * (r ^ (g & 1)) + q;
}

__global__ void k_stage(const v4i* rows, v4i* out, int qsel) {
  __shared__ __attribute__((aligned(16))) unsigned char s[1024];
  const int l = threadIdx.x;
  *(v4i*)(s + 16 * pos(l)) = rows[l];  // lane l holds logical row l
  __syncthreads();
  const int i = l & 15, g = l >> 4;
  // lane i of the group supplies (row q, half p) of its 8-row block: qsel 0: q = i >> 1, p = i & 1;
  // qsel 1: q = i & 7, p = i >> 3
  const int q = qsel ? (i & 7) : (i >> 1), p = qsel ? (i >> 3) : (i & 1);
  const int b0 = 256 * g + 128 * (g & 1) + 16 * q + 8 * p;  // logical slots 16 g .. 16 g + 7
  const v2i lo = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_v2i*)(s + b0));
  const v2i hh = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_v2i*)(s + (b0 ^ 128)));
  out[l] = (v4i){lo[0], lo[1], hh[0], hh[1]};
}

__global__ void k_dma(const unsigned char* x, unsigned char* out, int nrec, int base, int stride) {
  __shared__ __attribute__((aligned(16))) unsigned char s[1024];
  const int l = threadIdx.x;
  for (int i = l; i < 1024; i += 64) s[i] = 0xEE;
  __syncthreads();
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)x, (short)0, nrec, 0x00020000);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)s, 16, base + stride * l, 0, 0, 0);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  for (int i = l; i < 1024; i += 64) out[i] = s[i];
}

int main() {
  unsigned *d;
  hipMalloc(&d, 64 * 8);
  std::vector<unsigned> lo(128), hi(128);
  hipLaunchKernelGGL(k_map, 1, 64, 0, 0, d, 0);
  hipMemcpy(lo.data(), d, 512, hipMemcpyDeviceToHost);
  hipLaunchKernelGGL(k_map, 1, 64, 0, 0, d, 1);
  hipMemcpy(hi.data(), d, 512, hipMemcpyDeviceToHost);
  printf("1. ds_read_b64_tr_b8 with address 8 * lane: byte indices received (lane: 8 bytes)\n");
  for (int l = 0; l < 64; l++) {
    printf("  lane %2d:", l);
    for (int b = 0; b < 8; b++) {
      const int w = b / 4, sh = 8 * (b % 4);
      const int idx = ((lo[2 * l + w] >> sh) & 255) | (((hi[2 * l + w] >> sh) & 255) << 8);
      printf(" %4d", idx);
    }
    printf("\n");
  }
  // 2. staging form
  std::vector<int> rows(64 * 4);
  unsigned char* rb = (unsigned char*)rows.data();
  for (int k = 0; k < 64; k++)
    for (int j = 0; j < 16; j++) rb[16 * k + j] = (unsigned char)(k * 16 + j * 3 + 5);
  v4i *drows, *dout;
  hipMalloc(&drows, 1024); hipMalloc(&dout, 1024);
  hipMemcpy(drows, rows.data(), 1024, hipMemcpyHostToDevice);
  for (int qsel = 0; qsel < 2; qsel++) {
    hipLaunchKernelGGL(k_stage, 1, 64, 0, 0, drows, dout, qsel);
    std::vector<unsigned char> o(1024);
    hipMemcpy(o.data(), dout, 1024, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; l++) {
      const int j = l & 15, g = l >> 4;
      for (int jj = 0; jj < 16; jj++) bad += o[16 * l + jj] != rb[16 * (16 * g + jj) + j];
    }
    printf("2. staging form (lane map %s): %d wrong bytes of 1024\n", qsel ? "q = i & 7, p = i >> 3" : "q = i >> 1, p = i & 1", bad);
  }
  // 3. LDS-DMA
  const int N = 8192;
  std::vector<unsigned char> hx(N);
  for (int i = 0; i < N; i++) hx[i] = (unsigned char)(i * 7 + 3);
  unsigned char *dx, *dl;
  hipMalloc(&dx, N); hipMalloc(&dl, 1024);
  hipMemcpy(dx, hx.data(), N, hipMemcpyHostToDevice);
  for (int base : {0, 1, 2, 3, 1125}) {
    for (int nrec : {N, 1125 + 16 * 40 + 7}) {
      hipLaunchKernelGGL(k_dma, 1, 64, 0, 0, dx, dl, nrec, base, 17);
      std::vector<unsigned char> o(1024);
      hipMemcpy(o.data(), dl, 1024, hipMemcpyDeviceToHost);
      int bad = 0, zero = 0, kept = 0, partial = 0;
      for (int l = 0; l < 64; l++) {
        const int off = base + 17 * l;
        for (int i = 0; i < 16; i++) {
          const int src = off + i;
          const unsigned char got = o[16 * l + i];
          if (off + 16 <= nrec) bad += got != hx[src];
          else {
            zero += got == 0;
            kept += got == 0xEE;
            partial += (src < nrec && got == hx[src]);
          }
        }
      }
      printf("3. LDS-DMA base %4d stride 17 nrec %5d: in-range wrong bytes %d; straddling/out-of-range bytes: zero %d, untouched %d, data %d\n",
             base, nrec, bad, zero, kept, partial);
    }
  }
  return 0;
}
