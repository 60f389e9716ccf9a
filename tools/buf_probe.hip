// Raw buffer load range checking on gfx950 (diagnostic): dwordx4 at 4-byte-aligned offsets
// straddling num_records; offsets via VGPR and via the immediate field.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef unsigned v4u __attribute__((ext_vector_type(4)));
__global__ void k(const unsigned char* x, v4u* o, int nrec) {
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)x, (short)0, nrec, 0x00020000);
  const int t = threadIdx.x;  // offset nrec - 32 + 4 t
  o[t] = __builtin_amdgcn_raw_buffer_load_b128(r, nrec - 32 + 4 * t, 0, 2);
  o[64 + t] = __builtin_amdgcn_raw_buffer_load_b128(r, nrec - 32 - 704 + 4 * t + 0, 0, 2);  // then +704 imm below
  v4u b = __builtin_amdgcn_raw_buffer_load_b128(r, nrec - 32 - 704 + 4 * t, 0, 2);
  asm volatile("" ::: "memory");
  v4u c;
  const int vo = nrec - 32 - 704 + 4 * t;
  asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen offset:704 nt\n s_waitcnt vmcnt(0)" : "=v"(c) : "v"(vo), "s"(r));
  o[128 + t] = c;
  (void)b;
}
int main() {
  const int N = 4096, nrec = 2000;
  unsigned char h[N];
  for (int i = 0; i < N; i++) h[i] = (unsigned char)(i * 7 + 1);
  unsigned char* d; v4u* o;
  hipMalloc(&d, N); hipMalloc(&o, 192 * 16);
  hipMemcpy(d, h, N, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, 1, 16, 0, 0, d, o, nrec);
  v4u r[192]; hipMemcpy(r, o, sizeof(r), hipMemcpyDeviceToHost);
  for (int t = 0; t < 12; t++) {
    int off = nrec - 32 + 4 * t;
    printf("off %d (end %d):", off, off + 16);
    for (int w = 0; w < 4; w++) {
      unsigned want = 0;
      for (int b = 0; b < 4; b++) want |= (unsigned)h[off + 4 * w + b] << (8 * b);
      printf(" dw%d %s", w, r[t][w] == want ? "data" : r[t][w] == 0 ? "ZERO" : "????");
    }
    printf(" | imm-path:");
    for (int w = 0; w < 4; w++) {
      unsigned want = 0;
      for (int b = 0; b < 4; b++) want |= (unsigned)h[off + 4 * w + b] << (8 * b);
      printf(" %s", r[128 + t][w] == want ? "data" : r[128 + t][w] == 0 ? "ZERO" : "????");
    }
    printf("\n");
  }
  return 0;
}
