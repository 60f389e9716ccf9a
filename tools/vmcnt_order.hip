// Does s_waitcnt vmcnt(N) guarantee the data of the (5-N)th oldest of 5 outstanding
// global_load_dwordx4 ... nt (4-byte aligned, layer-1 address pattern) on gfx950?  (diagnostic)
// Each wave issues 5 loads into distinct registers (one asm block: exact order), then for
// k = 0..4: s_waitcnt vmcnt(4-k) and copies load k's registers (v_mov) -- a load whose data is
// not there yet shows the poison value the registers held before.  Counts mismatches per k.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

typedef int v4i __attribute__((ext_vector_type(4)));

__global__ void k(const int8_t* __restrict__ x, size_t trial_stride, int ntrials, unsigned* bad, int mode) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int j = lane & 15, g = lane >> 4;
  for (int t = blockIdx.x; t < ntrials; t += gridDim.x) {
    const int8_t* xt = x + (size_t)t * trial_stride;
    unsigned off[5];
    for (int i = 0; i < 5; i++) off[i] = (unsigned)(((wave * 5 + i) * 16 + j) * 44 + 16 * g);
    v4i r0, r1, r2, r3, r4;
    const int P = 0x7fc0dead;
    r0 = r1 = r2 = r3 = r4 = (v4i){P, P, P, P};
    asm volatile(
        "global_load_dwordx4 %0, %5, %10 nt\n"
        "global_load_dwordx4 %1, %6, %10 nt\n"
        "global_load_dwordx4 %2, %7, %10 nt\n"
        "global_load_dwordx4 %3, %8, %10 nt\n"
        "global_load_dwordx4 %4, %9, %10 nt\n"
        : "+&v"(r0), "+&v"(r1), "+&v"(r2), "+&v"(r3), "+&v"(r4)
        : "v"(off[0]), "v"(off[1]), "v"(off[2]), "v"(off[3]), "v"(off[4]), "s"(xt)
        : "memory");
    int c[5];
    asm volatile("s_waitcnt vmcnt(4)\n v_mov_b32 %0, %1" : "=v"(c[0]) : "v"(r0.w));
    asm volatile("s_waitcnt vmcnt(3)\n v_mov_b32 %0, %1" : "=v"(c[1]) : "v"(r1.w));
    asm volatile("s_waitcnt vmcnt(2)\n v_mov_b32 %0, %1" : "=v"(c[2]) : "v"(r2.w));
    asm volatile("s_waitcnt vmcnt(1)\n v_mov_b32 %0, %1" : "=v"(c[3]) : "v"(r3.w));
    asm volatile("s_waitcnt vmcnt(0)\n v_mov_b32 %0, %1" : "=v"(c[4]) : "v"(r4.w));
    asm volatile("" ::"v"(r0), "v"(r1), "v"(r2), "v"(r3), "v"(r4));  // loads' registers stay reserved
    for (int i = 0; i < 5; i++) {
      const int want = *(const int*)(xt + off[i] + 12);  // plain (ordered, waited) reference load
      if (c[i] == 0x7fc0dead) atomicAdd(&bad[i], 1u);
      else if (c[i] != want) atomicAdd(&bad[8 + i], 1u);
    }
  }
}

int main() {
  const int B = 65536;
  const size_t stride = 24768;
  int8_t* x;
  unsigned* bad;
  hipMalloc(&x, (size_t)B * stride + 65536);
  hipMalloc(&bad, 64);
  std::vector<int8_t> h((size_t)B * stride);
  for (size_t i = 0; i < h.size(); i++) h[i] = (int8_t)((i * 2654435761u) >> 13);
  hipMemcpy(x, h.data(), h.size(), hipMemcpyHostToDevice);
  hipMemset(bad, 0, 64);
  hipMemset(x + (size_t)B * stride, 0, 65536);
  for (int rep = 0; rep < 20; rep++) hipLaunchKernelGGL(k, dim3(512), dim3(512), 0, 0, x, stride, B, bad, 0);
  hipDeviceSynchronize();
  unsigned hb[16];
  hipMemcpy(hb, bad, 64, hipMemcpyDeviceToHost);
  printf("loads checked per slot: %lld\n", 20LL * B * 8 * 64);
  for (int i = 0; i < 5; i++) printf("slot %d (after vmcnt(%d)): %u still poison, %u other mismatches\n", i, 4 - i, hb[i], hb[8 + i]);
  return 0;
}
