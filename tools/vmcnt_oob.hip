// Do buffer loads that fetch nothing (every lane past num_records, or an empty view) keep the
// in-order return that s_waitcnt vmcnt(N) relies on, when they are issued behind loads that do go
// to HBM?  (diagnostic; the layer-1 and quantiser loads mix both kinds)
//
// Each wave issues 5 buffer_load_dwordx4 ... nt in one asm block (exact order): load 0 reads HBM,
// loads 1..4 follow the mode's pattern.  Then s_waitcnt vmcnt(4) and a copy of load 0's registers:
// if a younger no-fetch load completed first and decremented the counter, load 0's registers
// still hold the poison value they had before.  Then vmcnt(3..0) for loads 1..4 in turn.
//   mode 0: loads 1..4 read HBM too (control)
//   mode 1: loads 1..4 have every lane past num_records (offset 0x80000000)
//   mode 2: loads 1..4 go through an empty view (num_records = 0)
//   mode 3: loads 1..4 have lanes 48..63 past num_records, the rest in range (partial)
//   mode 4: load 0 has lanes 48..63 past num_records, loads 1..4 every lane
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
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)xt, (short)0, (int)trial_stride, 0x00020000);
    const __amdgpu_buffer_rsrc_t e = __builtin_amdgcn_make_buffer_rsrc((void*)xt, (short)0, 0, 0x00020000);
    unsigned off[5];
    for (int i = 0; i < 5; i++) off[i] = (unsigned)(((((wave * 5 + i) % 34) * 16 + j) * 44 + 16 * g));  // < stride - 16
    const bool far = mode == 1 || mode == 4 || (mode == 3 && g == 3);
    for (int i = 1; i < 5; i++)
      if (far) off[i] = 0x80000000u;
    if (mode == 4 && g == 3) off[0] = 0x80000000u;
    const __amdgpu_buffer_rsrc_t r1 = mode == 2 ? e : r;
    v4i r0, v1, v2, v3, v4;
    const int P = 0x7fc0dead;
    r0 = v1 = v2 = v3 = v4 = (v4i){P, P, P, P};
    asm volatile(
        "buffer_load_dwordx4 %0, %5, %10, 0 offen nt\n"
        "buffer_load_dwordx4 %1, %6, %11, 0 offen nt\n"
        "buffer_load_dwordx4 %2, %7, %11, 0 offen nt\n"
        "buffer_load_dwordx4 %3, %8, %11, 0 offen nt\n"
        "buffer_load_dwordx4 %4, %9, %11, 0 offen nt\n"
        : "+&v"(r0), "+&v"(v1), "+&v"(v2), "+&v"(v3), "+&v"(v4)
        : "v"(off[0]), "v"(off[1]), "v"(off[2]), "v"(off[3]), "v"(off[4]), "s"(r), "s"(r1)
        : "memory");
    int c[5];
    asm volatile("s_waitcnt vmcnt(4)\n v_mov_b32 %0, %1" : "=v"(c[0]) : "v"(r0.w));
    asm volatile("s_waitcnt vmcnt(3)\n v_mov_b32 %0, %1" : "=v"(c[1]) : "v"(v1.w));
    asm volatile("s_waitcnt vmcnt(2)\n v_mov_b32 %0, %1" : "=v"(c[2]) : "v"(v2.w));
    asm volatile("s_waitcnt vmcnt(1)\n v_mov_b32 %0, %1" : "=v"(c[3]) : "v"(v3.w));
    asm volatile("s_waitcnt vmcnt(0)\n v_mov_b32 %0, %1" : "=v"(c[4]) : "v"(v4.w));
    asm volatile("" ::"v"(r0), "v"(v1), "v"(v2), "v"(v3), "v"(v4));  // loads' registers stay reserved
    for (int i = 0; i < 5; i++) {
      const bool oob = off[i] >= 0x80000000u || (i > 0 && mode == 2);
      const int want = oob ? 0 : *(const int*)(xt + off[i] + 12);  // plain (ordered, waited) reference load
      if (c[i] == 0x7fc0dead) atomicAdd(&bad[16 * mode + i], 1u);
      else if (c[i] != want) atomicAdd(&bad[16 * mode + 8 + i], 1u);
    }
  }
}

int main() {
  const int B = 65536;
  const size_t stride = 24768;
  int8_t* x;
  unsigned* bad;
  hipMalloc(&x, (size_t)B * stride + 65536);
  hipMalloc(&bad, 5 * 64);
  std::vector<int8_t> h((size_t)B * stride);
  for (size_t i = 0; i < h.size(); i++) h[i] = (int8_t)((i * 2654435761u) >> 13);
  hipMemcpy(x, h.data(), h.size(), hipMemcpyHostToDevice);
  hipMemset(bad, 0, 5 * 64);
  hipMemset(x + (size_t)B * stride, 0, 65536);
  const int reps = 20;
  for (int mode = 0; mode < 5; mode++)
    for (int rep = 0; rep < reps; rep++) hipLaunchKernelGGL(k, dim3(512), dim3(512), 0, 0, x, stride, B, bad, mode);
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  unsigned hb[80];
  hipMemcpy(hb, bad, sizeof(hb), hipMemcpyDeviceToHost);
  printf("loads checked per slot and mode: %lld\n", (long long)reps * B * 8 * 64);
  for (int mode = 0; mode < 5; mode++)
    for (int i = 0; i < 5; i++)
      printf("mode %d slot %d (after vmcnt(%d)): %u still poison, %u other mismatches\n", mode, i, 4 - i,
             hb[16 * mode + i], hb[16 * mode + 8 + i]);
  return 0;
}
