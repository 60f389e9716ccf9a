// Hypothesis (ii) of the round-1 layer-1 row fault: an MFMA that reads its C-init
// tuple two wait states after the VALU moves that built it, while HBM loads are still returning
// into other registers of the wave, reads a stale C-init register in some lanes.  (diagnostic)
//
// The asm block below repeats the faulting build's stage-1 sequence: five buffer loads (the first
// into the registers that then become tile 0's C-init), vmcnt(4), the tile-0 C-init moves,
// vmcnt(3), MFMA 0, the tile-1 C-init moves, one unrelated VALU, s_nop 0 (so the last move is two
// wait states ahead of MFMA 1, the compiler's minimum), MFMA 1.  A = all 1s, B0 = all 1s,
// B1 = all 2s, so every accumulator element must be init + 64 (tile 0) and init + 128 (tile 1).
// Mode 0 runs it as is; mode 1 pads four more wait states before each MFMA (the control).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

typedef int v4i __attribute__((ext_vector_type(4)));

__global__ void k(const int8_t* __restrict__ x, size_t trial_stride, int ntrials, int iters, unsigned* bad, int mode) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int j = lane & 15, g = lane >> 4;
  const int INIT = 0x4B400000;  // the float magic of the layer-1 C-init
  int t = blockIdx.x;
  for (int it = 0; it < iters; it++, t += gridDim.x) {
    if (t >= ntrials) t -= ntrials;
    const int8_t* xt = x + (size_t)t * trial_stride;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)xt, (short)0, (int)trial_stride, 0x00020000);
    unsigned off[5];
    for (int i = 0; i < 5; i++) off[i] = (unsigned)(((((wave * 5 + i) % 34) * 16 + j) * 44 + 16 * g));
    v4i acc0, acc1;
    int junk = lane;
    // fixed registers: c0 v[40:43] (first load, then tile 0's C-init), loads v[44:59], c1 v[60:63],
    // acc v[64:71], A/B0/B1 v[72:83], init v84, junk v85, offsets v[86:90]
#define CINIT_SEQ(PAD)                                                                              \
  asm volatile(                                                                                     \
      "v_mov_b32 v72, %[a0]\n v_mov_b32 v73, %[a0]\n v_mov_b32 v74, %[a0]\n v_mov_b32 v75, %[a0]\n"   \
      "v_mov_b32 v76, %[a0]\n v_mov_b32 v77, %[a0]\n v_mov_b32 v78, %[a0]\n v_mov_b32 v79, %[a0]\n"   \
      "v_mov_b32 v80, %[b1]\n v_mov_b32 v81, %[b1]\n v_mov_b32 v82, %[b1]\n v_mov_b32 v83, %[b1]\n"   \
      "v_mov_b32 v84, %[init]\n v_mov_b32 v85, %[junk]\n"                                            \
      "v_mov_b32 v86, %[o0]\n v_mov_b32 v87, %[o1]\n v_mov_b32 v88, %[o2]\n v_mov_b32 v89, %[o3]\n" \
      "v_mov_b32 v90, %[o4]\n"                                                                     \
      "s_nop 7\n"                                                                                  \
      "buffer_load_dwordx4 v[40:43], v86, %[r], 0 offen nt\n"                                      \
      "buffer_load_dwordx4 v[44:47], v87, %[r], 0 offen nt\n"                                      \
      "buffer_load_dwordx4 v[48:51], v88, %[r], 0 offen nt\n"                                      \
      "buffer_load_dwordx4 v[52:55], v89, %[r], 0 offen nt\n"                                      \
      "buffer_load_dwordx4 v[56:59], v90, %[r], 0 offen nt\n"                                      \
      "s_waitcnt vmcnt(4)\n"                                                                       \
      "v_mov_b32 v40, v84\n v_mov_b32 v41, v84\n v_mov_b32 v42, v84\n v_mov_b32 v43, v84\n"       \
      "v_mov_b32 v60, v84\n v_mov_b32 v61, v84\n"                                                 \
      "s_waitcnt vmcnt(3)\n" PAD                                                                   \
      "v_mfma_i32_16x16x64_i8 v[64:67], v[72:75], v[76:79], v[40:43]\n"                             \
      "v_mov_b32 v62, v84\n v_mov_b32 v63, v84\n"                                                 \
      "v_or_b32 v85, 1, v85\n"                                                                     \
      "s_nop 0\n" PAD                                                                              \
      "v_mfma_i32_16x16x64_i8 v[68:71], v[72:75], v[80:83], v[60:63]\n"                             \
      "s_waitcnt vmcnt(0)\n"                                                                       \
      "s_nop 15\n s_nop 15\n"                                                                     \
      "v_mov_b32 %[x0], v64\n v_mov_b32 %[x1], v65\n v_mov_b32 %[x2], v66\n v_mov_b32 %[x3], v67\n" \
      "v_mov_b32 %[y0], v68\n v_mov_b32 %[y1], v69\n v_mov_b32 %[y2], v70\n v_mov_b32 %[y3], v71\n" \
      "v_mov_b32 %[junk], v85\n"                                                                   \
      : [x0] "=&v"(acc0[0]), [x1] "=&v"(acc0[1]), [x2] "=&v"(acc0[2]), [x3] "=&v"(acc0[3]),         \
        [y0] "=&v"(acc1[0]), [y1] "=&v"(acc1[1]), [y2] "=&v"(acc1[2]), [y3] "=&v"(acc1[3]),         \
        [junk] "+v"(junk)                                                                           \
      : [o0] "v"(off[0]), [o1] "v"(off[1]), [o2] "v"(off[2]), [o3] "v"(off[3]), [o4] "v"(off[4]),   \
        [r] "s"(r), [init] "v"(INIT), [a0] "v"(0x01010101), [b1] "v"(0x02020202)                      \
      : "memory", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", \
        "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64",   \
        "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77",   \
        "v78", "v79", "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90")
    if (mode == 0) {
      CINIT_SEQ("");
    } else {
      CINIT_SEQ("s_nop 3\n");
    }
    for (int q = 0; q < 4; q++) {
      if (acc0[q] != INIT + 64) atomicAdd(&bad[32 * mode + 4 * g + (acc0[q] == 64 ? 1 : 0)], 1u);
      if (acc1[q] != INIT + 128) atomicAdd(&bad[32 * mode + 16 + 4 * g + (acc1[q] == 128 ? 1 : 0)], 1u);
    }
  }
}

int main(int argc, char** argv) {
  const int B = 65536;
  const size_t stride = 24768;
  const int iters = argc > 1 ? atoi(argv[1]) : 2000;
  int8_t* x;
  unsigned* bad;
  if (hipMalloc(&x, (size_t)B * stride + 65536) != hipSuccess) return 1;
  hipMalloc(&bad, 64 * 4);
  std::vector<int8_t> h((size_t)B * stride);
  for (size_t i = 0; i < h.size(); i++) h[i] = (int8_t)((i * 2654435761u) >> 13);
  hipMemcpy(x, h.data(), h.size(), hipMemcpyHostToDevice);
  hipMemset(bad, 0, 64 * 4);
  for (int mode = 0; mode < 2; mode++) hipLaunchKernelGGL(k, dim3(1024), dim3(512), 0, 0, x, stride, B, iters, bad, mode);
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  unsigned hb[64];
  hipMemcpy(hb, bad, sizeof(hb), hipMemcpyDeviceToHost);
  printf("MFMA pairs per mode: %lld (each 64 lanes x 4 elements per tile)\n", (long long)iters * 1024 * 8);
  for (int mode = 0; mode < 2; mode++) {
    printf("mode %d (%s):\n", mode, mode ? "4 extra wait states" : "compiler-minimum wait states");
    for (int tile = 0; tile < 2; tile++)
      for (int g = 0; g < 4; g++)
        printf("  tile %d lanes %2d..%2d: %u wrong (of which %u equal the bare dot: C-init lost)\n", tile, 16 * g,
               16 * g + 15, hb[32 * mode + 16 * tile + 4 * g] + hb[32 * mode + 16 * tile + 4 * g + 1],
               hb[32 * mode + 16 * tile + 4 * g + 1]);
  }
  return 0;
}
