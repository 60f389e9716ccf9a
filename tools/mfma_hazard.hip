// Diagnostic probe (not part of the product): do gfx950 i8 MFMAs tolerate overwriting their
// source registers right after issue, and a destination that partially overlaps a source?
// Each case runs a hazard-free reference sequence and the suspect sequence on the same inputs.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef int v4i __attribute__((ext_vector_type(4)));
#define NOPS "s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n"

__global__ void k(const v4i* a, const v4i* b, v4i* out) {
  const int l = threadIdx.x;
  v4i A = a[l], Bv = b[l], r;
  // case 0: reference 16x16x64
  asm volatile(
      "v_mov_b32 v40, %1\n v_mov_b32 v41, %2\n v_mov_b32 v42, %3\n v_mov_b32 v43, %4\n"
      "v_mov_b32 v44, %5\n v_mov_b32 v45, %6\n v_mov_b32 v46, %7\n v_mov_b32 v47, %8\n" NOPS
      "v_mfma_i32_16x16x64_i8 v[48:51], v[40:43], v[44:47], 0\n" NOPS
      "v_mov_b32 %0, v48\n"
      : "=v"(r[0]) : "v"(A[0]), "v"(A[1]), "v"(A[2]), "v"(A[3]), "v"(Bv[0]), "v"(Bv[1]), "v"(Bv[2]), "v"(Bv[3])
      : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51");
  out[0 * 64 + l] = r;
  // case 1: overwrite srcA right after issue
  asm volatile(
      "v_mov_b32 v40, %1\n v_mov_b32 v41, %2\n v_mov_b32 v42, %3\n v_mov_b32 v43, %4\n"
      "v_mov_b32 v44, %5\n v_mov_b32 v45, %6\n v_mov_b32 v46, %7\n v_mov_b32 v47, %8\n" NOPS
      "v_mfma_i32_16x16x64_i8 v[48:51], v[40:43], v[44:47], 0\n"
      "v_mov_b32 v40, 0\n v_mov_b32 v41, 0\n v_mov_b32 v42, 0\n v_mov_b32 v43, 0\n" NOPS
      "v_mov_b32 %0, v48\n"
      : "=v"(r[0]) : "v"(A[0]), "v"(A[1]), "v"(A[2]), "v"(A[3]), "v"(Bv[0]), "v"(Bv[1]), "v"(Bv[2]), "v"(Bv[3])
      : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51");
  out[1 * 64 + l] = r;
  // case 2: overwrite srcB right after issue
  asm volatile(
      "v_mov_b32 v40, %1\n v_mov_b32 v41, %2\n v_mov_b32 v42, %3\n v_mov_b32 v43, %4\n"
      "v_mov_b32 v44, %5\n v_mov_b32 v45, %6\n v_mov_b32 v46, %7\n v_mov_b32 v47, %8\n" NOPS
      "v_mfma_i32_16x16x64_i8 v[48:51], v[40:43], v[44:47], 0\n"
      "v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v46, 0\n v_mov_b32 v47, 0\n" NOPS
      "v_mov_b32 %0, v48\n"
      : "=v"(r[0]) : "v"(A[0]), "v"(A[1]), "v"(A[2]), "v"(A[3]), "v"(Bv[0]), "v"(Bv[1]), "v"(Bv[2]), "v"(Bv[3])
      : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51");
  out[2 * 64 + l] = r;
  // case 3: dst v[38:41] overlaps the low half of srcA v[40:43]
  asm volatile(
      "v_mov_b32 v40, %1\n v_mov_b32 v41, %2\n v_mov_b32 v42, %3\n v_mov_b32 v43, %4\n"
      "v_mov_b32 v44, %5\n v_mov_b32 v45, %6\n v_mov_b32 v46, %7\n v_mov_b32 v47, %8\n" NOPS
      "v_mfma_i32_16x16x64_i8 v[38:41], v[40:43], v[44:47], 0\n" NOPS
      "v_mov_b32 %0, v38\n"
      : "=v"(r[0]) : "v"(A[0]), "v"(A[1]), "v"(A[2]), "v"(A[3]), "v"(Bv[0]), "v"(Bv[1]), "v"(Bv[2]), "v"(Bv[3])
      : "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47");
  out[3 * 64 + l] = r;
  // case 4: dst v[42:45] overlaps the high half of srcA v[40:43] and the low half of srcB
  asm volatile(
      "v_mov_b32 v40, %1\n v_mov_b32 v41, %2\n v_mov_b32 v42, %3\n v_mov_b32 v43, %4\n"
      "v_mov_b32 v44, %5\n v_mov_b32 v45, %6\n v_mov_b32 v46, %7\n v_mov_b32 v47, %8\n" NOPS
      "v_mfma_i32_16x16x64_i8 v[42:45], v[40:43], v[44:47], 0\n" NOPS
      "v_mov_b32 %0, v42\n"
      : "=v"(r[0]) : "v"(A[0]), "v"(A[1]), "v"(A[2]), "v"(A[3]), "v"(Bv[0]), "v"(Bv[1]), "v"(Bv[2]), "v"(Bv[3])
      : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47");
  out[4 * 64 + l] = r;
  // case 5: reference 16x16x32 on (A lo, B lo), then case 6: a 16x16x64 issued right after it
  // writes that 16x16x32's source registers
  asm volatile(
      "v_mov_b32 v40, %1\n v_mov_b32 v41, %2\n v_mov_b32 v42, %3\n v_mov_b32 v43, %4\n"
      "v_mov_b32 v44, %5\n v_mov_b32 v45, %6\n v_mov_b32 v46, %7\n v_mov_b32 v47, %8\n" NOPS
      "v_mfma_i32_16x16x32_i8 v[52:55], v[40:41], v[44:45], 0\n" NOPS
      "v_mov_b32 %0, v52\n"
      : "=v"(r[0]) : "v"(A[0]), "v"(A[1]), "v"(A[2]), "v"(A[3]), "v"(Bv[0]), "v"(Bv[1]), "v"(Bv[2]), "v"(Bv[3])
      : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v52", "v53", "v54", "v55");
  out[5 * 64 + l] = r;
  asm volatile(
      "v_mov_b32 v40, %1\n v_mov_b32 v41, %2\n v_mov_b32 v42, %3\n v_mov_b32 v43, %4\n"
      "v_mov_b32 v44, %5\n v_mov_b32 v45, %6\n v_mov_b32 v46, %7\n v_mov_b32 v47, %8\n" NOPS
      "v_mfma_i32_16x16x32_i8 v[52:55], v[40:41], v[44:45], 0\n"
      "v_mfma_i32_16x16x64_i8 v[40:43], v[44:47], v[44:47], 0\n" NOPS
      "v_mov_b32 %0, v52\n"
      : "=v"(r[0]) : "v"(A[0]), "v"(A[1]), "v"(A[2]), "v"(A[3]), "v"(Bv[0]), "v"(Bv[1]), "v"(Bv[2]), "v"(Bv[3])
      : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v52", "v53", "v54", "v55");
  out[6 * 64 + l] = r;
  // case 7: 16x16x32 followed by a VALU write of its srcA
  asm volatile(
      "v_mov_b32 v40, %1\n v_mov_b32 v41, %2\n v_mov_b32 v42, %3\n v_mov_b32 v43, %4\n"
      "v_mov_b32 v44, %5\n v_mov_b32 v45, %6\n v_mov_b32 v46, %7\n v_mov_b32 v47, %8\n" NOPS
      "v_mfma_i32_16x16x32_i8 v[52:55], v[40:41], v[44:45], 0\n"
      "v_mov_b32 v40, 0\n v_mov_b32 v41, 0\n" NOPS
      "v_mov_b32 %0, v52\n"
      : "=v"(r[0]) : "v"(A[0]), "v"(A[1]), "v"(A[2]), "v"(A[3]), "v"(Bv[0]), "v"(Bv[1]), "v"(Bv[2]), "v"(Bv[3])
      : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v52", "v53", "v54", "v55");
  out[7 * 64 + l] = r;
}

int main() {
  const int N = 64;
  v4i ha[N], hb[N], ho[8 * N];
  srand(1);
  for (int i = 0; i < N; i++)
    for (int j = 0; j < 4; j++) { ha[i][j] = rand(); hb[i][j] = rand(); }
  v4i *da, *db, *dout;
  hipMalloc(&da, sizeof(ha)); hipMalloc(&db, sizeof(hb)); hipMalloc(&dout, sizeof(ho));
  hipMemcpy(da, ha, sizeof(ha), hipMemcpyHostToDevice);
  hipMemcpy(db, hb, sizeof(hb), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, da, db, dout);
  if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
  hipMemcpy(ho, dout, sizeof(ho), hipMemcpyDeviceToHost);
  const char* names[] = {"ref 16x16x64", "VALU overwrites srcA after issue", "VALU overwrites srcB after issue",
                         "dst overlaps low half of srcA", "dst overlaps high half of srcA / low of srcB",
                         "ref 16x16x32", "next 16x16x64 writes 16x16x32's sources", "VALU overwrites 16x16x32 srcA"};
  for (int c = 1; c < 8; c++) {
    const int ref = c == 6 || c == 7 ? 5 : 0;
    if (c == 5) continue;
    int bad = 0;
    for (int l = 0; l < N; l++) bad += ho[c * N + l][0] != ho[ref * N + l][0];
    printf("case %d %-45s %s (%d/64 lanes differ)\n", c, names[c], bad ? "WRONG" : "ok", bad);
  }
  return 0;
}
