// Diagnostic probe (not part of the product): dependent i8 MFMA chains on gfx950 where a later
// MFMA (issued back to back) overwrites a source of an earlier, still-waiting MFMA.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef int v4i __attribute__((ext_vector_type(4)));
#define NOPS "s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n"
#define LOAD \
  "v_mov_b32 v40, %1\n v_mov_b32 v41, %2\n v_mov_b32 v42, %3\n v_mov_b32 v43, %4\n" \
  "v_mov_b32 v44, %5\n v_mov_b32 v45, %6\n v_mov_b32 v46, %7\n v_mov_b32 v47, %8\n" \
  "v_mov_b32 v56, %2\n v_mov_b32 v57, %3\n v_mov_b32 v58, %6\n v_mov_b32 v59, %7\n" NOPS
#define INS "v"(A[0]), "v"(A[1]), "v"(A[2]), "v"(A[3]), "v"(Bv[0]), "v"(Bv[1]), "v"(Bv[2]), "v"(Bv[3])
#define CLOB "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", \
  "v54", "v55", "v56", "v57", "v58", "v59"
#define CASE(idx, body, outreg) \
  asm volatile(LOAD body NOPS "v_mov_b32 %0, " outreg "\n" : "=v"(r) : INS : CLOB); out[(idx) * 64 + l] = r;

__global__ void k(const v4i* a, const v4i* b, int* out) {
  const int l = threadIdx.x;
  v4i A = a[l], Bv = b[l];
  int r;
  // reference: M1 then (serialised) M2 with srcC = M1's result
  CASE(0, "v_mfma_i32_16x16x64_i8 v[48:51], v[40:43], v[44:47], 0\n" NOPS
          "v_mfma_i32_16x16x32_i8 v[52:55], v[56:57], v[58:59], v[48:51]\n", "v53")
  // A: back to back, then M3 overwrites M2's srcA/srcB (v[56:59])
  CASE(1, "v_mfma_i32_16x16x64_i8 v[48:51], v[40:43], v[44:47], 0\n"
          "v_mfma_i32_16x16x32_i8 v[52:55], v[56:57], v[58:59], v[48:51]\n"
          "v_mfma_i32_16x16x64_i8 v[56:59], v[40:43], v[44:47], 0\n", "v53")
  // B: M3 overwrites M2's srcC (v[48:51])
  CASE(2, "v_mfma_i32_16x16x64_i8 v[48:51], v[40:43], v[44:47], 0\n"
          "v_mfma_i32_16x16x32_i8 v[52:55], v[56:57], v[58:59], v[48:51]\n"
          "v_mfma_i32_16x16x64_i8 v[48:51], v[40:43], v[44:47], 0\n", "v53")
  // C: M2's dst partially overlaps its srcC (v[50:53] <- srcC v[48:51]); reference: case 0 lane
  // value of D row 1 sits in v51 there (v53 in case 0 corresponds to v51 here)
  CASE(3, "v_mfma_i32_16x16x64_i8 v[48:51], v[40:43], v[44:47], 0\n"
          "v_mfma_i32_16x16x32_i8 v[50:53], v[56:57], v[58:59], v[48:51]\n", "v51")
  // D: like A, M3 a VALU write instead of an MFMA
  CASE(4, "v_mfma_i32_16x16x64_i8 v[48:51], v[40:43], v[44:47], 0\n"
          "v_mfma_i32_16x16x32_i8 v[52:55], v[56:57], v[58:59], v[48:51]\n"
          "v_mov_b32 v56, 0\n v_mov_b32 v57, 0\n v_mov_b32 v58, 0\n v_mov_b32 v59, 0\n", "v53")
  // E: like B, VALU overwrite of M2's srcC
  CASE(5, "v_mfma_i32_16x16x64_i8 v[48:51], v[40:43], v[44:47], 0\n"
          "v_mfma_i32_16x16x32_i8 v[52:55], v[56:57], v[58:59], v[48:51]\n"
          "v_mov_b32 v48, 0\n v_mov_b32 v49, 0\n v_mov_b32 v50, 0\n v_mov_b32 v51, 0\n", "v53")
  // F: 16x16x32 chain (srcC dependent) then a 16x16x32 overwriting the sources
  CASE(6, "v_mfma_i32_16x16x32_i8 v[48:51], v[40:41], v[44:45], 0\n" NOPS
          "v_mfma_i32_16x16x32_i8 v[52:55], v[56:57], v[58:59], v[48:51]\n", "v53")
  CASE(7, "v_mfma_i32_16x16x32_i8 v[48:51], v[40:41], v[44:45], 0\n"
          "v_mfma_i32_16x16x32_i8 v[52:55], v[56:57], v[58:59], v[48:51]\n"
          "v_mfma_i32_16x16x32_i8 v[56:59], v[40:41], v[44:45], 0\n", "v53")
  // G: 16x16x64 chain
  CASE(8, "v_mfma_i32_16x16x64_i8 v[48:51], v[40:43], v[44:47], 0\n" NOPS
          "v_mfma_i32_16x16x64_i8 v[52:55], v[56:59], v[40:43], v[48:51]\n", "v53")
  CASE(9, "v_mfma_i32_16x16x64_i8 v[48:51], v[40:43], v[44:47], 0\n"
          "v_mfma_i32_16x16x64_i8 v[52:55], v[56:59], v[40:43], v[48:51]\n"
          "v_mfma_i32_16x16x64_i8 v[56:59], v[44:47], v[44:47], 0\n", "v53")
}

int main() {
  const int N = 64;
  v4i ha[N], hb[N];
  int ho[10 * N];
  srand(2);
  for (int i = 0; i < N; i++)
    for (int j = 0; j < 4; j++) { ha[i][j] = rand(); hb[i][j] = rand(); }
  v4i *da, *db;
  int* dout;
  (void)hipMalloc(&da, sizeof(ha)); (void)hipMalloc(&db, sizeof(hb)); (void)hipMalloc(&dout, sizeof(ho));
  (void)hipMemcpy(da, ha, sizeof(ha), hipMemcpyHostToDevice);
  (void)hipMemcpy(db, hb, sizeof(hb), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, da, db, dout);
  if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
  (void)hipMemcpy(ho, dout, sizeof(ho), hipMemcpyDeviceToHost);
  struct { int c, ref; const char* name; } cs[] = {
      {1, 0, "x64 -> x32(srcC dep) ; x64 overwrites x32 srcA/B"},
      {2, 0, "x64 -> x32(srcC dep) ; x64 overwrites x32 srcC"},
      {3, 0, "x64 -> x32 with dst partially over srcC"},
      {4, 0, "x64 -> x32(srcC dep) ; VALU overwrites x32 srcA/B"},
      {5, 0, "x64 -> x32(srcC dep) ; VALU overwrites x32 srcC"},
      {7, 6, "x32 -> x32(srcC dep) ; x32 overwrites srcA/B"},
      {9, 8, "x64 -> x64(srcC dep) ; x64 overwrites srcA"}};
  for (auto& c : cs) {
    int bad = 0;
    for (int l = 0; l < N; l++) bad += ho[c.c * N + l] != ho[c.ref * N + l];
    printf("case %d %-52s %s (%d/64 lanes differ)\n", c.c, c.name, bad ? "WRONG" : "ok", bad);
  }
  return 0;
}
