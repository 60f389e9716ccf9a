// ISA probe (diagnostic, not part of the product): does an inline-asm v_pk_fma_f32 that reads an
// MFMA accumulator directly see the final result after the documented wait states?  Round 5's
// clamp-form experiment (plain BN) returned wrong logits at random when its asm read
// the layer-2 accumulator, with 12 or 24 wait states in front, and none when a compiler fma read it
// first.  Every wave of a full grid runs a chained 32x32x32 i8 MFMA triple on its own operands, then
// the variant below reads the accumulator; the compiler's own fma on the same accumulator (issued
// after, so the compiler pads it) is the reference.
//   variant 0: asm "s_nop 11; v_pk_fma_f32 ... op_sel ... clamp" (the failing form), 12 states
//   variant 1: the same with 24 wait states
//   variant 2: the same with 48 wait states
//   variant 3: the same without the clamp bit, 12 states
//   variant 4: asm v_pk_fma_f32 with plain VGPR operands, no op_sel, no clamp, 12 states
// usage: pkclamp_probe [iters]   prints the mismatching element count per variant
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ unsigned long long pair(float lo, float hi) {
  return (unsigned long long)__float_as_uint(hi) << 32 | __float_as_uint(lo);
}

template <int V>
__device__ __forceinline__ f2 asm_read(f2 a, float r, float c) {
  f2 p = a;
  if constexpr (V == 0)
    asm("s_nop 11\n\tv_pk_fma_f32 %0, %0, %1, %1 op_sel:[0,0,1] op_sel_hi:[1,0,1] clamp" : "+v"(p) : "s"(pair(r, c)));
  if constexpr (V == 1)
    asm("s_nop 11\n\ts_nop 11\n\tv_pk_fma_f32 %0, %0, %1, %1 op_sel:[0,0,1] op_sel_hi:[1,0,1] clamp"
        : "+v"(p) : "s"(pair(r, c)));
  if constexpr (V == 2)
    asm("s_nop 15\n\ts_nop 15\n\ts_nop 15\n\tv_pk_fma_f32 %0, %0, %1, %1 op_sel:[0,0,1] op_sel_hi:[1,0,1] clamp"
        : "+v"(p) : "s"(pair(r, c)));
  if constexpr (V == 3)
    asm("s_nop 11\n\tv_pk_fma_f32 %0, %0, %1, %1 op_sel:[0,0,1] op_sel_hi:[1,0,1]" : "+v"(p) : "s"(pair(r, c)));
  if constexpr (V == 4) {
    const f2 rr = {r, r}, cc = {c, c};
    asm("s_nop 11\n\tv_pk_fma_f32 %0, %0, %1, %2" : "+v"(p) : "v"(rr), "v"(cc));
  }
  return p;
}

template <int V>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_probe(const int* seed, unsigned* bad, int iters, float r, float c) {
  const int lane = threadIdx.x & 63;
  unsigned s = seed[blockIdx.x] ^ (threadIdx.x * 0x9E3779B9u);
  unsigned nbad = 0;
  for (int it = 0; it < iters; it++) {
    v4i a[3], b[3];
    for (int k = 0; k < 3; k++)
      for (int j = 0; j < 4; j++) {
        s = s * 1664525u + 1013904223u;
        a[k][j] = (int)s;
        s = s * 1664525u + 1013904223u;
        b[k][j] = (int)s;
      }
    // the asm is the accumulator's first reader, as in round 5's layer 2
    v16i acc = {};
    for (int k = 0; k < 3; k++) acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[k], b[k], acc, 0, 0, 0);
    const f2 got = asm_read<V>((f2){__int_as_float(acc[0]), __int_as_float(acc[1])}, r, c);
    // reference: the same chain again (operands laundered so that it is not merged with the first),
    // read by the compiler's own fma (which the compiler pads), then the clamp
    for (int k = 0; k < 3; k++) asm volatile("" : "+v"(a[k]), "+v"(b[k]));
    v16i acc2 = {};
    for (int k = 0; k < 3; k++) acc2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[k], b[k], acc2, 0, 0, 0);
    f2 want = __builtin_elementwise_fma((f2){__int_as_float(acc2[0]), __int_as_float(acc2[1])}, (f2){r, r}, (f2){c, c});
    if constexpr (V != 3 && V != 4) {
      want[0] = fminf(fmaxf(want[0], 0.0f), 1.0f);
      want[1] = fminf(fmaxf(want[1], 0.0f), 1.0f);
    }
    nbad += (__float_as_uint(got[0]) != __float_as_uint(want[0])) + (__float_as_uint(got[1]) != __float_as_uint(want[1]));
  }
  if (nbad) atomicAdd(bad, nbad);
  (void)lane;
}

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      std::printf("%s: %s\n", #x, hipGetErrorString(e_));                     \
      std::exit(1);                                                           \
    }                                                                         \
  } while (0)

template <int V>
void run(const int* dseed, unsigned* dbad, int iters, int grid) {
  CHECK(hipMemset(dbad, 0, 4));
  // r, c chosen so that the fma result lands inside (0, 1) for part of the accumulators' range
  k_probe<V><<<grid, 512>>>(dseed, dbad, iters, 1.0f / 4096.0f, 0.5f);
  CHECK(hipDeviceSynchronize());
  unsigned bad = 0;
  CHECK(hipMemcpy(&bad, dbad, 4, hipMemcpyDeviceToHost));
  std::printf("variant %d: %u of %ld elements differ\n", V, bad, (long)grid * 512 * iters * 2);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 200;
  const int grid = 1024;
  int* dseed;
  unsigned* dbad;
  CHECK(hipMalloc(&dseed, grid * 4));
  CHECK(hipMalloc(&dbad, 4));
  int* hseed = (int*)std::malloc(grid * 4);
  for (int i = 0; i < grid; i++) hseed[i] = 12345 + 7919 * i;
  CHECK(hipMemcpy(dseed, hseed, grid * 4, hipMemcpyHostToDevice));
  run<0>(dseed, dbad, iters, grid);
  run<1>(dseed, dbad, iters, grid);
  run<2>(dseed, dbad, iters, grid);
  run<3>(dseed, dbad, iters, grid);
  run<4>(dseed, dbad, iters, grid);
  return 0;
}
