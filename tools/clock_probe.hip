// In-kernel clock of the fused forward (diagnostic, not part of the product; MI355X_MICROARCH.md
// 'DVFS give-back' item 6).  Builds the library TU with -DMIB_CLOCK (plus any MIB_DIAG_* ablation):
// each workgroup sums one s_memtime / s_memrealtime pair around its trial loop into g_clk.
// The probe runs 65,536-trial launches back to back for `warm` seconds on one resident batch
// (uniform random int8, or all zero), then clears g_clk and times `iters` more launches with HIP
// events.  It prints the wall time per launch, the median over workgroups of
// d(memtime) / d(memrealtime) x 100 MHz (the clock the chip held inside the kernel), and the
// kernel's cycles per launch at that clock.
// usage: clock_probe <blob> [zero] [warm_s] [iters] [ct]   (ct = 1: channel-major [B][C][T] input,
//        net_model_compute_batch_ct)
#include "../mi-bminet_amd/csrc/mibminet.hip"
#include <algorithm>
#include <chrono>
#include <fstream>
#include <iterator>
#include <random>

int main(int argc, char** argv) {
  std::ifstream f(argv[1], std::ios::binary);
  std::vector<char> blob((std::istreambuf_iterator<char>(f)), {});
  if (net_params_load(blob.data(), blob.size())) { printf("load failed\n"); return 1; }
  const bool zero = argc > 2 && atoi(argv[2]) != 0;
  const double warm = argc > 3 ? atof(argv[3]) : 2.5;
  const int iters = argc > 4 ? atoi(argv[4]) : 200;
  const bool ct = argc > 5 && atoi(argv[5]) != 0;
  int32_t dims[7];
  net_params_dims(dims);
  const size_t B = 65536, stride = ct ? (size_t)dims[0] * dims[1] : net_trial_stride();
  auto run = [&](int8_t* x, int8_t* y) {
    return ct ? net_model_compute_batch_ct(x, y, B, 0, nullptr) : net_model_compute_batch_async(x, y, B, 0, nullptr);
  };
  int8_t *x, *y;
  if (hipMalloc(&x, B * stride) != hipSuccess || hipMalloc(&y, B * 4) != hipSuccess) return 1;
  std::vector<int8_t> hx(B * stride, 0);
  if (!zero) {
    std::mt19937 rng(7);
    for (auto& v : hx) v = (int8_t)(rng() & 255);
  }
  if (hipMemcpy(x, hx.data(), hx.size(), hipMemcpyHostToDevice) != hipSuccess) return 1;
  if (int rc = run(x, y)) { printf("run rc %d %s\n", rc, net_error_string(rc)); return 1; }
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  const auto t0 = std::chrono::steady_clock::now();
  long warm_launches = 0;
  while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < warm) {
    for (int i = 0; i < 100; i++) run(x, y);
    warm_launches += 100;
    if (hipDeviceSynchronize() != hipSuccess) return 1;
  }
  std::vector<unsigned long long> clk(2 * CLK_SLOTS, 0);
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_clk), clk.data(), clk.size() * 8) != hipSuccess) return 1;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, 0);
  for (int i = 0; i < iters; i++) run(x, y);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  if (hipMemcpyFromSymbol(clk.data(), HIP_SYMBOL(g_clk), clk.size() * 8) != hipSuccess) return 1;
  int32_t info[3];
  net_launch_info(B, 0, info);
  std::vector<double> ghz, cyc;
  for (int w = 0; w < info[0] && w < CLK_SLOTS; w++) {
    if (!clk[2 * w + 1]) continue;
    ghz.push_back(0.1 * (double)clk[2 * w] / (double)clk[2 * w + 1]);
    cyc.push_back((double)clk[2 * w] / iters);
  }
  std::sort(ghz.begin(), ghz.end());
  std::sort(cyc.begin(), cyc.end());
  const double med = ghz[ghz.size() / 2];
  printf("%s%s input, %.1f s warm (%ld launches), %d timed launches: %.4f ms/launch; in-kernel clock median %.3f GHz "
         "(p10 %.3f, p90 %.3f over %zu workgroups); loop cycles per launch median %.0f; ms x clock = %.0f K cycles\n",
         ct ? "channel-major " : "", zero ? "all-zero" : "random", warm, warm_launches, iters, ms / iters, med, ghz[ghz.size() / 10],
         ghz[ghz.size() * 9 / 10], ghz.size(), cyc[cyc.size() / 2], ms / iters * med * 1e3);
  return 0;
}
