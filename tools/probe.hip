// Diagnostic probe (not part of the product): builds the library TU with -DMIB_STAMPS and
// reports per-phase cycles of the forward kernel (s_memtime deltas accumulated by the flushing
// lane of every wave (one-wave kernel) or of one wave per workgroup (workgroup kernel)).
// usage: probe <blob> [B] [iters]
#include "../mi-bminet_amd/csrc/mibminet.hip"
#include <chrono>
#include <fstream>
#include <iterator>

int main(int argc, char** argv) {
  std::ifstream f(argv[1], std::ios::binary);
  std::vector<char> blob((std::istreambuf_iterator<char>(f)), {});
  int rc = net_params_load(blob.data(), blob.size());
  if (rc) { printf("load rc %d\n", rc); return 1; }
  size_t B = argc > 2 ? atol(argv[2]) : 65536;
  int iters = argc > 3 ? atoi(argv[3]) : 10;
  size_t stride = net_trial_stride();
  int8_t *x, *y;
  hipMalloc(&x, B * stride); hipMalloc(&y, B * 4);
  std::vector<int8_t> hx(B * stride);
  for (size_t i = 0; i < hx.size(); i++) hx[i] = (int8_t)(rand() & 255);
  hipMemcpy(x, hx.data(), hx.size(), hipMemcpyHostToDevice);
  rc = net_model_compute_batch(x, y, B, 0);
  if (rc) { printf("run rc %d %s\n", rc, net_error_string(rc)); return 1; }
  unsigned long long zero[16] = {0};
  hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), zero, sizeof(zero));
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0, 0);
  for (int i = 0; i < iters; i++) net_model_compute_batch_async(x, y, B, 0, nullptr);
  hipEventRecord(e1, 0); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  unsigned long long st[16];
  hipMemcpyFromSymbol(st, HIP_SYMBOL(g_stamps), sizeof(st));
  int32_t info[3]; net_launch_info(B, 0, info);
  const char* names[] = {"layer1", "layer2", "layer3", "layer4", "layer5+store", "loop top", "-", "-"};
  double trials = (double)B * iters;
  printf("B=%zu iters=%d  %.3f ms/launch  grid %d  lds %d\n", B, iters, ms / iters, info[0], info[2]);
  double tot = 0;
  for (int i = 0; i < 6; i++) tot += st[i];
  printf("  shader clock from s_memtime/s_memrealtime: %.3f GHz\n", 0.1 * (double)st[6] / (double)st[7]);
  for (int i = 0; i < 6; i++)
    printf("  %-18s %8.0f cycles/trial/flusher  (%4.1f%%)\n", names[i], st[i] / trials, 100.0 * st[i] / tot);
  printf("  total %8.0f cycles per trial per flusher (s_memtime ticks), flushers %llu\n", tot / trials, st[8]);
  return 0;
}
