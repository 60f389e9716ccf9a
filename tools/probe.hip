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
  unsigned long long zero[24] = {0};
  hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), zero, sizeof(zero));
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0, 0);
  for (int i = 0; i < iters; i++) net_model_compute_batch_async(x, y, B, 0, nullptr);
  hipEventRecord(e1, 0); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  unsigned long long st[24];
  hipMemcpyFromSymbol(st, HIP_SYMBOL(g_stamps), sizeof(st));
  int32_t info[3]; net_launch_info(B, 0, info);
  const char* names[] = {"layer1 work", "barrier A wait", "layer2 work", "layer3 work", "barrier B wait",
                         "layer4 (last wave)", "layer5 (last wave)", "loop top"};
  double trials = (double)B * iters;
  printf("B=%zu iters=%d  %.3f ms/launch  grid %d  lds %d\n", B, iters, ms / iters, info[0], info[2]);
  printf("  shader clock from s_memtime/s_memrealtime: %.3f GHz\n", 0.1 * (double)st[16] / (double)st[17]);
  printf("  %-20s %12s %12s   (cycles per trial, summed over the trial's wave)\n", "phase", "wave 0", "last wave");
  double t0 = 0, t1 = 0;
  for (int i = 0; i < 8; i++) {
    printf("  %-20s %12.0f %12.0f\n", names[i], st[i] / trials, st[8 + i] / trials);
    t0 += st[i]; t1 += st[8 + i];
  }
  printf("  %-20s %12.0f %12.0f\n", "total", t0 / trials, t1 / trials);
  return 0;
}
