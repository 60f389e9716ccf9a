// Diagnostic probe (not part of the product): builds the library TU with -DMIB_STAMPS and
// reports per-phase cycles of the forward kernel (s_memtime deltas accumulated by the flushing
// lane of every wave (one-wave kernel) or of one wave per workgroup (workgroup kernel)).
// usage: probe <blob> [B] [iters] [ct]   (ct = 1: channel-major [B][C][T] input, net_model_compute_batch_ct;
//                                        ct = 2: float32 [B][C][T], net_model_compute_batch_f32)
#include "../mi-bminet_amd/csrc/mibminet.hip"
#include <chrono>
#include <fstream>
#include <iterator>

int main(int argc, char** argv) {
  std::ifstream f(argv[1], std::ios::binary);
  std::vector<char> blob((std::istreambuf_iterator<char>(f)), {});
  int8_t *x, *y;
  if (getenv("MIB_FORCE_GENERAL")) mibminet_test_force_general(1);  // the run-time-dimension kernels
  int rc = net_params_load(blob.data(), blob.size());
  if (rc) { printf("load rc %d\n", rc); return 1; }
  size_t B = argc > 2 ? atol(argv[2]) : 65536;
  int iters = argc > 3 ? atoi(argv[3]) : 10;
  const int mode = argc > 4 ? atoi(argv[4]) : 0;
  const bool ct = mode != 0, f32 = mode == 2;
  int32_t dims[7];
  net_params_dims(dims);
  size_t stride = f32 ? (size_t)dims[0] * dims[1] * 4 : ct ? (size_t)dims[0] * dims[1] : net_trial_stride();
  auto run = [&]() {
    if (f32) return net_model_compute_batch_f32((const float*)x, y, B, 3.0f, 0, nullptr);
    return ct ? net_model_compute_batch_ct(x, y, B, 0, nullptr) : net_model_compute_batch_async(x, y, B, 0, nullptr);
  };
  hipMalloc(&x, B * stride); hipMalloc(&y, B * 16);
  std::vector<int8_t> hx(B * stride);
  for (size_t i = 0; i < hx.size(); i++) hx[i] = (int8_t)(rand() & 255);
  if (f32)  // floats in about [-4, 4]: exponent 0x40 / 0xC0 high byte, random mantissa
    for (size_t i = 3; i < hx.size(); i += 4) hx[i] = (int8_t)((rand() & 1) ? 0x40 : 0xC0);
  hipMemcpy(x, hx.data(), hx.size(), hipMemcpyHostToDevice);
  rc = run();
  if (!rc && hipDeviceSynchronize() != hipSuccess) rc = -1;
  if (rc) { printf("run rc %d %s\n", rc, net_error_string(rc)); return 1; }
  unsigned long long zero[72] = {0};
  hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), zero, sizeof(zero));
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0, 0);
  for (int i = 0; i < iters; i++) run();
  hipEventRecord(e1, 0); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  unsigned long long st[72];
  hipMemcpyFromSymbol(st, HIP_SYMBOL(g_stamps), sizeof(st));
  int32_t info[3]; net_launch_info(B, 0, info);
  const char* names[] = {"layer1 work", "barrier A wait", "layer2 work", "layer3 work", "barrier B wait",
                         "layer4 (last wave)", "layer5 (last wave)", "loop top"};
  double trials = (double)B * iters;
  printf("%sB=%zu iters=%d  %.3f ms/launch  grid %d  lds %d\n", f32 ? "float32 " : ct ? "channel-major " : "", B, iters,
         ms / iters, info[0], info[2]);
  printf("  shader clock from s_memtime/s_memrealtime: %.3f GHz\n", 0.1 * (double)st[64] / (double)st[65]);
  printf("  %-20s", "phase (cycles/trial)");
  for (int w = 0; w < 8; w++) printf("  wave %d", w);
  printf("\n");
  double tot[8] = {0};
  for (int i = 0; i < 8; i++) {
    printf("  %-20s", names[i]);
    for (int w = 0; w < 8; w++) { printf(" %7.0f", st[8 * w + i] / trials); tot[w] += st[8 * w + i]; }
    printf("\n");
  }
  printf("  %-20s", "total");
  for (int w = 0; w < 8; w++) printf(" %7.0f", tot[w] / trials);
  printf("\n");
  return 0;
}
