/*
 * net_host.c — a plain-C host for libmibminet, the way the reference's C callers use the path.
 *
 * The reference calls net_model_compute() from C on the cluster (src/cl/cluster.c:38; its model
 * test, test/cl/net/model/cluster.c:40-49, compares the logits with the golden model's).  This
 * program does the same against the MI355X library, through the C ABI only (include/mibminet.h
 * and the HIP runtime's C API for device buffers):
 *
 *   net_host check <params.blob> <x.bin> <want.bin> <n>
 *       x.bin: n trials in the reference single-trial layout [T][C_ALIGN] int8; want.bin: the
 *       expected logits [n][N] int8.  Runs every trial through net_model_compute (host
 *       buffers), then all n at once through net_model_compute_batch (device buffers, packed
 *       [n][trial_stride] layout) and through net_model_compute_batch_ct (channel-major
 *       [n][C][T], at an odd device address), and compares each with want.bin.  Exit 0 when all
 *       match.
 *   net_host bench <params.blob> [B=65536] [steps=50]
 *       Times `steps` back-to-back net_model_compute_batch_async launches over B resident
 *       random trials with HIP events and prints one line of trials/s.
 *
 * Built with -DMIB_NET_H against a generated net.h / net.c (the reference's weight globals,
 * gen_net_header.py; net_host_b22 / net_host_g19 in the Makefile), <params.blob> may be "-": the
 * parameters then come from the linked arrays through net_params_load_arrays
 * (include/mibminet_net_h.h), as the reference's callers link them (src/cl/cluster.c:38).
 */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mibminet.h"
#ifdef MIB_NET_H
#include "net.h"
#include "mibminet_net_h.h"
#endif

static void* read_file(const char* path, size_t* len) {
    FILE* f = fopen(path, "rb");
    if (!f) {
        perror(path);
        return NULL;
    }
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    void* buf = malloc(n > 0 ? (size_t)n : 1);
    if (!buf || fread(buf, 1, (size_t)n, f) != (size_t)n) {
        fprintf(stderr, "%s: read failed\n", path);
        free(buf);
        fclose(f);
        return NULL;
    }
    fclose(f);
    *len = (size_t)n;
    return buf;
}

static int load_params(const char* path, int32_t dims[7]) {
#ifdef MIB_NET_H
    if (!strcmp(path, "-")) {  /* the linked net.c: no blob, no file */
        const int rc = mibminet_load_net_h();
        if (rc) {
            fprintf(stderr, "net_params_load_arrays: %s\n", net_error_string(rc));
            return 1;
        }
        net_params_dims(dims);
        printf("parameters: linked net.c (C=%d T=%d N=%d)\n", NET_C, NET_T, NET_N);
        return 0;
    }
#endif
    size_t len = 0;
    void* blob = read_file(path, &len);
    if (!blob) return 1;
    int rc = net_params_load(blob, len);
    free(blob);
    if (rc) {
        fprintf(stderr, "net_params_load: %s\n", net_error_string(rc));
        return 1;
    }
    net_params_dims(dims);
    return 0;
}

#define HIP_OK(call)                                                                  \
    do {                                                                              \
        hipError_t e_ = (call);                                                       \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s: %s\n", #call, hipGetErrorString(e_));                \
            return 1;                                                                 \
        }                                                                             \
    } while (0)

static int check(const char* blob, const char* xpath, const char* wpath, long n) {
    int32_t d[7];
    if (load_params(blob, d)) return 1;
    const int C = d[0], T = d[1], N = d[4], CA = (C + 3) / 4 * 4;
    const size_t stride = net_trial_stride();
    size_t xl = 0, wl = 0;
    int8_t* x = read_file(xpath, &xl);
    int8_t* want = read_file(wpath, &wl);
    if (!x || !want || n <= 0 || xl != (size_t)n * T * CA || wl != (size_t)n * N) {
        fprintf(stderr, "check: input sizes do not match n=%ld (C=%d T=%d N=%d)\n", n, C, T, N);
        return 1;
    }
    long bad = 0;
    int8_t out[64];
    for (long b = 0; b < n; b++) {  /* the reference entry point, one trial at a time */
        net_model_compute(x + (size_t)b * T * CA, out);
        if (net_last_error()) {
            fprintf(stderr, "net_model_compute: %s\n", net_error_string(net_last_error()));
            return 1;
        }
        if (memcmp(out, want + (size_t)b * N, (size_t)N)) bad++;
    }
    printf("net_model_compute: %ld of %ld trials differ\n", bad, n);
    /* batched: pack [T][C_ALIGN] -> [T][C] per trial (the device layout, include/mibminet.h) */
    int8_t* packed = calloc((size_t)n, stride);
    for (long b = 0; b < n; b++)
        for (int t = 0; t < T; t++)
            memcpy(packed + (size_t)b * stride + (size_t)t * C, x + ((size_t)b * T + t) * CA, (size_t)C);
    int8_t *dx = NULL, *dy = NULL;
    HIP_OK(hipMalloc((void**)&dx, (size_t)n * stride));
    HIP_OK(hipMalloc((void**)&dy, (size_t)n * N));
    HIP_OK(hipMemcpy(dx, packed, (size_t)n * stride, hipMemcpyHostToDevice));
    int rc = net_model_compute_batch(dx, dy, (size_t)n, 0);
    if (rc) {
        fprintf(stderr, "net_model_compute_batch: %s\n", net_error_string(rc));
        return 1;
    }
    int8_t* y = malloc((size_t)n * N);
    HIP_OK(hipMemcpy(y, dy, (size_t)n * N, hipMemcpyDeviceToHost));
    long badb = 0;
    for (long b = 0; b < n; b++) badb += memcmp(y + (size_t)b * N, want + (size_t)b * N, (size_t)N) != 0;
    printf("net_model_compute_batch: %ld of %ld trials differ\n", badb, n);
    /* channel-major [n][C][T] (input.npz's layout) straight into net_model_compute_batch_ct,
       one byte into its allocation (the entry point takes any alignment) */
    int8_t* cm = malloc((size_t)n * C * T);
    for (long b = 0; b < n; b++)
        for (int c = 0; c < C; c++)
            for (int t = 0; t < T; t++) cm[((size_t)b * C + c) * T + t] = x[((size_t)b * T + t) * CA + c];
    int8_t* dxc = NULL;
    HIP_OK(hipMalloc((void**)&dxc, (size_t)n * C * T + 1));
    HIP_OK(hipMemcpy(dxc + 1, cm, (size_t)n * C * T, hipMemcpyHostToDevice));
    HIP_OK(hipMemset(dy, 0, (size_t)n * N));
    rc = net_model_compute_batch_ct(dxc + 1, dy, (size_t)n, 0, NULL);
    if (rc) {
        fprintf(stderr, "net_model_compute_batch_ct: %s\n", net_error_string(rc));
        return 1;
    }
    HIP_OK(hipMemcpy(y, dy, (size_t)n * N, hipMemcpyDeviceToHost));  /* null stream: after the launch */
    long badc = 0;
    for (long b = 0; b < n; b++) badc += memcmp(y + (size_t)b * N, want + (size_t)b * N, (size_t)N) != 0;
    printf("net_model_compute_batch_ct: %ld of %ld trials differ\n", badc, n);
    badb += badc;
    hipFree(dxc);
    free(cm);
    hipFree(dx);
    hipFree(dy);
    free(y);
    free(packed);
    free(x);
    free(want);
    if (bad || badb) return 1;
    printf("ok\n");
    return 0;
}

static int bench(const char* blob, long B, int steps) {
    int32_t d[7];
    if (load_params(blob, d)) return 1;
    const int C = d[0], T = d[1], N = d[4];
    const size_t stride = net_trial_stride();
    int8_t* h = malloc((size_t)B * stride);
    uint32_t s = 12345u;
    for (size_t i = 0; i < (size_t)B * stride; i++) {
        s = s * 1664525u + 1013904223u;
        h[i] = (i % stride) < (size_t)C * T ? (int8_t)(s >> 24) : 0;
    }
    int8_t *dx = NULL, *dy = NULL;
    HIP_OK(hipMalloc((void**)&dx, (size_t)B * stride));
    HIP_OK(hipMalloc((void**)&dy, (size_t)B * N));
    HIP_OK(hipMemcpy(dx, h, (size_t)B * stride, hipMemcpyHostToDevice));
    free(h);
    hipStream_t st;
    HIP_OK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    for (int i = 0; i < 200; i++) net_model_compute_batch_async(dx, dy, (size_t)B, 0, st);  /* clock settle */
    HIP_OK(hipStreamSynchronize(st));
    hipEvent_t e0, e1;
    HIP_OK(hipEventCreate(&e0));
    HIP_OK(hipEventCreate(&e1));
    HIP_OK(hipEventRecord(e0, st));
    for (int i = 0; i < steps; i++) {
        int rc = net_model_compute_batch_async(dx, dy, (size_t)B, 0, st);
        if (rc) {
            fprintf(stderr, "net_model_compute_batch_async: %s\n", net_error_string(rc));
            return 1;
        }
    }
    HIP_OK(hipEventRecord(e1, st));
    HIP_OK(hipEventSynchronize(e1));
    float ms = 0.f;
    HIP_OK(hipEventElapsedTime(&ms, e0, e1));
    const double per = ms / steps;
    printf("C host bench: B=%ld C=%d T=%d steps=%d  %.4f ms/launch  %.4g trials/s  %.1f GB/s algorithmic\n", B, C, T,
           steps, per, B / (per * 1e-3), (double)B * (C * T + N) / (per * 1e-3) / 1e9);
    hipFree(dx);
    hipFree(dy);
    hipStreamDestroy(st);
    return 0;
}

int main(int argc, char** argv) {
    if (argc >= 6 && !strcmp(argv[1], "check")) return check(argv[2], argv[3], argv[4], atol(argv[5]));
    if (argc >= 3 && !strcmp(argv[1], "bench"))
        return bench(argv[2], argc > 3 ? atol(argv[3]) : 65536, argc > 4 ? atoi(argv[4]) : 50);
    fprintf(stderr,
            "usage: %s check <params.blob> <x.bin> <want.bin> <n>\n"
            "       %s bench <params.blob> [B] [steps]\n",
            argv[0], argv[0]);
    return 2;
}
