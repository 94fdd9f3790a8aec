// probe: host cost per call, from C++ (no Python, no torch): back-to-back issue of an empty
// kernel vs the C-ABI forward at a decode size (N = 4, 4096 -> 4096, b = 128, fp32, AUTO), both
// timed on the host clock over 20000 calls with the queue kept short (a sync every 200 calls).
// Build (in the repo root): hipcc --offload-arch=gfx950 -O2 -Iinclude tools/probe/host_launch.hip
//   -Lllama-fft_amd/lib -lbcfft -Wl,-rpath,'$ORIGIN/../../llama-fft_amd/lib' -o tools/probe/host_launch
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <vector>
#include "bcfft.h"

__global__ void empty_k(float* p, int n) {
  if (threadIdx.x == 0 && blockIdx.x == n) p[0] = 1.f;   // never (n = grid)
}

template <class F>
double per_call_us(F&& f, int iters = 20000) {
  for (int i = 0; i < 500; ++i) f();
  (void)hipDeviceSynchronize();
  double total = 0.0;
  for (int rep = 0; rep < iters / 200; ++rep) {
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < 200; ++i) f();
    const auto t1 = std::chrono::steady_clock::now();
    total += std::chrono::duration<double, std::micro>(t1 - t0).count();
    (void)hipDeviceSynchronize();
  }
  return total / iters;
}

int main() {
  const int n = 4, k = 4096, m = 4096, b = 128;
  float *x, *y, *c;
  void* spec;
  (void)hipMalloc(&x, sizeof(float) * n * k);
  (void)hipMalloc(&y, sizeof(float) * n * m);
  (void)hipMalloc(&c, sizeof(float) * (m / b) * (k / b) * b);
  std::vector<float> hc((size_t)(m / b) * (k / b) * b, 0.01f);
  (void)hipMemcpy(c, hc.data(), hc.size() * sizeof(float), hipMemcpyHostToDevice);
  (void)hipMemset(x, 0, sizeof(float) * n * k);
  const int64_t sb = bcfft_spectra_bytes(m / b, k / b, b);
  (void)hipMalloc(&spec, sb);
  hipStream_t s;
  (void)hipStreamCreate(&s);
  int rc = bcfft_spectra(c, BCFFT_F32, m / b, k / b, b, 0, spec, s);
  (void)hipStreamSynchronize(s);
  if (rc != BCFFT_OK) { printf("spectra: %s\n", bcfft_status_string(rc)); return 1; }
  const double t_empty1 = per_call_us([&] { hipLaunchKernelGGL(empty_k, dim3(1), dim3(64), 0, s, y, 1); });
  const double t_empty = per_call_us([&] { hipLaunchKernelGGL(empty_k, dim3(64), dim3(512), 0, s, y, 64); });
  const double t_fwd = per_call_us([&] {
    rc |= bcfft_forward_algo(x, BCFFT_F32, n, k, m, b, spec, nullptr, BCFFT_NONE, y, BCFFT_F32, BCFFT_ALGO_AUTO, s);
  });
  const double t_res = per_call_us([&] { rc |= bcfft_forward_resolve(n, k, m, b, BCFFT_ALGO_AUTO, BCFFT_F32, BCFFT_F32) < 0; });
  printf("empty kernel 1 x 64 threads:    %6.2f us per call (host)\n", t_empty1);
  printf("empty kernel 64 x 512 threads:  %6.2f us per call (host)\n", t_empty);
  printf("bcfft_forward_algo N=%d AUTO:    %6.2f us per call (host), kernel %s\n", n, t_fwd,
         bcfft_forward_kernel_name(n, k, m, b, BCFFT_ALGO_AUTO, BCFFT_F32, BCFFT_F32));
  printf("bcfft_forward_resolve:          %6.2f us per call (host)\n", t_res);
  printf("status %s\n", rc == BCFFT_OK ? "ok" : "error");
  return rc == BCFFT_OK ? 0 : 1;
}
