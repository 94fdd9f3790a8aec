// probe: back-to-back launch time of an (almost) empty kernel by grid, block and LDS size,
// HIP events around 2000 launches: the floor under a short BC forward launch.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(float* p, int n) {
  extern __shared__ char lds[];
  if (threadIdx.x == 0 && blockIdx.x == n) { lds[0] = 1; p[0] = lds[0]; }   // never (n = grid)
}
__global__ void kstore(float* p) {   // each workgroup writes 64 KiB (the 1024-token shard's y per CU)
  const int t = threadIdx.x;
  float4* q = reinterpret_cast<float4*>(p) + (size_t)blockIdx.x * 4096;
  for (int i = t; i < 4096; i += blockDim.x) q[i] = make_float4(1.f, 2.f, 3.f, 4.f);
}
int main() {
  float* d;
  (void)hipMalloc(&d, 256ull * 65536);
  hipEvent_t a, b;
  (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  const int grids[] = {64, 256, 512};
  const int ldss[] = {0, 65536, 147648};
  for (int g : grids)
    for (int l : ldss) {
      (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      for (int i = 0; i < 100; ++i) hipLaunchKernelGGL(k, dim3(g), dim3(512), l, 0, d, g);
      (void)hipEventRecord(a);
      for (int i = 0; i < 2000; ++i) hipLaunchKernelGGL(k, dim3(g), dim3(512), l, 0, d, g);
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms; (void)hipEventElapsedTime(&ms, a, b);
      printf("empty grid %3d x 512, LDS %6d B: %6.2f us per launch\n", g, l, ms / 2000 * 1000);
    }
  for (int i = 0; i < 100; ++i) hipLaunchKernelGGL(kstore, dim3(256), dim3(512), 0, 0, d);
  (void)hipEventRecord(a);
  for (int i = 0; i < 2000; ++i) hipLaunchKernelGGL(kstore, dim3(256), dim3(512), 0, 0, d);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms; (void)hipEventElapsedTime(&ms, a, b);
  printf("store 16 MiB (256 x 64 KiB): %6.2f us per launch\n", ms / 2000 * 1000);
  return 0;
}
