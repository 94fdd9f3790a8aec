// probe: v_mfma_f32_16x16x32_fp8_bf8 / bf8_fp8 operand formats and lane mapping on gfx950.
// A[16][32] bytes, B[32][16] bytes (row-major), lane l supplies A[l%16][8(l/16)..+7] and
// B[8(l/16)..+7][l%16]; D[16][16] fp32 written row-major from the f32x4 accumulator layout
// (lane l: rows 4(l/16)..+3, column l%16).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
typedef float f32x4 __attribute__((ext_vector_type(4)));
__global__ void k(const uint8_t* A, const uint8_t* B, float* D, int which) {
  const int l = threadIdx.x;
  uint64_t a = 0, b = 0;
  for (int j = 0; j < 8; ++j) {
    a |= (uint64_t)A[(l % 16) * 32 + 8 * (l / 16) + j] << (8 * j);
    b |= (uint64_t)B[(8 * (l / 16) + j) * 16 + (l % 16)] << (8 * j);
  }
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (which == 0) acc = __builtin_amdgcn_mfma_f32_16x16x32_fp8_bf8((long)a, (long)b, acc, 0, 0, 0);
  else acc = __builtin_amdgcn_mfma_f32_16x16x32_bf8_fp8((long)a, (long)b, acc, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[(4 * (l / 16) + r) * 16 + (l % 16)] = acc[r];
}
int main(int argc, char** argv) {
  const int which = argc > 1 ? atoi(argv[1]) : 0;
  uint8_t hA[512], hB[512];
  FILE* f = fopen(argv[2], "rb"); fread(hA, 1, 512, f); fread(hB, 1, 512, f); fclose(f);
  uint8_t *dA, *dB; float* dD;
  hipMalloc(&dA, 512); hipMalloc(&dB, 512); hipMalloc(&dD, 1024);
  hipMemcpy(dA, hA, 512, hipMemcpyHostToDevice); hipMemcpy(dB, hB, 512, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dD, which);
  float hD[256];
  hipMemcpy(hD, dD, 1024, hipMemcpyDeviceToHost);
  f = fopen(argv[3], "wb"); fwrite(hD, 4, 256, f); fclose(f);
  printf("ok\n");
  return 0;
}
