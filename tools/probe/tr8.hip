// probe: fp8 A operand from ds_read_b64_tr_b16 over a byte-pair image (rows 2p, 2p+1 of a column
// in one 16-bit element), chained onto an f16 MFMA's accumulator, as the precise engine's stage 1.
// Pair image P: 16 pair-rows x 16 columns (16-bit), row stride 288 B. A[i][k] = byte (k & 1) of
// P[k >> 1][i] (k < 32). B: 32 x 16 bf8 bytes (row-major) and an f16 32x16 matrix H, A16 16x32 f16.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
__global__ void k(const uint8_t* P, const uint8_t* B, const _Float16* A16, const _Float16* H, float* D, int mode) {
  __shared__ __attribute__((aligned(16))) char lds[288 * 16];
  const int l = threadIdx.x;
  for (int i = l; i < 16 * 16; i += 64) {       // 16 pair-rows x 16 cols x 2 B
    const int r = i / 16, c = i % 16;
    lds[288 * r + 2 * c] = P[(r * 16 + c) * 2];
    lds[288 * r + 2 * c + 1] = P[(r * 16 + c) * 2 + 1];
  }
  __syncthreads();
  const int g = l >> 4, q4 = (l & 15) >> 2, p4 = l & 3;
  const s16x4 rl = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(lds + 288 * (4 * g + q4) + 8 * p4));
  uint64_t b = 0;
  for (int j = 0; j < 8; ++j) b |= (uint64_t)B[(8 * g + j) * 16 + (l % 16)] << (8 * j);
  f16x8 a16, h16;
  for (int j = 0; j < 8; ++j) { a16[j] = A16[(l % 16) * 32 + 8 * g + j]; h16[j] = H[(8 * g + j) * 16 + (l % 16)]; }
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (mode & 1) acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a16, h16, acc, 0, 0, 0);
  if (mode & 2) acc = __builtin_amdgcn_mfma_f32_16x16x32_fp8_bf8(__builtin_bit_cast(long, rl), (long)b, acc, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[(4 * g + r) * 16 + (l % 16)] = acc[r];
}
int main(int argc, char** argv) {
  const int mode = atoi(argv[1]);
  uint8_t hP[512], hB[512]; _Float16 hA[512], hH[512];
  FILE* f = fopen(argv[2], "rb");
  fread(hP, 1, 512, f); fread(hB, 1, 512, f); fread(hA, 2, 512, f); fread(hH, 2, 512, f); fclose(f);
  uint8_t *dP, *dB; _Float16 *dA, *dH; float* dD;
  (void)hipMalloc(&dP, 512); (void)hipMalloc(&dB, 512); (void)hipMalloc(&dA, 1024); (void)hipMalloc(&dH, 1024); (void)hipMalloc(&dD, 1024);
  (void)hipMemcpy(dP, hP, 512, hipMemcpyHostToDevice); (void)hipMemcpy(dB, hB, 512, hipMemcpyHostToDevice);
  (void)hipMemcpy(dA, hA, 1024, hipMemcpyHostToDevice); (void)hipMemcpy(dH, hH, 1024, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dP, dB, dA, dH, dD, mode);
  float hD[256];
  (void)hipMemcpy(hD, dD, 1024, hipMemcpyDeviceToHost);
  f = fopen(argv[3], "wb"); fwrite(hD, 4, 256, f); fclose(f);
  printf("ok %d\n", mode);
  return 0;
}
