// probe: is a VGPR that an issued MFMA reads as SrcB safe to overwrite by the next instructions?
// One asm block (no compiler hazard handling inside): four f16 MFMAs keep the matrix pipe busy,
// then the victim MFMA reads v (= 1.0 everywhere) as B; right behind it v is overwritten with 2.0
// by KIND: 0 v_mov (VALU), 1 ds_read_b128, 2 global_load_dwordx4, 3 ds_read_b64_tr_b16 (two reads),
// 4 no overwrite (control). The victim's D = C + 32 * B: 33.. if it read the old v, 65.. if the
// new. FP8 = 1: the victim is v_mfma_f32_16x16x32_fp8_bf8 with a 64-bit B (e5m2 1.0 -> 2.0, K 32).
// Launched with 64 threads (one wave) and with 512 (two waves per SIMD, all doing the same).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

template <int KIND, int FP8>
__global__ void k(float* out, const u32x4* two16, const u32x2* two8) {
  __shared__ u32x4 lds[64 * 2];
  const int l = threadIdx.x & 63;
  lds[threadIdx.x & 127] = FP8 ? u32x4{two8[0][0], two8[0][1], two8[0][0], two8[0][1]} : two16[0];
  __syncthreads();
  f16x8 a, b, one;
  for (int j = 0; j < 8; ++j) { a[j] = (_Float16)(0.001f * (l + j)); b[j] = (_Float16)(0.002f * (l - j)); one[j] = (_Float16)1.f; }
  f32x4 c = {1.f, 2.f, 3.f, 4.f}, d = {-7.f, -7.f, -7.f, -7.f};
  f32x4 q0 = {0, 0, 0, 0}, q1 = q0, q2 = q0, q3 = q0;
  u32x4 v = __builtin_bit_cast(u32x4, one);                                      // f16 1.0 x 8
  u32x2 v8 = {0x3c3c3c3cu, 0x3c3c3c3cu};                                        // e5m2 1.0 x 8
  const long fa = 0x3838383838383838L;                                           // e4m3 1.0 x 8
  const unsigned la = (unsigned)(uintptr_t)(lds + (threadIdx.x & 63));
  const u32x4* gp = two16;
  u32x2 vlo = {0u, 0u};                                   // (KIND 0, f16: a pair that is NOT the victim's B)
  const u32x2 two2 = {0x40004000u, 0x40004000u};
  const u32x2 two8p = {0x40404040u, 0x40404040u};
#define HEAD "v_mfma_f32_16x16x32_f16 %[q0], %[a], %[b], %[q0]\n v_mfma_f32_16x16x32_f16 %[q1], %[a], %[b], %[q1]\n" \
             "v_mfma_f32_16x16x32_f16 %[q2], %[a], %[b], %[q2]\n v_mfma_f32_16x16x32_f16 %[q3], %[a], %[b], %[q3]\n"
#define TAIL "s_waitcnt vmcnt(0) lgkmcnt(0)\n s_nop 7\n s_nop 7\n s_nop 7\n"
  if constexpr (FP8 == 0) {
    const char* dummy = "";
    (void)dummy;
    if constexpr (KIND == 0)
      asm volatile(HEAD "v_mfma_f32_16x16x32_f16 %[d], %[o], %[v], %[c]\n"
                   "v_pk_mov_b32 %[w], %[s], %[s] op_sel:[0,1]\n" TAIL
                   : [q0] "+v"(q0), [q1] "+v"(q1), [q2] "+v"(q2), [q3] "+v"(q3), [d] "+v"(d), [v] "+v"(v),
                     [w] "+v"(vlo)
                   : [a] "v"(a), [b] "v"(b), [o] "v"(one), [c] "v"(c), [s] "v"(two2) : "memory");
    else if constexpr (KIND == 1)
      asm volatile(HEAD "v_mfma_f32_16x16x32_f16 %[d], %[o], %[v], %[c]\n"
                   "ds_read_b128 %[v], %[la]\n" TAIL
                   : [q0] "+v"(q0), [q1] "+v"(q1), [q2] "+v"(q2), [q3] "+v"(q3), [d] "+v"(d), [v] "+v"(v)
                   : [a] "v"(a), [b] "v"(b), [o] "v"(one), [c] "v"(c), [la] "v"(la) : "memory");
    else if constexpr (KIND == 2)
      asm volatile(HEAD "v_mfma_f32_16x16x32_f16 %[d], %[o], %[v], %[c]\n"
                   "global_load_dwordx4 %[v], %[gp], off\n" TAIL
                   : [q0] "+v"(q0), [q1] "+v"(q1), [q2] "+v"(q2), [q3] "+v"(q3), [d] "+v"(d), [v] "+v"(v)
                   : [a] "v"(a), [b] "v"(b), [o] "v"(one), [c] "v"(c), [gp] "v"(gp) : "memory");
    else if constexpr (KIND == 3)
      asm volatile(HEAD "v_mfma_f32_16x16x32_f16 %[d], %[o], %[v], %[c]\n"
                   "ds_read_b128 %[v], %[la]\n" TAIL
                   : [q0] "+v"(q0), [q1] "+v"(q1), [q2] "+v"(q2), [q3] "+v"(q3), [d] "+v"(d), [v] "+v"(v)
                   : [a] "v"(a), [b] "v"(b), [o] "v"(one), [c] "v"(c), [la] "v"(la) : "memory");
    else
      asm volatile(HEAD "v_mfma_f32_16x16x32_f16 %[d], %[o], %[v], %[c]\n" TAIL
                   : [q0] "+v"(q0), [q1] "+v"(q1), [q2] "+v"(q2), [q3] "+v"(q3), [d] "+v"(d), [v] "+v"(v)
                   : [a] "v"(a), [b] "v"(b), [o] "v"(one), [c] "v"(c) : "memory");
  } else {
    if constexpr (KIND == 0)
      asm volatile(HEAD "v_mfma_f32_16x16x32_fp8_bf8 %[d], %[fa], %[v], %[c]\n"
                   "v_pk_mov_b32 %[v], %[s], %[s] op_sel:[0,1]\n" TAIL
                   : [q0] "+v"(q0), [q1] "+v"(q1), [q2] "+v"(q2), [q3] "+v"(q3), [d] "+v"(d), [v] "+v"(v8)
                   : [a] "v"(a), [b] "v"(b), [fa] "v"(fa), [c] "v"(c), [s] "v"(two8p) : "memory");
    else if constexpr (KIND == 1)
      asm volatile(HEAD "v_mfma_f32_16x16x32_fp8_bf8 %[d], %[fa], %[v], %[c]\n"
                   "ds_read_b64 %[v], %[la]\n" TAIL
                   : [q0] "+v"(q0), [q1] "+v"(q1), [q2] "+v"(q2), [q3] "+v"(q3), [d] "+v"(d), [v] "+v"(v8)
                   : [a] "v"(a), [b] "v"(b), [fa] "v"(fa), [c] "v"(c), [la] "v"(la) : "memory");
    else if constexpr (KIND == 2)
      asm volatile(HEAD "v_mfma_f32_16x16x32_fp8_bf8 %[d], %[fa], %[v], %[c]\n"
                   "global_load_dwordx2 %[v], %[gp], off\n" TAIL
                   : [q0] "+v"(q0), [q1] "+v"(q1), [q2] "+v"(q2), [q3] "+v"(q3), [d] "+v"(d), [v] "+v"(v8)
                   : [a] "v"(a), [b] "v"(b), [fa] "v"(fa), [c] "v"(c), [gp] "v"(two8) : "memory");
    else if constexpr (KIND == 3)
      asm volatile(HEAD "v_mfma_f32_16x16x32_fp8_bf8 %[d], %[fa], %[v], %[c]\n"
                   "ds_read_b64_tr_b16 %[v], %[la]\n" TAIL
                   : [q0] "+v"(q0), [q1] "+v"(q1), [q2] "+v"(q2), [q3] "+v"(q3), [d] "+v"(d), [v] "+v"(v8)
                   : [a] "v"(a), [b] "v"(b), [fa] "v"(fa), [c] "v"(c), [la] "v"(la) : "memory");
    else
      asm volatile(HEAD "v_mfma_f32_16x16x32_fp8_bf8 %[d], %[fa], %[v], %[c]\n" TAIL
                   : [q0] "+v"(q0), [q1] "+v"(q1), [q2] "+v"(q2), [q3] "+v"(q3), [d] "+v"(d), [v] "+v"(v8)
                   : [a] "v"(a), [b] "v"(b), [fa] "v"(fa), [c] "v"(c) : "memory");
  }
  const int w = threadIdx.x >> 6;
  float* o = out + w * 256 + 4 * l;
  o[0] = d[0]; o[1] = d[1]; o[2] = d[2]; o[3] = d[3];
  out[8 * 256 + threadIdx.x] = q0[0] + q1[1] + q2[2] + q3[3];
}

template <int KIND, int FP8>
void run(float* d, const u32x4* g16, const u32x2* g8, int threads) {
  static float h[8 * 256];
  hipLaunchKernelGGL((k<KIND, FP8>), dim3(1), dim3(threads), 0, 0, d, g16, g8);
  if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return; }
  (void)hipMemcpy(h, d, 8 * 256 * 4, hipMemcpyDeviceToHost);
  int oldv = 0, newv = 0, other = 0;
  for (int i = 0; i < threads * 4; ++i) {
    const float e = 1.f + (i & 3);
    if (h[i] == e + 32.f) ++oldv;
    else if (h[i] == e + 64.f) ++newv;
    else ++other;
  }
  printf("%s victim, overwrite %-18s threads %3d: old %4d new %4d other %4d   (elem0 %g)\n", FP8 ? "fp8" : "f16",
         KIND == 0 ? (FP8 ? "v_pk_mov_b32" : "v_pk_mov(other reg)") : KIND == 1 ? "ds_read" : KIND == 2 ? "global_load" : KIND == 3 ? (FP8 ? "ds_read_b64_tr_b16" : "ds_read_b128") : "none",
         threads, oldv, newv, other, h[0]);
}

int main() {
  float* d;
  u32x4* g16;
  u32x2* g8;
  (void)hipMalloc(&d, 8 * 256 * 4 + 512 * 4);
  (void)hipMalloc(&g16, 16);
  (void)hipMalloc(&g8, 16);
  const u32x4 h16 = {0x40004000u, 0x40004000u, 0x40004000u, 0x40004000u};   // f16 2.0 x 8
  const u32x2 h8 = {0x40404040u, 0x40404040u};                              // e5m2 2.0 x 8
  (void)hipMemcpy(g16, &h16, 16, hipMemcpyHostToDevice);
  (void)hipMemcpy(g8, &h8, 8, hipMemcpyHostToDevice);
  for (int threads : {64, 512}) {
    run<4, 0>(d, g16, g8, threads); run<0, 0>(d, g16, g8, threads); run<1, 0>(d, g16, g8, threads);
    run<2, 0>(d, g16, g8, threads); run<3, 0>(d, g16, g8, threads);
    run<4, 1>(d, g16, g8, threads); run<0, 1>(d, g16, g8, threads); run<1, 1>(d, g16, g8, threads);
    run<2, 1>(d, g16, g8, threads); run<3, 1>(d, g16, g8, threads);
  }
  return 0;
}
