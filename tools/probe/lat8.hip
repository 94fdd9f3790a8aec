// probe: after an fp8 MFMA whose destination differs from its srcC, issued behind four f16 MFMAs,
// how many wait states until a VALU read of its destination sees the result? The sequence is one
// asm block (no compiler hazard handling inside); NOPS s_nop cycles separate the MFMA and the read.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
template <int NOPS, int KIND>
__global__ void k(float* out) {
  const int l = threadIdx.x;
  f16x8 a, b;
  for (int j = 0; j < 8; ++j) { a[j] = (_Float16)(0.001f * (l + j)); b[j] = (_Float16)(0.002f * (l - j)); }
  const long fa = 0x3838383838383838L;   // e4m3 0x38 = 1.0
  const long fb = 0x3c3c3c3c3c3c3c3cL;   // e5m2 0x3c = 1.0
  f32x4 c = {1.f, 2.f, 3.f, 4.f}, d = {-7.f, -7.f, -7.f, -7.f};
  f32x4 q0 = {0, 0, 0, 0}, q1 = q0, q2 = q0, q3 = q0;
#define NOPSTR(n) "s_nop " #n "\n"
  if constexpr (KIND == 0) {           // fp8 MFMA, dst != srcC, behind 4 f16 MFMAs
    asm volatile(
        "v_mfma_f32_16x16x32_f16 %[q0], %[a], %[b], %[q0]\n"
        "v_mfma_f32_16x16x32_f16 %[q1], %[a], %[b], %[q1]\n"
        "v_mfma_f32_16x16x32_f16 %[q2], %[a], %[b], %[q2]\n"
        "v_mfma_f32_16x16x32_f16 %[q3], %[a], %[b], %[q3]\n"
        "v_mfma_f32_16x16x32_fp8_bf8 %[d], %[fa], %[fb], %[c]\n"
        "s_nop %[n]\n"
        "global_store_dwordx4 %[p], %[d], off\n"
        : [q0] "+v"(q0), [q1] "+v"(q1), [q2] "+v"(q2), [q3] "+v"(q3), [d] "+v"(d)
        : [a] "v"(a), [b] "v"(b), [fa] "v"(fa), [fb] "v"(fb), [c] "v"(c), [n] "n"(NOPS), [p] "v"(out + 4 * l)
        : "memory");
  } else {                             // same with an f16 MFMA in the fp8 one's place
    f16x8 one;
    for (int j = 0; j < 8; ++j) one[j] = (_Float16)1.f;
    asm volatile(
        "v_mfma_f32_16x16x32_f16 %[q0], %[a], %[b], %[q0]\n"
        "v_mfma_f32_16x16x32_f16 %[q1], %[a], %[b], %[q1]\n"
        "v_mfma_f32_16x16x32_f16 %[q2], %[a], %[b], %[q2]\n"
        "v_mfma_f32_16x16x32_f16 %[q3], %[a], %[b], %[q3]\n"
        "v_mfma_f32_16x16x32_f16 %[d], %[o], %[o], %[c]\n"
        "s_nop %[n]\n"
        "global_store_dwordx4 %[p], %[d], off\n"
        : [q0] "+v"(q0), [q1] "+v"(q1), [q2] "+v"(q2), [q3] "+v"(q3), [d] "+v"(d)
        : [a] "v"(a), [b] "v"(b), [o] "v"(one), [c] "v"(c), [n] "n"(NOPS), [p] "v"(out + 4 * l)
        : "memory");
  }
  out[256 + l] = q0[0] + q1[1] + q2[2] + q3[3];
}
template <int N, int KIND>
void run(float* d, float* h) {
  hipLaunchKernelGGL((k<N, KIND>), dim3(1), dim3(64), 0, 0, d);
  (void)hipMemcpy(h, d, 256 * 4, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int l = 0; l < 64; ++l)
    for (int r = 0; r < 4; ++r)                      // D = C + 32 (all-ones operands): {33, 34, 35, 36}
      if (h[4 * l + r] != 33.f + r) ++bad;
  printf("kind %d nops %2d: lane0 %g %g %g %g  bad %d of 256\n", KIND, N, h[0], h[1], h[2], h[3], bad);
}
int main() {
  float* d;
  float h[320];
  (void)hipMalloc(&d, 320 * 4);
  run<0, 0>(d, h); run<1, 0>(d, h); run<3, 0>(d, h); run<5, 0>(d, h); run<7, 0>(d, h);
  run<0, 1>(d, h); run<1, 1>(d, h); run<3, 1>(d, h); run<5, 1>(d, h); run<7, 1>(d, h);
  return 0;
}
