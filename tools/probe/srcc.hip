// probe: an MFMA that reads as SrcC the result of the MFMA right before it, of ANOTHER opcode
// (v_mfma_f32_16x16x32_f16 -> v_mfma_f32_16x16x32_fp8_bf8 and the reverse), with G independent
// VALU instructions between them; hipcc inserts no wait states for this pair (exact overlap), the
// same as for a same-opcode accumulation chain. One asm block (no compiler hazard handling):
// four f16 MFMAs keep the matrix pipe busy, then
//   CHAIN 0  P = R + 1*1 (K 32, f16)           ; Q = P + 1*1 (K 32, fp8)       Q expected R + 64
//   CHAIN 1  P = R + 1*1 (f16)                  ; R = P + 1*1 (fp8)             (the dftp stage-1
//            schedule: the second MFMA's D is the first one's C)                R expected R0 + 64
//   CHAIN 2  Q = R + 1*1 (fp8)                  ; P = Q + 1*1 (f16)             P expected R + 64
//   CHAIN 3  P = R + 1*1 (f16)                  ; Q = P + 1*1 (f16)  (control)  Q expected R + 64
// One wave (64 threads) and two waves per SIMD (512 threads).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

#define GAP0 ""
#define GAP1 "v_add_u32 %[z], 1, %[z]\n"
#define GAP3 GAP1 GAP1 GAP1
#define GAP6 GAP3 GAP3
#define HEAD "v_mfma_f32_16x16x32_f16 %[q0], %[a], %[b], %[q0]\n v_mfma_f32_16x16x32_f16 %[q1], %[a], %[b], %[q1]\n" \
             "v_mfma_f32_16x16x32_f16 %[q2], %[a], %[b], %[q2]\n v_mfma_f32_16x16x32_f16 %[q3], %[a], %[b], %[q3]\n"
#define TAIL "s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7\n"

template <int CHAIN, int G>
__global__ void k(float* out) {
  const int l = threadIdx.x & 63;
  f16x8 a, b, one;
  for (int j = 0; j < 8; ++j) { a[j] = (_Float16)(0.001f * (l + j)); b[j] = (_Float16)(0.002f * (l - j)); one[j] = (_Float16)1.f; }
  f32x4 q0 = {0, 0, 0, 0}, q1 = q0, q2 = q0, q3 = q0;
  f32x4 r = {100.f + l, 200.f, 300.f, 400.f}, p = {-1.f, -1.f, -1.f, -1.f}, q = p;
  const long e4 = 0x3838383838383838L, b8 = 0x3c3c3c3c3c3c3c3cL;   // e4m3 1.0, e5m2 1.0
  unsigned z = 0;
#define GAPS (G == 0 ? GAP0 : G == 1 ? GAP1 : G == 3 ? GAP3 : GAP6)
#define OPS [q0] "+v"(q0), [q1] "+v"(q1), [q2] "+v"(q2), [q3] "+v"(q3), [p] "+v"(p), [q] "+v"(q), [r] "+v"(r), [z] "+v"(z)
#define INS [a] "v"(a), [b] "v"(b), [o] "v"(one), [e] "v"(e4), [f] "v"(b8)
  if constexpr (CHAIN == 0) {
    if constexpr (G == 0) asm volatile(HEAD "v_mfma_f32_16x16x32_f16 %[p], %[o], %[o], %[r]\n" GAP0 "v_mfma_f32_16x16x32_fp8_bf8 %[q], %[e], %[f], %[p]\n" TAIL : OPS : INS);
    if constexpr (G == 1) asm volatile(HEAD "v_mfma_f32_16x16x32_f16 %[p], %[o], %[o], %[r]\n" GAP1 "v_mfma_f32_16x16x32_fp8_bf8 %[q], %[e], %[f], %[p]\n" TAIL : OPS : INS);
    if constexpr (G == 3) asm volatile(HEAD "v_mfma_f32_16x16x32_f16 %[p], %[o], %[o], %[r]\n" GAP3 "v_mfma_f32_16x16x32_fp8_bf8 %[q], %[e], %[f], %[p]\n" TAIL : OPS : INS);
    if constexpr (G == 6) asm volatile(HEAD "v_mfma_f32_16x16x32_f16 %[p], %[o], %[o], %[r]\n" GAP6 "v_mfma_f32_16x16x32_fp8_bf8 %[q], %[e], %[f], %[p]\n" TAIL : OPS : INS);
  } else if constexpr (CHAIN == 1) {
    if constexpr (G == 0) asm volatile(HEAD "v_mfma_f32_16x16x32_f16 %[p], %[o], %[o], %[r]\n" GAP0 "v_mfma_f32_16x16x32_fp8_bf8 %[r], %[e], %[f], %[p]\n" TAIL : OPS : INS);
    if constexpr (G == 1) asm volatile(HEAD "v_mfma_f32_16x16x32_f16 %[p], %[o], %[o], %[r]\n" GAP1 "v_mfma_f32_16x16x32_fp8_bf8 %[r], %[e], %[f], %[p]\n" TAIL : OPS : INS);
    if constexpr (G == 3) asm volatile(HEAD "v_mfma_f32_16x16x32_f16 %[p], %[o], %[o], %[r]\n" GAP3 "v_mfma_f32_16x16x32_fp8_bf8 %[r], %[e], %[f], %[p]\n" TAIL : OPS : INS);
    if constexpr (G == 6) asm volatile(HEAD "v_mfma_f32_16x16x32_f16 %[p], %[o], %[o], %[r]\n" GAP6 "v_mfma_f32_16x16x32_fp8_bf8 %[r], %[e], %[f], %[p]\n" TAIL : OPS : INS);
    q = r;
  } else if constexpr (CHAIN == 2) {
    if constexpr (G == 0) asm volatile(HEAD "v_mfma_f32_16x16x32_fp8_bf8 %[q], %[e], %[f], %[r]\n" GAP0 "v_mfma_f32_16x16x32_f16 %[p], %[o], %[o], %[q]\n" TAIL : OPS : INS);
    if constexpr (G == 1) asm volatile(HEAD "v_mfma_f32_16x16x32_fp8_bf8 %[q], %[e], %[f], %[r]\n" GAP1 "v_mfma_f32_16x16x32_f16 %[p], %[o], %[o], %[q]\n" TAIL : OPS : INS);
    if constexpr (G == 3) asm volatile(HEAD "v_mfma_f32_16x16x32_fp8_bf8 %[q], %[e], %[f], %[r]\n" GAP3 "v_mfma_f32_16x16x32_f16 %[p], %[o], %[o], %[q]\n" TAIL : OPS : INS);
    if constexpr (G == 6) asm volatile(HEAD "v_mfma_f32_16x16x32_fp8_bf8 %[q], %[e], %[f], %[r]\n" GAP6 "v_mfma_f32_16x16x32_f16 %[p], %[o], %[o], %[q]\n" TAIL : OPS : INS);
    q = p;
  } else {
    if constexpr (G == 0) asm volatile(HEAD "v_mfma_f32_16x16x32_f16 %[p], %[o], %[o], %[r]\n" GAP0 "v_mfma_f32_16x16x32_f16 %[q], %[o], %[o], %[p]\n" TAIL : OPS : INS);
    if constexpr (G == 1) asm volatile(HEAD "v_mfma_f32_16x16x32_f16 %[p], %[o], %[o], %[r]\n" GAP1 "v_mfma_f32_16x16x32_f16 %[q], %[o], %[o], %[p]\n" TAIL : OPS : INS);
    if constexpr (G == 3) asm volatile(HEAD "v_mfma_f32_16x16x32_f16 %[p], %[o], %[o], %[r]\n" GAP3 "v_mfma_f32_16x16x32_f16 %[q], %[o], %[o], %[p]\n" TAIL : OPS : INS);
    if constexpr (G == 6) asm volatile(HEAD "v_mfma_f32_16x16x32_f16 %[p], %[o], %[o], %[r]\n" GAP6 "v_mfma_f32_16x16x32_f16 %[q], %[o], %[o], %[p]\n" TAIL : OPS : INS);
  }
  // expected: the chain's final value = R0 + 64 in every component; report the max deviation
  const f32x4 r0 = {100.f + l, 200.f, 300.f, 400.f};
  float dev = 0.f;
  for (int i = 0; i < 4; ++i) dev = fmaxf(dev, fabsf(q[i] - (r0[i] + 64.f)));
  out[threadIdx.x] = dev + 0.f * (q0[0] + q1[0] + q2[0] + q3[0] + (float)z);
}

template <int CHAIN, int G>
void run(int threads, float* d, float* h) {
  hipLaunchKernelGGL((k<CHAIN, G>), dim3(1), dim3(threads), 0, 0, d);
  hipMemcpy(h, d, threads * sizeof(float), hipMemcpyDeviceToHost);
  float mx = 0.f; int bad = 0;
  for (int i = 0; i < threads; ++i) { mx = fmaxf(mx, h[i]); bad += h[i] != 0.f; }
  const char* names[] = {"f16->fp8 (Q = P + ..)", "f16->fp8, D of 2nd = C of 1st", "fp8->f16", "f16->f16 (control)"};
  printf("chain %-34s gap %d VALU, %3d threads: max |dev| %g, %d of %d lanes wrong\n", names[CHAIN], G, threads, mx, bad, threads);
}
int main() {
  float *d, h[512];
  hipMalloc(&d, 512 * sizeof(float));
  for (int t : {64, 512}) {
    run<0, 0>(t, d, h); run<0, 1>(t, d, h); run<0, 3>(t, d, h); run<0, 6>(t, d, h);
    run<1, 0>(t, d, h); run<1, 1>(t, d, h); run<1, 3>(t, d, h); run<1, 6>(t, d, h);
    run<2, 0>(t, d, h); run<2, 1>(t, d, h); run<2, 3>(t, d, h); run<2, 6>(t, d, h);
    run<3, 0>(t, d, h); run<3, 1>(t, d, h); run<3, 3>(t, d, h); run<3, 6>(t, d, h);
  }
  hipFree(d);
  return 0;
}
