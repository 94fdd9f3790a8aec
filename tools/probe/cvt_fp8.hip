// Probe: semantics of gfx950's v_cvt_scalef32_pk_fp8_f16 (two fp16 -> two OCP e4m3 bytes with an
// f32 scale): is the result fp8(v * scale) or fp8(v / scale), does it round to nearest even, does it
// saturate? Prints, per input, the byte for scales 1, 1/64 and 64, and the RNE reference from
// v_cvt_pk_fp8_f32 on the fp32 value v / 64 and v * 64.
// build: hipcc --offload-arch=gfx950 -O2 tools/probe/cvt_fp8.hip -o tools/probe/cvt_fp8
#include <hip/hip_runtime.h>
#include <cstdio>
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef short s16x2 __attribute__((ext_vector_type(2)));

__global__ void k(const float* in, unsigned* out, int n) {
  int i = threadIdx.x;
  if (i >= n) return;
  float v = in[i];
  f16x2 h = {(_Float16)v, (_Float16)0.f};
  s16x2 z = {0, 0};
  s16x2 a = __builtin_amdgcn_cvt_scalef32_pk_fp8_f16(z, h, 1.0f, false);
  s16x2 b = __builtin_amdgcn_cvt_scalef32_pk_fp8_f16(z, h, 1.0f / 64.0f, false);
  s16x2 c = __builtin_amdgcn_cvt_scalef32_pk_fp8_f16(z, h, 64.0f, false);
  int d = __builtin_amdgcn_cvt_pk_fp8_f32((float)(_Float16)v / 64.0f, 0.f, 0, false);
  int e = __builtin_amdgcn_cvt_pk_fp8_f32((float)(_Float16)v * 64.0f, 0.f, 0, false);
  int f = __builtin_amdgcn_cvt_pk_fp8_f32((float)(_Float16)v, 0.f, 0, false);
  out[6 * i + 0] = (unsigned)a[0] & 0xff;
  out[6 * i + 1] = (unsigned)b[0] & 0xff;
  out[6 * i + 2] = (unsigned)c[0] & 0xff;
  out[6 * i + 3] = (unsigned)d & 0xff;
  out[6 * i + 4] = (unsigned)e & 0xff;
  out[6 * i + 5] = (unsigned)f & 0xff;
}

int main() {
  const float vals[] = {1.0f, 1.0625f, 1.125f, 1.1875f, 1.25f, 3.0f, 100.0f, 300.0f, 448.0f, 500.0f, 1000.0f,
                        16384.0f, 0.015625f, 0.01f, -2.5f, 6.0f, 7.0f, 4095.0f};
  const int n = sizeof(vals) / sizeof(vals[0]);
  float* din;
  unsigned* dout;
  hipMalloc(&din, n * sizeof(float));
  hipMalloc(&dout, 6 * n * sizeof(unsigned));
  hipMemcpy(din, vals, n * sizeof(float), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, din, dout, n);
  unsigned h[6 * 64];
  hipMemcpy(h, dout, 6 * n * sizeof(unsigned), hipMemcpyDeviceToHost);
  printf("value      scale1 scale1/64 scale64 | ref(v/64) ref(v*64) ref(v)\n");
  for (int i = 0; i < n; ++i)
    printf("%-10g 0x%02x   0x%02x      0x%02x    | 0x%02x      0x%02x      0x%02x\n", vals[i], h[6 * i], h[6 * i + 1],
           h[6 * i + 2], h[6 * i + 3], h[6 * i + 4], h[6 * i + 5]);
  return 0;
}
