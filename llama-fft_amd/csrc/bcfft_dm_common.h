// bcfft_dm_common.h — fp16 fragment types and helpers shared by the DFT-on-MFMA kernels
// (bcfft_dm.hip: 4 tokens per M-tile, any x dtype; bcfft_dm8.hip: 8 tokens, bf16 I/O).
#pragma once
#include "bcfft_device.h"

namespace bcfft {
namespace dmh {
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(2))) _Float16 f16x2;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;

// F image: row t, 16-B chunk ch stored at chunk ch ^ fsw(t) (conflict-free for the stage-3 row
// reads and the stage-1 transposed reads)
__device__ __forceinline__ int fsw(int t) { return ((t & 3) << 1) | (t & 8); }
__device__ __forceinline__ uint32_t pk_rtz(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(a, b));
}
__device__ __forceinline__ uint32_t pk_rne(float a, float b) {
  const f16x2 h = {(_Float16)a, (_Float16)b};
  return __builtin_bit_cast(uint32_t, h);
}
__device__ __forceinline__ float lo16(uint32_t p) { return (float)__builtin_bit_cast(f16x2, p).x; }
__device__ __forceinline__ float hi16(uint32_t p) { return (float)__builtin_bit_cast(f16x2, p).y; }
// a - f32(fp16 half of h): one v_fma_mix_f32 (hipcc emits a conversion and a subtraction)
__device__ __forceinline__ float sub_lo16(float a, uint32_t h) {
  float r;
  asm("v_fma_mix_f32 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]" : "=v"(r) : "v"(a), "v"(h));
  return r;
}
__device__ __forceinline__ float sub_hi16(float a, uint32_t h) {
  float r;
  asm("v_fma_mix_f32 %0, %1, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "=v"(r) : "v"(a), "v"(h));
  return r;
}
// (a, b) -> fp16 hi (toward zero) and lo = the rest (toward zero)
__device__ __forceinline__ void split2(float a, float b, uint32_t& hi, uint32_t& lo) {
  hi = pk_rtz(a, b);
  lo = pk_rtz(sub_lo16(a, hi), sub_hi16(b, hi));
}
// max(m, |a|, |b|) in one v_max3_f32 (hipcc canonicalises |a| through an extra v_max first)
__device__ __forceinline__ float amax3(float m, float a, float b) {
  float r;
  asm("v_max3_f32 %0, |%1|, |%2|, %3" : "=v"(r) : "v"(a), "v"(b), "v"(m));
  return r;
}
// max |v| over the wave as an integer max of the magnitude bits (no NaN canonicalisation)
__device__ __forceinline__ uint32_t wave_umax(uint32_t v) {
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, true));   // quad xor 1
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, true));   // quad xor 2
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, true));  // row half mirror
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, true));  // row mirror
  const uint32_t a = max((uint32_t)__builtin_amdgcn_readlane((int)v, 0), (uint32_t)__builtin_amdgcn_readlane((int)v, 16));
  const uint32_t b = max((uint32_t)__builtin_amdgcn_readlane((int)v, 32), (uint32_t)__builtin_amdgcn_readlane((int)v, 48));
  return max(a, b);
}
__device__ __forceinline__ f16x8 frag(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  return __builtin_bit_cast(f16x8, make_uint4(a, b, c, d));
}
// s_setprio(p) for a p the unrolled loops fold to a constant (the instruction takes an immediate).
// The streamed-weight kernels lower a wave's priority as it works through a stage, so that of
// the two waves on a SIMD the one behind issues first instead of the older one (bcfft_dm64k.hip)
__device__ __forceinline__ void set_prio(int p) {
  if (p >= 3) __builtin_amdgcn_s_setprio(3);
  else if (p == 2) __builtin_amdgcn_s_setprio(2);
  else if (p == 1) __builtin_amdgcn_s_setprio(1);
  else __builtin_amdgcn_s_setprio(0);
}
}  // namespace dmh
}  // namespace bcfft
