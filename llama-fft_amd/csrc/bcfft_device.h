// bcfft_device.h — device helpers shared by the gfx950 kernels of libbcfft.so (internal).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bcfft.h"
#include "bcfft_analysis.h"

namespace bcfft {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

// ------------------------------------------------------------------ scalar conversions
__device__ __forceinline__ float bf16_to_f32(uint32_t h) { return __uint_as_float(h << 16); }
// hardware round-to-nearest-even (v_cvt_pk_bf16_f32; NaN stays a quiet NaN, denormals kept),
// the rounding of torch's float -> bfloat16. A software RNE with its NaN test compiled to an
// exec-masked branch per value here.
__device__ __forceinline__ uint32_t f32_to_bf16(float f) {
  return __builtin_bit_cast(uint16_t, (__bf16)f);
}
__device__ __forceinline__ float f16_to_f32(uint32_t h) {
  _Float16 v;
  uint16_t s = (uint16_t)h;
  __builtin_memcpy(&v, &s, 2);
  return (float)v;
}
__device__ __forceinline__ uint32_t f32_to_f16(float f) {
  _Float16 v = (_Float16)f;
  uint16_t s;
  __builtin_memcpy(&s, &v, 2);
  return s;
}
// two values -> packed 16-bit pair (low = a), one conversion instruction for bf16
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
typedef __attribute__((ext_vector_type(2))) _Float16 h16x2;
template <int DT>
__device__ __forceinline__ uint32_t pack16(float a, float b) {
  if constexpr (DT == BCFFT_BF16) {
    const bf16x2 h = {(__bf16)a, (__bf16)b};
    return __builtin_bit_cast(uint32_t, h);
  } else {
    const h16x2 h = {(_Float16)a, (_Float16)b};
    return __builtin_bit_cast(uint32_t, h);
  }
}
// packed 16-bit pair (low = first) -> two floats (exact)
template <int DT>
__device__ __forceinline__ float2 unpack16(uint32_t p) {
  if constexpr (DT == BCFFT_BF16) return make_float2(__uint_as_float(p << 16), __uint_as_float(p & 0xffff0000u));
  else return make_float2(f16_to_f32(p & 0xffffu), f16_to_f32(p >> 16));
}
// torch's SiLU in fp32, x * sigmoid(x) = x / (1 + e^-x): hardware exp and reciprocal (~1 ulp each;
// e^-x -> inf gives -0 / NaN as torch does for x -> -inf)
__device__ __forceinline__ float silu(float x) {
  return x * __builtin_amdgcn_rcpf(1.f + __expf(-x));
}
// round a pair to DT and back: the packed pair's halves widened (exact)
template <int DT>
__device__ __forceinline__ float2 round_pair(float a, float b) {
  if constexpr (DT == BCFFT_F32) {
    return make_float2(a, b);
  } else {
    const uint32_t p = pack16<DT>(a, b);
    if constexpr (DT == BCFFT_BF16) return make_float2(__uint_as_float(p << 16), __uint_as_float(p & 0xffff0000u));
    else return make_float2(f16_to_f32(p & 0xffffu), f16_to_f32(p >> 16));
  }
}
// value-exact emulation of tensor.to(dtype) read back as fp32
__device__ __forceinline__ float round_to(float v, int dt) {
  if (dt == BCFFT_BF16) return bf16_to_f32(f32_to_bf16(v));
  if (dt == BCFFT_F16) return f16_to_f32(f32_to_f16(v));
  return v;
}
__device__ __forceinline__ float load_scalar(const void* p, int64_t i, int dt) {
  if (dt == BCFFT_F32) return ((const float*)p)[i];
  uint32_t h = ((const uint16_t*)p)[i];
  return dt == BCFFT_BF16 ? bf16_to_f32(h) : f16_to_f32(h);
}
// elements i .. i + 3 (i a multiple of 4; p 16-B aligned) as fp32: one 16-B or 8-B load
__device__ __forceinline__ float4 load4(const void* p, int64_t i, int dt) {
  if (dt == BCFFT_F32) return *reinterpret_cast<const float4*>((const float*)p + i);
  const uint2 w = *reinterpret_cast<const uint2*>((const uint16_t*)p + i);
  if (dt == BCFFT_BF16)
    return make_float4(bf16_to_f32(w.x & 0xffffu), bf16_to_f32(w.x >> 16), bf16_to_f32(w.y & 0xffffu), bf16_to_f32(w.y >> 16));
  return make_float4(f16_to_f32(w.x & 0xffffu), f16_to_f32(w.x >> 16), f16_to_f32(w.y & 0xffffu), f16_to_f32(w.y >> 16));
}
// v = hi + lo with hi, lo bf16 (hardware RNE, one v_cvt_pk_bf16_f32 per pair): returns packed
// (lo16 = first, hi16 = second) pairs
__device__ __forceinline__ void split_bf16(float2 v, uint32_t& hi, uint32_t& lo) {
  const bf16x2 h = {(__bf16)v.x, (__bf16)v.y};
  hi = __builtin_bit_cast(uint32_t, h);
  const bf16x2 l = {(__bf16)(v.x - __uint_as_float(hi << 16)),
                    (__bf16)(v.y - __uint_as_float(hi & 0xffff0000u))};
  lo = __builtin_bit_cast(uint32_t, l);
}

typedef __attribute__((ext_vector_type(2))) _Float16 f16x2_t;
// ------------------------------------------------------------------ cross-lane / scaling helpers
// (stationary and DFT-on-MFMA kernels)
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, true));
}
constexpr int DPP_XOR1 = 0xB1;   // quad_perm [1,0,3,2]
constexpr int DPP_XOR2 = 0x4E;   // quad_perm [2,3,0,1]
constexpr int DPP_XOR3 = 0x1B;   // quad_perm [3,2,1,0]
constexpr int DPP_P0 = 0xB4;     // quad_perm [0,1,3,2]

// v_mov through inline asm: the compiler cannot hoist or CSE what depends on it, so per-lane
// addresses are rematerialised inside each phase instead of being kept (and spilled) across the
// persistent loop next to the 128 VGPRs of stationary weights
__device__ __forceinline__ int opaque(int v) {
  int r;
  asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "v"(v));
  return r;
}

// packed fp16 product of two fp16 pairs (v_pk_mul_f16)
__device__ __forceinline__ uint32_t pkmul(uint32_t a, uint32_t b) {
  return __builtin_bit_cast(uint32_t, __builtin_bit_cast(f16x2_t, a) * __builtin_bit_cast(f16x2_t, b));
}

// max over the wave's 64 lanes, uniform: quad and row by DPP, the four rows by readlane
__device__ __forceinline__ float wave_max(float v) {
  v = fmaxf(v, dpp<DPP_XOR1>(v));
  v = fmaxf(v, dpp<DPP_XOR2>(v));
  v = fmaxf(v, dpp<0x141>(v));                     // row_half_mirror
  v = fmaxf(v, dpp<0x140>(v));                     // row_mirror
  const int u = __float_as_int(v);
  const float a = fmaxf(__int_as_float(__builtin_amdgcn_readlane(u, 0)), __int_as_float(__builtin_amdgcn_readlane(u, 16)));
  const float b = fmaxf(__int_as_float(__builtin_amdgcn_readlane(u, 32)), __int_as_float(__builtin_amdgcn_readlane(u, 48)));
  return fmaxf(a, b);
}

// scale exponent for fp16 hi/lo: 2^nsc mx < 2^15, clamped so 2^nsc and 2^-nsc stay normal. An
// all-zero piece (mx == 0; frexp gives exponent 0) takes the largest exponent, i.e. "quieter than
// anything": the kernels align a token's pieces to the smallest exponent among them, so a zero
// piece must never become that reference (a quiet piece aligned to it would flush to zero).
__device__ __forceinline__ int stat_scale_exp(float mx) {
  if (mx == 0.f) return 126;
  const int nsc = 15 - __builtin_amdgcn_frexp_expf(mx);
  return nsc < -126 ? -126 : (nsc > 126 ? 126 : nsc);
}

// Cache policy of the streamed activations (per translation unit): with BCFFT_STREAM_POLICY=1
// the x LDS-DMA loads are nt (each token is read once, by one CU) and the y stores sc1 (aux 16:
// write-through, the line leaves the XCD's L2), so that neither evicts the weight fragments every
// CU re-reads from L2 per tile (MI355X_MICROARCH.md: plain and nt stores keep the line in L2,
// sc1 drops it; nt loads are L2-served). Measured (tools/ab_stream.py, profiles/r04_ab_stream_policy.log):
// 6-7 % faster for the multi-group kernels that stream every group's fragments per tile (dmg,
// dm64g, the one-launch MLP); the K-chunk kernels (dmk, dm64k) gain from the write-through stores
// alone (policy 3: 4-5 % at 11008 -> 4096 b = 128), and the VGPR-resident kernels keep the default.
// nt x loads alone were slower everywhere (profiles/r04_ab_stream_policy_split.log).
#ifndef BCFFT_STREAM_POLICY
#define BCFFT_STREAM_POLICY 0
#endif
#if BCFFT_STREAM_POLICY == 1                       // nt x loads, write-through y stores
#define BCFFT_XPOL " nt"
#define BCFFT_YAUX 16
#elif BCFFT_STREAM_POLICY == 2                     // analysis builds: nt x loads only
#define BCFFT_XPOL " nt"
#define BCFFT_YAUX 0
#elif BCFFT_STREAM_POLICY == 3                     // analysis builds: write-through y stores only
#define BCFFT_XPOL ""
#define BCFFT_YAUX 16
#else
#define BCFFT_XPOL ""
#define BCFFT_YAUX 0
#endif

// ------------------------------------------------------------------ LDS-DMA (inline asm)
// hipcc neither counts an asm load in its s_waitcnt bookkeeping nor drains it at a barrier, so
// the x stream stays in flight across compute phases; every wait on it is explicit below.
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
// LDS[m0 + 16 * lane] <- 16 B at the lane's global address (m0 = wave-uniform LDS byte address)
__device__ __forceinline__ void dma16(const void* gsrc, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds) : "memory");
}
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  // a real S_WAITCNT (not inline asm): the compiler's waitcnt pass sees it and knows every older
  // load has landed, so it adds no vmcnt(0) of its own later (those drain in-flight DMA/stores)
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
  asm volatile("" ::: "memory");
}
// workgroup rendezvous on LDS: own LDS traffic complete, then s_barrier; VMEM stays in flight
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }


// ------------------------------------------------------------------ complex helpers
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 w) {
  return make_float2(fmaf(a.x, w.x, -a.y * w.y), fmaf(a.x, w.y, a.y * w.x));
}
__device__ __forceinline__ float2 cmulc(float2 a, float2 w) {  // a * conj(w)
  return make_float2(fmaf(a.x, w.x, a.y * w.y), fmaf(a.y, w.x, -a.x * w.y));
}

// exp(-2*pi*i*m/16) for m < 8: the constant twiddles of the in-register radix-2 DFTs
__device__ __forceinline__ float2 tw16(int m) {
  constexpr float C1 = 0.92387953251128674f, S1 = 0.38268343236508978f, R = 0.70710678118654752f;
  switch (m) {
    case 1: return make_float2(C1, -S1);
    case 2: return make_float2(R, -R);
    case 3: return make_float2(S1, -C1);
    case 5: return make_float2(-S1, -C1);
    case 6: return make_float2(-R, -R);
    case 7: return make_float2(-C1, -S1);
    default: return make_float2(1.f, 0.f);
  }
}

template <bool INV>
__device__ __forceinline__ float2 twiddle16(float2 b, int m) {  // b * W16^m (conj if INV)
  if (m == 0) return b;
  if (m == 4) return INV ? make_float2(-b.y, b.x) : make_float2(b.y, -b.x);
  float2 w = tw16(m);
  return INV ? cmulc(b, w) : cmul(b, w);
}

template <int N>
constexpr int bitrev(int x) {
  int r = 0;
  for (int i = 1; i < N; i <<= 1) { r = (r << 1) | (x & 1); x >>= 1; }
  return r;
}

// In-register N-point DFT (N = 2,4,8,16), natural order in and out.
// Forward: sum_n v[n] e^{-2 pi i nk/N}; INV: e^{+2 pi i nk/N} (unnormalised).
template <int N, bool INV>
__device__ __forceinline__ void dft(float2 (&v)[N]) {
  float2 t[N];
#pragma unroll
  for (int i = 0; i < N; ++i) t[i] = v[bitrev<N>(i)];
#pragma unroll
  for (int len = 2; len <= N; len <<= 1) {
#pragma unroll
    for (int s = 0; s < N; s += len) {
#pragma unroll
      for (int j = 0; j < len / 2; ++j) {
        float2 a = t[s + j];
        float2 b = twiddle16<INV>(t[s + j + len / 2], j * (16 / len));
        t[s + j] = cadd(a, b);
        t[s + j + len / 2] = csub(a, b);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = t[i];
}

// LDS ordering between lanes of ONE wave (the lanes of an FFT group share a wave):
// DS instructions of a wave execute in order; this only stops the compiler from moving
// LDS accesses across the point.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// four consecutive fp32 outputs y32[off .. off+3] of a BC forward -> y, with the reference's
// roundings (patch_llama_fft.py:266-271): .to(x dtype), + bias in fp32, rounded to the y dtype
// (= promote(x dtype, bias dtype): the x dtype, or fp32 when YF32). bias is 16-B aligned.
template <int XT, bool YF32>
__device__ __forceinline__ void store4(float4 val, void* yv, int64_t off, const void* bias, int64_t bcol,
                                       int bias_dt) {
  float vv[4] = {round_to(val.x, XT), round_to(val.y, XT), round_to(val.z, XT), round_to(val.w, XT)};
  if (bias_dt != BCFFT_NONE) {
    float bb[4];
    if (bias_dt == BCFFT_F32) {
      const float4 b4 = *reinterpret_cast<const float4*>((const float*)bias + bcol);
      bb[0] = b4.x; bb[1] = b4.y; bb[2] = b4.z; bb[3] = b4.w;
    } else {
      const uint2 b2 = *reinterpret_cast<const uint2*>((const uint16_t*)bias + bcol);
      const uint32_t w[4] = {b2.x & 0xffffu, b2.x >> 16, b2.y & 0xffffu, b2.y >> 16};
#pragma unroll
      for (int e = 0; e < 4; ++e) bb[e] = bias_dt == BCFFT_BF16 ? bf16_to_f32(w[e]) : f16_to_f32(w[e]);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) vv[e] += bb[e];
  }
  if constexpr (YF32 || XT == BCFFT_F32) {
    *reinterpret_cast<float4*>((float*)yv + off) = make_float4(vv[0], vv[1], vv[2], vv[3]);
  } else {
    uint32_t h[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) h[e] = XT == BCFFT_BF16 ? f32_to_bf16(vv[e]) : f32_to_f16(vv[e]);
    *reinterpret_cast<uint2*>((uint16_t*)yv + off) = make_uint2(h[0] | (h[1] << 16), h[2] | (h[3] << 16));
  }
}

// ------------------------------------------------------------------ FFT building blocks
// One transform per L-lane group, on an LDS row of SROW floats.
template <int B>
struct Fft {
  static constexpr int H = B / 2;                 // complex FFT length / packed bins
  static constexpr int L = (H <= 32) ? 4 : 8;     // lanes per transform (four-step H = L x P)
  static constexpr int P = H / L;                 // points per lane
  static constexpr int Q = P / L > 0 ? P / L : 1; // k2 values per lane in step 2
  static constexpr int ROWA = B + 2 * L;
  static constexpr int ROWB = 2 * P * (L + 1);
  static constexpr int SROW = ((ROWA > ROWB ? ROWA : ROWB) + 3) / 4 * 4;

  // steps 1-2 of the four-step FFT on v (v[n2] = z[gl + L*n2]); on return the row holds
  // the result in natural order (complex index k at floats 2k, 2k+1).
  template <bool INV>
  static __device__ __forceinline__ void core(float* row, int gl, const float2* tw, float2 (&v)[P]) {
    dft<P, INV>(v);
#pragma unroll
    for (int k2 = 1; k2 < P; ++k2) {                                  // W_H^(+-n1 k2)
      const float2 w = tw[(2 * gl * k2) % B];
      v[k2] = INV ? cmulc(v[k2], w) : cmul(v[k2], w);
    }
    wave_lds_sync();
#pragma unroll
    for (int k2 = 0; k2 < P; ++k2)                                    // transpose through the row
      *reinterpret_cast<float2*>(row + 2 * (k2 * (L + 1) + gl)) = v[k2];
    wave_lds_sync();
    float2 u[Q][L];
#pragma unroll
    for (int m = 0; m < Q; ++m)
#pragma unroll
      for (int n1 = 0; n1 < L; ++n1)
        u[m][n1] = *reinterpret_cast<const float2*>(row + 2 * ((gl + L * m) * (L + 1) + n1));
#pragma unroll
    for (int m = 0; m < Q; ++m) dft<L, INV>(u[m]);
    wave_lds_sync();
#pragma unroll
    for (int m = 0; m < Q; ++m)
#pragma unroll
      for (int k1 = 0; k1 < L; ++k1)                                  // index P*k1 + k2
        *reinterpret_cast<float2*>(row + 2 * (P * k1 + gl + L * m)) = u[m][k1];
    wave_lds_sync();
  }

  // forward: row holds x (B reals, fp32 or the raw 16-bit input when RAW16 is the dtype);
  // afterwards Z = FFT_H(x_even + i x_odd) in natural order (fp32 complex)
  template <int RAW = BCFFT_F32>
  static __device__ __forceinline__ void forward(float* row, int gl, const float2* tw) {
    float2 v[P];
#pragma unroll
    for (int n2 = 0; n2 < P; ++n2) {
      const int j = gl + L * n2;
      if constexpr (RAW == BCFFT_F32) {
        v[n2] = *reinterpret_cast<const float2*>(row + 2 * j);
      } else {
        const uint32_t w = reinterpret_cast<const uint32_t*>(row)[j];
        v[n2] = RAW == BCFFT_BF16 ? make_float2(bf16_to_f32(w & 0xffffu), bf16_to_f32(w >> 16))
                                  : make_float2(f16_to_f32(w & 0xffffu), f16_to_f32(w >> 16));
      }
    }
    core<false>(row, gl, tw, v);
  }

  // packed spectrum X'[k] = 2 X[k] (bin 0: (2 X_0, 2 X_{H})) from Z in the row
  static __device__ __forceinline__ float2 untangle(const float* row, int k, const float2* tw) {
    const float2 zk = *reinterpret_cast<const float2*>(row + 2 * k);
    const float2 zh = *reinterpret_cast<const float2*>(row + 2 * ((H - k) & (H - 1)));
    const float sr = zk.x + zh.x, si = zk.y - zh.y;   // Zk + conj(Z[H-k])
    const float dr = zk.x - zh.x, di = zk.y + zh.y;   // Zk - conj(Z[H-k])
    const float2 w = tw[k];
    float2 o;
    o.x = sr + w.x * di + w.y * dr;                    // (Zk+Zm) - i W^k (Zk-Zm)
    o.y = si - w.x * dr + w.y * di;
    if (k == 0) o = make_float2(2.f * (zk.x + zk.y), 2.f * (zk.x - zk.y));
    return o;
  }

  // inverse: the row holds packed Y (complex index k stored at column k ^ swz); afterwards
  // it holds the b real outputs y[0..B) in order (1/b already folded into the spectra).
  static __device__ __forceinline__ void inverse(float* row, int gl, const float2* tw, int swz) {
    float2 v[P];
#pragma unroll
    for (int n2 = 0; n2 < P; ++n2) {
      const int k = gl + L * n2;
      const float2 yk = *reinterpret_cast<const float2*>(row + 2 * (k ^ swz));
      const float2 yh = *reinterpret_cast<const float2*>(row + 2 * (((H - k) & (H - 1)) ^ swz));
      const float er = yk.x + yh.x, ei = yk.y - yh.y;   // E = Y[k] + conj(Y[H-k])
      const float dr = yk.x - yh.x, di = yk.y + yh.y;   // D = Y[k] - conj(Y[H-k])
      const float2 w = tw[k];                           // O = D conj(W^k); Zi = E + iO
      float2 z;
      z.x = er - (di * w.x - dr * w.y);
      z.y = ei + (dr * w.x + di * w.y);
      if (k == 0) z = make_float2(yk.x + yk.y, yk.x - yk.y);   // packed bin 0
      v[n2] = z;
    }
    core<true>(row, gl, tw, v);
  }

  // epilogue store of one transform's b outputs: y32 -> x dtype -> + bias -> y dtype.
  // y dtype = promote(x dtype, bias dtype) is the x dtype or fp32 (YF32); bias is 16-B aligned.
  template <int XT, bool YF32>
  static __device__ __forceinline__ void store(const float* row, int gl, void* yv, int64_t off,
                                               const void* bias, int64_t bcol, int bias_dt) {
#pragma unroll
    for (int pc = 0; pc < B / (4 * L); ++pc) {
      const int p4 = (gl + L * pc) * 4;
      store4<XT, YF32>(*reinterpret_cast<const float4*>(row + p4), yv, off + p4, bias, bcol + p4, bias_dt);
    }
  }

  // split-K partial: one transform's b fp32 outputs to the slice's workspace row (plain 16-B
  // stores; the finishing pass adds the slices in a fixed order)
  static __device__ __forceinline__ void store_partial(const float* row, int gl, float* dst) {
#pragma unroll
    for (int pc = 0; pc < B / (4 * L); ++pc) {
      const int p4 = (gl + L * pc) * 4;
      *reinterpret_cast<float4*>(dst + p4) = *reinterpret_cast<const float4*>(row + p4);
    }
  }
};

template <int XT> struct XTraits;
template <> struct XTraits<BCFFT_F32> { static constexpr int ES = 4; };
template <> struct XTraits<BCFFT_F16> { static constexpr int ES = 2; };
template <> struct XTraits<BCFFT_BF16> { static constexpr int ES = 2; };

// 16 B of x (VEC elements) -> fp32 in LDS
template <int XT>
__device__ __forceinline__ void stage_store(float* dst, uint4 v) {
  if constexpr (XT == BCFFT_F32) {
    *reinterpret_cast<uint4*>(dst) = v;
  } else {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    float f[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if constexpr (XT == BCFFT_BF16) {
        f[2 * k] = bf16_to_f32(w[k] & 0xffffu);
        f[2 * k + 1] = bf16_to_f32(w[k] >> 16);
      } else {
        f[2 * k] = f16_to_f32(w[k] & 0xffffu);
        f[2 * k + 1] = f16_to_f32(w[k] >> 16);
      }
    }
    *reinterpret_cast<float4*>(dst) = make_float4(f[0], f[1], f[2], f[3]);
    *reinterpret_cast<float4*>(dst + 4) = make_float4(f[4], f[5], f[6], f[7]);
  }
}

// ------------------------------------------------------------------ persistent grids
// Output group and tile lane of a persistent 1-D grid's workgroup, and the lane stride. When
// the grid is a multiple of 8 x groups the map is XCD-aware: blocks are dealt round-robin over
// the 8 XCDs (MI355X_MICROARCH.md, workgroup dispatch), so block b = 8 i + xcd takes group
// i % groups and lane 8 (i / groups) + xcd. Every group's workgroup of one tile lane then sits
// on the same XCD and the tile's x is fetched from HBM once, not once per group. Otherwise
// group = b % groups.
struct GroupMap { int grp, lane, stride; };
__device__ __forceinline__ GroupMap group_map(int n_groups) {
  const int b = blockIdx.x;
  if (n_groups > 1 && gridDim.x % (8 * n_groups) == 0)
    return {(b / 8) % n_groups, (b / 8 / n_groups) * 8 + b % 8, (int)gridDim.x / n_groups};
  const int g = b % n_groups;
  return {g, b / n_groups, ((int)gridDim.x - g + n_groups - 1) / n_groups};
}
// grid for group_map: one workgroup per CU, never more than groups x tiles nor fewer than
// groups. It is not trimmed to a multiple of 8 x groups. Trimming 256 CUs to 240 for 3 groups
// cut the HBM reads at 4096 -> 11008 bf16 from 196 to 74 MB (PMC), but it did not save time:
// these kernels are compute-bound. In one A/B session
// (profiles/r02_ab_xcd_map.log; the trim is in the git history of this file) config 2 was level (83-86 us either way),
// while the fused gate/up went from 180 to 189 us and b = 64 4096 -> 11008 from 136 to 140 us.
inline int64_t group_grid(int64_t cus, int groups, int64_t n_mtiles) {
  int64_t total = cus;
  if (total > groups * n_mtiles) total = groups * n_mtiles;
  if (total < groups) total = groups;
  return total;
}

// ------------------------------------------------------------------ spectra buffer layout
// [packed fp32: nO*nI*H float2][twiddles: B float2][MFMA image (b <= 128)][stationary image]
// MFMA image: dword ((c*H + f)*2 + prec)*nOp*8 + o*8 + j  = split-bf16 pair of bin f of
// block (o, 8c + j): bin 0 (C0, C_H) as is, other bins conj(C); prec 0 = hi, 1 = lo.
// Stationary image (stat_eligible geometries, bc_forward_stat_kernel): a 16-B header, then per
// output group of 32 blocks, per wave (8), per register piece, per lane, the 16-B fp16 B fragment
// that lane keeps in VGPRs for the whole launch (bcfft_stat.hip has the exact map), then the
// inverse weight scales 1/s_o of the groups' 32 x groups output blocks (fp32, at osc_off_u32).
// Output block o's fragments hold conj(S) s_o, s_o = 2^(15 - E_o) with max |S[o][.][.]| < 2^E_o:
// every output block keeps fp16's full range, however quiet it is next to the others (one global
// scale pushed the per-bin products of a 1e-4-quiet block into fp16 subnormals).
struct SpecLayout {
  int64_t packed_f2, tw_off_f2, img_off_u32, img_u32, stat_off_u32, stat_u32, osc_off_u32, lo8_off_u32, lo8_u32,
      total_bytes;
  int n_chunk, n_out_pad, stat_groups, stat_pieces;
};
int device_cu_count();         // CUs of the current device (bcfft_stat.hip)
constexpr int BCFFT_MFMA_MAXB = 128;   // largest block size with a split-bf16 MFMA image
__host__ __device__ inline int mfma_out_per_wg(int b) { return 4096 / b; }   // 16 * NTL
// stationary-weight kernel geometries: fp16 B fragments of 32 output blocks x all inputs fit
// 128 VGPRs per lane of 8 waves (K <= 4096), and the A image swizzle needs >= 8 block quads
__host__ __device__ inline bool stat_eligible(int n_in, int b) {
  return (b == 128 && n_in == 32) || (b == 64 && (n_in == 32 || n_in == 64));
}
constexpr int STAT_OUT_BLOCKS = 32;    // output blocks per stationary group (two 16-wide N-tiles)
// the b = 256 DFT kernels (bcfft_dm256.hip): K = 4096 (16 input blocks, weights VGPR-resident)
// and any other K up to 127 blocks (16-block chunks, weights streamed). Their weights are the STAT
// image's (ceil(n_in / 16) K-steps, 16 bins per wave); a workgroup takes one N-tile (16 output
// blocks) of a group. n_in <= 127 keeps Y = acc 2^-21 below fp16's max.
__host__ __device__ inline bool dm256_geometry(int n_in, int b) { return b == 256 && n_in >= 1 && n_in <= 127; }
// the b = 64 streamed-weight DFT kernel (bcfft_dm64k.hip): K > 4096, 32-block chunks of the STAT
// image's K-steps (ceil(n_in / 16)); n_in <= 255 keeps Y = acc 2^-21 below fp16's max at b = 64
__host__ __device__ inline bool dm64k_geometry(int n_in, int b) { return b == 64 && n_in > 64 && n_in <= 255; }
// streamed-weight DFT kernel geometries (bcfft_dmk.hip): b = 128 with K > 4096. The same 16-B
// header, then per output group of 32 blocks, per 16-block K-chunk, per wave (4), per bin of
// the wave (16), per N-tile (2), per lane: the fp16 B fragment the lane loads for that chunk
__host__ __device__ inline bool dmk_geometry(int n_in, int b) { return b == 128 && n_in > 32 && n_in <= 127; }
constexpr int DMK_FRAGS_PER_CHUNK = 4 * 16 * 2;   // waves x bins per wave x N-tiles
__host__ __device__ inline SpecLayout spec_layout(int n_out, int n_in, int b) {
  SpecLayout s;
  const int h = b / 2;
  s.packed_f2 = (int64_t)n_out * n_in * h;
  s.tw_off_f2 = s.packed_f2;
  const int64_t head_f2 = s.packed_f2 + b;
  s.img_off_u32 = head_f2 * 2;
  if (b <= BCFFT_MFMA_MAXB) {
    const int opw = mfma_out_per_wg(b);
    s.n_chunk = (n_in + 7) / 8;
    s.n_out_pad = (n_out + opw - 1) / opw * opw;
    s.img_u32 = (int64_t)s.n_chunk * h * 2 * s.n_out_pad * 8;
  } else {
    s.n_chunk = 0;
    s.n_out_pad = 0;
    s.img_u32 = 0;
  }
  s.stat_off_u32 = s.img_off_u32 + s.img_u32;
  if (stat_eligible(n_in, b) || dm256_geometry(n_in, b) || dm64k_geometry(n_in, b)) {
    s.stat_groups = (n_out + STAT_OUT_BLOCKS - 1) / STAT_OUT_BLOCKS;
    s.stat_pieces = (h / 8) * ((n_in + 15) / 16) * 2;   // bins/wave x K-steps x N-tiles
    s.stat_u32 = 4 + (int64_t)s.stat_groups * 8 * s.stat_pieces * 64 * 4;
  } else if (dmk_geometry(n_in, b)) {
    s.stat_groups = (n_out + STAT_OUT_BLOCKS - 1) / STAT_OUT_BLOCKS;
    s.stat_pieces = (n_in + 15) / 16 * DMK_FRAGS_PER_CHUNK;   // fragments per group
    s.stat_u32 = 4 + (int64_t)s.stat_groups * s.stat_pieces * 64 * 4;
  } else {
    s.stat_groups = 0;
    s.stat_pieces = 0;
    s.stat_u32 = 0;
  }
  s.osc_off_u32 = s.stat_off_u32 + s.stat_u32;         // per-output-block inverse scales
  s.stat_u32 += (int64_t)s.stat_groups * STAT_OUT_BLOCKS;
  // the precise engine's weight residual (bcfft_dm.hip, EP): b = 128, K = 4096 only. Per output
  // group, per wave (8), per bin of the wave (8), per K-step (2), per lane: 16 B = the e4m3 of
  // conj(C) s_o - fp16(conj(C) s_o) for the lane's 8 B-fragment elements of N-tile 0, then N-tile 1
  s.lo8_off_u32 = s.stat_off_u32 + s.stat_u32;
  s.lo8_u32 = (b == 128 && n_in == 32) ? (int64_t)s.stat_groups * 8 * 8 * 2 * 64 * 4 : 0;
  s.total_bytes = (s.lo8_off_u32 + s.lo8_u32) * 4;
  return s;
}

// host launchers of the stationary-weight kernel (bcfft_stat.hip); return false when the
// geometry / dtype combination has no instantiation
bool launch_forward_stat(int b, int n_in, int xdt, bool yf32, const void* x, int64_t n, int n_out,
                         const void* spec, const void* bias, int bias_dt, void* y, hipStream_t s);
// fused gate/up + SwiGLU: h = silu(x Cg) * (x Cu); spec holds ceil(n_gate/16) groups of 32
// interleaved blocks (16 gate, 16 up). false if the geometry is not stationary-eligible.
bool launch_forward_glu(int b, int n_in, int xdt, const void* x, int64_t n, int n_gate, const void* spec,
                        void* h, hipStream_t s);
void launch_stat_image(int b, int n_out, int n_in, void* spec, hipStream_t s);
// the precise engine's e4m3 weight residual image (b = 128, K = 4096; after launch_stat_image)
void launch_lo8_image(int n_out, void* spec, hipStream_t s);
// short-N DFT kernel (bcfft_sn.hip): the STAT image's geometries, one workgroup per 4-token tile (2-token where those fit: sn_tt2)
// and 16-wide N-tile, one workgroup per CU (LDS). AUTO takes it while those workgroups fit one
// round on the device (sn_pays): measured against the persistent engines (tools/time_algos.py
// --short, profiles/r05e_time_short.log) it wins through one round and loses from two (e.g.
// 4096 -> 4096 b = 128 fp32: 9.9 vs 11.3 us at N = 512 = 256 workgroups, 19.6 vs 14.1 at 1024)
bool sn_eligible(int n_in, int b);
bool launch_forward_sn(int b, int n_in, int xdt, bool yf32, const void* x, int64_t n, int n_out, const void* spec,
                       const void* bias, int bias_dt, void* y, hipStream_t s);
inline int64_t sn_workgroups(int64_t n_tokens, int n_out) { return (n_tokens + 3) / 4 * ((n_out + 15) / 16); }
inline bool sn_pays(int64_t n_tokens, int n_out) {
  return n_tokens > 0 && sn_workgroups(n_tokens, n_out) <= device_cu_count();
}
// 2-token tiles (launch_forward_sn) while their workgroups also fit one round
inline bool sn_tt2(int64_t n_tokens, int n_out) {
  return n_tokens > 0 && (n_tokens + 1) / 2 * ((n_out + 15) / 16) <= device_cu_count();
}
// DFT-on-MFMA kernel (bcfft_dm.hip): the STAT image's geometry subset b = 128, K = 4096
bool dm_eligible(int n_in, int b);
bool dftp_serves(int xdt, bool yf32, int bias_dt);   // the precise engine's I/O forms (bcfft_dm.hip)
bool launch_forward_dm(int b, int n_in, int xdt, bool yf32, int mode, const void* x, int64_t n, int n_out,
                       const void* spec, const void* bias, int bias_dt, void* y, hipStream_t s);
bool launch_forward_dm_glu(int b, int n_in, int xdt, int mode, const void* x, int64_t n, int n_gate,
                           const void* spec, void* h, hipStream_t s);
bool dm8_eligible(int n_in, int b, int xdt, bool yf32);
// several output groups at bf16 I/O (bcfft_dmg.hip): one workgroup runs a token tile's stage 1
// once and loops over the groups with their weight fragments streamed from L2
bool dmg_eligible(int n_in, int b, int xdt, bool yf32, int n_out, bool glu);
// The multi-group kernels give one workgroup an 8-token tile for ALL its output groups, so a
// launch has only ceil(N / 8) workgroups; the per-group kernels spread (tile, group) pairs over
// the CUs. They pay once the tiles fill `eighths` / 8 of the CUs. Measured at bf16 on 256 CUs
// (profiles/r03h_dmg_switch.log, profiles/r03i_mg_switch.log; multi-group vs per-group):
//   b = 128 4096 -> 11008 and q/k/v: 3/8 (N = 768: 18.2 vs 18.9 us; N = 20: 15.6 vs 9.7 us)
//   b = 128 fused gate/up + SwiGLU:   5/8 (N = 1024: 38.7 vs 36.2 us; N = 1536: 42.3 vs 43.2 us)
//   b = 64 4096 -> 11008:             4/8 (N = 768: 25.4 vs 23.7 us; N = 1024: 26.9 vs 28.7 us)
//   b = 64 fused gate/up + SwiGLU:    5/8 (N = 1024: 48.1 vs 42.4 us; N = 1536: 50.0 vs 59.2 us)
//   b = 256 4096 -> 11008:            3/8 (N = 512: 18.5 vs 12.2 us; N = 768: 19.2 vs 19.9 us)
// Past one round of tiles a persistent multi-group launch takes ceil(tiles / CUs) whole tile
// times, so it also needs the last round well filled: at least 3/4 of the CUs' share per round
// (N = 2380, 298 tiles on 256 CUs: 2 rounds of 149 -> per-group; N = 3072: 2 rounds of 192 ->
// level with per-group, 78.4 vs 76.9 us for the fused gate/up; N = 4096 and up: multi-group).
inline bool multigroup_pays(int64_t n_tokens, int eighths) {
  const int64_t tiles8 = (n_tokens + 7) / 8, cus = device_cu_count();
  if (tiles8 * 8 < cus * eighths) return false;
  const int64_t rounds = (tiles8 + cus - 1) / cus;
  return rounds == 1 || tiles8 * 4 >= rounds * cus * 3;
}
void launch_forward_dmg(const void* x, int64_t n, int n_out, const void* spec, const void* bias, int bias_dt, void* y,
                        bool glu, hipStream_t s);
bool dm64_eligible(int n_in, int b, int xdt, bool yf32);
void launch_forward_dm64(const void* x, int64_t n, int n_out, const void* spec, const void* bias, int bias_dt,
                         void* y, bool glu, hipStream_t s);
// several output groups at b = 64 (bcfft_dm64g.hip): stage 1 once per tile, the groups' weight
// fragments streamed from L2
bool dm64g_eligible(int n_in, int b, int xdt, bool yf32, int n_out, bool glu);
void launch_forward_dm64g(const void* x, int64_t n, int n_out, const void* spec, const void* bias, int bias_dt,
                          void* y, bool glu, hipStream_t s);
void launch_forward_dm8(const void* x, int64_t n, int n_out, const void* spec, const void* bias, int bias_dt, void* y,
                        bool glu, hipStream_t s);
// b = 256, n_in <= 127, bf16 x and bf16 y (no bias or a bf16 bias) (bcfft_dm256.hip)
bool dm256_eligible(int n_in, int b, int xdt, bool yf32);
void launch_forward_dm256(const void* x, int64_t n, int n_in, int n_out, const void* spec, const void* bias,
                          int bias_dt, void* y, hipStream_t s);
bool dm256_glu_eligible(int n_in, int b, int xdt, int n_gate);
const char* dm256_kernel_name(int64_t n, int n_in, int n_out);   // the kernel launch_forward_dm256 runs
void launch_forward_dm256_glu(const void* x, int64_t n, int n_gate, const void* spec, void* h, hipStream_t s);
// b = 64, K > 4096 (up to 255 input blocks), bf16 x and bf16 y (bcfft_dm64k.hip)
bool dm64k_eligible(int n_in, int b, int xdt, bool yf32);
bool dm64k_pairs(int groups);   // two output groups per workgroup (even group counts)
constexpr int BCFFT_DM64K_MIN_TOKENS = 128;   // AUTO picks the b = 64 streamed-weight kernel from this many tokens
void launch_forward_dm64k(const void* x, int64_t n, int n_in, int n_out, const void* spec, const void* bias,
                          int bias_dt, void* y, hipStream_t s);
// streamed-weight DFT kernel (bcfft_dmk.hip): b = 128, K > 4096, bf16 x and bf16 y
bool dmk_eligible(int n_in, int b, int xdt, bool yf32);
constexpr int BCFFT_DMK_MIN_TOKENS = 1;       // AUTO picks the streamed-weight kernel from this many tokens
void launch_forward_dmk(const void* x, int64_t n, int n_in, int n_out, const void* spec, const void* bias,
                        int bias_dt, void* y, hipStream_t s);
void launch_dmk_image(int n_out, int n_in, void* spec, hipStream_t s);
// its K-chunk split for short grids (decode sizes): kz slices write fp32 partials to a caller
// workspace of kz x n x n_out * 128 floats, a finishing pass sums them; dmk_ksplit: 1 = no split
int dmk_ksplit(int64_t n, int n_in, int n_out);
void launch_forward_dmk_split(const void* x, int64_t n, int n_in, int n_out, const void* spec, const void* bias,
                              int bias_dt, void* y, float* ws, int kz, hipStream_t s);
// the split forms' finishing pass: y (bf16, n x M) = bf16(sum of the kz fp32 partial slabs in order) + bias
void launch_partials_finish(const float* ws, int kz, int64_t n, int64_t M, const void* bias, int bias_dt, void* y,
                            hipStream_t s);
// fused BC-MLP (bcfft_dmm.hip): y = down(silu(gate(x)) * up(x)) in one launch; bf16 x and y,
// b = 128, hidden 4096 (n_in = n_out = 32 blocks), intermediate n_h blocks with 32 < n_h <= 127
bool dmm_eligible(int n_in, int b, int xdt, int n_h, int n_out);
// the MLP's AUTO mode takes the fused kernel once its 8-token tiles fill 3/8 of the CUs (N = 768 on
// 256 CUs: 53.7 us vs 53.2 split; N = 1024: 57.7 vs 60.3; N = 256: 52.6 vs 34.0, the split form's
// per-group gate/up kernel spreading over more CUs; profiles/r03h_dmg_switch.log)
inline bool dmm_pays(int64_t n_tokens) { return multigroup_pays(n_tokens, 3); }
void launch_mlp_dmm(const void* x, int64_t n, int n_h, const void* spec_gu, const void* spec_dn, void* y,
                    hipStream_t s);
// its group split for short grids: kz slices of the gate/up groups (= the down projection's
// K-chunks) per 8-token tile, fp32 partial y slabs (kz x n x 4096 floats) and the finishing
// pass; dmm_ksplit: 1 = no split
int dmm_ksplit(int64_t n, int n_h);
void launch_mlp_dmm_split(const void* x, int64_t n, int n_h, const void* spec_gu, const void* spec_dn, void* y,
                          float* ws, int kz, hipStream_t s);

// weight prep (bcfft_prep.hip): loss-aware circulant projection of a dense (n_out*b, n_in*b)
// weight into c (n_out, n_in, b) fp32; false for an unsupported block size
bool launch_project(int b, const void* w, int dt, int n_out, int n_in, float eps, float* c, hipStream_t s);

// dc of the BC forward (bcfft_grad.hip): token split and workspace of the two-launch reduction
struct GradPlan { int64_t tiles, splits, tokens_per_split, workspace_bytes; };
GradPlan grad_plan(int b, int64_t n, int n_in, int n_out);
void launch_grad_c(int b, const void* x, int x_dt, const void* dy, int dy_dt, int64_t n, int n_in, int n_out,
                   void* ws, void* dc, int dc_dt, hipStream_t s);

}  // namespace bcfft
