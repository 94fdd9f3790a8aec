// bcfft_kernels.hip — CDNA4 (gfx950) kernels of the block-circulant (BC) linear engine.
//
// Hot path: BlockCirculantLinear.forward of the reference (patch_llama_fft.py:226-275):
//   y[n, o*b:(o+1)*b] = sum_i C(c[o,i]) x[n, i*b:(i+1)*b] (+ bias),  C[r,s] = c[(r-s) mod b]
// computed as rfft -> per-bin complex MAC over input blocks -> irfft, all in ONE launch:
//
//   per workgroup: TT=16 tokens x OUT_PER_WG output blocks, 512 threads (8 waves)
//   loop over chunks of IC input blocks:
//     x chunk  --(16 B/lane coalesced loads, prefetched one chunk ahead)--> LDS rows
//     real FFT of every (token, block) row: b/2-point complex FFT of z = x_even + i x_odd,
//        four-step L x P with an L-lane group per transform, untangled into packed bins
//        (bin 0 carries (X_0, X_{b/2}), both real) -> Xf chunk in LDS [block][bin][token]
//     CMAC on the VALU: lane = bin, registers hold acc[bin][out][token] (128 fp32/lane);
//        weight spectra (fp32, L2-resident) streamed straight to registers.
//   epilogue: per output round, accumulators -> LDS rows -> inverse four-step FFT ->
//        cast to x dtype, + bias, cast to y dtype -> 16 B stores.
//
// The 1/b of irfft and the 1/2 of the real-FFT untangling are folded into the spectra.
// See DESIGN.md for the data layout and the roofline accounting.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bcfft.h"

namespace bcfft {

// ------------------------------------------------------------------ scalar conversions
__device__ __forceinline__ float bf16_to_f32(uint32_t h) { return __uint_as_float(h << 16); }
__device__ __forceinline__ uint32_t f32_to_bf16(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (u >> 16) | 0x40u;  // keep NaN a (quiet) NaN
  u += 0x7fffu + ((u >> 16) & 1u);                                 // round to nearest even
  return u >> 16;
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

// ------------------------------------------------------------------ geometry
template <int B>
struct Geo {
  static constexpr int H = B / 2;                 // complex FFT length / packed bins
  static constexpr int L = (H <= 32) ? 4 : 8;     // lanes per transform (four-step H = L x P)
  static constexpr int P = H / L;                 // points per lane
  static constexpr int Q = P / L > 0 ? P / L : 1; // k2 values per lane in step 2
  static constexpr int LBINS = H < 64 ? H : 64;   // bins covered by one pass of 64 lanes
  static constexpr int BPL = H / LBINS;           // bins per lane
  static constexpr int LS = 64 / LBINS;           // lane sub-groups (outputs) per wave
  static constexpr int OPL = (B == 256) ? 2 : 4;  // outputs per lane
  static constexpr int TT = 16;                   // tokens per workgroup
  static constexpr int NW = 8;                    // waves per workgroup
  static constexpr int NT = NW * 64;
  static constexpr int OUT_PER_WG = NW * LS * OPL;
  static constexpr int NGROUPS = NT / L;          // FFT groups in the workgroup
  static constexpr int IC = NGROUPS / TT;         // input blocks per chunk
  // LDS row (floats) of one transform: staging / transpose / natural-order scratch
  static constexpr int ROWA = B + 2 * L;
  static constexpr int ROWB = 2 * P * (L + 1);
  static constexpr int SROW = ((ROWA > ROWB ? ROWA : ROWB) + 3) / 4 * 4;
  static constexpr int XROW = 2 * (TT + 2);       // floats per (block, bin) row of Xf
  // LDS carve (floats)
  static constexpr int TW_OFF = 0;                          // B float2 twiddles
  static constexpr int MAIN_OFF = 2 * B;
  static constexpr int STAGE_FLOATS = NGROUPS * SROW;       // x staging / FFT scratch
  static constexpr int XF_OFF = MAIN_OFF + STAGE_FLOATS;
  static constexpr int XF_FLOATS = IC * H * XROW;
  static constexpr int EPI_ROWS = NW * LS * TT;             // transforms per epilogue round
  static constexpr int EPI_FLOATS = EPI_ROWS * SROW;
  static constexpr int MAIN_FLOATS = STAGE_FLOATS + XF_FLOATS;
  static constexpr int LDS_FLOATS =
      MAIN_OFF + (MAIN_FLOATS > EPI_FLOATS ? MAIN_FLOATS : EPI_FLOATS);
  static_assert(NGROUPS % TT == 0, "FFT groups must cover whole token columns");
  static_assert(EPI_ROWS % NGROUPS == 0, "epilogue rows per group");
  static_assert(LDS_FLOATS * 4 <= 160 * 1024, "LDS budget");
  static_assert(BPL * OPL * TT * 2 == 128, "accumulator budget");
};

template <int XT> struct XTraits;
template <> struct XTraits<BCFFT_F32> { static constexpr int ES = 4; };
template <> struct XTraits<BCFFT_F16> { static constexpr int ES = 2; };
template <> struct XTraits<BCFFT_BF16> { static constexpr int ES = 2; };

// ------------------------------------------------------------------ forward kernel
template <int B, int XT>
__global__ __launch_bounds__(512) void bc_forward_kernel(
    const void* __restrict__ xv, int64_t n_tokens, int n_in, int n_out,
    const float2* __restrict__ spec, const void* __restrict__ bias, int bias_dt,
    void* __restrict__ yv, int y_dt) {
  using G = Geo<B>;
  constexpr int H = G::H, L = G::L, P = G::P, Q = G::Q, TT = G::TT, IC = G::IC;
  constexpr int SROW = G::SROW, XROW = G::XROW;
  constexpr int VEC = 16 / XTraits<XT>::ES;             // elements per 16 B load
  constexpr int CHUNK_ELEMS = TT * IC * B;
  constexpr int NLD = CHUNK_ELEMS / (G::NT * VEC);     // 16 B loads per thread per chunk
  static_assert(CHUNK_ELEMS % (G::NT * VEC) == 0, "chunk/loader mismatch");

  __shared__ __attribute__((aligned(16))) float lds[G::LDS_FLOATS];
  float2* tw = reinterpret_cast<float2*>(lds + G::TW_OFF);   // W_b^m = exp(-2 pi i m / b)
  float* stage = lds + G::MAIN_OFF;
  float* xf = lds + G::XF_OFF;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int64_t t0 = (int64_t)blockIdx.x * TT;
  const int o_base = blockIdx.y * G::OUT_PER_WG;
  const int K = n_in * B;
  const int64_t M = (int64_t)n_out * B;

  // twiddle table (stored by bcfft_spectra after the packed bins)
  const float2* twg = spec + (int64_t)n_out * n_in * H;
  for (int m = tid; m < B; m += G::NT) tw[m] = twg[m];

  // ---- FFT group identity: group g = il*TT + t handles (token t, chunk block il)
  const int g = tid / L;
  const int gl = tid % L;                 // lane within the FFT group
  const int g_t = g % TT;
  const int g_il = g / TT;

  // ---- CMAC identity
  const int lb = lane % G::LBINS;         // first bin of this lane
  const int ls = lane / G::LBINS;         // output sub-group
  const int o_lane = o_base + (wave * G::LS + ls) * G::OPL;   // first output of this lane
  const bool wave_active = (o_base + wave * G::LS * G::OPL) < n_out;

  float acc[G::BPL][G::OPL][TT][2];
#pragma unroll
  for (int j = 0; j < G::BPL; ++j)
#pragma unroll
    for (int q = 0; q < G::OPL; ++q)
#pragma unroll
      for (int t = 0; t < TT; ++t) acc[j][q][t][0] = acc[j][q][t][1] = 0.f;

  // ---- chunk loader (x -> registers, prefetched one chunk ahead)
  uint4 xr[NLD];
  auto load_chunk = [&](int i0) {
#pragma unroll
    for (int u = 0; u < NLD; ++u) {
      const int e = (u * G::NT + tid) * VEC;
      const int t = e / (IC * B);
      const int r = e % (IC * B);
      const int il = r / B;
      const int pos = r % B;
      const int64_t tok = t0 + t;
      if (tok < n_tokens && i0 + il < n_in) {
        const char* src = (const char*)xv +
                          ((tok * K + (int64_t)(i0 + il) * B + pos) * XTraits<XT>::ES);
        xr[u] = *reinterpret_cast<const uint4*>(src);
      } else {
        xr[u] = make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto store_chunk = [&]() {
#pragma unroll
    for (int u = 0; u < NLD; ++u) {
      const int e = (u * G::NT + tid) * VEC;
      const int t = e / (IC * B);
      const int r = e % (IC * B);
      const int il = r / B;
      const int pos = r % B;
      float* dst = stage + (il * TT + t) * SROW + pos;
      if constexpr (XT == BCFFT_F32) {
        *reinterpret_cast<uint4*>(dst) = xr[u];
      } else {
        const uint32_t w[4] = {xr[u].x, xr[u].y, xr[u].z, xr[u].w};
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
  };

  // ---- spectra coefficient loads for one input block (o-major, bins contiguous)
  auto load_coef = [&](int i, float2 (&c)[G::BPL][G::OPL]) {
#pragma unroll
    for (int j = 0; j < G::BPL; ++j)
#pragma unroll
      for (int q = 0; q < G::OPL; ++q) {
        const int o = o_lane + q;
        c[j][q] = (o < n_out && i < n_in)
                      ? spec[((int64_t)o * n_in + i) * H + lb + G::LBINS * j]
                      : make_float2(0.f, 0.f);
      }
  };

  const int n_chunks = (n_in + IC - 1) / IC;
  load_chunk(0);
  __syncthreads();  // twiddles visible

  for (int ch = 0; ch < n_chunks; ++ch) {
    const int i0 = ch * IC;
    __syncthreads();  // previous chunk's CMAC is done with xf / stage
    store_chunk();
    float2 cbuf[2][G::BPL][G::OPL];
    if (wave_active) load_coef(i0, cbuf[0]);
    __syncthreads();

    // ================= forward real FFT of row g (token g_t, block i0+g_il)
    {
      float* row = stage + g * SROW;
      float2 v[P];
#pragma unroll
      for (int n2 = 0; n2 < P; ++n2)
        v[n2] = *reinterpret_cast<const float2*>(row + 2 * (gl + L * n2));
      dft<P, false>(v);
#pragma unroll
      for (int k2 = 1; k2 < P; ++k2) v[k2] = cmul(v[k2], tw[(2 * gl * k2) % B]);   // W_H^(n1 k2)
      wave_lds_sync();
#pragma unroll
      for (int k2 = 0; k2 < P; ++k2)
        *reinterpret_cast<float2*>(row + 2 * (k2 * (L + 1) + gl)) = v[k2];
      wave_lds_sync();
      float2 u[Q][L];
#pragma unroll
      for (int m = 0; m < Q; ++m)
#pragma unroll
        for (int n1 = 0; n1 < L; ++n1)
          u[m][n1] = *reinterpret_cast<const float2*>(row + 2 * ((gl + L * m) * (L + 1) + n1));
#pragma unroll
      for (int m = 0; m < Q; ++m) dft<L, false>(u[m]);
      wave_lds_sync();
#pragma unroll
      for (int m = 0; m < Q; ++m)
#pragma unroll
        for (int k1 = 0; k1 < L; ++k1)   // Z[P*k1 + k2], k2 = gl + L*m, natural order
          *reinterpret_cast<float2*>(row + 2 * (P * k1 + gl + L * m)) = u[m][k1];
      wave_lds_sync();
      // untangle: X'[k] = (Zk + Zm) - i W_b^k (Zk - Zm), Zm = conj(Z[H-k]); k = gl + L*jj
      float* xdst = xf + (g_il * H) * XROW + 2 * g_t;
#pragma unroll
      for (int jj = 0; jj < P; ++jj) {
        const int k = gl + L * jj;
        const float2 zk = *reinterpret_cast<const float2*>(row + 2 * k);
        const float2 zh = *reinterpret_cast<const float2*>(row + 2 * ((H - k) & (H - 1)));
        const float sr = zk.x + zh.x, si = zk.y - zh.y;   // Zk + conj(Z[H-k])
        const float dr = zk.x - zh.x, di = zk.y + zh.y;   // Zk - conj(Z[H-k])
        const float2 w = tw[k];
        float2 o;
        o.x = sr + w.x * di + w.y * dr;
        o.y = si - w.x * dr + w.y * di;
        if (jj == 0 && gl == 0) {   // packed bin 0: (2(ReZ0+ImZ0), 2(ReZ0-ImZ0))
          o.x = 2.f * (zk.x + zk.y);
          o.y = 2.f * (zk.x - zk.y);
        }
        *reinterpret_cast<float2*>(xdst + k * XROW) = o;
      }
    }
    // prefetch the next chunk behind the CMAC (live only during the CMAC)
    if (ch + 1 < n_chunks) load_chunk(i0 + IC);
    __syncthreads();

    // ================= CMAC: acc[bin][out][tok] += S[out][i][bin] * X'[tok][i][bin]
    if (wave_active) {
#pragma unroll
      for (int il = 0; il < IC; ++il) {
        const int i = i0 + il;
        if (i >= n_in) break;
        float2(&cc)[G::BPL][G::OPL] = cbuf[il & 1];
        if (il + 1 < IC) load_coef(i + 1, cbuf[(il + 1) & 1]);
#pragma unroll
        for (int j = 0; j < G::BPL; ++j) {
          const bool bin0 = (j == 0) && (lb == 0);
          float cr[G::OPL], ci[G::OPL], crp[G::OPL];
#pragma unroll
          for (int q = 0; q < G::OPL; ++q) {
            cr[q] = cc[j][q].x;
            ci[q] = bin0 ? 0.f : cc[j][q].y;
            crp[q] = bin0 ? cc[j][q].y : cc[j][q].x;
          }
          const float* xs = xf + (il * H + lb + G::LBINS * j) * XROW;
#pragma unroll
          for (int tp = 0; tp < TT / 2; ++tp) {
            const float4 xx = *reinterpret_cast<const float4*>(xs + 4 * tp);
            const float xr0[2] = {xx.x, xx.z}, xi0[2] = {xx.y, xx.w};
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const int t = 2 * tp + h;
#pragma unroll
              for (int q = 0; q < G::OPL; ++q) {
                float re = acc[j][q][t][0], im = acc[j][q][t][1];
                re = fmaf(cr[q], xr0[h], re);
                re = fmaf(-ci[q], xi0[h], re);
                im = fmaf(crp[q], xi0[h], im);
                im = fmaf(ci[q], xr0[h], im);
                acc[j][q][t][0] = re;
                acc[j][q][t][1] = im;
              }
            }
          }
        }
      }
    }
  }

  // ================= epilogue: inverse real FFT per (output, token), + bias, store
  constexpr int TPG = G::EPI_ROWS / G::NGROUPS;    // transforms per FFT group per round
#pragma unroll
  for (int q = 0; q < G::OPL; ++q) {
    __syncthreads();   // previous round (or the last CMAC) is done with the LDS
    // rows: R = (wave*LS + ls)*TT + t, complex index = bin
#pragma unroll
    for (int j = 0; j < G::BPL; ++j)
#pragma unroll
      for (int t = 0; t < TT; ++t) {
        const int R = (wave * G::LS + ls) * TT + t;
        *reinterpret_cast<float2*>(stage + R * SROW + 2 * (lb + G::LBINS * j)) =
            make_float2(acc[j][q][t][0], acc[j][q][t][1]);
      }
    __syncthreads();
#pragma unroll 1
    for (int u2 = 0; u2 < TPG; ++u2) {
      const int R = g + G::NGROUPS * u2;
      const int sub = R / TT;                // = wave*LS + ls of the writer
      const int t = R % TT;
      const int o = o_base + sub * G::OPL + q;
      float* row = stage + R * SROW;
      // pre-process + step-1 load: Zi[k] = E + iO, E = Y[k] + conj(Y[H-k]),
      // O = (Y[k] - conj(Y[H-k])) W_b^-k; k = gl + L*n2
      float2 v[P];
#pragma unroll
      for (int n2 = 0; n2 < P; ++n2) {
        const int k = gl + L * n2;
        const float2 yk = *reinterpret_cast<const float2*>(row + 2 * k);
        const float2 yh = *reinterpret_cast<const float2*>(row + 2 * ((H - k) & (H - 1)));
        const float er = yk.x + yh.x, ei = yk.y - yh.y;
        const float dr = yk.x - yh.x, di = yk.y + yh.y;
        const float2 w = tw[k];                       // use conj(w)
        float2 z;
        z.x = er - (di * w.x - dr * w.y);
        z.y = ei + (dr * w.x + di * w.y);
        if (n2 == 0 && gl == 0) {   // packed bin 0: (Y0 + YH) + i (Y0 - YH)
          z.x = yk.x + yk.y;
          z.y = yk.x - yk.y;
        }
        v[n2] = z;
      }
      dft<P, true>(v);
#pragma unroll
      for (int k2 = 1; k2 < P; ++k2) v[k2] = cmulc(v[k2], tw[(2 * gl * k2) % B]);
      wave_lds_sync();
#pragma unroll
      for (int k2 = 0; k2 < P; ++k2)
        *reinterpret_cast<float2*>(row + 2 * (k2 * (L + 1) + gl)) = v[k2];
      wave_lds_sync();
      float2 uu[Q][L];
#pragma unroll
      for (int m = 0; m < Q; ++m)
#pragma unroll
        for (int n1 = 0; n1 < L; ++n1)
          uu[m][n1] = *reinterpret_cast<const float2*>(row + 2 * ((gl + L * m) * (L + 1) + n1));
#pragma unroll
      for (int m = 0; m < Q; ++m) dft<L, true>(uu[m]);
      wave_lds_sync();
#pragma unroll
      for (int m = 0; m < Q; ++m)
#pragma unroll
        for (int k1 = 0; k1 < L; ++k1)   // z[m'] = (y[2m'], y[2m'+1]), m' = P*k1 + k2
          *reinterpret_cast<float2*>(row + 2 * (P * k1 + gl + L * m)) = uu[m][k1];
      wave_lds_sync();
      // store: lane gl writes float4 pieces gl, gl+L, ... of the b outputs
      const int64_t tok = t0 + t;
      if (tok < n_tokens && o < n_out) {
#pragma unroll
        for (int pc = 0; pc < B / (4 * L); ++pc) {
          const int p4 = (gl + L * pc) * 4;
          float4 val = *reinterpret_cast<const float4*>(row + p4);
          float vv[4] = {val.x, val.y, val.z, val.w};
          const int64_t col = (int64_t)o * B + p4;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float r = round_to(vv[e], XT);                  // y32.to(x.dtype)  (:266)
            if (bias_dt != BCFFT_NONE) r += load_scalar(bias, col + e, bias_dt);  // (:270-271)
            vv[e] = r;
          }
          const int64_t off = tok * M + col;
          if (y_dt == BCFFT_F32) {
            *reinterpret_cast<float4*>((float*)yv + off) = make_float4(vv[0], vv[1], vv[2], vv[3]);
          } else {
            uint32_t h[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) h[e] = y_dt == BCFFT_BF16 ? f32_to_bf16(vv[e]) : f32_to_f16(vv[e]);
            *reinterpret_cast<uint2*>((uint16_t*)yv + off) = make_uint2(h[0] | (h[1] << 16), h[2] | (h[3] << 16));
          }
        }
      }
    }
  }
}

// ------------------------------------------------------------------ spectra kernel
// One thread per packed bin: direct DFT of the b-point column in fp64, scaled 1/(2b).
template <int B>
__global__ void bc_spectra_kernel(const void* __restrict__ c, int c_dt, int n_out, int n_in,
                                  int transpose_conj, float2* __restrict__ spec) {
  constexpr int H = B / 2;
  const int64_t blk = blockIdx.x;            // (o, i) pair
  const int k = threadIdx.x;                 // packed bin
  if (blk < (int64_t)n_out * n_in && k < H) {
    const int o = (int)(blk / n_in), i = (int)(blk % n_in);
    const int64_t base = blk * B;
    double re = 0.0, im = 0.0, re_h = 0.0;
    for (int n = 0; n < B; ++n) {
      const double v = (double)load_scalar(c, base + n, c_dt);
      double s, co;
      sincospi(2.0 * (double)((k * n) % B) / (double)B, &s, &co);
      re += v * co;
      im -= v * s;
      if (k == 0) re_h += (n & 1) ? -v : v;   // Nyquist bin
    }
    const double sc = 1.0 / (2.0 * B);
    float2 out;
    if (k == 0) out = make_float2((float)(re * sc), (float)(re_h * sc));
    else out = make_float2((float)(re * sc), (float)((transpose_conj ? -im : im) * sc));
    const int64_t dst = transpose_conj ? ((int64_t)i * n_out + o) : ((int64_t)o * n_in + i);
    spec[dst * H + k] = out;
  }
  if (blk == 0) {   // twiddle table W_b^m, m < b
    for (int m = threadIdx.x; m < B; m += blockDim.x) {
      double s, co;
      sincospi(2.0 * (double)m / (double)B, &s, &co);
      spec[(int64_t)n_out * n_in * H + m] = make_float2((float)co, (float)(-s));
    }
  }
}

// ------------------------------------------------------------------ circulant matvec
__global__ void circulant_matvec_kernel(const void* __restrict__ c, const void* __restrict__ x,
                                        int dt, int n, void* __restrict__ y) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  double acc = 0.0;
  for (int s = 0; s < n; ++s) {
    int d = r - s;
    d += (d < 0) ? n : 0;
    acc += (double)load_scalar(c, d, dt) * (double)load_scalar(x, s, dt);
  }
  const float v = (float)acc;
  if (dt == BCFFT_F32) ((float*)y)[r] = v;
  else ((uint16_t*)y)[r] = (uint16_t)(dt == BCFFT_BF16 ? f32_to_bf16(v) : f32_to_f16(v));
}

}  // namespace bcfft

// ====================================================================== C ABI
namespace {
thread_local char g_last_hip_error[256] = {0};

int record_launch() {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    snprintf(g_last_hip_error, sizeof(g_last_hip_error), "%s", hipGetErrorString(e));
    return BCFFT_ERR_HIP;
  }
  return BCFFT_OK;
}
bool valid_dt(int d) { return d == BCFFT_F32 || d == BCFFT_F16 || d == BCFFT_BF16; }
bool valid_block(int b) { return b == 32 || b == 64 || b == 128 || b == 256; }
int promote(int a, int b) { return (b == BCFFT_NONE || a == b) ? a : BCFFT_F32; }
bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

template <int B, int XT>
void launch_forward(const void* x, int64_t n, int n_in, int n_out, const void* spec,
                    const void* bias, int bias_dt, void* y, int y_dt, hipStream_t s) {
  using G = bcfft::Geo<B>;
  dim3 grid((unsigned)((n + G::TT - 1) / G::TT), (unsigned)((n_out + G::OUT_PER_WG - 1) / G::OUT_PER_WG));
  hipLaunchKernelGGL((bcfft::bc_forward_kernel<B, XT>), grid, dim3(G::NT), 0, s, x, n, n_in,
                     n_out, (const float2*)spec, bias, bias_dt, y, y_dt);
}

template <int B>
void launch_forward_b(int xdt, const void* x, int64_t n, int n_in, int n_out, const void* spec,
                      const void* bias, int bias_dt, void* y, int y_dt, hipStream_t s) {
  if (xdt == BCFFT_F32) launch_forward<B, BCFFT_F32>(x, n, n_in, n_out, spec, bias, bias_dt, y, y_dt, s);
  else if (xdt == BCFFT_F16) launch_forward<B, BCFFT_F16>(x, n, n_in, n_out, spec, bias, bias_dt, y, y_dt, s);
  else launch_forward<B, BCFFT_BF16>(x, n, n_in, n_out, spec, bias, bias_dt, y, y_dt, s);
}
}  // namespace

extern "C" {

int bcfft_abi_version(void) { return BCFFT_ABI_VERSION; }

const char* bcfft_status_string(int status) {
  switch (status) {
    case BCFFT_OK: return "ok";
    case BCFFT_ERR_SHAPE: return "shape error: features must be positive multiples of block_size";
    case BCFFT_ERR_BLOCK: return "unsupported block_size (supported: 32, 64, 128, 256)";
    case BCFFT_ERR_DTYPE: return "unsupported dtype or y dtype != promote(x dtype, bias dtype)";
    case BCFFT_ERR_ALIGN: return "x, y and spectra must be 16-byte aligned";
    case BCFFT_ERR_HIP: return "HIP launch failed";
    case BCFFT_ERR_ARG: return "NULL pointer argument";
    default: return "unknown status";
  }
}

const char* bcfft_last_hip_error(void) { return g_last_hip_error; }

int64_t bcfft_spectra_bytes(int n_out_blocks, int n_in_blocks, int block_size) {
  if (n_out_blocks <= 0 || n_in_blocks <= 0 || !valid_block(block_size)) return -1;
  return ((int64_t)n_out_blocks * n_in_blocks * (block_size / 2) + block_size) * 8;
}

int bcfft_spectra(const void* c, int c_dtype, int n_out_blocks, int n_in_blocks, int block_size,
                  int transpose_conj, void* spectra, void* stream) {
  if (!c || !spectra) return BCFFT_ERR_ARG;
  if (!valid_block(block_size)) return BCFFT_ERR_BLOCK;
  if (n_out_blocks <= 0 || n_in_blocks <= 0) return BCFFT_ERR_SHAPE;
  if (!valid_dt(c_dtype)) return BCFFT_ERR_DTYPE;
  if (!aligned16(spectra)) return BCFFT_ERR_ALIGN;
  hipStream_t s = (hipStream_t)stream;
  const unsigned nblk = (unsigned)((int64_t)n_out_blocks * n_in_blocks);
  const int h = block_size / 2;
  const unsigned threads = h < 64 ? 64 : (unsigned)h;
  float2* out = (float2*)spectra;
  switch (block_size) {
    case 32: hipLaunchKernelGGL(bcfft::bc_spectra_kernel<32>, dim3(nblk), dim3(threads), 0, s, c, c_dtype, n_out_blocks, n_in_blocks, transpose_conj, out); break;
    case 64: hipLaunchKernelGGL(bcfft::bc_spectra_kernel<64>, dim3(nblk), dim3(threads), 0, s, c, c_dtype, n_out_blocks, n_in_blocks, transpose_conj, out); break;
    case 128: hipLaunchKernelGGL(bcfft::bc_spectra_kernel<128>, dim3(nblk), dim3(threads), 0, s, c, c_dtype, n_out_blocks, n_in_blocks, transpose_conj, out); break;
    default: hipLaunchKernelGGL(bcfft::bc_spectra_kernel<256>, dim3(nblk), dim3(threads), 0, s, c, c_dtype, n_out_blocks, n_in_blocks, transpose_conj, out); break;
  }
  return record_launch();
}

int bcfft_forward(const void* x, int x_dtype, int64_t n_tokens, int in_features,
                  int out_features, int block_size, const void* spectra, const void* bias,
                  int bias_dtype, void* y, int y_dtype, void* stream) {
  if (!valid_block(block_size)) return BCFFT_ERR_BLOCK;
  if (n_tokens < 0 || in_features <= 0 || out_features <= 0 || in_features % block_size ||
      out_features % block_size)
    return BCFFT_ERR_SHAPE;
  if (!valid_dt(x_dtype) || !valid_dt(y_dtype) || (bias_dtype != BCFFT_NONE && !valid_dt(bias_dtype)))
    return BCFFT_ERR_DTYPE;
  if (y_dtype != promote(x_dtype, bias_dtype)) return BCFFT_ERR_DTYPE;
  if ((bias == nullptr) != (bias_dtype == BCFFT_NONE)) return BCFFT_ERR_ARG;
  if (n_tokens == 0) return BCFFT_OK;
  if (!x || !y || !spectra) return BCFFT_ERR_ARG;
  if (!aligned16(x) || !aligned16(y) || !aligned16(spectra)) return BCFFT_ERR_ALIGN;
  const int n_in = in_features / block_size, n_out = out_features / block_size;
  hipStream_t s = (hipStream_t)stream;
  switch (block_size) {
    case 32: launch_forward_b<32>(x_dtype, x, n_tokens, n_in, n_out, spectra, bias, bias_dtype, y, y_dtype, s); break;
    case 64: launch_forward_b<64>(x_dtype, x, n_tokens, n_in, n_out, spectra, bias, bias_dtype, y, y_dtype, s); break;
    case 128: launch_forward_b<128>(x_dtype, x, n_tokens, n_in, n_out, spectra, bias, bias_dtype, y, y_dtype, s); break;
    default: launch_forward_b<256>(x_dtype, x, n_tokens, n_in, n_out, spectra, bias, bias_dtype, y, y_dtype, s); break;
  }
  return record_launch();
}

int bcfft_circulant_matvec(const void* c, const void* x, int dtype, int n, void* y, void* stream) {
  if (!c || !x || !y) return BCFFT_ERR_ARG;
  if (n <= 0) return BCFFT_ERR_SHAPE;
  if (!valid_dt(dtype)) return BCFFT_ERR_DTYPE;
  hipLaunchKernelGGL(bcfft::circulant_matvec_kernel, dim3((n + 255) / 256), dim3(256), 0,
                     (hipStream_t)stream, c, x, dtype, n, y);
  return record_launch();
}

}  // extern "C"
