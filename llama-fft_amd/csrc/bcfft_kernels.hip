// bcfft_kernels.hip — CDNA4 (gfx950) kernels of the block-circulant (BC) linear engine.
//
// Hot path: BlockCirculantLinear.forward of the reference (patch_llama_fft.py:226-275):
//   y[n, o*b:(o+1)*b] = sum_i C(c[o,i]) x[n, i*b:(i+1)*b] (+ bias),  C[r,s] = c[(r-s) mod b]
// computed as rfft -> per-bin complex MAC over input blocks -> irfft, in ONE launch.
//
// Two forward kernels share the FFT building blocks below:
//   * bc_forward_mfma_kernel (BCFFT_ALGO_MFMA, default for b <= 128): the per-bin complex MAC
//     runs on the matrix cores as a dense bf16 GEMM with 4-term hi/lo splitting
//     ((Xhi+Xlo)(Chi+Clo), fp32 accumulate, ~1e-5 relative), the FFTs on the VALU.
//   * bc_forward_valu_kernel (BCFFT_ALGO_VALU): the complex MAC in fp32 FMAs (exact fp32
//     arithmetic, the reference's precision); also the b = 256 path.
//
// Per workgroup: TT = 16 tokens x OUT_PER_WG output blocks, 512 threads (8 waves):
//   loop over chunks of input blocks:
//     x chunk  --(16 B/lane coalesced loads, prefetched one chunk ahead)--> LDS rows
//     real FFT of every (token, block) row: b/2-point complex FFT of z = x_even + i x_odd,
//        four-step L x P, an L-lane group per transform, untangled into packed bins
//        (bin 0 carries (X_0, X_{b/2}), both real)
//     complex MAC into register accumulators (MFMA or VALU)
//   epilogue: accumulators -> LDS rows -> inverse four-step FFT -> cast to x dtype, + bias,
//        cast to y dtype -> 16 B stores.
// The 1/b of irfft and the 1/2 of the real-FFT untangling are folded into the spectra.
// DESIGN.md has the layouts and the roofline accounting.
#include "bcfft_device.h"
#include "bcfft.h"

namespace bcfft {

// ================================================================== VALU forward kernel
template <int B>
struct GeoV {
  using F = Fft<B>;
  static constexpr int H = B / 2, L = F::L, SROW = F::SROW;
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
  static constexpr int XROW = 2 * (TT + 2);       // floats per (block, bin) row of Xf
  static constexpr int MAIN_OFF = 2 * B;          // after B float2 twiddles
  static constexpr int STAGE_FLOATS = NGROUPS * SROW;
  static constexpr int XF_OFF = MAIN_OFF + STAGE_FLOATS;
  static constexpr int XF_FLOATS = IC * H * XROW;
  static constexpr int EPI_ROWS = NW * LS * TT;
  static constexpr int EPI_FLOATS = EPI_ROWS * SROW;
  static constexpr int MAIN_FLOATS = STAGE_FLOATS + XF_FLOATS;
  static constexpr int LDS_FLOATS = MAIN_OFF + (MAIN_FLOATS > EPI_FLOATS ? MAIN_FLOATS : EPI_FLOATS);
  static_assert(NGROUPS % TT == 0, "FFT groups must cover whole token columns");
  static_assert(EPI_ROWS % NGROUPS == 0, "epilogue rows per group");
  static_assert(LDS_FLOATS * 4 <= 160 * 1024, "LDS budget");
  static_assert(BPL * OPL * TT * 2 == 128, "accumulator budget");
};

template <int B, int XT, bool YF32>
__global__ __launch_bounds__(512) void bc_forward_valu_kernel(
    const void* __restrict__ xv, int64_t n_tokens, int n_in, int n_out,
    const float2* __restrict__ spec, const void* __restrict__ bias, int bias_dt,
    void* __restrict__ yv, float* __restrict__ yacc) {
  using G = GeoV<B>;
  using F = Fft<B>;
  constexpr int H = G::H, L = G::L, TT = G::TT, IC = G::IC, SROW = G::SROW, XROW = G::XROW;
  constexpr int VEC = 16 / XTraits<XT>::ES;
  constexpr int CHUNK_ELEMS = TT * IC * B;
  constexpr int NLD = CHUNK_ELEMS / (G::NT * VEC);
  static_assert(CHUNK_ELEMS % (G::NT * VEC) == 0, "chunk/loader mismatch");

  __shared__ __attribute__((aligned(16))) float lds[G::LDS_FLOATS];
  float2* tw = reinterpret_cast<float2*>(lds);
  float* stage = lds + G::MAIN_OFF;
  float* xf = lds + G::XF_OFF;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform (SGPR)
  const int64_t t0 = (int64_t)blockIdx.x * TT;
  const int o_base = blockIdx.y * G::OUT_PER_WG;
  const int K = n_in * B;
  const int64_t M = (int64_t)n_out * B;

  const float2* twg = spec + spec_layout(n_out, n_in, B).tw_off_f2;
  for (int m = tid; m < B; m += G::NT) tw[m] = twg[m];

  const int g = tid / L, gl = tid % L;    // FFT group (token g % TT, chunk block g / TT)
  const int g_t = g % TT, g_il = g / TT;
  const int lb = lane % G::LBINS;         // first bin of this lane
  const int ls = lane / G::LBINS;         // output sub-group
  const int o_lane = o_base + (wave * G::LS + ls) * G::OPL;
  const bool wave_active = (o_base + wave * G::LS * G::OPL) < n_out;

  float acc[G::BPL][G::OPL][TT][2];
#pragma unroll
  for (int j = 0; j < G::BPL; ++j)
#pragma unroll
    for (int q = 0; q < G::OPL; ++q)
#pragma unroll
      for (int t = 0; t < TT; ++t) acc[j][q][t][0] = acc[j][q][t][1] = 0.f;

  uint4 xr[NLD];
  auto load_chunk = [&](int i0) {
#pragma unroll
    for (int u = 0; u < NLD; ++u) {
      const int e = (u * G::NT + tid) * VEC;
      const int t = e / (IC * B), r = e % (IC * B), il = r / B, pos = r % B;
      const int64_t tok = t0 + t;
      xr[u] = (tok < n_tokens && i0 + il < n_in)
                  ? *reinterpret_cast<const uint4*>((const char*)xv +
                        ((tok * K + (int64_t)(i0 + il) * B + pos) * XTraits<XT>::ES))
                  : make_uint4(0, 0, 0, 0);
    }
  };
  auto store_chunk = [&]() {
#pragma unroll
    for (int u = 0; u < NLD; ++u) {
      const int e = (u * G::NT + tid) * VEC;
      const int t = e / (IC * B), r = e % (IC * B), il = r / B, pos = r % B;
      stage_store<XT>(stage + (il * TT + t) * SROW + pos, xr[u]);
    }
  };
  auto load_coef = [&](int i, float2 (&c)[G::BPL][G::OPL]) {
#pragma unroll
    for (int j = 0; j < G::BPL; ++j)
#pragma unroll
      for (int q = 0; q < G::OPL; ++q) {
        const int o = o_lane + q;
        c[j][q] = (o < n_out && i < n_in) ? spec[((int64_t)o * n_in + i) * H + lb + G::LBINS * j]
                                          : make_float2(0.f, 0.f);
      }
  };

  // split-K (gridDim.z slices, yacc != nullptr): as in bc_forward_mfma_kernel, slice z walks
  // chunks [c_lo, c_hi) and writes its partial rows to slab z of yacc
  const int n_chunks = (n_in + IC - 1) / IC;
  const int cps = (n_chunks + (int)gridDim.z - 1) / (int)gridDim.z;
  const int c_lo = (int)blockIdx.z * cps;
  const int c_hi = c_lo + cps < n_chunks ? c_lo + cps : n_chunks;
  load_chunk(c_lo * IC);
  __syncthreads();

  for (int ch = c_lo; ch < c_hi; ++ch) {
    const int i0 = ch * IC;
    __syncthreads();
    store_chunk();
    float2 cbuf[2][G::BPL][G::OPL];
    if (wave_active) load_coef(i0, cbuf[0]);
    __syncthreads();
    {
      float* row = stage + g * SROW;
      F::template forward<BCFFT_F32>(row, gl, tw);
      float* xdst = xf + (g_il * H) * XROW + 2 * g_t;
#pragma unroll
      for (int jj = 0; jj < F::P; ++jj) {
        const int k = gl + L * jj;
        *reinterpret_cast<float2*>(xdst + k * XROW) = F::untangle(row, k, tw);
      }
    }
    if (ch + 1 < c_hi) load_chunk(i0 + IC);
    __syncthreads();

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

  constexpr int TPG = G::EPI_ROWS / G::NGROUPS;
#pragma unroll
  for (int q = 0; q < G::OPL; ++q) {
    __syncthreads();
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
      const int t = R % TT;
      const int o = o_base + (R / TT) * G::OPL + q;
      float* row = stage + R * SROW;
      F::inverse(row, gl, tw, 0);
      const int64_t tok = t0 + t;
      if (tok < n_tokens && o < n_out) {
        if (yacc)
          F::store_partial(row, gl, yacc + ((int64_t)blockIdx.z * n_tokens + tok) * M + (int64_t)o * B);
        else
          F::template store<XT, YF32>(row, gl, yv, tok * M + (int64_t)o * B, bias, (int64_t)o * B, bias_dt);
      }
    }
  }
}

// ================================================================== MFMA forward kernel
// CMAC per bin f as a real GEMM on v_mfma_f32_16x16x32_bf16:
//   rows (M=16) = 8 tokens x {re, im} of the output, cols (N=16) = 16 output blocks,
//   K = 32 = {X hi, X lo} x 8 input blocks x {re, im} of the input.
//   A[(t,re)][(i,*)] = (xr, xi), A[(t,im)][(i,*)] = (xi, -xr), B[(i,*)][o] = conj(C[o,i])
//   => D[(t,re)][o] = sum_i Re(C X), D[(t,im)][o] = sum_i Im(C X).
//   Bin 0 (packed DC/Nyquist, both real): A = (X0, 0) / (0, X_H), B = (C0, C_H).
//   Two MFMAs per tile: B = C_hi and B = C_lo -> (Xhi + Xlo)(Chi + Clo), fp32 accumulate.
// x streams through two half-chunk LDS buffers by inline-asm LDS-DMA: half 0 of chunk c+1 is
// issued as soon as the FFTs of half 0 of chunk c are done (it lands under the half-1 FFTs and
// the MFMAs), half 1 after the MFMAs (it lands under the next half-0 FFTs). Waits are counted
// (every wave issues exactly NH DMAs per half), barriers are raw s_barrier + lgkmcnt(0).
template <int B>
struct GeoM {
  using F = Fft<B>;
  static constexpr int H = B / 2, L = F::L, SROW = F::SROW;
  static constexpr int TT = 8, NW = 4, NT = NW * 64;   // 8 tokens = one MFMA row tile
  static constexpr int KB = 8, KH = KB / 2;       // input blocks per chunk (MFMA K = 32) / half
  static constexpr int BPW = H / NW;              // bins per wave
  static constexpr int NTL = 32 / BPW;            // 16-output N-tiles per workgroup
  static constexpr int OUT_PER_WG = 16 * NTL;
  static constexpr int NGROUPS = NT / L;
  static constexpr int HROWS = TT * KH;           // x rows per half-chunk, row r = (r / KH, r % KH)
  static constexpr int HTPG = (HROWS + NGROUPS - 1) / NGROUPS;   // transforms per group per half
  static constexpr int NH = HROWS / NW;           // DMA instructions per wave per half-chunk
  static constexpr int XS = 2 * TT * KB + 4;      // dwords per bin of the split-X image (+4 pad)
  static constexpr int MAIN_OFF = 2 * B;
  static constexpr int STAGE_FLOATS = 2 * HROWS * SROW;
  static constexpr int XL_OFF = MAIN_OFF + STAGE_FLOATS;
  static constexpr int XL_FLOATS = H * XS;
  static constexpr int EPI_ROWS = 16 * TT;        // one N-tile: 16 outputs x TT tokens
  static constexpr int EPI_FLOATS = EPI_ROWS * SROW;
  static constexpr int MAIN_FLOATS = STAGE_FLOATS + XL_FLOATS;
  static constexpr int LDS_FLOATS = MAIN_OFF + (MAIN_FLOATS > EPI_FLOATS ? MAIN_FLOATS : EPI_FLOATS);
  static constexpr int STEPS = BPW * NTL;         // (bin, N-tile) steps per wave per chunk
  static constexpr int RING = 4;                  // B-fragment prefetch depth (steps)

  static_assert(BPW * NTL * 4 == 128, "accumulator budget");
  static_assert(HROWS % NW == 0 && EPI_ROWS % NGROUPS == 0, "row tiling");
  static_assert(H >= 16, "bin swizzle needs H >= 16");
  static_assert(LDS_FLOATS * 4 <= (B <= 128 ? 80 : 160) * 1024, "LDS budget: two workgroups per CU (b <= 128)");
};

template <int B, int XT, bool YF32>
__global__ __launch_bounds__(256, 2) void bc_forward_mfma_kernel(
    const void* __restrict__ xv, int64_t n_tokens, int n_in, int n_out,
    const float2* __restrict__ spec, const void* __restrict__ bias, int bias_dt,
    void* __restrict__ yv, float* __restrict__ yacc) {
  using G = GeoM<B>;
  using F = Fft<B>;
  constexpr int H = G::H, L = G::L, TT = G::TT, KB = G::KB, KH = G::KH, SROW = G::SROW, XS = G::XS;
  constexpr int NTL = G::NTL, BPW = G::BPW, STEPS = G::STEPS, RING = G::RING, NH = G::NH;
  constexpr int ES = XTraits<XT>::ES;
  constexpr int DMA_LANES = B * ES / 16;          // one 16-B-per-lane DMA instruction per x row
  static_assert(DMA_LANES <= 64, "x row fits one DMA instruction");

  ANALYSIS_INIT;
  __shared__ __attribute__((aligned(16))) float lds[G::LDS_FLOATS];
  float2* tw = reinterpret_cast<float2*>(lds);
  float* stage = lds + G::MAIN_OFF;
  uint32_t* xl = reinterpret_cast<uint32_t*>(lds + G::XL_OFF);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform (SGPR)
  const int64_t t0 = (int64_t)blockIdx.x * TT;
  const int o_base = blockIdx.y * G::OUT_PER_WG;
  const int K = n_in * B;
  const int64_t M = (int64_t)n_out * B;

  const SpecLayout sl = spec_layout(n_out, n_in, B);
  const float2* twg = spec + sl.tw_off_f2;
  const uint32_t* img = reinterpret_cast<const uint32_t*>(spec) + sl.img_off_u32;
  const int64_t prec_stride = (int64_t)sl.n_out_pad * 8;      // dwords between hi and lo slabs
  for (int m = tid; m < B; m += G::NT) tw[m] = twg[m];

  const int g = tid / L, gl = tid % L;    // FFT group
  // MFMA lane roles
  const int row = lane & 15, kb = lane >> 4;
  const int a_prec = kb >> 1, a_half = kb & 1;
  const int p_out = row & 1;
  const uint32_t a_sel = p_out ? 0x01000302u : 0x03020100u;   // im rows: swap (xr, xi)
  const uint32_t a_xor = p_out ? 0x80000000u : 0u;            //   -> (xi, -xr)
  const uint32_t a_bin0 = p_out ? 0xffff0000u : 0x0000ffffu;  // bin 0: (X0, 0) / (0, X_H)

  f32x4 acc[BPW][NTL];
#pragma unroll
  for (int fb = 0; fb < BPW; ++fb)
#pragma unroll
    for (int nt = 0; nt < NTL; ++nt) acc[fb][nt] = f32x4{0.f, 0.f, 0.f, 0.f};

  // half-chunk h of the chunk starting at input block i0 -> stage buffer h, raw x dtype.
  // Out-of-range rows read clamped (valid, finite-if-x-is) sources instead of branching, so every
  // wave issues exactly NH DMAs: past-the-end tokens are never stored, and blocks >= n_in meet
  // zero weights in the MFMA image.
  const int64_t last_tok = n_tokens - 1;
  auto dma_half = [&](int i0, int h) {
#pragma unroll
    for (int q = 0; q < NH; ++q) {
      const int r = q * G::NW + wave;
      const int t = r / KH, blk = h * KH + r % KH;
      const int64_t tok = t0 + t < n_tokens ? t0 + t : last_tok;
      const int ib = i0 + blk < n_in ? i0 + blk : 0;
      const char* src = (const char*)xv + (tok * K + (int64_t)ib * B) * ES + lane * 16;
      const uint32_t dst = __builtin_amdgcn_readfirstlane(lds_addr(stage + (h * G::HROWS + r) * SROW));
      if (ABLATE(16)) continue;
      if (lane < DMA_LANES) dma16(src, dst);
    }
  };
  // forward FFTs of half-chunk h -> split-X image [bin][prec][token][block]
  auto fft_half = [&](int h) {
#pragma unroll 1
    for (int u = 0; u < G::HTPG; ++u) {
      const int r = g + G::NGROUPS * u;
      if (r < G::HROWS) {                       // b <= 64: half the groups idle per half-chunk
        float* rowp = stage + (h * G::HROWS + r) * SROW;
        if (!ABLATE(4)) F::template forward<XT>(rowp, gl, tw);
        uint32_t* dst = xl + (r / KH) * KB + h * KH + r % KH;
#pragma unroll
        for (int jj = 0; jj < F::P; ++jj) {
          const int k = gl + L * jj;
          uint32_t hi, lo;
          split_bf16(F::untangle(rowp, k, tw), hi, lo);
          dst[k * XS] = hi;
          dst[k * XS + TT * KB] = lo;
        }
      }
    }
  };
  // B fragments (hi, lo) for step s of chunk c: 16 B each, 8 blocks of output o
  auto load_b = [&](int c, int s, uint4 (&dst)[2]) {
    const int fb = s / NTL, nt = s % NTL;
    const int f = wave * BPW + fb;
    const int o = o_base + 16 * nt + row;
    const uint32_t* p = img + ((int64_t)(c * H + f) * 2) * prec_stride + o * 8 + a_half * 4;
    dst[0] = *reinterpret_cast<const uint4*>(p);
    dst[1] = *reinterpret_cast<const uint4*>(p + prec_stride);
  };

  // split-K (gridDim.z slices, yacc != nullptr): slice z walks chunks [c_lo, c_hi) and writes
  // its inverse-transformed partial rows to slab z of yacc (the inverse FFT is linear); the
  // host only splits when every slice is non-empty
  const int cps = (sl.n_chunk + (int)gridDim.z - 1) / (int)gridDim.z;
  const int c_lo = (int)blockIdx.z * cps;
  const int c_hi = c_lo + cps < sl.n_chunk ? c_lo + cps : sl.n_chunk;
  STAMP(0);
  dma_half(c_lo * KB, 0);
  dma_half(c_lo * KB, 1);

  for (int ch = c_lo; ch < c_hi; ++ch) {
    const int i0 = ch * KB;
    const bool more = ch + 1 < c_hi;
    const int sb = 1 + 6 * (ch & 7);
    STAMP(sb);
    wait_vmcnt<NH>();     // half 0 of this chunk landed (half 1 may still be in flight) ...
    lds_barrier();        // ... for every wave; the previous chunk's MFMAs are done with xl
    STAMP(sb + 1);
    fft_half(0);
    STAMP(sb + 2);
    wait_vmcnt<0>();      // half 1 landed (no other VMEM is outstanding here)
    lds_barrier();        // every wave is done with stage half 0
    STAMP(sb + 3);
    if (more) dma_half(i0 + KB, 0);
    uint4 bring[RING][2];
#pragma unroll
    for (int s = 0; s < RING; ++s) load_b(ch, s, bring[s]);   // behind the DMA: waits stay exact
    fft_half(1);
    STAMP(sb + 4);
    lds_barrier();        // split-X image complete
    STAMP(sb + 5);

    // ---- MFMA complex MAC over the chunk's 8 blocks
    uint4 afrag;
#pragma unroll
    for (int s = 0; s < STEPS; ++s) {
      const int fb = s / NTL, nt = s % NTL;
      const int f = wave * BPW + fb;
      if (nt == 0) {
        const int t = row >> 1;
        uint4 raw = *reinterpret_cast<const uint4*>(xl + f * XS + (a_prec * TT + t) * KB + a_half * 4);
        if (f == 0) {
          raw.x &= a_bin0; raw.y &= a_bin0; raw.z &= a_bin0; raw.w &= a_bin0;
        } else {
          raw.x = __builtin_amdgcn_perm(raw.x, raw.x, a_sel) ^ a_xor;
          raw.y = __builtin_amdgcn_perm(raw.y, raw.y, a_sel) ^ a_xor;
          raw.z = __builtin_amdgcn_perm(raw.z, raw.z, a_sel) ^ a_xor;
          raw.w = __builtin_amdgcn_perm(raw.w, raw.w, a_sel) ^ a_xor;
        }
        afrag = raw;
      }
      uint4 bcur[2] = {bring[s % RING][0], bring[s % RING][1]};
      if (s + RING < STEPS && !ABLATE(2)) load_b(ch, s + RING, bring[s % RING]);
      if (ABLATE(1)) {   // keep the operands live, skip the MFMAs
        asm volatile("" :: "v"(bcur[0].x), "v"(bcur[1].x), "v"(afrag.x));
        continue;
      }
      const bf16x8 a = __builtin_bit_cast(bf16x8, afrag);
      acc[fb][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, __builtin_bit_cast(bf16x8, bcur[0]), acc[fb][nt], 0, 0, 0);
      acc[fb][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, __builtin_bit_cast(bf16x8, bcur[1]), acc[fb][nt], 0, 0, 0);
    }
    if (more) dma_half(i0 + KB, 1);   // after the last B-fragment wait: lands under the next FFTs
  }

  STAMP(49);
  // ---- epilogue, one 16-output N-tile per round (no DMA is in flight any more). D layout:
  //      col = lane & 15 (output), row = 4*(lane >> 4) + r -> token 2*(lane >> 4) + (r >> 1),
  //      part r & 1. LDS row R = o_local*TT + t holds bin f at complex column f ^ o_local.
#pragma unroll
  for (int nt = 0; nt < NTL; ++nt) {
    __syncthreads();
#pragma unroll
    for (int fb = 0; fb < BPW; ++fb) {
      const int f = wave * BPW + fb;
      const int R = row * TT + 2 * kb;
      const f32x4 a = acc[fb][nt];
      float* p = stage + R * SROW + 2 * (f ^ row);
      *reinterpret_cast<float2*>(p) = make_float2(a[0], a[1]);
      *reinterpret_cast<float2*>(p + SROW) = make_float2(a[2], a[3]);
    }
    __syncthreads();
    STAMP(50 + 2 * nt);
#pragma unroll 1
    for (int u2 = 0; u2 < G::EPI_ROWS / G::NGROUPS; ++u2) {
      const int R = g + G::NGROUPS * u2;
      const int ol = R / TT, t = R % TT;
      const int o = o_base + 16 * nt + ol;
      float* rowp = stage + R * SROW;
      if (!ABLATE(8)) F::inverse(rowp, gl, tw, ol);
      const int64_t tok = t0 + t;
      if (tok < n_tokens && o < n_out) {
        if (yacc)
          F::store_partial(rowp, gl, yacc + ((int64_t)blockIdx.z * n_tokens + tok) * M + (int64_t)o * B);
        else
          F::template store<XT, YF32>(rowp, gl, yv, tok * M + (int64_t)o * B, bias, (int64_t)o * B, bias_dt);
      }
    }
    STAMP(51 + 2 * nt);
  }
}

// split-K finish: y = slab 0 + slab 1 + ... (fixed order: bit-reproducible) with the epilogue's
// roundings and bias (store4, the same code as the unsplit epilogue). One thread per 4 outputs;
// M is a multiple of b >= 32.
template <int XT, bool YF32>
__global__ void bc_splitk_finish_kernel(const float* __restrict__ acc, int kz, int64_t n_quads, int64_t M,
                                        const void* __restrict__ bias, int bias_dt, void* __restrict__ yv) {
  const int64_t slab = n_quads * 4;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n_quads;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e0 = q * 4;
    float4 a = *reinterpret_cast<const float4*>(acc + e0);
    for (int z = 1; z < kz; ++z) {
      const float4 b = *reinterpret_cast<const float4*>(acc + z * slab + e0);
      a = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
    }
    store4<XT, YF32>(a, yv, e0, bias, e0 % M, bias_dt);
  }
}

// ================================================================== spectra kernels
// Packed spectra of the OPERATOR (n_out x n_in blocks; transpose_conj: the adjoint built
// from c's (n_in x n_out) grid): one thread per packed bin, direct DFT in fp64, 1/(2b).
template <int B>
__global__ void bc_spectra_kernel(const void* __restrict__ c, int c_dt, int n_out, int n_in,
                                  int transpose_conj, float2* __restrict__ spec) {
  constexpr int H = B / 2;
  const int64_t blk = blockIdx.x;            // operator (o, i) pair
  const int k = threadIdx.x;
  if (blk < (int64_t)n_out * n_in && k < H) {
    const int o = (int)(blk / n_in), i = (int)(blk % n_in);
    // c is (n_out, n_in, B) for the plain operator and (n_in, n_out, B) for the adjoint
    const int64_t base = (transpose_conj ? ((int64_t)i * n_out + o) : blk) * B;
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
    spec[blk * H + k] = out;
  }
  if (blk == 0) {
    const int64_t tw_off = spec_layout(n_out, n_in, B).tw_off_f2;
    for (int m = threadIdx.x; m < B; m += blockDim.x) {
      double s, co;
      sincospi(2.0 * (double)m / (double)B, &s, &co);
      spec[tw_off + m] = make_float2((float)co, (float)(-s));
    }
  }
}

// MFMA image from the packed spectra (one thread per image dword pair hi/lo)
template <int B>
__global__ void bc_mfma_image_kernel(int n_out, int n_in, float2* __restrict__ spec) {
  constexpr int H = B / 2;
  const SpecLayout sl = spec_layout(n_out, n_in, B);
  uint32_t* img = reinterpret_cast<uint32_t*>(spec) + sl.img_off_u32;
  const int64_t per_prec = (int64_t)sl.n_out_pad * 8;
  const int64_t total = (int64_t)sl.n_chunk * H * per_prec;   // (c, f, o, j) quadruples
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int j = (int)(idx & 7);
    const int o = (int)((idx >> 3) % sl.n_out_pad);
    const int64_t cf = (idx >> 3) / sl.n_out_pad;
    const int f = (int)(cf % H), c = (int)(cf / H);
    const int i = 8 * c + j;
    float2 v = make_float2(0.f, 0.f);
    if (o < n_out && i < n_in) {
      v = spec[((int64_t)o * n_in + i) * H + f];
      if (f != 0) v.y = -v.y;                 // conj(C); bin 0 keeps (C0, C_H)
    }
    uint32_t hi, lo;
    split_bf16(v, hi, lo);
    const int64_t d = ((int64_t)(c * H + f) * 2) * per_prec + (int64_t)o * 8 + j;
    img[d] = hi;
    img[d + per_prec] = lo;
  }
}

// ================================================================== circulant matvec
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
thread_local char g_last_detail[256] = {0};     // why the last call was refused (engine, geometry)

const char* dt_name(int d) {
  return d == BCFFT_F32 ? "fp32" : d == BCFFT_F16 ? "fp16" : d == BCFFT_BF16 ? "bf16" : d == BCFFT_NONE ? "none" : "?";
}
const char* algo_name(int a) {
  switch (a) {
    case BCFFT_ALGO_AUTO: return "auto";
    case BCFFT_ALGO_MFMA: return "mfma";
    case BCFFT_ALGO_VALU: return "valu";
    case BCFFT_ALGO_STAT: return "stationary";
    case BCFFT_ALGO_DFT: return "dft";
    case BCFFT_ALGO_DFTX: return "dftx";
    case BCFFT_ALGO_DFTP: return "dftp";
    case BCFFT_ALGO_SHORT: return "short";
    default: return "?";
  }
}
// BCFFT_ERR_BLOCK with the refused engine and geometry in bcfft_last_error_detail()
int refuse(const char* what, int algo, int n_in, int b, int xdt, int ydt) {
  snprintf(g_last_detail, sizeof(g_last_detail),
           "%s: engine '%s' does not serve block_size %d with %d input blocks (in_features %d), x %s -> y %s",
           what, algo_name(algo), b, n_in, n_in * b, dt_name(xdt), dt_name(ydt));
  return BCFFT_ERR_BLOCK;
}

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
// K-slices of the MFMA kernel. One workgroup walks every chunk of 8 input blocks for its 8 tokens,
// so a grid of fewer 8-token rows than CUs (LLaMA's down projection at prefill and decode sizes)
// takes one whole walk regardless of N. Such grids split the chunks over kz >= 2 slices, as many
// as fill two workgroups per CU, with >= 2 chunks per slice (each slice also pays the inverse
// transforms and stores); no split below 4 chunks. Independent of n_out, so a fused launch
// (q/k/v) splits exactly like its parts. kz is rounded so that no slice is empty.
// rows = workgroup rows of the unsplit grid, slots = resident workgroups per CU, min_chunks =
// chunks per slice at least (a slice also pays the inverse transforms and stores: 2 measured
// best for the MFMA kernel, 1 for the VALU kernel; profiles/r01_splitk_timing.jsonl)
int ksplit_rows(int64_t rows, int n_chunks, int slots, int min_chunks) {
  const int64_t cus = bcfft::device_cu_count();
  if (n_chunks < 4 || rows >= cus || 2 * rows > slots * cus) return 1;
  int64_t kz = slots * cus / rows;
  const int64_t kmax = (n_chunks + min_chunks - 1) / min_chunks;
  if (kz > kmax) kz = kmax;
  if (kz < 2) kz = 2;
  const int64_t cps = (n_chunks + kz - 1) / kz;
  return (int)((n_chunks + cps - 1) / cps);
}
int mfma_ksplit(int64_t n, int n_in, int b) {
  if (b > bcfft::BCFFT_MFMA_MAXB || n <= 0) return 1;
  // one chunk per slice pays at decode sizes (<= 4 rows: 24.0 vs 27.7 us at N = 20), two above
  // (35.1 vs 37.3 us at N = 256)
  const int64_t rows = (n + 7) / 8;
  return ksplit_rows(rows, (n_in + 7) / 8, 2, rows <= 4 ? 1 : 2);
}
// the VALU kernel: 16-token rows, chunks of 64 / L input blocks (bcfft::GeoV<B>::IC); its LDS
// allows two workgroups per CU at b = 128, one at b = 64 and 256 (b = 32 is counted as one)
int valu_ksplit(int64_t n, int n_in, int b) {
  if (n <= 0) return 1;
  const int ic = 512 / (b / 2 <= 32 ? 4 : 8) / 16;
  return ksplit_rows((n + 15) / 16, (n_in + ic - 1) / ic, b == 128 ? 2 : 1, 1);
}

template <int XT, bool YF32>
void launch_finish(const float* ws, int kz, int64_t n, int64_t m, const void* bias, int bias_dt, void* y,
                   hipStream_t s) {
  const int64_t quads = n * m / 4;
  const unsigned blocks = (unsigned)((quads + 255) / 256 < 65535 ? (quads + 255) / 256 : 65535);
  hipLaunchKernelGGL((bcfft::bc_splitk_finish_kernel<XT, YF32>), dim3(blocks), dim3(256), 0, s, ws, kz, quads,
                     m, bias, bias_dt, y);
}

template <int B, int XT, bool YF32>
void launch_forward(int algo, const void* x, int64_t n, int n_in, int n_out, const void* spec,
                    const void* bias, int bias_dt, void* y, float* ws, hipStream_t s) {
  if constexpr (B <= bcfft::BCFFT_MFMA_MAXB) {
    if (algo == BCFFT_ALGO_MFMA) {
      using G = bcfft::GeoM<B>;
      const int kz = ws ? mfma_ksplit(n, n_in, B) : 1;
      dim3 grid((unsigned)((n + G::TT - 1) / G::TT), (unsigned)((n_out + G::OUT_PER_WG - 1) / G::OUT_PER_WG),
                (unsigned)kz);
      const int64_t m = (int64_t)n_out * B;
      hipLaunchKernelGGL((bcfft::bc_forward_mfma_kernel<B, XT, YF32>), grid, dim3(G::NT), 0, s, x, n,
                         n_in, n_out, (const float2*)spec, bias, bias_dt, y, kz > 1 ? ws : nullptr);
      if (kz > 1) launch_finish<XT, YF32>(ws, kz, n, m, bias, bias_dt, y, s);
      return;
    }
  }
  using G = bcfft::GeoV<B>;
  static_assert(G::IC == 512 / (B / 2 <= 32 ? 4 : 8) / 16, "valu_ksplit's chunk size");
  const int kz = ws ? valu_ksplit(n, n_in, B) : 1;
  dim3 grid((unsigned)((n + G::TT - 1) / G::TT), (unsigned)((n_out + G::OUT_PER_WG - 1) / G::OUT_PER_WG),
            (unsigned)kz);
  hipLaunchKernelGGL((bcfft::bc_forward_valu_kernel<B, XT, YF32>), grid, dim3(G::NT), 0, s, x, n, n_in,
                     n_out, (const float2*)spec, bias, bias_dt, y, kz > 1 ? ws : nullptr);
  if (kz > 1) launch_finish<XT, YF32>(ws, kz, n, (int64_t)n_out * B, bias, bias_dt, y, s);
}

template <int B>
void launch_forward_b(int algo, int xdt, const void* x, int64_t n, int n_in, int n_out,
                      const void* spec, const void* bias, int bias_dt, void* y, int y_dt, float* ws,
                      hipStream_t s) {
  // y dtype = promote(x dtype, bias dtype): the x dtype, or fp32 for 16-bit x with another bias dtype
  const bool yf32 = y_dt == BCFFT_F32;
  if (xdt == BCFFT_F32) launch_forward<B, BCFFT_F32, true>(algo, x, n, n_in, n_out, spec, bias, bias_dt, y, ws, s);
  else if (xdt == BCFFT_F16 && yf32) launch_forward<B, BCFFT_F16, true>(algo, x, n, n_in, n_out, spec, bias, bias_dt, y, ws, s);
  else if (xdt == BCFFT_F16) launch_forward<B, BCFFT_F16, false>(algo, x, n, n_in, n_out, spec, bias, bias_dt, y, ws, s);
  else if (yf32) launch_forward<B, BCFFT_BF16, true>(algo, x, n, n_in, n_out, spec, bias, bias_dt, y, ws, s);
  else launch_forward<B, BCFFT_BF16, false>(algo, x, n, n_in, n_out, spec, bias, bias_dt, y, ws, s);
}

template <int B>
void launch_spectra(const void* c, int c_dt, int n_out, int n_in, int tc, float2* out, hipStream_t s) {
  const unsigned nblk = (unsigned)((int64_t)n_out * n_in);
  const unsigned threads = (B / 2) < 64 ? 64u : (unsigned)(B / 2);
  hipLaunchKernelGGL(bcfft::bc_spectra_kernel<B>, dim3(nblk), dim3(threads), 0, s, c, c_dt,
                     n_out, n_in, tc, out);
  if constexpr (B <= bcfft::BCFFT_MFMA_MAXB) {
    const bcfft::SpecLayout sl = bcfft::spec_layout(n_out, n_in, B);
    const int64_t total = sl.img_u32 / 2;
    const unsigned blocks = (unsigned)((total + 255) / 256 < 65535 ? (total + 255) / 256 : 65535);
    hipLaunchKernelGGL(bcfft::bc_mfma_image_kernel<B>, dim3(blocks), dim3(256), 0, s, n_out, n_in, out);
  }
  bcfft::launch_stat_image(B, n_out, n_in, out, s);   // no-op unless stat_eligible
  if (B == 128 && n_in == 32) bcfft::launch_lo8_image(n_out, out, s);   // the precise engine's residual
}
}  // namespace

extern "C" {

int bcfft_abi_version(void) { return BCFFT_ABI_VERSION; }

const char* bcfft_status_string(int status) {
  switch (status) {
    case BCFFT_OK: return "ok";
    case BCFFT_ERR_SHAPE: return "shape error: features must be positive multiples of block_size";
    case BCFFT_ERR_BLOCK: return "block_size / engine not supported for this geometry (block sizes: 32, 64, 128, 256)";
    case BCFFT_ERR_DTYPE: return "unsupported dtype or y dtype != promote(x dtype, bias dtype)";
    case BCFFT_ERR_ALIGN: return "x, y, spectra and bias must be 16-byte aligned";
    case BCFFT_ERR_HIP: return "HIP launch failed";
    case BCFFT_ERR_ARG: return "NULL pointer or invalid argument";
    default: return "unknown status";
  }
}

const char* bcfft_last_hip_error(void) { return g_last_hip_error; }

const char* bcfft_last_error_detail(void) { return g_last_detail; }

int64_t bcfft_spectra_bytes(int n_out_blocks, int n_in_blocks, int block_size) {
  if (n_out_blocks <= 0 || n_in_blocks <= 0 || !valid_block(block_size)) return -1;
  return bcfft::spec_layout(n_out_blocks, n_in_blocks, block_size).total_bytes;
}

int bcfft_spectra(const void* c, int c_dtype, int n_out_blocks, int n_in_blocks, int block_size,
                  int transpose_conj, void* spectra, void* stream) {
  if (!c || !spectra) return BCFFT_ERR_ARG;
  if (!valid_block(block_size)) return BCFFT_ERR_BLOCK;
  if (n_out_blocks <= 0 || n_in_blocks <= 0) return BCFFT_ERR_SHAPE;
  if (!valid_dt(c_dtype)) return BCFFT_ERR_DTYPE;
  if (!aligned16(spectra)) return BCFFT_ERR_ALIGN;
  hipStream_t s = (hipStream_t)stream;
  float2* out = (float2*)spectra;
  const int tc = transpose_conj ? 1 : 0;
  switch (block_size) {
    case 32: launch_spectra<32>(c, c_dtype, n_out_blocks, n_in_blocks, tc, out, s); break;
    case 64: launch_spectra<64>(c, c_dtype, n_out_blocks, n_in_blocks, tc, out, s); break;
    case 128: launch_spectra<128>(c, c_dtype, n_out_blocks, n_in_blocks, tc, out, s); break;
    default: launch_spectra<256>(c, c_dtype, n_out_blocks, n_in_blocks, tc, out, s); break;
  }
  return record_launch();
}

// the algorithm bcfft_forward_algo runs for this geometry (AUTO resolved). xdt = -2: the caller
// did not say (bcfft_forward_workspace_bytes); the I/O-dependent choices are then not taken.
// fp32 outputs take DFTX at b = 128 (its hi + lo products keep the layer linear in x to ~1e-6,
// which fp32 training gradients through dx rely on); 16-bit outputs take the one-term DFT, whose
// noise sits far below their own rounding.
static int resolve_algo(int algo, int n_in, int block_size, int xdt = -2, bool yf32 = true, int64_t n_tokens = -1,
                        int n_out = 0) {
  if (algo != BCFFT_ALGO_AUTO) return algo;
  // short token counts on the STAT geometries: one workgroup per (4-token tile, 16 output blocks)
  // instead of a persistent grid of ceil(N / 4) x groups workgroups (bcfft_sn.hip)
  if (n_tokens >= 0 && n_out > 0 && bcfft::sn_eligible(n_in, block_size) && bcfft::sn_pays(n_tokens, n_out))
    return BCFFT_ALGO_SHORT;
  if (bcfft::dm_eligible(n_in, block_size)) return yf32 ? BCFFT_ALGO_DFTX : BCFFT_ALGO_DFT;
  if (bcfft::dm64_eligible(n_in, block_size, xdt, yf32)) return BCFFT_ALGO_DFT;
  if (bcfft::dm256_eligible(n_in, block_size, xdt, yf32)) return BCFFT_ALGO_DFT;
  // K > 4096 at b = 64 (bf16): the streamed-weight DFT kernel once its 16-token tiles fill a few
  // CUs (N = 64: 36.9 us vs the split-K MFMA kernel's 31.4; N = 1024: 39.5 vs 71.9)
  if (bcfft::dm64k_eligible(n_in, block_size, xdt, yf32) && n_tokens >= bcfft::BCFFT_DM64K_MIN_TOKENS) return BCFFT_ALGO_DFT;
  // K > 4096 at b = 128 (bf16): the streamed-weight DFT kernel, from one token up (it beats the
  // split-K MFMA kernel at every measured N: 20.9 vs 23.4 us at N = 1, profiles/r02_dmk_decode_sizes.log)
  if (bcfft::dmk_eligible(n_in, block_size, xdt, yf32) && n_tokens >= bcfft::BCFFT_DMK_MIN_TOKENS) return BCFFT_ALGO_DFT;
  return bcfft::stat_eligible(n_in, block_size) ? BCFFT_ALGO_STAT
                                                : (block_size <= 128 ? BCFFT_ALGO_MFMA : BCFFT_ALGO_VALU);
}

static int64_t ws_bytes_for(int64_t n_tokens, int in_features, int out_features, int block_size, int algo,
                               int xdt, bool yf32) {
  if (!valid_block(block_size) || n_tokens < 0 || in_features <= 0 || out_features <= 0 ||
      in_features % block_size || out_features % block_size)
    return -1;
  const int n_in = in_features / block_size;
  const int a = resolve_algo(algo, n_in, block_size, xdt, yf32, n_tokens, out_features / block_size);
  // the DFT engines take no workspace, except the down projection's streamed-weight kernel at
  // short grids (its K-chunk split: kz fp32 partial slabs)
  if (a == BCFFT_ALGO_DFT && bcfft::dmk_eligible(in_features / block_size, block_size, xdt, yf32)) {
    const int kz = bcfft::dmk_ksplit(n_tokens, in_features / block_size, out_features / block_size);
    return kz < 2 ? 0 : kz * n_tokens * (int64_t)out_features * (int64_t)sizeof(float);
  }
  if (a == BCFFT_ALGO_DFT || a == BCFFT_ALGO_DFTX || a == BCFFT_ALGO_DFTP || a == BCFFT_ALGO_STAT ||
      a == BCFFT_ALGO_SHORT)
    return 0;
  int kz = 1;
  if (a == BCFFT_ALGO_MFMA && block_size <= bcfft::BCFFT_MFMA_MAXB) kz = mfma_ksplit(n_tokens, n_in, block_size);
  else if (a == BCFFT_ALGO_VALU || a == BCFFT_ALGO_MFMA) kz = valu_ksplit(n_tokens, n_in, block_size);
  if (kz < 2) return 0;
  return kz * n_tokens * (int64_t)out_features * (int64_t)sizeof(float);   // one fp32 slab per slice
}

int64_t bcfft_forward_workspace_bytes(int64_t n_tokens, int in_features, int out_features, int block_size,
                                      int algo) {
  return ws_bytes_for(n_tokens, in_features, out_features, block_size, algo, -2, true);
}

int64_t bcfft_forward_workspace_bytes_io(int64_t n_tokens, int in_features, int out_features, int block_size,
                                         int algo, int x_dtype, int y_dtype) {
  if (!valid_dt(x_dtype) || !valid_dt(y_dtype)) return -1;
  return ws_bytes_for(n_tokens, in_features, out_features, block_size, algo, x_dtype, y_dtype == BCFFT_F32);
}

int bcfft_forward_ws(const void* x, int x_dtype, int64_t n_tokens, int in_features,
                     int out_features, int block_size, const void* spectra, const void* bias,
                     int bias_dtype, void* y, int y_dtype, int algo, void* workspace,
                     int64_t workspace_bytes, void* stream) {
  g_last_detail[0] = 0;
  if (!valid_block(block_size)) return refuse("bcfft_forward", algo, 0, block_size, x_dtype, y_dtype);
  if (n_tokens < 0 || in_features <= 0 || out_features <= 0 || in_features % block_size ||
      out_features % block_size)
    return BCFFT_ERR_SHAPE;
  if (!valid_dt(x_dtype) || !valid_dt(y_dtype) || (bias_dtype != BCFFT_NONE && !valid_dt(bias_dtype)))
    return BCFFT_ERR_DTYPE;
  if (y_dtype != promote(x_dtype, bias_dtype)) return BCFFT_ERR_DTYPE;
  if ((bias == nullptr) != (bias_dtype == BCFFT_NONE)) return BCFFT_ERR_ARG;
  if (algo < BCFFT_ALGO_AUTO || algo > BCFFT_ALGO_SHORT) return BCFFT_ERR_ARG;
  if (n_tokens == 0) return BCFFT_OK;
  if (!x || !y || !spectra) return BCFFT_ERR_ARG;
  if (!aligned16(x) || !aligned16(y) || !aligned16(spectra) || (bias && !aligned16(bias)) ||
      (workspace && !aligned16(workspace)))
    return BCFFT_ERR_ALIGN;
  const int n_in = in_features / block_size, n_out = out_features / block_size;
  const bool stat_ok = bcfft::stat_eligible(n_in, block_size);
  if (algo == BCFFT_ALGO_STAT && !stat_ok) return refuse("bcfft_forward", algo, n_in, block_size, x_dtype, y_dtype);
  if (algo == BCFFT_ALGO_SHORT && !bcfft::sn_eligible(n_in, block_size))
    return refuse("bcfft_forward", algo, n_in, block_size, x_dtype, y_dtype);
  const bool dm64 = bcfft::dm64_eligible(n_in, block_size, x_dtype, y_dtype == BCFFT_F32);
  if ((algo == BCFFT_ALGO_DFTX || algo == BCFFT_ALGO_DFTP) && !bcfft::dm_eligible(n_in, block_size))
    return refuse("bcfft_forward", algo, n_in, block_size, x_dtype, y_dtype);
  const bool dmk = bcfft::dmk_eligible(n_in, block_size, x_dtype, y_dtype == BCFFT_F32);
  const bool dm256 = bcfft::dm256_eligible(n_in, block_size, x_dtype, y_dtype == BCFFT_F32);
  const bool dm64k = bcfft::dm64k_eligible(n_in, block_size, x_dtype, y_dtype == BCFFT_F32);
  if (algo == BCFFT_ALGO_DFT && !bcfft::dm_eligible(n_in, block_size) && !dm64 && !dmk && !dm256 && !dm64k)
    return refuse("bcfft_forward", algo, n_in, block_size, x_dtype, y_dtype);
  algo = resolve_algo(algo, n_in, block_size, x_dtype, y_dtype == BCFFT_F32, n_tokens, n_out);
  // the workspace is used only when it is as large as bcfft_forward_workspace_bytes_io asks
  const int64_t need = ws_bytes_for(n_tokens, in_features, out_features, block_size, algo, x_dtype,
                                       y_dtype == BCFFT_F32);
  float* ws = (workspace && need > 0 && workspace_bytes >= need) ? (float*)workspace : nullptr;
  hipStream_t s = (hipStream_t)stream;
  if (algo == BCFFT_ALGO_SHORT) {
    // eligibility was checked by resolve_algo; a launcher that still declines (a future geometry or
    // dtype rule out of step with it) must not report BCFFT_OK over an unwritten y
    if (!bcfft::launch_forward_sn(block_size, n_in, x_dtype, y_dtype == BCFFT_F32, x, n_tokens, n_out, spectra, bias,
                                  bias_dtype, y, s))
      return refuse("bcfft_forward", algo, n_in, block_size, x_dtype, y_dtype);
    return record_launch();
  }
  if (algo == BCFFT_ALGO_DFT && dmk) {
    if (ws) bcfft::launch_forward_dmk_split(x, n_tokens, n_in, n_out, spectra, bias, bias_dtype, y, ws,
                                            bcfft::dmk_ksplit(n_tokens, n_in, n_out), s);
    else bcfft::launch_forward_dmk(x, n_tokens, n_in, n_out, spectra, bias, bias_dtype, y, s);
    return record_launch();
  }
  if (algo == BCFFT_ALGO_DFT && dm256) {
    bcfft::launch_forward_dm256(x, n_tokens, n_in, n_out, spectra, bias, bias_dtype, y, s);
    return record_launch();
  }
  if (algo == BCFFT_ALGO_DFT && dm64k) {
    bcfft::launch_forward_dm64k(x, n_tokens, n_in, n_out, spectra, bias, bias_dtype, y, s);
    return record_launch();
  }
  if (algo == BCFFT_ALGO_DFT && block_size == 64) {
    bcfft::launch_forward_dm64(x, n_tokens, n_out, spectra, bias, bias_dtype, y, false, s);
    return record_launch();
  }
  if (algo == BCFFT_ALGO_DFT || algo == BCFFT_ALGO_DFTX || algo == BCFFT_ALGO_DFTP) {
    bcfft::launch_forward_dm(block_size, n_in, x_dtype, y_dtype == BCFFT_F32,
                             algo == BCFFT_ALGO_DFTP ? 2 : algo == BCFFT_ALGO_DFTX ? 1 : 0, x, n_tokens,
                             n_out, spectra, bias, bias_dtype, y, s);
    return record_launch();
  }
  if (algo == BCFFT_ALGO_STAT) {
    bcfft::launch_forward_stat(block_size, n_in, x_dtype, y_dtype == BCFFT_F32, x, n_tokens, n_out,
                               spectra, bias, bias_dtype, y, s);
    return record_launch();
  }
  switch (block_size) {
    case 32: launch_forward_b<32>(algo, x_dtype, x, n_tokens, n_in, n_out, spectra, bias, bias_dtype, y, y_dtype, ws, s); break;
    case 64: launch_forward_b<64>(algo, x_dtype, x, n_tokens, n_in, n_out, spectra, bias, bias_dtype, y, y_dtype, ws, s); break;
    case 128: launch_forward_b<128>(algo, x_dtype, x, n_tokens, n_in, n_out, spectra, bias, bias_dtype, y, y_dtype, ws, s); break;
    default: launch_forward_b<256>(algo, x_dtype, x, n_tokens, n_in, n_out, spectra, bias, bias_dtype, y, y_dtype, ws, s); break;
  }
  return record_launch();
}

// The engine and kernel bcfft_forward_ws runs for these arguments (with the workspace that
// bcfft_forward_workspace_bytes_io asks for): the same refusals, resolve_algo, and each launcher's
// own choice between its per-group, multi-group and split forms. Host logic only (no launch).
static int forward_plan(int64_t n_tokens, int in_features, int out_features, int block_size, int algo, int x_dtype,
                        int y_dtype, const char** kernel) {
  *kernel = "";
  if (!valid_block(block_size) || n_tokens < 0 || in_features <= 0 || out_features <= 0 ||
      in_features % block_size || out_features % block_size)
    return -1;
  if (!valid_dt(x_dtype) || !valid_dt(y_dtype)) return -1;
  if (algo < BCFFT_ALGO_AUTO || algo > BCFFT_ALGO_SHORT) return -1;
  const int n_in = in_features / block_size, n_out = out_features / block_size;
  const bool yf32 = y_dtype == BCFFT_F32;
  const bool dm = bcfft::dm_eligible(n_in, block_size);
  const bool dm64 = bcfft::dm64_eligible(n_in, block_size, x_dtype, yf32);
  const bool dmk = bcfft::dmk_eligible(n_in, block_size, x_dtype, yf32);
  const bool dm256 = bcfft::dm256_eligible(n_in, block_size, x_dtype, yf32);
  const bool dm64k = bcfft::dm64k_eligible(n_in, block_size, x_dtype, yf32);
  if (algo == BCFFT_ALGO_STAT && !bcfft::stat_eligible(n_in, block_size)) return -1;
  if (algo == BCFFT_ALGO_SHORT && !bcfft::sn_eligible(n_in, block_size)) return -1;
  if ((algo == BCFFT_ALGO_DFTX || algo == BCFFT_ALGO_DFTP) && !dm) return -1;
  if (algo == BCFFT_ALGO_DFT && !dm && !dm64 && !dmk && !dm256 && !dm64k) return -1;
  int a = resolve_algo(algo, n_in, block_size, x_dtype, yf32, n_tokens, n_out);
  // the precise engine serves fp32 outputs (launch_forward_dm runs DFTX for 16-bit outputs, and for
  // a 16-bit bias on 16-bit x, which this query does not see: bcfft.h)
  if (a == BCFFT_ALGO_DFTP && !bcfft::dftp_serves(x_dtype, yf32, BCFFT_NONE)) a = BCFFT_ALGO_DFTX;
  if (a == BCFFT_ALGO_SHORT) *kernel = "bc_forward_sn_kernel";
  else if (a == BCFFT_ALGO_DFT && dmk) *kernel = "bc_forward_dmk_kernel";
  else if (a == BCFFT_ALGO_DFT && dm256) *kernel = bcfft::dm256_kernel_name(n_tokens, n_in, n_out);
  else if (a == BCFFT_ALGO_DFT && dm64k) *kernel = "bc_forward_dm64k_kernel";
  else if (a == BCFFT_ALGO_DFT && block_size == 64)
    *kernel = bcfft::dm64g_eligible(64, 64, BCFFT_BF16, false, n_out, false) && bcfft::multigroup_pays(n_tokens, 4)
                  ? "bc_forward_dm64g_kernel" : "bc_forward_dm64_kernel";
  else if (a == BCFFT_ALGO_DFT && bcfft::dm8_eligible(n_in, block_size, x_dtype, yf32))
    *kernel = bcfft::dmg_eligible(n_in, block_size, x_dtype, yf32, n_out, false) && bcfft::multigroup_pays(n_tokens, 3)
                  ? "bc_forward_dmg_kernel" : "bc_forward_dm8_kernel";
  else if (a == BCFFT_ALGO_DFT || a == BCFFT_ALGO_DFTX || a == BCFFT_ALGO_DFTP) *kernel = "bc_forward_dm_kernel";
  else if (a == BCFFT_ALGO_STAT) *kernel = "bc_forward_stat_kernel";
  else if (a == BCFFT_ALGO_MFMA && block_size <= bcfft::BCFFT_MFMA_MAXB) *kernel = "bc_forward_mfma_kernel";
  else *kernel = "bc_forward_valu_kernel";
  return a;
}

int bcfft_forward_resolve(int64_t n_tokens, int in_features, int out_features, int block_size, int algo, int x_dtype,
                          int y_dtype) {
  const char* k;
  return forward_plan(n_tokens, in_features, out_features, block_size, algo, x_dtype, y_dtype, &k);
}

const char* bcfft_forward_kernel_name(int64_t n_tokens, int in_features, int out_features, int block_size, int algo,
                                      int x_dtype, int y_dtype) {
  const char* k;
  forward_plan(n_tokens, in_features, out_features, block_size, algo, x_dtype, y_dtype, &k);
  return k;
}

int bcfft_forward_algo(const void* x, int x_dtype, int64_t n_tokens, int in_features,
                       int out_features, int block_size, const void* spectra, const void* bias,
                       int bias_dtype, void* y, int y_dtype, int algo, void* stream) {
  return bcfft_forward_ws(x, x_dtype, n_tokens, in_features, out_features, block_size, spectra, bias,
                          bias_dtype, y, y_dtype, algo, nullptr, 0, stream);
}

int bcfft_forward_glu_algo(const void* x, int x_dtype, int64_t n_tokens, int in_features, int gate_features,
                           int block_size, const void* spectra_gu, void* h, int algo, void* stream) {
  g_last_detail[0] = 0;
  if (algo != BCFFT_ALGO_AUTO && algo != BCFFT_ALGO_STAT && algo != BCFFT_ALGO_DFT && algo != BCFFT_ALGO_DFTX &&
      algo != BCFFT_ALGO_DFTP)
    return BCFFT_ERR_ARG;
  if (!valid_block(block_size)) return refuse("bcfft_forward_glu", algo, 0, block_size, x_dtype, x_dtype);
  if (n_tokens < 0 || in_features <= 0 || gate_features <= 0 || in_features % block_size ||
      gate_features % block_size)
    return BCFFT_ERR_SHAPE;
  if (!valid_dt(x_dtype)) return BCFFT_ERR_DTYPE;
  const int n_in = in_features / block_size, n_gate = gate_features / block_size;
  const bool g256 = bcfft::dm256_glu_eligible(n_in, block_size, x_dtype, n_gate);   // b = 256, K = 4096, bf16
  if (!bcfft::stat_eligible(n_in, block_size) && !g256)
    return refuse("bcfft_forward_glu", algo, n_in, block_size, x_dtype, x_dtype);
  if (g256) {
    if (algo != BCFFT_ALGO_AUTO && algo != BCFFT_ALGO_DFT)
      return refuse("bcfft_forward_glu", algo, n_in, block_size, x_dtype, x_dtype);
    if (n_tokens == 0) return BCFFT_OK;
    if (!x || !h || !spectra_gu) return BCFFT_ERR_ARG;
    if (!aligned16(x) || !aligned16(h) || !aligned16(spectra_gu)) return BCFFT_ERR_ALIGN;
    bcfft::launch_forward_dm256_glu(x, n_tokens, n_gate, spectra_gu, h, (hipStream_t)stream);
    return record_launch();
  }
  const bool dm = bcfft::dm_eligible(n_in, block_size);
  const bool dm64 = bcfft::dm64_eligible(n_in, block_size, x_dtype, false);   // h has x's dtype
  // AUTO: fp32 h takes the hi + lo products (DFTX), as bcfft_forward does for fp32 outputs
  if (algo == BCFFT_ALGO_AUTO)
    algo = dm ? (x_dtype == BCFFT_F32 ? BCFFT_ALGO_DFTX : BCFFT_ALGO_DFT) : dm64 ? BCFFT_ALGO_DFT : BCFFT_ALGO_STAT;
  if ((algo == BCFFT_ALGO_DFTX || algo == BCFFT_ALGO_DFTP) && !dm)
    return refuse("bcfft_forward_glu", algo, n_in, block_size, x_dtype, x_dtype);
  if (algo == BCFFT_ALGO_DFT && !dm && !dm64)
    return refuse("bcfft_forward_glu", algo, n_in, block_size, x_dtype, x_dtype);
  if (n_tokens == 0) return BCFFT_OK;
  if (!x || !h || !spectra_gu) return BCFFT_ERR_ARG;
  if (!aligned16(x) || !aligned16(h) || !aligned16(spectra_gu)) return BCFFT_ERR_ALIGN;
  if (algo == BCFFT_ALGO_STAT)
    bcfft::launch_forward_glu(block_size, n_in, x_dtype, x, n_tokens, n_gate, spectra_gu, h, (hipStream_t)stream);
  else if (block_size == 64)
    bcfft::launch_forward_dm64(x, n_tokens, n_gate, spectra_gu, nullptr, BCFFT_NONE, h, true, (hipStream_t)stream);
  else
    bcfft::launch_forward_dm_glu(block_size, n_in, x_dtype,
                                 algo == BCFFT_ALGO_DFTP ? 2 : algo == BCFFT_ALGO_DFTX ? 1 : 0, x, n_tokens, n_gate, spectra_gu,
                                 h, (hipStream_t)stream);
  return record_launch();
}

int bcfft_forward_glu(const void* x, int x_dtype, int64_t n_tokens, int in_features, int gate_features,
                      int block_size, const void* spectra_gu, void* h, void* stream) {
  return bcfft_forward_glu_algo(x, x_dtype, n_tokens, in_features, gate_features, block_size, spectra_gu, h,
                                BCFFT_ALGO_AUTO, stream);
}

// the fused BC-MLP's resolved mode: FUSED_SPLITK where bcfft_dmm.hip serves the geometry at a
// short grid (bcfft::dmm_ksplit >= 2); FUSED where its tiles fill the CUs (bcfft::dmm_pays); else
// SPLIT. Explicit modes are kept (a FUSED_SPLITK that would not
// split runs as FUSED). < 0 for invalid arguments.
static int mlp_mode(int64_t n_tokens, int hidden_features, int inter_features, int block_size, int x_dtype, int mode) {
  if (mode != BCFFT_MLP_AUTO && mode != BCFFT_MLP_FUSED && mode != BCFFT_MLP_SPLIT && mode != BCFFT_MLP_FUSED_SPLITK)
    return -1;
  if (!valid_block(block_size) || !valid_dt(x_dtype) || n_tokens < 0 || hidden_features <= 0 || inter_features <= 0 ||
      hidden_features % block_size || inter_features % block_size)
    return -1;
  const int n_hid = hidden_features / block_size, n_h = inter_features / block_size;
  const bool ok = bcfft::dmm_eligible(n_hid, block_size, x_dtype, n_h, n_hid);
  const bool splits = ok && bcfft::dmm_ksplit(n_tokens, n_h) >= 2;
  // AUTO: the group split wherever it applies (measured faster than the one launch up to its limit
  // of half the CUs' worth of tiles: N = 1024 49.6 vs 56.7 us, N = 20 20.9 vs 52.0;
  // profiles/r03p_mlp_time.log), the one launch where its tiles fill the CUs, else two launches
  if (mode == BCFFT_MLP_AUTO)
    return !ok ? BCFFT_MLP_SPLIT
               : splits ? BCFFT_MLP_FUSED_SPLITK : bcfft::dmm_pays(n_tokens) ? BCFFT_MLP_FUSED : BCFFT_MLP_SPLIT;
  if (mode == BCFFT_MLP_FUSED_SPLITK && ok && !splits) return BCFFT_MLP_FUSED;
  return mode;
}

static int64_t dt_bytes(int dt) { return dt == BCFFT_F32 ? 4 : 2; }

int bcfft_forward_mlp_mode(int64_t n_tokens, int hidden_features, int inter_features, int block_size, int x_dtype,
                           int mode) {
  return mlp_mode(n_tokens, hidden_features, inter_features, block_size, x_dtype, mode);
}

int64_t bcfft_forward_mlp_workspace_bytes(int64_t n_tokens, int hidden_features, int inter_features, int block_size,
                                          int x_dtype, int mode) {
  const int m = mlp_mode(n_tokens, hidden_features, inter_features, block_size, x_dtype, mode);
  if (m < 0) return -1;
  if (m == BCFFT_MLP_FUSED) return 0;
  if (m == BCFFT_MLP_FUSED_SPLITK)
    return (int64_t)bcfft::dmm_ksplit(n_tokens, inter_features / block_size) * n_tokens * hidden_features * 4;
  return (n_tokens * (int64_t)inter_features * dt_bytes(x_dtype) + 15) / 16 * 16;   // h
}

int bcfft_forward_mlp(const void* x, int x_dtype, int64_t n_tokens, int hidden_features, int inter_features,
                      int block_size, const void* spectra_gu, const void* spectra_down, void* y, int mode,
                      void* workspace, int64_t workspace_bytes, void* stream) {
  g_last_detail[0] = 0;
  if (mode != BCFFT_MLP_AUTO && mode != BCFFT_MLP_FUSED && mode != BCFFT_MLP_SPLIT && mode != BCFFT_MLP_FUSED_SPLITK)
    return BCFFT_ERR_ARG;
  if (!valid_block(block_size)) return refuse("bcfft_forward_mlp", BCFFT_ALGO_AUTO, 0, block_size, x_dtype, x_dtype);
  if (n_tokens < 0 || hidden_features <= 0 || inter_features <= 0 || hidden_features % block_size ||
      inter_features % block_size)
    return BCFFT_ERR_SHAPE;
  if (!valid_dt(x_dtype)) return BCFFT_ERR_DTYPE;
  const int n_hid = hidden_features / block_size, n_h = inter_features / block_size;
  const int m = mlp_mode(n_tokens, hidden_features, inter_features, block_size, x_dtype, mode);
  if ((m == BCFFT_MLP_FUSED || m == BCFFT_MLP_FUSED_SPLITK) && !bcfft::dmm_eligible(n_hid, block_size, x_dtype, n_h, n_hid)) {
    snprintf(g_last_detail, sizeof(g_last_detail),
             "bcfft_forward_mlp: the fused kernel serves bf16, block_size 128, hidden 4096 and intermediate "
             "4224..16256; got block_size %d, hidden %d, intermediate %d, x %s",
             block_size, hidden_features, inter_features, dt_name(x_dtype));
    return BCFFT_ERR_BLOCK;
  }
  if (n_tokens == 0) return BCFFT_OK;
  if (!x || !y || !spectra_gu || !spectra_down) return BCFFT_ERR_ARG;
  if (!aligned16(x) || !aligned16(y) || !aligned16(spectra_gu) || !aligned16(spectra_down) ||
      (workspace && !aligned16(workspace)))
    return BCFFT_ERR_ALIGN;
  hipStream_t s = (hipStream_t)stream;
  const int64_t need = bcfft_forward_mlp_workspace_bytes(n_tokens, hidden_features, inter_features, block_size,
                                                         x_dtype, m);
  if (m == BCFFT_MLP_FUSED) {
    bcfft::launch_mlp_dmm(x, n_tokens, n_h, spectra_gu, spectra_down, y, s);
    return record_launch();
  }
  if (!workspace || workspace_bytes < need) return BCFFT_ERR_ARG;
  if (m == BCFFT_MLP_FUSED_SPLITK) {
    bcfft::launch_mlp_dmm_split(x, n_tokens, n_h, spectra_gu, spectra_down, y, (float*)workspace,
                                bcfft::dmm_ksplit(n_tokens, n_h), s);
    return record_launch();
  }
  // SPLIT: h = silu(gate(x)) * up(x) into the workspace, then down(h) (two launches, AUTO engines)
  int st = bcfft_forward_glu(x, x_dtype, n_tokens, hidden_features, inter_features, block_size, spectra_gu, workspace,
                             stream);
  if (st != BCFFT_OK) return st;
  return bcfft_forward(workspace, x_dtype, n_tokens, inter_features, hidden_features, block_size, spectra_down,
                       nullptr, BCFFT_NONE, y, x_dtype, stream);
}

int bcfft_forward(const void* x, int x_dtype, int64_t n_tokens, int in_features,
                  int out_features, int block_size, const void* spectra, const void* bias,
                  int bias_dtype, void* y, int y_dtype, void* stream) {
  return bcfft_forward_algo(x, x_dtype, n_tokens, in_features, out_features, block_size, spectra,
                            bias, bias_dtype, y, y_dtype, BCFFT_ALGO_AUTO, stream);
}

#ifdef BCFFT_ANALYSIS
// analysis builds only: phase switches of the MFMA kernel (results are WRONG when set):
// 1 skip MFMAs, 2 skip B-fragment loads, 4 skip forward FFT math, 8 skip inverse FFT math,
// 16 skip x DMA
int bcfft_set_ablation(int flags) {
  return hipMemcpyToSymbol(HIP_SYMBOL(bcfft::g_ablate), &flags, sizeof(int)) == hipSuccess ? BCFFT_OK : BCFFT_ERR_HIP;
}
// phase timeline: 64 u64 slots per wave (s_memtime), indexed (block * waves + wave) * 64 + id;
// NULL switches stamping off
int bcfft_set_stamps(void* buf) {
  unsigned long long* p = (unsigned long long*)buf;
  return hipMemcpyToSymbol(HIP_SYMBOL(bcfft::g_stamps), &p, sizeof(p)) == hipSuccess ? BCFFT_OK : BCFFT_ERR_HIP;
}
#endif

int bcfft_project_circulant(const void* w, int w_dtype, int out_features, int in_features, int block_size,
                            float* c, void* stream) {
  if (!valid_block(block_size)) return BCFFT_ERR_BLOCK;
  if (out_features <= 0 || in_features <= 0 || out_features % block_size || in_features % block_size)
    return BCFFT_ERR_SHAPE;
  if (!valid_dt(w_dtype)) return BCFFT_ERR_DTYPE;
  if (!w || !c) return BCFFT_ERR_ARG;
  bcfft::launch_project(block_size, w, w_dtype, out_features / block_size, in_features / block_size, 1e-12f, c,
                        (hipStream_t)stream);
  return record_launch();
}

int64_t bcfft_grad_c_workspace_bytes(int64_t n_tokens, int in_features, int out_features, int block_size) {
  if (!valid_block(block_size) || n_tokens < 0 || in_features <= 0 || out_features <= 0 ||
      in_features % block_size || out_features % block_size)
    return -1;
  return bcfft::grad_plan(block_size, n_tokens, in_features / block_size, out_features / block_size).workspace_bytes;
}

int bcfft_grad_c(const void* x, int x_dtype, const void* dy, int dy_dtype, int64_t n_tokens, int in_features,
                 int out_features, int block_size, void* workspace, void* dc, int dc_dtype, void* stream) {
  if (!valid_block(block_size)) return BCFFT_ERR_BLOCK;
  if (n_tokens < 0 || in_features <= 0 || out_features <= 0 || in_features % block_size ||
      out_features % block_size)
    return BCFFT_ERR_SHAPE;
  if (!valid_dt(x_dtype) || !valid_dt(dy_dtype) || !valid_dt(dc_dtype)) return BCFFT_ERR_DTYPE;
  if (!dc || (n_tokens > 0 && (!x || !dy))) return BCFFT_ERR_ARG;
  const int n_in = in_features / block_size, n_out = out_features / block_size;
  if (bcfft::grad_plan(block_size, n_tokens, n_in, n_out).workspace_bytes > 0 && !workspace) return BCFFT_ERR_ARG;
  if ((x && !aligned16(x)) || (dy && !aligned16(dy)) || (workspace && !aligned16(workspace))) return BCFFT_ERR_ALIGN;
  bcfft::launch_grad_c(block_size, x, x_dtype, dy, dy_dtype, n_tokens, n_in, n_out, workspace, dc, dc_dtype,
                       (hipStream_t)stream);
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
