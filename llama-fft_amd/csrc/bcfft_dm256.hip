// bcfft_dm256.hip — the DFT-on-MFMA block-circulant forward at b = 256 (the reference's default
// block size, patch_llama_fft.py:13) for K = 4096, bf16 I/O (gfx950).
//
// Same operator (BlockCirculantLinear.forward, patch_llama_fft.py:226-275; per block
// src/fft_utils.py:3-34) and the same three matrix-core stages as bcfft_dm8.hip. A 256-point
// dense DFT table would take 64 KiB of LDS beside the two 64 KiB token regions, so every 256-point
// transform is built from the 128-point fp16 table of the b = 128 kernels (bcfft_dm_table.h)
// applied to three 128-point "virtual rows" (tests/dm256_model.py restates the algebra):
//
//  * forward (stage 1): a_t = x_t + x_{t+128}, d_t = x_t - x_{t+128}, psi_t = 2 pi t / 256;
//    p_t = d_t cos psi_t, q_t = -d_t sin psi_t (t < 128). With A, P, Q the packed 128-point
//    spectra of a, p, q: X_{2j} = A_j (bin 0 = (X_0, X_128)) and X_{2j+1} = P_j + i Q_j
//    (P_0, Q_0 from the re slot of packed bin 0), j < 64. The three virtual rows share the
//    table fragments; the P / Q combination is lane-local.
//  * stage 2: per b = 256 bin (16 per wave), the 16-input-block complex MAC against the
//    VGPR-resident weights of the workgroup's 16 output blocks (one N-tile: 64 VGPRs).
//  * inverse (stage 3): per output block three 128-point inverses of bcfft_dm8.hip's stage 3:
//    E (the even bins), W (the odd bins Z_j = Y_{2j+1}, packed bin 0 (Re Z_0, 0)) and
//    W' = -i Z (packed bin 0 (Im Z_0, 0)); y_t = e_t + cos psi_t w_t - sin psi_t w'_t,
//    y_{t+128} = e_t - cos psi_t w_t + sin psi_t w'_t. With the b = 256 spectra (1/(2b) folded
//    in) the output scale is the b = 128 kernels'.
//
// Wave roles, LDS regions and the pipeline are bcfft_dm8.hip's: 8 tokens per tile, wave w does
// stage 1 and stage 3 of token w and streams that token's x; all waves run stage 2.
// Numerics: one power-of-two scale per token (|a + a'|, |p + p'| <= 4 max |x|); a, p, q, X and
// Y one RNE fp16 term each, C (per-output-block scale) and the table one term each, fp32
// accumulation.
//
// LDS (150,784 B): two regions x 8 token slots of 8,256 B (x rows of 512 B -> X units (bin k,
// block quad q) at 64 k + 16 q -> Y units -> y staging), the DFT table, the (cos, sin) psi
// table, scales, the group's inverse weight scales.
#include "bcfft_device.h"
#include "bcfft_dm_table.h"
#include "bcfft_dm_common.h"

namespace bcfft {

namespace d256 {
using namespace dmh;

constexpr int B = 256, NI = 16, TT = 8, NW = 8;
constexpr int BPW = 16;                             // b = 256 bins per wave in stage 2
constexpr int NOB = 16;                             // output blocks per workgroup (one N-tile)
constexpr int K = NI * B;
constexpr int SLOT = 8192 + 64;                     // one token
constexpr int REGION = TT * SLOT;
constexpr int F_OFF = 2 * REGION;                   // DFT table image, 64 rows x 256 B
constexpr int CS_OFF = F_OFF + 16384;               // (cos, sin) psi_t, t < 128, float2
constexpr int SC_OFF = CS_OFF + 1024;               // scale exponents [2 parity][8 token][2]
constexpr int OS_OFF = SC_OFF + 128;                // the group's 16 inverse weight scales
constexpr int LDS_BYTES = OS_OFF + 64;
constexpr int NPIECE = BPW * 2;                     // STAT image pieces per wave: 16 bins x 2 N-tiles
constexpr int NDMA = K * 2 / 1024;                  // 1-KiB LDS-DMA pieces per token (bf16 x)
static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
static_assert(F_OFF % 256 == 0, "table rows on the bank period");

// X unit (16 B: input blocks 4q..4q+3 x (re, im) fp16 of b = 256 bin k) in a token slot
__device__ __forceinline__ int xunit(int k, int q) { return 64 * k + 16 * q; }
// Y unit (16 B = 4 virtual bins 8w + par + 2i of spectrum s (0: E, the even bins; 1: Z, the odd
// bins) x (re, im) fp16) of output block o. Wave w's 64 units fill exactly the 1 KiB of its own
// stage-2 X units (bins 16 w .. 16 w + 15), so it writes them as soon as its reads are issued
// (in-order DS per wave) without a barrier in between.
__device__ __forceinline__ int yunit(int s, int w, int o, int par) { return 1024 * w + 512 * s + 256 * par + 16 * o; }
}  // namespace d256

// HB: a bias is added (the runtime bias_dt then names its dtype); without one the store path is
// straight-line (a runtime test per stored quad split stage 3 into hundreds of basic blocks)
template <bool HB>
__global__ __launch_bounds__(512, 2) void bc_forward_dm256_kernel(
    const void* __restrict__ xv, int64_t n_tokens, int n_out, const uint32_t* __restrict__ stat,
    const float* __restrict__ osc, const void* __restrict__ bias, int bias_dt, void* __restrict__ yv) {
  using namespace d256;
  constexpr int XT = BCFFT_BF16;
  constexpr int ES = 2, ESY = 2;

  __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];
  int* wsc = reinterpret_cast<int*>(lds + SC_OFF);
  const float2* cs_l = reinterpret_cast<const float2*>(lds + CS_OFF);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n_groups = (n_out + NOB - 1) / NOB;
  const GroupMap gm = group_map(n_groups);
  const int grp_o = gm.grp, wg_in_grp = gm.lane;
  const int64_t M = (int64_t)n_out * B;
  const int64_t n_mtiles = (n_tokens + TT - 1) / TT;
  const int gstride = gm.stride;
  const uint32_t lds_base = __builtin_amdgcn_readfirstlane(lds_addr(lds));

  // ---- x of token `wave` of M-tile m -> its slot by LDS-DMA. Rows of 512 B; logical 16-B unit
  // u of block row r sits at u ^ (r & 15) (conflict-free stage-1 reads), applied to the global
  // source offsets. Piece q = rows 2q + (lane >> 5).
  auto dma_token = [&](int64_t m, char* region) {
    const int64_t tok = m * TT + wave;
    const bool ok = tok < n_tokens;
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<char*>((const char*)xv) + (ok ? tok : 0) * K * ES, 0, ok ? K * ES : 0, 0x00020000);
    const int dl = opaque(lane);
    const uint32_t dst0 = lds_base + (uint32_t)(region - lds) + wave * SLOT;
    int vb[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int h = dl >> 5;
      vb[c] = h * 512 + 16 * ((dl & 31) ^ ((2 * c + h) & 15));
    }
#pragma unroll
    for (int q = 0; q < NDMA; ++q) {
      uint32_t keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen" BCFFT_XPOL " lds\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep) : "v"(vb[q & 7]), "s"(xrs), "s"(dst0 + q * 1024), "s"(q * 1024) : "memory");
    }
  };

  // ---- prologue: first tile's x, the DFT table, the psi table, the stationary B fragments of
  // the group's 16 output blocks (STAT image group grp_o >> 1, N-tile grp_o & 1)
  if (wg_in_grp < n_mtiles) dma_token(wg_in_grp, lds);
  {
    const uint4* tab = reinterpret_cast<const uint4*>(kDmF);
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int c = tid + 512 * r;                  // chunk c: row c >> 4, chunk c & 15
      const int t = c >> 4, ch = c & 15;
      *reinterpret_cast<uint4*>(lds + F_OFF + 256 * t + 16 * (ch ^ fsw(t))) = tab[c];
    }
    if (tid < 128) {
      double sn, cn;
      sincospi((double)tid / 128.0, &sn, &cn);     // psi_t = 2 pi t / 256
      reinterpret_cast<float2*>(lds + CS_OFF)[tid] = make_float2((float)cn, (float)sn);
    }
  }
  f16x8 creg[BPW];
  {
    const uint4* img = reinterpret_cast<const uint4*>(stat + 4) + ((int64_t)((grp_o >> 1) * NW + wave) * NPIECE) * 64 + lane;
#pragma unroll
    for (int fb = 0; fb < BPW; ++fb) creg[fb] = __builtin_bit_cast(f16x8, img[(fb * 2 + (grp_o & 1)) * 64]);
#pragma unroll
    for (int fb = 0; fb < BPW; ++fb) asm volatile("" : "+v"(creg[fb]));   // pin the loads here
  }
  // the group's inverse weight scales 1 / s_o -> LDS (after the weight loads)
  if (tid < NOB) reinterpret_cast<float*>(lds + OS_OFF)[tid] = osc[grp_o * NOB + tid];
  wait_vmcnt<0>();
  lds_barrier();

  // ---- stage 1 (wave w, token slot w): x rows -> X units (one fp16 term), in place. Lane
  // (b16 = block, g): t = 32 ks + 8 g + j (j < 8) and t + 64, t + 128, t + 192. Virtual rows a
  // (even bins) and p, q (odd bins) through the 128-point table; the x rows are all read (into
  // the B fragments) before the first X unit is written.
  auto stage1 = [&](char* region, int par) {
    const int l = opaque(lane);
    const int b16 = l & 15, g = l >> 4;
    char* slot = region + wave * SLOT;
    const int q4 = (l & 15) >> 2, p4 = l & 3;
    const int cx = (p4 >> 1) ^ fsw(8 * g + q4);
    const int trb = F_OFF + 256 * (8 * g + q4) + 8 * (p4 & 1);
    const char* rowp = slot + b16 * (B * ES);
    // x[4 quarter + ...]: unit (8 qt + 4 ks + g) of the row, 8 bf16 each
    uint32_t xr[4][2][4];
#pragma unroll
    for (int qt = 0; qt < 4; ++qt)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const uint4 w = *reinterpret_cast<const uint4*>(rowp + 16 * ((8 * qt + 4 * ks + g) ^ b16));
        xr[qt][ks][0] = w.x; xr[qt][ks][1] = w.y; xr[qt][ks][2] = w.z; xr[qt][ks][3] = w.w;
      }
    float m0f = 0.f, m1f = 0.f;                     // max |x| over the token
#pragma unroll
    for (int qt = 0; qt < 4; ++qt)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int e = 0; e < 4; e += 2) {
          const float2 f0 = unpack16<XT>(xr[qt][ks][e]), f1 = unpack16<XT>(xr[qt][ks][e + 1]);
          m0f = amax3(m0f, f0.x, f0.y);
          m1f = amax3(m1f, f1.x, f1.y);
        }
    const float mxf = __builtin_fmaxf(m0f, m1f);
    // |a + a'|, |p +- p'|, |q +- q'| <= 4 max |x|
    const int sx = stat_scale_exp(4.f * __uint_as_float(wave_umax(__float_as_uint(mxf))));
    if (l < 2) wsc[par * 16 + wave * 2 + l] = sx - 7;   // X = D 2^-(sx - 7): the table's 2^-7
    const float S = __int_as_float((sx + 127) << 23);
    // B fragments (8 t each) of the six transform inputs per K-step
    uint32_t fa[2][2][4], fp[2][2][4], fq[2][2][4];   // [ks][prime / double prime][e]
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const float4* csp = reinterpret_cast<const float4*>(cs_l + 32 * ks + 8 * g);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float4 cs2 = csp[e];                   // (cos, sin) of t = 32 ks + 8 g + 2 e, + 1
        const float2 x0 = unpack16<XT>(xr[0][ks][e]), x1 = unpack16<XT>(xr[1][ks][e]);
        const float2 x2 = unpack16<XT>(xr[2][ks][e]), x3 = unpack16<XT>(xr[3][ks][e]);
        float ap[2], app[2], pp[2], ppp[2], qp[2], qpp[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const float xt = h ? x0.y : x0.x, xt64 = h ? x1.y : x1.x, xt128 = h ? x2.y : x2.x, xt192 = h ? x3.y : x3.x;
          const float c = h ? cs2.z : cs2.x, s = h ? cs2.w : cs2.y;
          const float u = (xt + xt128) * S, v = (xt64 + xt192) * S;
          const float d0 = (xt - xt128) * S, d1 = (xt64 - xt192) * S;
          ap[h] = u + v;
          app[h] = u - v;
          pp[h] = fmaf(d0, c, -d1 * s);             // p_t + p_{t+64}
          ppp[h] = fmaf(d0, c, d1 * s);             // p_t - p_{t+64}
          qp[h] = -fmaf(d0, s, d1 * c);             // q_t + q_{t+64}
          qpp[h] = fmaf(d1, c, -d0 * s);            // q_t - q_{t+64}
        }
        fa[ks][0][e] = pk_rne(ap[0], ap[1]);
        fa[ks][1][e] = pk_rne(app[0], app[1]);
        fp[ks][0][e] = pk_rne(pp[0], pp[1]);
        fp[ks][1][e] = pk_rne(ppp[0], ppp[1]);
        fq[ks][0][e] = pk_rne(qp[0], qp[1]);
        fq[ks][1][e] = pk_rne(qpp[0], qpp[1]);
      }
    }
    // X write lane bases: D^T row 4 g + r of tile (pr, mt) is b = 128 packed bin
    // f = 16 mt + 4 g + pr (+ 2 for r >= 2): b = 256 bin 2 f (a) or 2 f + 1 (p, q)
    // pass 1: the a rows -> even bins
    {
      f32x4 acc[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int pr = 0; pr < 2; ++pr)
#pragma unroll
          for (int mt = 0; mt < 4; ++mt) {
            const int cb = 16 * ((8 * pr + 2 * mt) ^ cx);
            const char* p0 = lds + trb + 256 * 32 * ks + cb;
            const s16x4 r0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p0));
            const s16x4 r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p0 + 256 * 4));
            const f16x8 af = __builtin_bit_cast(f16x8, __builtin_shufflevector(r0, r1, 0, 1, 2, 3, 4, 5, 6, 7));
            acc[4 * pr + mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
                af, frag(fa[ks][pr][0], fa[ks][pr][1], fa[ks][pr][2], fa[ks][pr][3]), acc[4 * pr + mt], 0, 0, 0);
          }
      // stage-1 outputs of pass 2 (p, q) come from the same registers-only inputs, so the even
      // X units may overwrite the x rows now: every x read of this wave is done (in-order DS)
#pragma unroll
      for (int pr = 0; pr < 2; ++pr)
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          const int f = 16 * mt + 4 * g + pr;
          *reinterpret_cast<uint32_t*>(slot + xunit(2 * f, 0) + 4 * b16) = pk_rne(acc[4 * pr + mt][0], acc[4 * pr + mt][1]);
          *reinterpret_cast<uint32_t*>(slot + xunit(2 * f + 4, 0) + 4 * b16) = pk_rne(acc[4 * pr + mt][2], acc[4 * pr + mt][3]);
        }
    }
    // pass 2: the p and q rows -> odd bins X_{2f+1} = P_f + i Q_f (bin 1: (P_0, Q_0))
    {
      f32x4 accp[8], accq[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        accp[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        accq[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int pr = 0; pr < 2; ++pr)
#pragma unroll
          for (int mt = 0; mt < 4; ++mt) {
            const int cb = 16 * ((8 * pr + 2 * mt) ^ cx);
            const char* p0 = lds + trb + 256 * 32 * ks + cb;
            const s16x4 r0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p0));
            const s16x4 r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p0 + 256 * 4));
            const f16x8 af = __builtin_bit_cast(f16x8, __builtin_shufflevector(r0, r1, 0, 1, 2, 3, 4, 5, 6, 7));
            accp[4 * pr + mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
                af, frag(fp[ks][pr][0], fp[ks][pr][1], fp[ks][pr][2], fp[ks][pr][3]), accp[4 * pr + mt], 0, 0, 0);
            accq[4 * pr + mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
                af, frag(fq[ks][pr][0], fq[ks][pr][1], fq[ks][pr][2], fq[ks][pr][3]), accq[4 * pr + mt], 0, 0, 0);
          }
#pragma unroll
      for (int pr = 0; pr < 2; ++pr)
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          const f32x4 P = accp[4 * pr + mt], Q = accq[4 * pr + mt];
          const int f = 16 * mt + 4 * g + pr;
          float re0 = P[0] - Q[1], im0 = P[1] + Q[0];
          if (mt == 0 && pr == 0 && g == 0) {       // packed bin 0 = (P_0, P_64): X_1 = P_0 + i Q_0
            re0 = P[0];
            im0 = Q[0];
          }
          *reinterpret_cast<uint32_t*>(slot + xunit(2 * f + 1, 0) + 4 * b16) = pk_rne(re0, im0);
          *reinterpret_cast<uint32_t*>(slot + xunit(2 * f + 5, 0) + 4 * b16) = pk_rne(P[2] - Q[3], P[3] + Q[2]);
        }
    }
  };

  // ---- stage 2 (all waves): per-bin complex MAC on b = 256 bins k = 16 wave + fb for all 8
  // tokens (bcfft_dm8.hip's A rows: re rows [Xr, Xi], im rows [Xi, -Xr] by v_perm + v_pk_mul_f16;
  // bin 0 (X_0, X_128) with the extra 1/2). Y units: even bins -> spectrum E, odd -> Z, over the
  // wave's own X units.
  auto stage2 = [&](char* region, int par) {
    uint32_t yh[BPW][2];
    const int ml = opaque(lane);
    const int arow = ml & 15, kb = ml >> 4;
    const int a_t = arow >> 1, a_reim = arow & 1;
    const uint32_t a_sel = a_reim ? 0x01000302u : 0x03020100u;
    const int nk = wsc[par * 16 + a_t * 2];
    (void)nk;                                       // one scale per token: no alignment
    const uint32_t hh = 15u << 10;                  // 1.0
    const uint32_t h0 = 14u << 10;                  // bin 0: 1/2
    const uint32_t amul = a_reim ? (hh | ((hh | 0x8000u) << 16)) : (hh | (hh << 16));
    const uint32_t amul0 = a_reim ? (h0 << 16) : h0;
    const char* ab = region + a_t * SLOT + 16 * kb;
#pragma unroll
    for (int fb = 0; fb < BPW; ++fb) {
      const int k = wave * BPW + fb;
      uint4 raw = *reinterpret_cast<const uint4*>(ab + xunit(k, 0));
      if (k == 0) {
        raw.x = pkmul(raw.x, amul0); raw.y = pkmul(raw.y, amul0);
        raw.z = pkmul(raw.z, amul0); raw.w = pkmul(raw.w, amul0);
      } else {
        raw.x = pkmul(__builtin_amdgcn_perm(raw.x, raw.x, a_sel), amul);
        raw.y = pkmul(__builtin_amdgcn_perm(raw.y, raw.y, a_sel), amul);
        raw.z = pkmul(__builtin_amdgcn_perm(raw.z, raw.z, a_sel), amul);
        raw.w = pkmul(__builtin_amdgcn_perm(raw.w, raw.w, a_sel), amul);
      }
      const f32x4 acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, raw), creg[fb],
                                                                f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      constexpr float YS = 1.f / 2097152.f;          // 2^-21: |Y| < 2^13 in fp16 (16 input blocks)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) yh[fb][s2] = pk_rne(acc[2 * s2] * YS, acc[2 * s2 + 1] * YS);
    }
    const int yt = ml >> 4;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      char* yb = region + (2 * yt + s2) * SLOT + 16 * (ml & 15);
      // spectrum E: bins fb = 4 i (+2 for parity 1); Z: fb = 4 i + 1 (+2)
      *reinterpret_cast<uint4*>(yb + yunit(0, wave, 0, 0)) = make_uint4(yh[0][s2], yh[4][s2], yh[8][s2], yh[12][s2]);
      *reinterpret_cast<uint4*>(yb + yunit(0, wave, 0, 1)) = make_uint4(yh[2][s2], yh[6][s2], yh[10][s2], yh[14][s2]);
      *reinterpret_cast<uint4*>(yb + yunit(1, wave, 0, 0)) = make_uint4(yh[1][s2], yh[5][s2], yh[9][s2], yh[13][s2]);
      *reinterpret_cast<uint4*>(yb + yunit(1, wave, 0, 1)) = make_uint4(yh[3][s2], yh[7][s2], yh[11][s2], yh[15][s2]);
    }
  };

  // ---- stage 3 (wave w, token slot w of the previous tile): three 128-point inverses per
  // output block (E, W, W') -> y rows of 512 B staged in the slot -> 1 KiB stores (2 rows each)
  auto stage3 = [&](char* region, int par, int64_t mp) {
    const int l = opaque(lane);
    const int o16 = l & 15, g = l >> 4;
    char* slot = region + wave * SLOT;
    const int nmin = wsc[par * 16 + wave * 2];
    const float ysc = __builtin_ldexpf(reinterpret_cast<const float*>(lds + OS_OFF)[o16], 30 - nmin);
    // Y fragments: B[k = 8 g + j][o] of virtual wave 4 ks + g, parity pr, spectrum s
    uint4 ye[2][2], yz[2][2], yw[2][2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        ye[ks][pr] = *reinterpret_cast<const uint4*>(slot + yunit(0, 4 * ks + g, o16, pr));
        yz[ks][pr] = *reinterpret_cast<const uint4*>(slot + yunit(1, 4 * ks + g, o16, pr));
      }
    const int gx = g ^ fsw(o16);
    const char* gb = lds + F_OFF + 256 * o16;
    auto gload = [&](int mt, f16x8 (&gf)[2][2]) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int pr = 0; pr < 2; ++pr)
          gf[ks][pr] = *reinterpret_cast<const f16x8*>(gb + 4096 * mt + 16 * ((8 * pr + 4 * ks) ^ gx));
    };
    f16x8 gcur[2][2];
    gload(0, gcur);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // Y is in registers: the slot is free
    // W' = -i Z: (re, im) -> (im, -re); W and W' packed bin 0 (virtual bin 0 of wave 0: g == 0,
    // ks 0, parity 0, first pair) = (Re Z_0, 0) and (Im Z_0, 0)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        const uint4 z = yz[ks][pr];
        yw[ks][pr] = make_uint4(__builtin_amdgcn_perm(z.x, z.x, 0x01000302u) ^ 0x80000000u,
                                __builtin_amdgcn_perm(z.y, z.y, 0x01000302u) ^ 0x80000000u,
                                __builtin_amdgcn_perm(z.z, z.z, 0x01000302u) ^ 0x80000000u,
                                __builtin_amdgcn_perm(z.w, z.w, 0x01000302u) ^ 0x80000000u);
      }
    if (g == 0) {
      yw[0][0].x = yz[0][0].x >> 16;
      yz[0][0].x &= 0xffffu;
    }
    const int64_t tok = mp * TT + wave;
    const bool tok_ok = tok < n_tokens;
    const int nvalid = n_out - grp_o * NOB;
    // staging: row o16 (512 B = 64 units of 8 B), outputs t..t+3 (t = 16 mt + 4 g + 64 hf) in
    // unit 4 mt + g + 16 hf, t + 128 in unit 32 + ...; physical unit u ^ 2 o16
    const int sw = 2 * o16;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      f32x4 E[3], O[3];
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        E[s] = f32x4{0.f, 0.f, 0.f, 0.f};
        O[s] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        E[0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(gcur[ks][0], __builtin_bit_cast(f16x8, ye[ks][0]), E[0], 0, 0, 0);
        O[0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(gcur[ks][1], __builtin_bit_cast(f16x8, ye[ks][1]), O[0], 0, 0, 0);
        E[1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(gcur[ks][0], __builtin_bit_cast(f16x8, yz[ks][0]), E[1], 0, 0, 0);
        O[1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(gcur[ks][1], __builtin_bit_cast(f16x8, yz[ks][1]), O[1], 0, 0, 0);
        E[2] = __builtin_amdgcn_mfma_f32_16x16x32_f16(gcur[ks][0], __builtin_bit_cast(f16x8, yw[ks][0]), E[2], 0, 0, 0);
        O[2] = __builtin_amdgcn_mfma_f32_16x16x32_f16(gcur[ks][1], __builtin_bit_cast(f16x8, yw[ks][1]), O[2], 0, 0, 0);
      }
      if (mt < 3) gload(mt + 1, gcur);
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        const float4 c01 = *reinterpret_cast<const float4*>(cs_l + 16 * mt + 4 * g + 64 * hf);
        const float4 c23 = *reinterpret_cast<const float4*>(cs_l + 16 * mt + 4 * g + 64 * hf + 2);
        const float cc[4] = {c01.x, c01.z, c23.x, c23.z}, ss[4] = {c01.y, c01.w, c23.y, c23.w};
        float lo[4], hi[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float e = hf ? E[0][r] - O[0][r] : E[0][r] + O[0][r];
          const float w = hf ? E[1][r] - O[1][r] : E[1][r] + O[1][r];
          const float wp = hf ? E[2][r] - O[2][r] : E[2][r] + O[2][r];
          const float o = fmaf(cc[r], w, -ss[r] * wp);
          lo[r] = (e + o) * ysc;                    // y_t
          hi[r] = (e - o) * ysc;                    // y_{t+128}
        }
        if (HB) {                                   // .to(x dtype) :266, + bias :270-271
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            lo[r] = round_to(lo[r], XT);
            hi[r] = round_to(hi[r], XT);
          }
          if (o16 < nvalid) {
            const int64_t cc0 = (int64_t)(grp_o * NOB + o16) * B + 16 * mt + 4 * g + 64 * hf;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              lo[r] += load_scalar(bias, cc0 + r, bias_dt);
              hi[r] += load_scalar(bias, cc0 + 128 + r, bias_dt);
            }
          }
        }
        const int u = 4 * mt + g + 16 * hf;
        *reinterpret_cast<uint2*>(slot + 512 * o16 + 8 * (u ^ sw)) = make_uint2(pack16<XT>(lo[0], lo[1]), pack16<XT>(lo[2], lo[3]));
        *reinterpret_cast<uint2*>(slot + 512 * o16 + 8 * ((u + 32) ^ sw)) = make_uint2(pack16<XT>(hi[0], hi[1]), pack16<XT>(hi[2], hi[3]));
      }
    }
    // staged rows -> global: each instruction stores 1 KiB = 2 whole rows (32 lanes per row):
    // 16-B unit w of row r at physical 16-B unit w ^ r (the 8-B swizzle by 2 r keeps pairs)
    constexpr int RB = B * ESY;
    const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
        (char*)yv + (tok_ok ? tok : 0) * M * ESY + (int64_t)grp_o * NOB * RB, 0,
        tok_ok ? (int)((M - (int64_t)grp_o * NOB * B) * ESY) : 0, 0x00020000);
    const int w = l & 31, lr = l >> 5;
    uint4 d[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int row = 2 * q + lr;
      d[q] = *reinterpret_cast<const uint4*>(slot + 512 * row + 16 * (w ^ row));
    }
#pragma unroll
    for (int q = 0; q < 8; ++q)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, d[q]), yrs, (2 * q + lr) * RB + 16 * w, 0, BCFFT_YAUX);
  };

  // Pipeline (bcfft_dm8.hip's), two workgroup barriers per M-tile; iteration it: region R =
  // it & 1 holds tile m, R' tile m - stride:
  //   P1  wave w: stage 3 of token w of tile m - stride from R' (stores); LDS-DMA of
  //       x(m + stride, token w) into that slot; its own x(m) landed (a whole iteration after
  //       its issue) -> stage 1 of token w of tile m in R                                 | Ba |
  //   P2  stage 2 of tile m in R (Y units over each wave's own X units)                     | Bb |
  // The x(m) waits count the younger VMEM operations: 8 stage-3 stores, then NDMA DMA pieces.
  int64_t m = wg_in_grp;
  for (int it = 0; m < n_mtiles || it > 0; ++it, m += gstride) {
    char* region = lds + (it & 1) * REGION;
    char* other = lds + ((it + 1) & 1) * REGION;
    const int par = it & 1;
    const bool have = m < n_mtiles;
    const bool pf = m + gstride < n_mtiles;
    if (wave < 4 && it > 0 && have) {
      // waves 0-3: stage 3 of the previous tile, the next tile's x DMA, then stage 1
      if (it > 0) stage3(other, par ^ 1, m - gstride);
      if (pf) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the slot's staging reads are done
        dma_token(m + gstride, other);
      }
      if (!have) break;
      if (pf) {
        if (it > 0) wait_vmcnt<8 + NDMA>();
        else wait_vmcnt<NDMA>();
      } else {
        if (it > 0) wait_vmcnt<8>();
        else wait_vmcnt<0>();
      }
      stage1(region, par);
    } else {
      // waves 4-7, and every wave of the first and last iterations): stage 1 first, at a
      // higher priority than the partner wave's stage 3 (bcfft_dm8.hip's mixed order and YPRIO):
      // 39.2 -> 36.8 us over six interleaved passes, the order alone 38.7
      // (profiles/r05ad_ab_dm256_mix_yprio.log)
      if (have) {
        wait_vmcnt<0>();                            // this wave's x (issued an iteration ago)
        __builtin_amdgcn_s_setprio(1);
        stage1(region, par);
        __builtin_amdgcn_s_setprio(0);
      }
      if (it > 0) stage3(other, par ^ 1, m - gstride);
      if (pf) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the slot's staging reads are done
        dma_token(m + gstride, other);
      }
      if (!have) break;
    }
    lds_barrier();                                  // Ba: X units and scales complete
    stage2(region, par);
    lds_barrier();                                  // Bb: Y units complete
  }
}

// ============================================================== K > 4096: streamed weights
// bc_forward_dm256k_kernel: b = 256 with more than 16 input blocks (the LLaMA down projection
// 11008 -> 4096: 43 blocks). A workgroup's 16 output blocks x n_in input blocks of fp16 spectra
// (88 KiB per 11 blocks) do not fit its VGPRs, so the K axis is cut into 16-block chunks
// (bcfft_dmk.hip's scheme at b = 256): per chunk, stage 1 of the 8 tokens' chunk rows (x DMA one
// chunk ahead), then stage 2 against the chunk's B fragments streamed from L2 (16 per wave, the
// next chunk's loaded bin by bin into the same registers as each bin is done), accumulating in
// 64 fp32 VGPRs over all chunks. At the tile end the Y units go into the last chunk's region and
// stage 3 of token w runs at the start of the next tile, beside its first stage 1.
// Numerics: per-(token, chunk) power-of-two scales with HEAD bits of headroom (stage 2 aligns
// each chunk to the token's reference exponent with an exact fp16 power-of-two factor and scales
// the accumulator rows down once if a chunk is more than 2^HEAD louder: tests/dm_model.py's
// head = 4 scheme); otherwise bc_forward_dm256_kernel's.
namespace d256 {
constexpr int HEAD = 4;
// wave priority falling through stage 1 (1) and stage 2 (2): set_prio, bcfft_dm64k.hip's finding
constexpr int PRIO = 3;
constexpr int SC2_OFF = CS_OFF + 1024;              // chunk scale exponents [8 tokens]
constexpr int RR_OFF = SC2_OFF + 64;                // per-token reference exponents [8]
constexpr int OS2_OFF = RR_OFF + 64;                // the workgroup's 16 inverse weight scales
constexpr int LDS2_BYTES = OS2_OFF + 64;
static_assert(LDS2_BYTES <= 160 * 1024, "LDS budget");
constexpr int NDMA_C = NI * B * 2 / 1024;           // 1-KiB x DMA pieces per token and chunk
// fp16 factor 2^-d (d >= -15) as a (lo, hi) pair: subnormal below 2^-14, zero below 2^-24
__device__ __forceinline__ uint32_t f16_pow2_neg(int d) {
  return d <= 14 ? (uint32_t)(15 - d) << 10 : (d <= 24 ? 1u << (24 - d) : 0u);
}
}  // namespace d256

template <bool HB>
__global__ __launch_bounds__(512, 2) void bc_forward_dm256k_kernel(
    const void* __restrict__ xv, int64_t n_tokens, int n_in, int n_out, const uint32_t* __restrict__ stat,
    const float* __restrict__ osc, const void* __restrict__ bias, int bias_dt, void* __restrict__ yv) {
  using namespace d256;
  constexpr int XT = BCFFT_BF16;
  constexpr int ES = 2, ESY = 2;

  __shared__ __attribute__((aligned(16))) char lds[LDS2_BYTES];
  int* wsc = reinterpret_cast<int*>(lds + SC2_OFF);
  int* wrr = reinterpret_cast<int*>(lds + RR_OFF);
  const float2* cs_l = reinterpret_cast<const float2*>(lds + CS_OFF);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n_groups = (n_out + NOB - 1) / NOB;
  const GroupMap gm = group_map(n_groups);
  const int grp_o = gm.grp, wg_in_grp = gm.lane;
  const int64_t KX = (int64_t)n_in * B;
  const int64_t M = (int64_t)n_out * B;
  const int nch = (n_in + NI - 1) / NI;
  const int64_t n_mtiles = (n_tokens + TT - 1) / TT;
  const int gstride = gm.stride;
  const uint32_t lds_base = __builtin_amdgcn_readfirstlane(lds_addr(lds));

  // ---- chunk c of token `wave` of M-tile m -> its slot by LDS-DMA (rows of 512 B, unit swizzle
  // u ^ (r & 15)); the buffer range ends at the token's row end, so a partial last chunk and
  // tokens / tiles past the end land as zeros
  auto dma_chunk = [&](int64_t m, int c, char* region) {
    const int64_t tok = m * TT + wave;
    const bool ok = m < n_mtiles && tok < n_tokens;
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<char*>((const char*)xv) + (ok ? tok * KX * ES + (int64_t)c * (NI * B * ES) : 0), 0,
        ok ? (int)(KX * ES - (int64_t)c * (NI * B * ES)) : 0, 0x00020000);
    const int dl = opaque(lane);
    const uint32_t dst0 = lds_base + (uint32_t)(region - lds) + wave * SLOT;
    int vb[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int h = dl >> 5;
      vb[q] = h * 512 + 16 * ((dl & 31) ^ ((2 * q + h) & 15));
    }
#pragma unroll
    for (int q = 0; q < NDMA_C; ++q) {
      uint32_t keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen" BCFFT_XPOL " lds\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep) : "v"(vb[q & 7]), "s"(xrs), "s"(dst0 + q * 1024), "s"(q * 1024) : "memory");
    }
  };

  // ---- B fragments: STAT image group grp_o >> 1, wave, piece (fb KS + c) 2 + (grp_o & 1). Asm
  // loads (bcfft_dmk.hip's scheme): the compiler does not count them, so its waits never drain
  // the x DMA issued after them; wait_b is the one wait, with the exact number of younger VMEM
  // operations, and it redefines the registers it waited for.
  const int KS = nch;
  const int npiece = BPW * KS * 2;
  const __amdgpu_buffer_rsrc_t brs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint32_t*>(stat + 4) + ((int64_t)((grp_o >> 1) * NW + wave) * npiece) * 256, 0, npiece * 1024,
      0x00020000);
  // live = false: an empty-range load (the offset lies past the buffer: zeros, no memory access)
  auto load_b1 = [&](int c, int fb, u32x4 (&breg)[BPW], bool live = true) {
    const int vo = opaque(lane) * 16 + (live ? (c * 2 + (grp_o & 1)) * 1024 : npiece * 1024);
    asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen"
                 : "=v"(breg[fb]) : "v"(vo), "s"(brs), "s"(fb * KS * 2048));
  };
  auto wait_b = [&](auto n_tag, u32x4 (&breg)[BPW]) {
    constexpr int N = decltype(n_tag)::value;
    static_assert(N >= 0 && N < 64, "vmcnt");
    asm volatile("s_waitcnt vmcnt(%16) ; bcfft-wait %0 %1 %2 %3 %4 %5 %6 %7 %8 %9 %10 %11 %12 %13 %14 %15"
                 : "+v"(breg[0]), "+v"(breg[1]), "+v"(breg[2]), "+v"(breg[3]), "+v"(breg[4]), "+v"(breg[5]),
                   "+v"(breg[6]), "+v"(breg[7]), "+v"(breg[8]), "+v"(breg[9]), "+v"(breg[10]), "+v"(breg[11]),
                   "+v"(breg[12]), "+v"(breg[13]), "+v"(breg[14]), "+v"(breg[15])
                 : "n"(N) : "memory");
  };
  static_assert(BPW == 16, "wait_b names sixteen fragments");

  // ---- prologue: the first tile's chunk 0, the DFT and psi tables, the inverse weight scales
  dma_chunk(wg_in_grp, 0, lds);
  {
    const uint4* tab = reinterpret_cast<const uint4*>(kDmF);
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int c = tid + 512 * r;
      const int t = c >> 4, ch = c & 15;
      *reinterpret_cast<uint4*>(lds + F_OFF + 256 * t + 16 * (ch ^ fsw(t))) = tab[c];
    }
    if (tid < 128) {
      double sn, cn;
      sincospi((double)tid / 128.0, &sn, &cn);
      reinterpret_cast<float2*>(lds + CS_OFF)[tid] = make_float2((float)cn, (float)sn);
    }
  }
  if (tid < NOB) reinterpret_cast<float*>(lds + OS2_OFF)[tid] = osc[grp_o * NOB + tid];
  wait_vmcnt<0>();
  lds_barrier();

  // ---- stage 1 (wave w, token slot w): bc_forward_dm256_kernel's on one 16-block chunk, with
  // the per-(token, chunk) scale lowered by HEAD bits, and the odd-bin pass split by parity
  auto stage1 = [&](char* region) {
    const int l = opaque(lane);
    const int b16 = l & 15, g = l >> 4;
    char* slot = region + wave * SLOT;
    const int q4 = (l & 15) >> 2, p4 = l & 3;
    const int cx = (p4 >> 1) ^ fsw(8 * g + q4);
    const int trb = F_OFF + 256 * (8 * g + q4) + 8 * (p4 & 1);
    const char* rowp = slot + b16 * (B * ES);
    if constexpr ((PRIO & 1) != 0) set_prio(2);
    uint32_t xr[4][2][4];
#pragma unroll
    for (int qt = 0; qt < 4; ++qt)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const uint4 w = *reinterpret_cast<const uint4*>(rowp + 16 * ((8 * qt + 4 * ks + g) ^ b16));
        xr[qt][ks][0] = w.x; xr[qt][ks][1] = w.y; xr[qt][ks][2] = w.z; xr[qt][ks][3] = w.w;
      }
    float m0f = 0.f, m1f = 0.f;
#pragma unroll
    for (int qt = 0; qt < 4; ++qt)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int e = 0; e < 4; e += 2) {
          const float2 f0 = unpack16<XT>(xr[qt][ks][e]), f1 = unpack16<XT>(xr[qt][ks][e + 1]);
          m0f = amax3(m0f, f0.x, f0.y);
          m1f = amax3(m1f, f1.x, f1.y);
        }
    const float mxf = __builtin_fmaxf(m0f, m1f);
    const int sx = stat_scale_exp(4.f * __uint_as_float(wave_umax(__float_as_uint(mxf)))) - HEAD;
    if (l == 0) wsc[wave] = sx - 7;                 // X = D 2^-(sx - 7): the table's 2^-7
    const float S = __int_as_float((sx + 127) << 23);
    uint32_t fa[2][2][4], fp[2][2][4], fq[2][2][4];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const float4* csp = reinterpret_cast<const float4*>(cs_l + 32 * ks + 8 * g);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float4 cs2 = csp[e];
        const float2 x0 = unpack16<XT>(xr[0][ks][e]), x1 = unpack16<XT>(xr[1][ks][e]);
        const float2 x2 = unpack16<XT>(xr[2][ks][e]), x3 = unpack16<XT>(xr[3][ks][e]);
        float ap[2], app[2], pp[2], ppp[2], qp[2], qpp[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const float xt = h ? x0.y : x0.x, xt64 = h ? x1.y : x1.x, xt128 = h ? x2.y : x2.x, xt192 = h ? x3.y : x3.x;
          const float c = h ? cs2.z : cs2.x, s = h ? cs2.w : cs2.y;
          const float u = (xt + xt128) * S, v = (xt64 + xt192) * S;
          const float d0 = (xt - xt128) * S, d1 = (xt64 - xt192) * S;
          ap[h] = u + v;
          app[h] = u - v;
          pp[h] = fmaf(d0, c, -d1 * s);
          ppp[h] = fmaf(d0, c, d1 * s);
          qp[h] = -fmaf(d0, s, d1 * c);
          qpp[h] = fmaf(d1, c, -d0 * s);
        }
        fa[ks][0][e] = pk_rne(ap[0], ap[1]);
        fa[ks][1][e] = pk_rne(app[0], app[1]);
        fp[ks][0][e] = pk_rne(pp[0], pp[1]);
        fp[ks][1][e] = pk_rne(ppp[0], ppp[1]);
        fq[ks][0][e] = pk_rne(qp[0], qp[1]);
        fq[ks][1][e] = pk_rne(qpp[0], qpp[1]);
      }
    }
    {
      f32x4 acc8[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) acc8[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int pr = 0; pr < 2; ++pr)
#pragma unroll
          for (int mt = 0; mt < 4; ++mt) {
            const int cb = 16 * ((8 * pr + 2 * mt) ^ cx);
            const char* p0 = lds + trb + 256 * 32 * ks + cb;
            const s16x4 r0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p0));
            const s16x4 r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p0 + 256 * 4));
            const f16x8 af = __builtin_bit_cast(f16x8, __builtin_shufflevector(r0, r1, 0, 1, 2, 3, 4, 5, 6, 7));
            acc8[4 * pr + mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
                af, frag(fa[ks][pr][0], fa[ks][pr][1], fa[ks][pr][2], fa[ks][pr][3]), acc8[4 * pr + mt], 0, 0, 0);
          }
#pragma unroll
      for (int pr = 0; pr < 2; ++pr)
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          const int f = 16 * mt + 4 * g + pr;
          *reinterpret_cast<uint32_t*>(slot + xunit(2 * f, 0) + 4 * b16) = pk_rne(acc8[4 * pr + mt][0], acc8[4 * pr + mt][1]);
          *reinterpret_cast<uint32_t*>(slot + xunit(2 * f + 4, 0) + 4 * b16) = pk_rne(acc8[4 * pr + mt][2], acc8[4 * pr + mt][3]);
        }
    }
    if constexpr ((PRIO & 1) != 0) set_prio(1);
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
      f32x4 accp[4], accq[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        accp[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        accq[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          const int cb = 16 * ((8 * pr + 2 * mt) ^ cx);
          const char* p0 = lds + trb + 256 * 32 * ks + cb;
          const s16x4 r0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p0));
          const s16x4 r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p0 + 256 * 4));
          const f16x8 af = __builtin_bit_cast(f16x8, __builtin_shufflevector(r0, r1, 0, 1, 2, 3, 4, 5, 6, 7));
          accp[mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
              af, frag(fp[ks][pr][0], fp[ks][pr][1], fp[ks][pr][2], fp[ks][pr][3]), accp[mt], 0, 0, 0);
          accq[mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
              af, frag(fq[ks][pr][0], fq[ks][pr][1], fq[ks][pr][2], fq[ks][pr][3]), accq[mt], 0, 0, 0);
        }
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const f32x4 P = accp[mt], Q = accq[mt];
        const int f = 16 * mt + 4 * g + pr;
        float re0 = P[0] - Q[1], im0 = P[1] + Q[0];
        if (mt == 0 && pr == 0 && g == 0) {         // packed bin 0 = (P_0, P_64): X_1 = P_0 + i Q_0
          re0 = P[0];
          im0 = Q[0];
        }
        *reinterpret_cast<uint32_t*>(slot + xunit(2 * f + 1, 0) + 4 * b16) = pk_rne(re0, im0);
        *reinterpret_cast<uint32_t*>(slot + xunit(2 * f + 5, 0) + 4 * b16) = pk_rne(P[2] - Q[3], P[3] + Q[2]);
      }
    }
  };

  // accumulators [bin of the wave]: rows 4 yt + r = token 2 yt + (r >> 1), re / im r & 1; the
  // reference exponents of the lane's A-row token and accumulator-row tokens
  f32x4 acc[BPW];
#pragma unroll
  for (int fb = 0; fb < BPW; ++fb) acc[fb] = f32x4{0.f, 0.f, 0.f, 0.f};
  int ra = 0;
  int rc[2] = {0, 0};

  // ---- stage 2 (all waves): chunk c's per-bin complex MAC on bins 16 wave + fb, accumulated
  // (the accumulators are zero at a tile's first chunk); the fragment of each bin for the next
  // (tile, chunk) step is loaded into its registers right after its MFMA (nb < 0: none). One call
  // site: the fragments stay in the same registers from their load to their use.
  auto stage2 = [&](char* region, u32x4 (&breg)[BPW], int nb, bool first, bool tile0) {
    const int ml = opaque(lane);
    const int arow = ml & 15, kb = ml >> 4;
    const int a_t = arow >> 1, a_reim = arow & 1;
    const uint32_t a_sel = a_reim ? 0x01000302u : 0x03020100u;
    const int yt = ml >> 4;
    const int nka = wsc[a_t];
    if (first) {
      ra = nka;
      rc[0] = wsc[2 * yt];
      rc[1] = wsc[2 * yt + 1];
    } else {
      ra = min(ra, nka + HEAD);
      float fct[2];
      bool need = false;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int nn = wsc[2 * yt + s] + HEAD;
        const int d = rc[s] - nn;
        fct[s] = d > 0 ? __builtin_ldexpf(1.f, -d) : 1.f;
        need |= d > 0;
        rc[s] = min(rc[s], nn);
      }
      if (__builtin_amdgcn_ballot_w64(need)) {
#pragma unroll
        for (int fb = 0; fb < BPW; ++fb)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[fb][r] *= fct[r >> 1];
      }
    }
    const int d = nka - ra;                         // >= -HEAD: factor 2^-d <= 2^HEAD
    const uint32_t hh = f16_pow2_neg(d);
    const uint32_t h0 = f16_pow2_neg(d + 1);        // bin 0: the extra 1/2
    const uint32_t amul = a_reim ? (hh | ((hh | 0x8000u) << 16)) : (hh | (hh << 16));
    const uint32_t amul0 = a_reim ? (h0 << 16) : h0;
    const char* ab = region + a_t * SLOT + 16 * kb;
    // B of this step: the younger VMEM is this step's x DMA and, at a tile's first chunk, the
    // previous tile's stage-3 stores before it. One operand-carrying wait on every path (one per
    // branch made the compiler copy the 16 fragments where the paths joined)
    if (!tile0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NDMA_C) : "memory");
    wait_b(std::integral_constant<int, 8 + NDMA_C>{}, breg);
    const bool more = nb >= 0;
    const int nc = more ? nb : 0;
    // A rows one bin ahead (the LDS latency off the MFMA chain); bin 0 (wave 0, fb 0) branch-free
    const bool bin0 = wave == 0;
    uint4 anext = *reinterpret_cast<const uint4*>(ab + xunit(wave * BPW, 0));
#pragma unroll
    for (int fb = 0; fb < BPW; ++fb) {
      if constexpr ((PRIO & 2) != 0) set_prio(3 - 4 * fb / BPW);
      const int k = wave * BPW + fb;
      uint4 raw = anext;
      if (fb + 1 < BPW) anext = *reinterpret_cast<const uint4*>(ab + xunit(k + 1, 0));
      const uint32_t sel = (fb == 0 && bin0) ? 0x03020100u : a_sel;
      const uint32_t mul = (fb == 0 && bin0) ? amul0 : amul;
      raw.x = pkmul(__builtin_amdgcn_perm(raw.x, raw.x, sel), mul);
      raw.y = pkmul(__builtin_amdgcn_perm(raw.y, raw.y, sel), mul);
      raw.z = pkmul(__builtin_amdgcn_perm(raw.z, raw.z, sel), mul);
      raw.w = pkmul(__builtin_amdgcn_perm(raw.w, raw.w, sel), mul);
      acc[fb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, raw),
                                                       __builtin_bit_cast(f16x8, breg[fb]), acc[fb], 0, 0, 0);
      load_b1(nc, fb, breg, more);                  // past the last step: an empty-range load
    }
  };

  // ---- Y of the tile (fp16 units, bc_forward_dm256_kernel's layout) into a region; the
  // reference exponents into wrr
  auto ywrite = [&](char* region) {
    const int ml = opaque(lane);
    const int yt = ml >> 4;
    constexpr float YS = 1.f / 2097152.f;            // 2^-21: |Y| <= n_in 2^9 < 65504 (n_in <= 127)
    if (wave == 0 && (ml & 15) == 0) {
      wrr[2 * yt] = rc[0];
      wrr[2 * yt + 1] = rc[1];
    }
    uint32_t yh[BPW][2];
#pragma unroll
    for (int fb = 0; fb < BPW; ++fb)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) yh[fb][s2] = pk_rne(acc[fb][2 * s2] * YS, acc[fb][2 * s2 + 1] * YS);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      char* yb = region + (2 * yt + s2) * SLOT + 16 * (ml & 15);
      *reinterpret_cast<uint4*>(yb + yunit(0, wave, 0, 0)) = make_uint4(yh[0][s2], yh[4][s2], yh[8][s2], yh[12][s2]);
      *reinterpret_cast<uint4*>(yb + yunit(0, wave, 0, 1)) = make_uint4(yh[2][s2], yh[6][s2], yh[10][s2], yh[14][s2]);
      *reinterpret_cast<uint4*>(yb + yunit(1, wave, 0, 0)) = make_uint4(yh[1][s2], yh[5][s2], yh[9][s2], yh[13][s2]);
      *reinterpret_cast<uint4*>(yb + yunit(1, wave, 0, 1)) = make_uint4(yh[3][s2], yh[7][s2], yh[11][s2], yh[15][s2]);
    }
#pragma unroll
    for (int fb = 0; fb < BPW; ++fb) acc[fb] = f32x4{0.f, 0.f, 0.f, 0.f};
  };

  // ---- stage 3 (wave w, token slot w): bc_forward_dm256_kernel's, with the token's reference
  // exponent rref; tok < 0 stores nothing (the stores are still issued, with an empty range)
  auto stage3 = [&](char* region, int rref, int64_t tok) {
    const int l = opaque(lane);
    const int o16 = l & 15, g = l >> 4;
    char* slot = region + wave * SLOT;
    const float ysc = __builtin_ldexpf(reinterpret_cast<const float*>(lds + OS2_OFF)[o16], 30 - rref);
    uint4 ye[2][2], yz[2][2], yw[2][2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        ye[ks][pr] = *reinterpret_cast<const uint4*>(slot + yunit(0, 4 * ks + g, o16, pr));
        yz[ks][pr] = *reinterpret_cast<const uint4*>(slot + yunit(1, 4 * ks + g, o16, pr));
      }
    const int gx = g ^ fsw(o16);
    const char* gb = lds + F_OFF + 256 * o16;
    auto gload = [&](int mt, f16x8 (&gf)[2][2]) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int pr = 0; pr < 2; ++pr)
          gf[ks][pr] = *reinterpret_cast<const f16x8*>(gb + 4096 * mt + 16 * ((8 * pr + 4 * ks) ^ gx));
    };
    f16x8 gcur[2][2];
    gload(0, gcur);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        const uint4 z = yz[ks][pr];
        yw[ks][pr] = make_uint4(__builtin_amdgcn_perm(z.x, z.x, 0x01000302u) ^ 0x80000000u,
                                __builtin_amdgcn_perm(z.y, z.y, 0x01000302u) ^ 0x80000000u,
                                __builtin_amdgcn_perm(z.z, z.z, 0x01000302u) ^ 0x80000000u,
                                __builtin_amdgcn_perm(z.w, z.w, 0x01000302u) ^ 0x80000000u);
      }
    if (g == 0) {
      yw[0][0].x = yz[0][0].x >> 16;
      yz[0][0].x &= 0xffffu;
    }
    const bool tok_ok = tok >= 0 && tok < n_tokens;
    const int nvalid = n_out - grp_o * NOB;
    const int sw = 2 * o16;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      f32x4 E[3], O[3];
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        E[s] = f32x4{0.f, 0.f, 0.f, 0.f};
        O[s] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        E[0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(gcur[ks][0], __builtin_bit_cast(f16x8, ye[ks][0]), E[0], 0, 0, 0);
        O[0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(gcur[ks][1], __builtin_bit_cast(f16x8, ye[ks][1]), O[0], 0, 0, 0);
        E[1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(gcur[ks][0], __builtin_bit_cast(f16x8, yz[ks][0]), E[1], 0, 0, 0);
        O[1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(gcur[ks][1], __builtin_bit_cast(f16x8, yz[ks][1]), O[1], 0, 0, 0);
        E[2] = __builtin_amdgcn_mfma_f32_16x16x32_f16(gcur[ks][0], __builtin_bit_cast(f16x8, yw[ks][0]), E[2], 0, 0, 0);
        O[2] = __builtin_amdgcn_mfma_f32_16x16x32_f16(gcur[ks][1], __builtin_bit_cast(f16x8, yw[ks][1]), O[2], 0, 0, 0);
      }
      if (mt < 3) gload(mt + 1, gcur);
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        const float4 c01 = *reinterpret_cast<const float4*>(cs_l + 16 * mt + 4 * g + 64 * hf);
        const float4 c23 = *reinterpret_cast<const float4*>(cs_l + 16 * mt + 4 * g + 64 * hf + 2);
        const float cc[4] = {c01.x, c01.z, c23.x, c23.z}, ss[4] = {c01.y, c01.w, c23.y, c23.w};
        float lo[4], hi[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float e = hf ? E[0][r] - O[0][r] : E[0][r] + O[0][r];
          const float w = hf ? E[1][r] - O[1][r] : E[1][r] + O[1][r];
          const float wp = hf ? E[2][r] - O[2][r] : E[2][r] + O[2][r];
          const float o = fmaf(cc[r], w, -ss[r] * wp);
          lo[r] = (e + o) * ysc;
          hi[r] = (e - o) * ysc;
        }
        if (HB) {                                   // .to(x dtype) :266, + bias :270-271
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            lo[r] = round_to(lo[r], XT);
            hi[r] = round_to(hi[r], XT);
          }
          if (o16 < nvalid) {
            const int64_t cc0 = (int64_t)(grp_o * NOB + o16) * B + 16 * mt + 4 * g + 64 * hf;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              lo[r] += load_scalar(bias, cc0 + r, bias_dt);
              hi[r] += load_scalar(bias, cc0 + 128 + r, bias_dt);
            }
          }
        }
        const int u = 4 * mt + g + 16 * hf;
        *reinterpret_cast<uint2*>(slot + 512 * o16 + 8 * (u ^ sw)) = make_uint2(pack16<XT>(lo[0], lo[1]), pack16<XT>(lo[2], lo[3]));
        *reinterpret_cast<uint2*>(slot + 512 * o16 + 8 * ((u + 32) ^ sw)) = make_uint2(pack16<XT>(hi[0], hi[1]), pack16<XT>(hi[2], hi[3]));
      }
    }
    constexpr int RB = B * ESY;
    const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
        (char*)yv + (tok_ok ? tok : 0) * M * ESY + (int64_t)grp_o * NOB * RB, 0,
        tok_ok ? (int)((M - (int64_t)grp_o * NOB * B) * ESY) : 0, 0x00020000);
    const int w = l & 31, lr = l >> 5;
    uint4 dd[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int row = 2 * q + lr;
      dd[q] = *reinterpret_cast<const uint4*>(slot + 512 * row + 16 * (w ^ row));
    }
#pragma unroll
    for (int q = 0; q < 8; ++q)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, dd[q]), yrs, (2 * q + lr) * RB + 16 * w, 0, BCFFT_YAUX);
  };

  // Pipeline: one step per (M-tile m of 8 tokens, chunk c), two barriers per step (rsel: the
  // region holding chunk c's x; the other holds the previous chunk's X or, at c = 0, the
  // previous tile's Y units):
  //   c = 0   stage 3 of the previous tile's token w from the other region (8 stores)
  //           x DMA of the next step's chunk into the other region (zeros past the last tile);
  //           x(m, c) landed; stage 1                                                        | Ba |
  //           stage 2 on B(c) (loaded in the previous step), loading the next step's B      | Bb |
  //   c last  Y of the tile into this region                                                 | Be |
  // VMEM younger than x(m, c) when it is waited for: B(c) 16 (the previous step's stage 2), at
  // c = 0 the 8 stores, then the DMA (the first step's x and B were waited for in the prologue).
  u32x4 breg[BPW];
#pragma unroll
  for (int fb = 0; fb < BPW; ++fb) load_b1(0, fb, breg);   // B(0), waited for by the prologue
  wait_vmcnt<0>();
  int rsel = 0;
  int64_t mprev = -1;
  int64_t m = wg_in_grp;
  int c = 0;
  while (m < n_mtiles) {
    char* region = lds + rsel * REGION;
    char* other = lds + (rsel ^ 1) * REGION;
    const bool tile0 = c == 0;
    if (tile0) {
      // B(0) of this tile (the previous step's stage-2 loads, asm: invisible to the compiler) has
      // landed before stage 3: its register pressure made hipcc rotate the 16 fragment registers
      // around stage 3 (v_mov copies of registers an in-flight load still writes; found by
      // tools/vmem_audit.py). The wait names the fragments, so copies made
      // after it carry the landed values. Nothing younger is in flight here.
      wait_b(std::integral_constant<int, 0>{}, breg);
      stage3(other, wrr[wave], mprev >= 0 ? mprev * TT + wave : -1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the slot's staging reads are done
    }
    const bool last = c + 1 == nch;
    const int64_t mn = last ? m + gstride : m;
    const int cn = last ? 0 : c + 1;
    dma_chunk(mn, cn, other);
    if (tile0) wait_vmcnt<16 + 8 + NDMA_C>();
    else wait_vmcnt<16 + NDMA_C>();
    stage1(region);
    lds_barrier();                                  // Ba: X units and chunk scales complete
    stage2(region, breg, mn < n_mtiles ? cn : -1, tile0, tile0);
    lds_barrier();                                  // Bb: every read of this chunk's X done
    if (last) {
      ywrite(region);
      lds_barrier();                                // Be: Y units and reference exponents
      mprev = m;
    }
    rsel ^= 1;
    m = mn;
    c = cn;
  }
  stage3(lds + (rsel ^ 1) * REGION, wrr[wave], mprev >= 0 ? mprev * TT + wave : -1);
  // the last step's empty-range B loads: waited for with the fragments as operands, so their
  // registers are not reused by ywrite / stage 3 while the loads are in flight
  wait_b(std::integral_constant<int, 0>{}, breg);
}

// ---- weight image at b = 256: the generic STAT image kernels instantiated for B = 256 (groups
// of 32 output blocks = two N-tiles; a b = 256 workgroup takes one N-tile)

// ============================================================== several output groups
// bc_forward_dm256g_kernel: b = 256, K = 4096, M > 4096 (three or more groups of 16 output
// blocks: the sweep's 4096 -> 11008). bcfft_dmg.hip's scheme on the b = 256 stages: stage 1 once
// per 8-token tile (bc_forward_dm256_kernel's), the A fragments of the wave's 16 bins for all 8
// tokens into VGPRs (64), then per output group: stage 2 against the group's 16 B fragments per
// wave, streamed from L2 in two passes of 8 (double-buffered, compiler-visible loads), Y units
// into the tile's slots, stage 3 of token w with the group's 16 rows stored. Numerics are
// bc_forward_dm256_kernel's in the same order: bit-identical to it run per group.
namespace d256 {
constexpr int MAXG = 64;
constexpr int OSG_OFF = SC_OFF + 128;               // inverse weight scales [MAXG][16]
constexpr int LDSG_BYTES = OSG_OFF + MAXG * NOB * 4;
static_assert(LDSG_BYTES <= 160 * 1024, "LDS budget");
}  // namespace d256

template <bool GLU, bool HB>
__global__ __launch_bounds__(512, 2) void bc_forward_dm256g_kernel(
    const void* __restrict__ xv, int64_t n_tokens, int n_out, const uint32_t* __restrict__ stat,
    const float* __restrict__ osc, const void* __restrict__ bias, int bias_dt, void* __restrict__ yv) {
  using namespace d256;
  constexpr int XT = BCFFT_BF16;
  constexpr int ES = 2, ESY = 2;
  constexpr int PF = 8;                             // fragments per stage-2 pass

  __shared__ __attribute__((aligned(16))) char lds[LDSG_BYTES];
  int* wsc = reinterpret_cast<int*>(lds + SC_OFF);
  const float2* cs_l = reinterpret_cast<const float2*>(lds + CS_OFF);
  const float* osl = reinterpret_cast<const float*>(lds + OSG_OFF);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // GLU (fused gate/up + SwiGLU): n_out counts h blocks and the spectra hold ceil(n_out / 16)
  // STAT groups of 16 gate + 16 up blocks (bcfft.ops.glu_weights). Virtual group v takes gate
  // blocks 16 (v >> 1) + 8 (v & 1) + [0, 8) in output columns 0-7 and the matching up blocks in
  // columns 8-15, so stage 3 pairs gate and up with one DPP row rotation and stores 8 h rows.
  const int n_groups = GLU ? 2 * ((n_out + 15) / 16) : (n_out + NOB - 1) / NOB;
  const int64_t M = (int64_t)n_out * B;
  const int64_t n_mtiles = (n_tokens + TT - 1) / TT;
  const int64_t gstride = gridDim.x;
  const uint32_t lds_base = __builtin_amdgcn_readfirstlane(lds_addr(lds));
  const uint4* bimg = reinterpret_cast<const uint4*>(stat + 4);

  auto dma_token = [&](int64_t m, char* region) {
    const int64_t tok = m * TT + wave;
    const bool ok = tok < n_tokens;
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<char*>((const char*)xv) + (ok ? tok : 0) * K * ES, 0, ok ? K * ES : 0, 0x00020000);
    const int dl = opaque(lane);
    const uint32_t dst0 = lds_base + (uint32_t)(region - lds) + wave * SLOT;
    int vb[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int h = dl >> 5;
      vb[c] = h * 512 + 16 * ((dl & 31) ^ ((2 * c + h) & 15));
    }
#pragma unroll
    for (int q = 0; q < NDMA; ++q) {
      uint32_t keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen" BCFFT_XPOL " lds\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep) : "v"(vb[q & 7]), "s"(xrs), "s"(dst0 + q * 1024), "s"(q * 1024) : "memory");
    }
  };

  // ---- B fragments of output group g (STAT image group g >> 1, N-tile g & 1), pass p: bins
  // 8p .. 8p + 7 of the wave (piece (fb * 1 + 0) * 2 + nt)
  typedef u32x4 Breg[PF];
  auto b_rsrc = [&](int g) {
    return __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint4*>(bimg + ((int64_t)((g >> 1) * NW + wave) * NPIECE) * 64), 0, NPIECE * 1024, 0x00020000);
  };
  auto load_pass = [&](int g, int p, Breg& br) {
    const __amdgpu_buffer_rsrc_t brs = b_rsrc(g);
    const int ol = opaque(lane);
    int vo;
    if constexpr (GLU) {                            // column c of N-tile nt: lane c + 16 (lane >> 4)
      const int o16 = ol & 15, h8 = 8 * (g & 1);
      vo = (o16 < 8 ? 0 : 1024) + 16 * (h8 + (o16 & 7) + 16 * (ol >> 4));
    } else {
      vo = ol * 16 + (g & 1) * 1024;
    }
#pragma unroll
    for (int j = 0; j < PF; ++j) br[j] = __builtin_amdgcn_raw_buffer_load_b128(brs, vo, (8 * p + j) * 2048, 0);
  };

  // ---- prologue: the first tile's x, the tables, every group's inverse weight scales, the first
  // group's first B pass
  Breg breg[2];
  const int64_t m0 = blockIdx.x;
  if (m0 < n_mtiles) dma_token(m0, lds);
  {
    const uint4* tab = reinterpret_cast<const uint4*>(kDmF);
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int c = tid + 512 * r;
      const int t = c >> 4, ch = c & 15;
      *reinterpret_cast<uint4*>(lds + F_OFF + 256 * t + 16 * (ch ^ fsw(t))) = tab[c];
    }
    if (tid < 128) {
      double sn, cn;
      sincospi((double)tid / 128.0, &sn, &cn);
      reinterpret_cast<float2*>(lds + CS_OFF)[tid] = make_float2((float)cn, (float)sn);
    }
    for (int e = tid; e < n_groups * NOB; e += 512) reinterpret_cast<float*>(lds + OSG_OFF)[e] = osc[e];
  }
  wait_vmcnt<0>();
  load_pass(0, 0, breg[0]);
  lds_barrier();

  auto stage1 = [&](char* region, int par) {
    const int l = opaque(lane);
    const int b16 = l & 15, g = l >> 4;
    char* slot = region + wave * SLOT;
    const int q4 = (l & 15) >> 2, p4 = l & 3;
    const int cx = (p4 >> 1) ^ fsw(8 * g + q4);
    const int trb = F_OFF + 256 * (8 * g + q4) + 8 * (p4 & 1);
    const char* rowp = slot + b16 * (B * ES);
    // x[4 quarter + ...]: unit (8 qt + 4 ks + g) of the row, 8 bf16 each
    uint32_t xr[4][2][4];
#pragma unroll
    for (int qt = 0; qt < 4; ++qt)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const uint4 w = *reinterpret_cast<const uint4*>(rowp + 16 * ((8 * qt + 4 * ks + g) ^ b16));
        xr[qt][ks][0] = w.x; xr[qt][ks][1] = w.y; xr[qt][ks][2] = w.z; xr[qt][ks][3] = w.w;
      }
    float m0f = 0.f, m1f = 0.f;                     // max |x| over the token
#pragma unroll
    for (int qt = 0; qt < 4; ++qt)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int e = 0; e < 4; e += 2) {
          const float2 f0 = unpack16<XT>(xr[qt][ks][e]), f1 = unpack16<XT>(xr[qt][ks][e + 1]);
          m0f = amax3(m0f, f0.x, f0.y);
          m1f = amax3(m1f, f1.x, f1.y);
        }
    const float mxf = __builtin_fmaxf(m0f, m1f);
    // |a + a'|, |p +- p'|, |q +- q'| <= 4 max |x|
    const int sx = stat_scale_exp(4.f * __uint_as_float(wave_umax(__float_as_uint(mxf))));
    if (l < 2) wsc[par * 16 + wave * 2 + l] = sx - 7;   // X = D 2^-(sx - 7): the table's 2^-7
    const float S = __int_as_float((sx + 127) << 23);
    // B fragments (8 t each) of the six transform inputs per K-step
    uint32_t fa[2][2][4], fp[2][2][4], fq[2][2][4];   // [ks][prime / double prime][e]
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const float4* csp = reinterpret_cast<const float4*>(cs_l + 32 * ks + 8 * g);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float4 cs2 = csp[e];                   // (cos, sin) of t = 32 ks + 8 g + 2 e, + 1
        const float2 x0 = unpack16<XT>(xr[0][ks][e]), x1 = unpack16<XT>(xr[1][ks][e]);
        const float2 x2 = unpack16<XT>(xr[2][ks][e]), x3 = unpack16<XT>(xr[3][ks][e]);
        float ap[2], app[2], pp[2], ppp[2], qp[2], qpp[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const float xt = h ? x0.y : x0.x, xt64 = h ? x1.y : x1.x, xt128 = h ? x2.y : x2.x, xt192 = h ? x3.y : x3.x;
          const float c = h ? cs2.z : cs2.x, s = h ? cs2.w : cs2.y;
          const float u = (xt + xt128) * S, v = (xt64 + xt192) * S;
          const float d0 = (xt - xt128) * S, d1 = (xt64 - xt192) * S;
          ap[h] = u + v;
          app[h] = u - v;
          pp[h] = fmaf(d0, c, -d1 * s);             // p_t + p_{t+64}
          ppp[h] = fmaf(d0, c, d1 * s);             // p_t - p_{t+64}
          qp[h] = -fmaf(d0, s, d1 * c);             // q_t + q_{t+64}
          qpp[h] = fmaf(d1, c, -d0 * s);            // q_t - q_{t+64}
        }
        fa[ks][0][e] = pk_rne(ap[0], ap[1]);
        fa[ks][1][e] = pk_rne(app[0], app[1]);
        fp[ks][0][e] = pk_rne(pp[0], pp[1]);
        fp[ks][1][e] = pk_rne(ppp[0], ppp[1]);
        fq[ks][0][e] = pk_rne(qp[0], qp[1]);
        fq[ks][1][e] = pk_rne(qpp[0], qpp[1]);
      }
    }
    // X write lane bases: D^T row 4 g + r of tile (pr, mt) is b = 128 packed bin
    // f = 16 mt + 4 g + pr (+ 2 for r >= 2): b = 256 bin 2 f (a) or 2 f + 1 (p, q)
    // pass 1: the a rows -> even bins
    {
      f32x4 acc[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int pr = 0; pr < 2; ++pr)
#pragma unroll
          for (int mt = 0; mt < 4; ++mt) {
            const int cb = 16 * ((8 * pr + 2 * mt) ^ cx);
            const char* p0 = lds + trb + 256 * 32 * ks + cb;
            const s16x4 r0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p0));
            const s16x4 r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p0 + 256 * 4));
            const f16x8 af = __builtin_bit_cast(f16x8, __builtin_shufflevector(r0, r1, 0, 1, 2, 3, 4, 5, 6, 7));
            acc[4 * pr + mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
                af, frag(fa[ks][pr][0], fa[ks][pr][1], fa[ks][pr][2], fa[ks][pr][3]), acc[4 * pr + mt], 0, 0, 0);
          }
      // stage-1 outputs of pass 2 (p, q) come from the same registers-only inputs, so the even
      // X units may overwrite the x rows now: every x read of this wave is done (in-order DS)
#pragma unroll
      for (int pr = 0; pr < 2; ++pr)
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          const int f = 16 * mt + 4 * g + pr;
          *reinterpret_cast<uint32_t*>(slot + xunit(2 * f, 0) + 4 * b16) = pk_rne(acc[4 * pr + mt][0], acc[4 * pr + mt][1]);
          *reinterpret_cast<uint32_t*>(slot + xunit(2 * f + 4, 0) + 4 * b16) = pk_rne(acc[4 * pr + mt][2], acc[4 * pr + mt][3]);
        }
    }
    // pass 2: the p and q rows -> odd bins X_{2f+1} = P_f + i Q_f (bin 1: (P_0, Q_0))
    {
      f32x4 accp[8], accq[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        accp[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        accq[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int pr = 0; pr < 2; ++pr)
#pragma unroll
          for (int mt = 0; mt < 4; ++mt) {
            const int cb = 16 * ((8 * pr + 2 * mt) ^ cx);
            const char* p0 = lds + trb + 256 * 32 * ks + cb;
            const s16x4 r0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p0));
            const s16x4 r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p0 + 256 * 4));
            const f16x8 af = __builtin_bit_cast(f16x8, __builtin_shufflevector(r0, r1, 0, 1, 2, 3, 4, 5, 6, 7));
            accp[4 * pr + mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
                af, frag(fp[ks][pr][0], fp[ks][pr][1], fp[ks][pr][2], fp[ks][pr][3]), accp[4 * pr + mt], 0, 0, 0);
            accq[4 * pr + mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
                af, frag(fq[ks][pr][0], fq[ks][pr][1], fq[ks][pr][2], fq[ks][pr][3]), accq[4 * pr + mt], 0, 0, 0);
          }
#pragma unroll
      for (int pr = 0; pr < 2; ++pr)
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          const f32x4 P = accp[4 * pr + mt], Q = accq[4 * pr + mt];
          const int f = 16 * mt + 4 * g + pr;
          float re0 = P[0] - Q[1], im0 = P[1] + Q[0];
          if (mt == 0 && pr == 0 && g == 0) {       // packed bin 0 = (P_0, P_64): X_1 = P_0 + i Q_0
            re0 = P[0];
            im0 = Q[0];
          }
          *reinterpret_cast<uint32_t*>(slot + xunit(2 * f + 1, 0) + 4 * b16) = pk_rne(re0, im0);
          *reinterpret_cast<uint32_t*>(slot + xunit(2 * f + 5, 0) + 4 * b16) = pk_rne(P[2] - Q[3], P[3] + Q[2]);
        }
    }
  };

  // ---- A fragments of the wave's bins k = 16 wave + fb for all 8 tokens, once per tile
  // (bc_forward_dm256_kernel's stage-2 operand: re rows [Xr, Xi], im rows [Xi, -Xr]; bin 0 with
  // the extra 1/2; one scale per token, so no alignment)
  f16x8 areg[BPW];
  auto load_a = [&](char* region) {
    const int ml = opaque(lane);
    const int arow = ml & 15, kb = ml >> 4;
    const int a_t = arow >> 1, a_reim = arow & 1;
    const uint32_t a_sel = a_reim ? 0x01000302u : 0x03020100u;
    const uint32_t hh = 15u << 10, h0 = 14u << 10;
    const uint32_t amul = a_reim ? (hh | ((hh | 0x8000u) << 16)) : (hh | (hh << 16));
    const uint32_t amul0 = a_reim ? (h0 << 16) : h0;
    const char* ab = region + a_t * SLOT + 16 * kb;
#pragma unroll
    for (int fb = 0; fb < BPW; ++fb) {
      const int k = wave * BPW + fb;
      uint4 raw = *reinterpret_cast<const uint4*>(ab + xunit(k, 0));
      if (k == 0) {
        raw.x = pkmul(raw.x, amul0); raw.y = pkmul(raw.y, amul0);
        raw.z = pkmul(raw.z, amul0); raw.w = pkmul(raw.w, amul0);
      } else {
        raw.x = pkmul(__builtin_amdgcn_perm(raw.x, raw.x, a_sel), amul);
        raw.y = pkmul(__builtin_amdgcn_perm(raw.y, raw.y, a_sel), amul);
        raw.z = pkmul(__builtin_amdgcn_perm(raw.z, raw.z, a_sel), amul);
        raw.w = pkmul(__builtin_amdgcn_perm(raw.w, raw.w, a_sel), amul);
      }
      areg[fb] = __builtin_bit_cast(f16x8, raw);
    }
  };

  // ---- stage 2 of group g: two passes of 8 bins over the double-buffered B registers (both in
  // flight on entry); Y units (bc_forward_dm256_kernel's map) into the tile's slots
  auto stage2 = [&](char* region) {
    constexpr float YS = 1.f / 2097152.f;
    uint32_t yh[BPW][2];
#pragma unroll
    for (int fb = 0; fb < BPW; ++fb) {
      const f32x4 acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(areg[fb], __builtin_bit_cast(f16x8, breg[fb >> 3][fb & 7]),
                                                                f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) yh[fb][s2] = pk_rne(acc[2 * s2] * YS, acc[2 * s2 + 1] * YS);
    }
    const int ml = opaque(lane);
    const int yt = ml >> 4;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      char* yb = region + (2 * yt + s2) * SLOT + 16 * (ml & 15);
      *reinterpret_cast<uint4*>(yb + yunit(0, wave, 0, 0)) = make_uint4(yh[0][s2], yh[4][s2], yh[8][s2], yh[12][s2]);
      *reinterpret_cast<uint4*>(yb + yunit(0, wave, 0, 1)) = make_uint4(yh[2][s2], yh[6][s2], yh[10][s2], yh[14][s2]);
      *reinterpret_cast<uint4*>(yb + yunit(1, wave, 0, 0)) = make_uint4(yh[1][s2], yh[5][s2], yh[9][s2], yh[13][s2]);
      *reinterpret_cast<uint4*>(yb + yunit(1, wave, 0, 1)) = make_uint4(yh[3][s2], yh[7][s2], yh[11][s2], yh[15][s2]);
    }
  };

  auto stage3 = [&](char* region, int par, int64_t mp, int grp, auto&& before_stores) {
    const int l = opaque(lane);
    const int o16 = l & 15, g = l >> 4;
    char* slot = region + wave * SLOT;
    const int nmin = wsc[par * 16 + wave * 2];
    const int oidx = GLU ? 32 * (grp >> 1) + (o16 < 8 ? 8 * (grp & 1) + o16 : 16 + 8 * (grp & 1) + (o16 - 8))
                         : grp * NOB + o16;
    const float ysc = __builtin_ldexpf(osl[oidx], 30 - nmin);
    // Y fragments: B[k = 8 g + j][o] of virtual wave 4 ks + g, parity pr, spectrum s
    uint4 ye[2][2], yz[2][2], yw[2][2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        ye[ks][pr] = *reinterpret_cast<const uint4*>(slot + yunit(0, 4 * ks + g, o16, pr));
        yz[ks][pr] = *reinterpret_cast<const uint4*>(slot + yunit(1, 4 * ks + g, o16, pr));
      }
    const int gx = g ^ fsw(o16);
    const char* gb = lds + F_OFF + 256 * o16;
    auto gload = [&](int mt, f16x8 (&gf)[2][2]) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int pr = 0; pr < 2; ++pr)
          gf[ks][pr] = *reinterpret_cast<const f16x8*>(gb + 4096 * mt + 16 * ((8 * pr + 4 * ks) ^ gx));
    };
    f16x8 gcur[2][2];
    gload(0, gcur);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // Y is in registers: the slot is free
    // W' = -i Z: (re, im) -> (im, -re); W and W' packed bin 0 (virtual bin 0 of wave 0: g == 0,
    // ks 0, parity 0, first pair) = (Re Z_0, 0) and (Im Z_0, 0)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        const uint4 z = yz[ks][pr];
        yw[ks][pr] = make_uint4(__builtin_amdgcn_perm(z.x, z.x, 0x01000302u) ^ 0x80000000u,
                                __builtin_amdgcn_perm(z.y, z.y, 0x01000302u) ^ 0x80000000u,
                                __builtin_amdgcn_perm(z.z, z.z, 0x01000302u) ^ 0x80000000u,
                                __builtin_amdgcn_perm(z.w, z.w, 0x01000302u) ^ 0x80000000u);
      }
    if (g == 0) {
      yw[0][0].x = yz[0][0].x >> 16;
      yz[0][0].x &= 0xffffu;
    }
    const int64_t tok = mp * TT + wave;
    const bool tok_ok = tok < n_tokens;
    const int nvalid = n_out - grp * NOB;
    // staging: row o16 (512 B = 64 units of 8 B), outputs t..t+3 (t = 16 mt + 4 g + 64 hf) in
    // unit 4 mt + g + 16 hf, t + 128 in unit 32 + ...; physical unit u ^ 2 o16
    const int sw = 2 * o16;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      f32x4 E[3], O[3];
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        E[s] = f32x4{0.f, 0.f, 0.f, 0.f};
        O[s] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        E[0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(gcur[ks][0], __builtin_bit_cast(f16x8, ye[ks][0]), E[0], 0, 0, 0);
        O[0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(gcur[ks][1], __builtin_bit_cast(f16x8, ye[ks][1]), O[0], 0, 0, 0);
        E[1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(gcur[ks][0], __builtin_bit_cast(f16x8, yz[ks][0]), E[1], 0, 0, 0);
        O[1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(gcur[ks][1], __builtin_bit_cast(f16x8, yz[ks][1]), O[1], 0, 0, 0);
        E[2] = __builtin_amdgcn_mfma_f32_16x16x32_f16(gcur[ks][0], __builtin_bit_cast(f16x8, yw[ks][0]), E[2], 0, 0, 0);
        O[2] = __builtin_amdgcn_mfma_f32_16x16x32_f16(gcur[ks][1], __builtin_bit_cast(f16x8, yw[ks][1]), O[2], 0, 0, 0);
      }
      if (mt < 3) gload(mt + 1, gcur);
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        const float4 c01 = *reinterpret_cast<const float4*>(cs_l + 16 * mt + 4 * g + 64 * hf);
        const float4 c23 = *reinterpret_cast<const float4*>(cs_l + 16 * mt + 4 * g + 64 * hf + 2);
        const float cc[4] = {c01.x, c01.z, c23.x, c23.z}, ss[4] = {c01.y, c01.w, c23.y, c23.w};
        float lo[4], hi[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float e = hf ? E[0][r] - O[0][r] : E[0][r] + O[0][r];
          const float w = hf ? E[1][r] - O[1][r] : E[1][r] + O[1][r];
          const float wp = hf ? E[2][r] - O[2][r] : E[2][r] + O[2][r];
          const float o = fmaf(cc[r], w, -ss[r] * wp);
          lo[r] = (e + o) * ysc;                    // y_t
          hi[r] = (e - o) * ysc;                    // y_{t+128}
        }
        if constexpr (GLU) {                        // gate (columns 0-7) x up (8-15), torch's roundings
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            lo[r] = round_to(lo[r], XT);
            hi[r] = round_to(hi[r], XT);
            const float ulo = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(lo[r]), 0x128, 0xF, 0xF, false));
            const float uhi = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(hi[r]), 0x128, 0xF, 0xF, false));
            lo[r] = round_to(round_to(silu(lo[r]), XT) * ulo, XT);
            hi[r] = round_to(round_to(silu(hi[r]), XT) * uhi, XT);
          }
        } else if (HB) {                            // .to(x dtype) :266, + bias :270-271
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            lo[r] = round_to(lo[r], XT);
            hi[r] = round_to(hi[r], XT);
          }
          if (o16 < nvalid) {
            const int64_t cc0 = (int64_t)(grp * NOB + o16) * B + 16 * mt + 4 * g + 64 * hf;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              lo[r] += load_scalar(bias, cc0 + r, bias_dt);
              hi[r] += load_scalar(bias, cc0 + 128 + r, bias_dt);
            }
          }
        }
        if (GLU && o16 >= 8) continue;              // GLU: the up columns stage nothing
        const int u = 4 * mt + g + 16 * hf;
        *reinterpret_cast<uint2*>(slot + 512 * o16 + 8 * (u ^ sw)) = make_uint2(pack16<XT>(lo[0], lo[1]), pack16<XT>(lo[2], lo[3]));
        *reinterpret_cast<uint2*>(slot + 512 * o16 + 8 * ((u + 32) ^ sw)) = make_uint2(pack16<XT>(hi[0], hi[1]), pack16<XT>(hi[2], hi[3]));
      }
    }
    before_stores();
    // staged rows -> global: each instruction stores 1 KiB = 2 whole rows (32 lanes per row):
    // 16-B unit w of row r at physical 16-B unit w ^ r (the 8-B swizzle by 2 r keeps pairs)
    constexpr int RB = B * ESY;
    constexpr int NQ = GLU ? 4 : 8;                 // 1 KiB stores: 2 rows each
    const int64_t row0 = GLU ? 16 * (grp >> 1) + 8 * (grp & 1) : (int64_t)grp * NOB;
    const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
        (char*)yv + (tok_ok ? tok : 0) * M * ESY + row0 * RB, 0,
        tok_ok ? (int)((M - row0 * B) * ESY) : 0, 0x00020000);
    const int w = l & 31, lr = l >> 5;
    uint4 d[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int row = 2 * q + lr;
      d[q] = *reinterpret_cast<const uint4*>(slot + 512 * row + 16 * (w ^ row));
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, d[q]), yrs, (2 * q + lr) * RB + 16 * w, 0, BCFFT_YAUX);
  };

  // Pipeline per 8-token tile m (bcfft_dmg.hip's; region R = it & 1 holds its x, R' is free):
  //   LDS-DMA of x(m + stride) into R'; stage 1 of token w in R                       | Ba |
  //   A fragments -> VGPRs; B pass 1 of group 0                                        | Bx |
  //   per group g: stage 2 (Y units into R)                                            | Bb |
  //                B pass 0 of the next group (or of the next tile's group 0); stage 3
  //                of token w, B pass 1 of the next group, stores                      | Bc |
  int it = 0;
  for (int64_t m = m0; m < n_mtiles; m += gstride, ++it) {
    char* region = lds + (it & 1) * REGION;
    char* other = lds + ((it + 1) & 1) * REGION;
    const int par = it & 1;
    const bool dma = m + gstride < n_mtiles;
    if (dma) dma_token(m + gstride, other);
    stage1(region, par);
    lds_barrier();                                  // Ba: X units and scales complete
    load_a(region);
    load_pass(0, 1, breg[1]);
    lds_barrier();                                  // Bx: every wave holds its A fragments
    for (int g = 0; g < n_groups; ++g) {
      stage2(region);
      lds_barrier();                                // Bb: Y units complete
      const bool more = g + 1 < n_groups;
      if (more) load_pass(g + 1, 0, breg[0]);
      else if (dma) load_pass(0, 0, breg[0]);
      stage3(region, par, m, g, [&] {
        if (more) load_pass(g + 1, 1, breg[1]);
      });
      lds_barrier();                                // Bc: staging reads done (slots reusable)
    }
  }
}
}  // namespace bcfft

namespace bcfft {
bool dm256_eligible(int n_in, int b, int xdt, bool yf32) {
  return dm256_geometry(n_in, b) && xdt == BCFFT_BF16 && !yf32;
}

// the multi-group kernel (stage 1 once per 8-token tile) serves K = 4096 from three output groups
// of 16 blocks, up to MAXG, once its tiles fill the CUs (bcfft::multigroup_pays)
bool dm256g_taken(int64_t n, int n_in, int n_out) {
  const int groups = (n_out + d256::NOB - 1) / d256::NOB;
  return n_in == d256::NI && groups >= 3 && groups <= d256::MAXG && multigroup_pays(n, 3);
}

const char* dm256_kernel_name(int64_t n, int n_in, int n_out) {
  return dm256g_taken(n, n_in, n_out) ? "bc_forward_dm256g_kernel"
                                      : n_in == d256::NI ? "bc_forward_dm256_kernel" : "bc_forward_dm256k_kernel";
}

void launch_forward_dm256(const void* x, int64_t n, int n_in, int n_out, const void* spec, const void* bias,
                          int bias_dt, void* y, hipStream_t s) {
  const int groups = (n_out + d256::NOB - 1) / d256::NOB;
  const SpecLayout sl = spec_layout(n_out, n_in, 256);
  const int64_t n_mtiles = (n + 7) / 8;
  const int64_t total = group_grid(device_cu_count(), groups, n_mtiles);
  const uint32_t* stat = reinterpret_cast<const uint32_t*>(spec) + sl.stat_off_u32;
  const float* osc = reinterpret_cast<const float*>(spec) + sl.osc_off_u32;
  if (dm256g_taken(n, n_in, n_out)) {             // x transformed once
    const int64_t wgs = device_cu_count() < n_mtiles ? device_cu_count() : n_mtiles;
    if (bias_dt != BCFFT_NONE)
      hipLaunchKernelGGL((bc_forward_dm256g_kernel<false, true>), dim3((unsigned)wgs), dim3(512), 0, s, x, n, n_out, stat,
                         osc, bias, bias_dt, y);
    else
      hipLaunchKernelGGL((bc_forward_dm256g_kernel<false, false>), dim3((unsigned)wgs), dim3(512), 0, s, x, n, n_out, stat,
                         osc, bias, bias_dt, y);
    return;
  }
  const bool hb = bias_dt != BCFFT_NONE;
  if (n_in == d256::NI && hb)
    hipLaunchKernelGGL(bc_forward_dm256_kernel<true>, dim3((unsigned)total), dim3(512), 0, s, x, n, n_out, stat, osc,
                       bias, bias_dt, y);
  else if (n_in == d256::NI)
    hipLaunchKernelGGL(bc_forward_dm256_kernel<false>, dim3((unsigned)total), dim3(512), 0, s, x, n, n_out, stat, osc,
                       bias, bias_dt, y);
  else if (hb)
    hipLaunchKernelGGL(bc_forward_dm256k_kernel<true>, dim3((unsigned)total), dim3(512), 0, s, x, n, n_in, n_out, stat,
                       osc, bias, bias_dt, y);
  else
    hipLaunchKernelGGL(bc_forward_dm256k_kernel<false>, dim3((unsigned)total), dim3(512), 0, s, x, n, n_in, n_out, stat,
                       osc, bias, bias_dt, y);
}
}  // namespace bcfft

namespace bcfft {
// fused gate/up + SwiGLU at b = 256, K = 4096, bf16 (the multi-group kernel's GLU form): spec
// holds ceil(n_gate / 16) STAT groups of 16 gate + 16 up blocks
// the GLU form splits each 32-block group into two virtual groups of 16, whose inverse weight scales
// the kernel stages in an LDS array of MAXG groups: 2 ceil(n_gate / 16) <= MAXG (n_gate <= 512 blocks)
bool dm256_glu_eligible(int n_in, int b, int xdt, int n_gate) {
  return b == 256 && n_in == d256::NI && xdt == BCFFT_BF16 && n_gate >= 1 && 2 * ((n_gate + 15) / 16) <= d256::MAXG;
}

void launch_forward_dm256_glu(const void* x, int64_t n, int n_gate, const void* spec, void* h, hipStream_t s) {
  const int stat_groups = (n_gate + 15) / 16;
  const SpecLayout sl = spec_layout(32 * stat_groups, d256::NI, 256);
  const int64_t n_mtiles = (n + 7) / 8;
  const int64_t wgs = device_cu_count() < n_mtiles ? device_cu_count() : n_mtiles;
  const uint32_t* stat = reinterpret_cast<const uint32_t*>(spec) + sl.stat_off_u32;
  const float* osc = reinterpret_cast<const float*>(spec) + sl.osc_off_u32;
  hipLaunchKernelGGL((bc_forward_dm256g_kernel<true, false>), dim3((unsigned)wgs), dim3(512), 0, s, x, n, n_gate, stat, osc,
                     nullptr, BCFFT_NONE, h);
}
}  // namespace bcfft
