// bcfft_dm64k.hip — the DFT-on-MFMA block-circulant forward at b = 64 for K > 4096, bf16 I/O
// (gfx950): the LLaMA down projection 11008 -> 4096 at b = 64 (172 input blocks) and every other
// wide-input layer at that block size.
//
// Same operator (BlockCirculantLinear.forward, patch_llama_fft.py:226-275; per block
// src/fft_utils.py:3-34) and the same three matrix-core stages as bcfft_dm64.hip. An output
// group's fp16 spectra at K = 11008 (32 x 172 blocks x 32 bins x 4 B = 704 KiB) do not fit the
// register file, so the K axis is cut into 32-block chunks (two 16-block K-steps) and each
// chunk's B fragments (16 per wave: 4 bins x 2 K-steps x 2 N-tiles, 64 VGPRs) are streamed from
// L2 once per 16-token tile, the next step's fragment of a bin loaded into its registers as soon
// as the bin's MFMAs are issued. Per-bin products accumulate in 64 fp32 VGPRs over all chunks.
//
//  * Workgroup: 8 waves, persistent, one per CU; wave w owns tokens w and w + 8 of the tile for
//    the x DMA, stage 1 and stage 3 (so no barrier is needed between its stage 3 and the DMA
//    into the same slots), and bins 4w .. 4w + 3 in stage 2 for all 16 tokens.
//  * One step per (tile, chunk): [tile's first chunk: stage 3 of the previous tile's tokens w,
//    w + 8] -> stage 1 (issuing, per token, the x DMA of the next step's chunk into the other
//    region) | Ba | stage 2 | Bb | [last chunk: Y of the 16 tokens into the chunk's region | Be].
//  * Stage 1 on raw bf16 x: the 64-point transform as bf16 MFMAs against F 2^-7 in bf16 hi + lo
//    (round 5; it replaced an even / odd fp16 form: git history of this file before round 6).
//  * Numerics: per-(token, 16-block quarter) power-of-two scales from stage 1 with HEAD bits of
//    headroom; stage 2 aligns each quarter to the token's running reference exponent (an exact
//    fp16 power of two on the A rows) and scales the accumulator rows down once when a chunk is
//    more than 2^HEAD louder (bcfft_dmk.hip's scheme). |X| <= 2^(13 - HEAD) at b = 64, so
//    Y = acc 2^-21 <= n_in 2^8 stays below fp16's max for n_in <= 255.
//
// LDS (145,728 B): two regions x 16 token slots of 4,160 B (a token's 32-block x chunk, 32 rows x
// 128 B -> X units (2 K-steps x 2 KiB, bcfft_dm64.hip's map) -> at the tile end Y half-units ->
// y staging), the 4 KiB DFT table (stage 3), stage 1's 8 KiB bf16 A fragments, the scales.
#ifndef BCFFT_STREAM_POLICY
#define BCFFT_STREAM_POLICY 3                       // write-through y stores (level to 1 % faster; nt x loads slower, profiles/r04_ab_stream_policy_split.log)
// (the two-group workgroups (NG = 2) read x with nt on top, below: each token is read once by one
// CU, and the fragments of both groups then stay in L2: HBM reads 235 -> 201 MB for 180 MB of x,
// 116.5 -> 113.8 us at 11008 -> 4096, N = 8192; profiles/r06f_ab_dm64k_pairs_nt.log)
#endif
#include "bcfft_device.h"
#include "bcfft_dm_table.h"
#include "bcfft_dm_common.h"

namespace bcfft {

namespace dm64k {
using namespace dmh;

constexpr int B = 64, NW = 8, BW = 4, NT = 2, KC = 2, NOG = 32;
// NG output groups per workgroup (the template parameter of the kernel): NG = 1, 16-token tiles
// (two M-tiles of 8, tokens w and w + 8 per wave); NG = 2, 8-token tiles (one M-tile, token w per
// wave) whose stage 1 serves both groups' stage 2 and stage 3
template <int NG> struct Geo {
  static constexpr int TT = 16 / NG, MT = 2 / NG, TPW = 2 / NG;   // tokens per tile / M-tiles / per wave
  // token slot: the 32-block x chunk (4 KiB) -> X units -> the NG groups' Y units (4 KiB each, at
  // 4096 g) -> y staging; the stride stays 64 B off the 256-B bank period
  static constexpr int XS = NG == 1 ? 4096 + 64 : 8192 + 64;
  static constexpr int REGION = TT * XS;
  static constexpr int F_OFF = 2 * REGION;          // DFT table image, 32 rows x 128 B
  static constexpr int SC_OFF = F_OFF + 4096;       // scale exponents [TT tokens][2 quarters]
  static constexpr int RR_OFF = SC_OFF + 128;       // per-token reference exponents [TT]
  static constexpr int OS_OFF = RR_OFF + 64;        // the groups' 32 NG inverse weight scales
  static constexpr int TB_OFF = OS_OFF + 128 * NG;  // stage 1's bf16 hi + lo A fragments (kDmB64)
  static constexpr int LDS_BYTES = TB_OFF + 8192;
  static constexpr int NDMA = TPW * 4;              // 1-KiB x DMA pieces per wave and chunk
  static constexpr int NST = TPW * NG * 4;          // y stores per wave at a tile's first chunk
  static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
  static_assert(XS % 256 == 64, "slot stride 64 B off the bank period");
};
constexpr int FRAGS = BW * KC * NT;                 // B fragments per wave, chunk and group
constexpr int HEAD = 4;
// wave priority falling with the work done in stage 1 (1) and stage 2 (2) (s_setprio, 0 = lowest):
// waves 4-7, younger than their SIMD partners 0-3, lose every age-ordered arbitration and finished
// both stages ~1.1 k cycles later; with the priority a wave that is behind issues first (117.7 vs
// 119.6 us at N = 8192, profiles/r05ll_ab_dm64k_prio.log)
constexpr int PRIO = 3;
// analysis builds only (results are WRONG when set): 1 no B loads, 2 no stage-1 arithmetic, 4 no
// stage-2 MFMAs, 8 no stage 3, 16 no x DMA, 32 no y stores
#ifdef BCFFT_DM64K_ABL
constexpr int ABL = BCFFT_DM64K_ABL;
#else
constexpr int ABL = 0;
#endif

__device__ __forceinline__ int fsw64(int t) { return (((t >> 1) & 1) << 1) | (((t >> 3) & 1) << 2); }
__device__ __forceinline__ int yhalf64(int w, int o, int par) { return 2048 * par + 256 * w + 8 * (o ^ (16 * ((w >> 1) & 1))); }
// fp16 factor 2^-d (d >= -15) as a (lo, hi) pair: subnormal below 2^-14, zero below 2^-24
__device__ __forceinline__ uint32_t f16_pow2_neg(int d) {
  return d <= 14 ? (uint32_t)(15 - d) << 10 : (d <= 24 ? 1u << (24 - d) : 0u);
}
// fp16 pair (a s, b s), each rounded once (v_fma_mix: f32 operands, f16 result in a half)
__device__ __forceinline__ uint32_t pk_scaled(float a, float b, float s) {
  uint32_t r;
  asm("v_fma_mixlo_f16 %0, %1, %3, 0\n\tv_fma_mixhi_f16 %0, %2, %3, 0" : "=&v"(r) : "v"(a), "v"(b), "v"(s));
  return r;
}
// per-half max of the bf16 magnitudes of two packed pairs (v_pk_max_u16 on the sign-cleared bits)
typedef __attribute__((ext_vector_type(2))) unsigned short u16x2;
__device__ __forceinline__ uint32_t pk_umax(uint32_t m, uint32_t w) {
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(u16x2, m),
                                                                __builtin_bit_cast(u16x2, w & 0x7fff7fffu)));
}
}  // namespace dm64k

// HB: a bias is added (the runtime bias_dt then names its dtype); without one the store path is
// straight-line (a runtime test per stored quad split stage 3 into hundreds of basic blocks)
// NG: output groups per workgroup (dm64k::Geo); NG = 2 needs an even group count
template <bool HB, int NG>
__global__ __launch_bounds__(512, 2) void bc_forward_dm64k_kernel(
    const void* __restrict__ xv, int64_t n_tokens, int n_in, int n_out, const uint32_t* __restrict__ stat,
    const float* __restrict__ osc, const void* __restrict__ bias, int bias_dt, void* __restrict__ yv) {
  using namespace dm64k;
  using G = Geo<NG>;
  constexpr int XT = BCFFT_BF16;
  constexpr int ES = 2, ESY = 2;
  constexpr int TT = G::TT, MT = G::MT, TPW = G::TPW, XS = G::XS, REGION = G::REGION;
  constexpr int F_OFF = G::F_OFF, SC_OFF = G::SC_OFF, RR_OFF = G::RR_OFF, OS_OFF = G::OS_OFF, TB_OFF = G::TB_OFF;
  constexpr int LDS_BYTES = G::LDS_BYTES, NDMA = G::NDMA, NST = G::NST;

  __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];
  int* wsc = reinterpret_cast<int*>(lds + SC_OFF);
  int* wrr = reinterpret_cast<int*>(lds + RR_OFF);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n_groups = (n_out + NOG - 1) / NOG;
  const GroupMap gm = group_map((n_groups + NG - 1) / NG);
  const int sgrp = gm.grp, wg_in_grp = gm.lane;     // groups NG sgrp .. NG sgrp + NG - 1
  const int64_t KX = (int64_t)n_in * B;
  const int64_t M = (int64_t)n_out * B;
  const int nch = (n_in + 31) / 32;
  const int KS = (n_in + 15) / 16;                  // K-steps of the STAT image
  const int64_t n_mtiles = (n_tokens + TT - 1) / TT;
  const int gstride = gm.stride;
  const uint32_t lds_base = __builtin_amdgcn_readfirstlane(lds_addr(lds));
  ANALYSIS_INIT;

  // ---- chunk c of token w + 8 t2 of M-tile m -> its slot by LDS-DMA: piece q = rows 8q +
  // (lane >> 3) of 128 B, unit u of row r at u ^ (r & 7); the buffer range ends at the row end, so
  // a partial last chunk and tokens / tiles past the end land as zeros. Issued inside stage 1
  // (which has no other VMEM), so that its issue cost overlaps the stage's MFMAs
  auto dma_tok = [&](int64_t m, int c, char* region, int t2) {
    const int tl = wave + 8 * t2;
    if constexpr ((ABL & 16) != 0) {                // keep the VMEM count: 4 empty-range loads
      const __amdgpu_buffer_rsrc_t zr = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(xv), 0, 0, 0x00020000);
      const uint32_t d0 = lds_base + (uint32_t)(region - lds) + tl * XS;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        uint32_t keep;
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen" BCFFT_XPOL " lds\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(0), "s"(zr), "s"(d0) : "memory");
      }
      return;
    }
    const int dl = opaque(lane);
    const int r = dl >> 3;
    const int vb = r * 128 + 16 * ((dl & 7) ^ r);
    const int64_t tok = m * TT + tl;
    const bool ok = m < n_mtiles && tok < n_tokens;
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<char*>((const char*)xv) + (ok ? tok * KX * ES + (int64_t)c * 4096 : 0), 0,
        ok ? (int)(KX * ES - (int64_t)c * 4096) : 0, 0x00020000);
    const uint32_t dst0 = lds_base + (uint32_t)(region - lds) + tl * XS;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      uint32_t keep;
      if constexpr (NG == 2)
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen nt lds\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(vb), "s"(xrs), "s"(dst0 + q * 1024), "s"(q * 1024) : "memory");
      else
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen" BCFFT_XPOL " lds\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(vb), "s"(xrs), "s"(dst0 + q * 1024), "s"(q * 1024) : "memory");
    }
  };

  // ---- B fragments (STAT image group NG sgrp + g, wave, piece (fb KS + 2c + j) 2 + nt), asm loads
  // counted by hand (bcfft_dmk.hip's scheme): wait_b is their one wait, with the exact number of
  // younger VMEM operations, and it redefines the registers it waited for
  const int npiece = BW * KS * NT;
  __amdgpu_buffer_rsrc_t brs[NG];
#pragma unroll
  for (int g = 0; g < NG; ++g)
    brs[g] = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint32_t*>(stat + 4) + ((int64_t)((NG * sgrp + g) * NW + wave) * npiece) * 256, 0, npiece * 1024,
        0x00020000);
  // fragment (fb, j, nt) of group g, chunk c; K-step 2c + 1 past the image (odd KS, last chunk)
  // reads zeros
  auto load_b1 = [&](int g, int c, int fb, int j, int nt, u32x4 (&breg)[BW][KC][NT], bool live) {
    const int ks = 2 * c + j;
    const int vo = opaque(lane) * 16 + (live && ks < KS && (ABL & 1) == 0 ? (fb * KS + ks) * 2 + nt : npiece) * 1024;
    asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(breg[fb][j][nt]) : "v"(vo), "s"(brs[g]));
  };
  // NG = 2: the wait for one bin's four fragments, with the number of younger loads (always 12:
  // the later bins of the same group, then the next group's fragments of the earlier bins)
  auto wait_bin = [&](int fb, u32x4 (&breg)[BW][KC][NT]) {
    asm volatile("s_waitcnt vmcnt(12) ; bcfft-wait %0 %1 %2 %3"
                 : "+v"(breg[fb][0][0]), "+v"(breg[fb][0][1]), "+v"(breg[fb][1][0]), "+v"(breg[fb][1][1]) :: "memory");
  };
  auto wait_b = [&](auto n_tag, u32x4 (&breg)[BW][KC][NT]) {
    constexpr int N = decltype(n_tag)::value;
    static_assert(N >= 0 && N < 64, "vmcnt");
    asm volatile("s_waitcnt vmcnt(%16) ; bcfft-wait %0 %1 %2 %3 %4 %5 %6 %7 %8 %9 %10 %11 %12 %13 %14 %15"
                 : "+v"(breg[0][0][0]), "+v"(breg[0][0][1]), "+v"(breg[0][1][0]), "+v"(breg[0][1][1]),
                   "+v"(breg[1][0][0]), "+v"(breg[1][0][1]), "+v"(breg[1][1][0]), "+v"(breg[1][1][1]),
                   "+v"(breg[2][0][0]), "+v"(breg[2][0][1]), "+v"(breg[2][1][0]), "+v"(breg[2][1][1]),
                   "+v"(breg[3][0][0]), "+v"(breg[3][0][1]), "+v"(breg[3][1][0]), "+v"(breg[3][1][1])
                 : "n"(N) : "memory");
  };
  static_assert(FRAGS == 16, "wait_b names sixteen fragments");

  // ---- prologue: the first tile's chunk 0, the DFT table, the inverse weight scales
  dma_tok(wg_in_grp, 0, lds, 0);
  dma_tok(wg_in_grp, 0, lds, 1);
  if (tid < 256) {                                  // chunk c: row c >> 3, chunk c & 7
    const uint4* tab = reinterpret_cast<const uint4*>(kDmF64);
    const int t = tid >> 3, ch = tid & 7;
    *reinterpret_cast<uint4*>(lds + F_OFF + 128 * t + 16 * (ch ^ fsw64(t))) = tab[tid];
  }
  if (tid < 32 * NG) reinterpret_cast<float*>(lds + OS_OFF)[tid] = osc[NG * sgrp * 32 + tid];
  reinterpret_cast<uint4*>(lds + TB_OFF)[tid] = reinterpret_cast<const uint4*>(kDmB64)[tid];
  wait_vmcnt<0>();
  lds_barrier();

  // ---- stage 1 (wave w: tokens w, w + 8) on the raw bf16 x of the chunk's two quarters: the
  // 64-point transform F x as bf16 MFMAs, F 2^-7 as hi + lo A fragments (kDmB64, ~16 significant
  // bits; x_{t+32} enters the odd-bin tiles negated, F_{t+32} = -F_t there), fp32 accumulation,
  // then X 2^sx rounded once to fp16. sx is the per-(token, quarter) scale of the even / odd
  // form below (max |x| from the bf16 magnitude bits, HEAD bits lower), so X keeps its bound and
  // stage 2 is unchanged. Per quarter and lane: 17 VALU for the max and 16 for scale + rounding
  // against ~100 for unpack / scale / a, d / rounding; 16 MFMAs instead of 4, issued as soon as
  // x is read (the max reduction runs under them). Products of x below ~2^-110 fall into fp32's
  // subnormal range, as in the reference's fp32 rfft.
  auto stage1 = [&](char* region, auto&& dma) {
    if constexpr ((ABL & 2) != 0) {
#pragma unroll
      for (int t2 = 0; t2 < TPW; ++t2) {
        if (lane < 2) wsc[(wave + 8 * t2) * 2 + lane] = 0;
        dma(t2);
      }
      return;
    }
    const int l = opaque(lane);
    const int b16 = l & 15, g = l >> 4;
    int xwb[2];
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) xwb[pr] = 256 * g + 64 * (pr ^ (g & 1)) + 4 * b16;
    if constexpr ((PRIO & 1) != 0) __builtin_amdgcn_s_setprio(2);
    // the table fragments read once for both tokens (the DMA's memory clobber kept the compiler
    // from hoisting them): 16 of the 20 1-KiB LDS reads per token were these (116.2 vs 117.6 us,
    // profiles/r05rr_ab_dm64k_table_once.log)
    bf16x8 tab[2][2][2];
#pragma unroll
    for (int pr = 0; pr < 2; ++pr)
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int tm = 0; tm < 2; ++tm)
          tab[pr][mt][tm] = *reinterpret_cast<const bf16x8*>(lds + TB_OFF + 2048 * (2 * pr + mt) + 1024 * tm + 16 * l);
#pragma unroll 1
    for (int t2 = 0; t2 < TPW; ++t2) {
      const int tl = wave + 8 * t2;
      char* slot = region + tl * XS;
      uint4 xr[KC][2];
#pragma unroll
      for (int h = 0; h < KC; ++h)
#pragma unroll
        for (int pt = 0; pt < 2; ++pt)
          xr[h][pt] = *reinterpret_cast<const uint4*>(slot + (16 * h + b16) * (B * ES) + 16 * ((g + 4 * pt) ^ (b16 & 7)));
      dma(t2);                                      // the next step's x of this token slot
      f32x4 acc4[KC][4];
#pragma unroll
      for (int h = 0; h < KC; ++h) {
        const uint4 xn = make_uint4(xr[h][1].x ^ 0x80008000u, xr[h][1].y ^ 0x80008000u, xr[h][1].z ^ 0x80008000u,
                                    xr[h][1].w ^ 0x80008000u);
        const bf16x8 b0 = __builtin_bit_cast(bf16x8, xr[h][0]), b1 = __builtin_bit_cast(bf16x8, xr[h][1]);
        const bf16x8 b1n = __builtin_bit_cast(bf16x8, xn);
#pragma unroll
        for (int pr = 0; pr < 2; ++pr)
#pragma unroll
          for (int mt = 0; mt < 2; ++mt) {
            const bf16x8 th = tab[pr][mt][0], tlo = tab[pr][mt][1];
            f32x4 a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(th, b0, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
            a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tlo, b0, a, 0, 0, 0);
            a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(th, pr ? b1n : b1, a, 0, 0, 0);
            acc4[h][2 * pr + mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tlo, pr ? b1n : b1, a, 0, 0, 0);
          }
      }
      uint32_t mq[KC];
#pragma unroll
      for (int h = 0; h < KC; ++h) {
        uint32_t m0 = pk_umax(0u, xr[h][0].x), m1 = pk_umax(0u, xr[h][0].y);
        m0 = pk_umax(m0, xr[h][0].z); m1 = pk_umax(m1, xr[h][0].w);
        m0 = pk_umax(m0, xr[h][1].x); m1 = pk_umax(m1, xr[h][1].y);
        m0 = pk_umax(m0, xr[h][1].z); m1 = pk_umax(m1, xr[h][1].w);
        const uint32_t m = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(u16x2, m0),
                                                                                  __builtin_bit_cast(u16x2, m1)));
        mq[h] = max(m & 0xffffu, m >> 16) << 16;    // fp32 bits of the lane's max |x|
      }
#pragma unroll
      for (int h = 0; h < KC; ++h) mq[h] = wave_umax(mq[h]);
#pragma unroll
      for (int h = 0; h < KC; ++h) {
        const int sx = stat_scale_exp(2.f * __uint_as_float(mq[h])) - HEAD;
        if (l == 0) wsc[tl * 2 + h] = sx - 7;      // X = D 2^-(sx - 7): the table's 2^-7
        const float S = __int_as_float((sx + 127) << 23);
        char* xb = slot + 2048 * h;
#pragma unroll
        for (int pr = 0; pr < 2; ++pr)
#pragma unroll
          for (int mt = 0; mt < 2; ++mt) {
            const f32x4 v = acc4[h][2 * pr + mt];
            *reinterpret_cast<uint32_t*>(xb + xwb[pr] + 1024 * mt) = pk_scaled(v[0], v[1], S);
            *reinterpret_cast<uint32_t*>(xb + xwb[pr] + 1024 * mt + 128) = pk_scaled(v[2], v[3], S);
          }
      }
      if constexpr ((PRIO & 1) != 0) __builtin_amdgcn_s_setprio(1);
    }
  };

  // accumulators [bin of the wave][M-tile][N-tile]: rows 4 yt + r = token 8 mt + 2 yt + (r >> 1),
  // re / im r & 1; reference exponents of the A-row tokens and the accumulator-row tokens
  f32x4 acc[NG][BW][MT][NT];
#pragma unroll
  for (int g = 0; g < NG; ++g)
#pragma unroll
    for (int fb = 0; fb < BW; ++fb)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[g][fb][mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  int ra[MT], rc[MT][2];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) ra[mt] = rc[mt][0] = rc[mt][1] = 0;

  // ---- stage 2 (all waves): the chunk's per-bin complex MAC on bins 4 wave + fb for the TT
  // tokens, accumulated. NG = 1: each fragment's successor for the next step (nb >= 0) is loaded
  // into its registers after its last MFMA. NG = 2: group 0's fragments are in the registers at
  // entry; after each group-0 bin its group-1 fragments are loaded into them, and after each
  // group-1 bin the next step's group-0 ones. One call site.
  auto stage2 = [&](char* region, u32x4 (&breg)[BW][KC][NT], int c_now, int nb, bool first, bool tile0) {
    const int ml = opaque(lane);
    const int arow = ml & 15, kb = ml >> 4;
    const int a_t = arow >> 1, a_reim = arow & 1;
    const uint32_t a_sel = a_reim ? 0x01000302u : 0x03020100u;
    const int yt = ml >> 4;
    int nk[MT][KC];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int j = 0; j < KC; ++j) nk[mt][j] = wsc[(8 * mt + a_t) * 2 + j];
    if (first) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        ra[mt] = min(nk[mt][0], nk[mt][1]);
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int* sc = wsc + (8 * mt + 2 * yt + s) * 2;
          rc[mt][s] = min(sc[0], sc[1]);
        }
      }
    } else {
      float fct[MT][2];
      bool need = false;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        ra[mt] = min(ra[mt], min(nk[mt][0], nk[mt][1]) + HEAD);
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int* sc = wsc + (8 * mt + 2 * yt + s) * 2;
          const int nn = min(sc[0], sc[1]) + HEAD;
          const int d = rc[mt][s] - nn;
          fct[mt][s] = d > 0 ? __builtin_ldexpf(1.f, -d) : 1.f;
          need |= d > 0;
          rc[mt][s] = min(rc[mt][s], nn);
        }
      }
      if (__builtin_amdgcn_ballot_w64(need)) {
#pragma unroll
        for (int g = 0; g < NG; ++g)
#pragma unroll
          for (int fb = 0; fb < BW; ++fb)
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
#pragma unroll
              for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                for (int r = 0; r < 4; ++r) acc[g][fb][mt][nt][r] *= fct[mt][r >> 1];
      }
    }
    uint32_t amul[MT][KC], amul0[MT][KC];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int j = 0; j < KC; ++j) {
        const int d = nk[mt][j] - ra[mt];           // >= -HEAD: factor 2^-d <= 2^HEAD
        const uint32_t hh = f16_pow2_neg(d);
        const uint32_t h0 = f16_pow2_neg(d + 1);    // bin 0: the inverse's 1/b vs 2/b
        amul[mt][j] = a_reim ? (hh | ((hh | 0x8000u) << 16)) : (hh | (hh << 16));
        amul0[mt][j] = a_reim ? (h0 << 16) : h0;
      }
    const int sw = 64 * (wave & 1);
    // B of this step: younger VMEM is this step's x DMA and, at a tile's first chunk, the
    // previous tile's stage-3 stores before it. One operand-carrying wait on every path (a wait
    // per branch made the compiler copy the 16 fragments where the paths join)
    if (!tile0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NDMA) : "memory");
    wait_b(std::integral_constant<int, NST + NDMA>{}, breg);
    const bool more = nb >= 0;
    const int nc = more ? nb : 0;
    // A rows of bin 4 wave + fb: X units of the 8 tokens of M-tile mt, K-step j; the next bin's
    // four units are read while this bin's are scaled and multiplied (LDS latency off the chain)
    const char* abase = region + a_t * XS + 256 * wave + 16 * kb;
    auto a_off = [&](int fb, int j, int mt) { return 8 * mt * XS + ((fb & 1) ? -sw : sw) + 64 * fb + 2048 * j; };
    const bool bin0 = wave == 0;                    // bin 0 (wave 0, fb 0): (X_0, X_32), no swap
    // NG = 2 (one M-tile): group 0's scaled A rows are kept for group 1
    f16x8 acache[NG == 2 ? BW : 1][KC];
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const bool reuse = NG == 2 && g == 1;
      uint4 araw[2][KC][MT];
      if (!reuse) {
#pragma unroll
        for (int j = 0; j < KC; ++j)
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) araw[0][j][mt] = *reinterpret_cast<const uint4*>(abase + a_off(0, j, mt));
      }
#pragma unroll
      for (int fb = 0; fb < BW; ++fb) {
        if constexpr ((PRIO & 2) != 0) set_prio(3 - (fb + g * BW) * 4 / (NG * BW));
        if (!reuse && fb + 1 < BW) {
#pragma unroll
          for (int j = 0; j < KC; ++j)
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
              araw[(fb + 1) & 1][j][mt] = *reinterpret_cast<const uint4*>(abase + a_off(fb + 1, j, mt));
        }
        if (NG == 2 && g == 1) wait_bin(fb, breg);   // this bin's group-1 fragments
        const uint32_t sel = (fb == 0 && bin0) ? 0x03020100u : a_sel;
#pragma unroll
        for (int j = 0; j < KC; ++j) {
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) {
            f16x8 a;
            if (reuse) {
              a = acache[fb][j];
            } else {
              const uint32_t mul = (fb == 0 && bin0) ? amul0[mt][j] : amul[mt][j];
              uint4 raw = araw[fb & 1][j][mt];
              raw.x = pkmul(__builtin_amdgcn_perm(raw.x, raw.x, sel), mul);
              raw.y = pkmul(__builtin_amdgcn_perm(raw.y, raw.y, sel), mul);
              raw.z = pkmul(__builtin_amdgcn_perm(raw.z, raw.z, sel), mul);
              raw.w = pkmul(__builtin_amdgcn_perm(raw.w, raw.w, sel), mul);
              a = __builtin_bit_cast(f16x8, raw);
              if (NG == 2) acache[fb][j] = a;
            }
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
              if constexpr ((ABL & 4) != 0)
                acc[g][fb][mt][nt] += f32x4{a[0], a[1], __builtin_bit_cast(f16x8, breg[fb][j][nt])[0], 0.f};
              else
                acc[g][fb][mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, __builtin_bit_cast(f16x8, breg[fb][j][nt]),
                                                                            acc[g][fb][mt][nt], 0, 0, 0);
          }
          // the next fragments into these registers (NG = 2, group 0: group 1's of this step;
          // otherwise the next step's group 0); past the last step an empty-range load (no
          // branch, no copy)
          if (NG == 2 && g == 0) {
            load_b1(1, c_now, fb, j, 0, breg, true);
            load_b1(1, c_now, fb, j, 1, breg, true);
          } else {
            load_b1(0, nc, fb, j, 0, breg, more);
            load_b1(0, nc, fb, j, 1, breg, more);
          }
        }
      }
    }
  };

  // ---- Y of the TT tokens (fp16 half-units, bcfft_dm64.hip's map; group g's at 4096 g of the
  // slot) into their slots of a region; the reference exponents into wrr; the accumulators
  // restart at zero
  auto ywrite = [&](char* region) {
    const int ml = opaque(lane);
    const int yt = ml >> 4;
    constexpr float YS = 1.f / 2097152.f;            // 2^-21: |Y| <= n_in 2^8 < 65504 (n_in <= 255)
    if (wave == 0 && (ml & 15) == 0) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        wrr[8 * mt + 2 * yt] = rc[mt][0];
        wrr[8 * mt + 2 * yt + 1] = rc[mt][1];
      }
    }
    const int ox = 16 * ((wave >> 1) & 1);
#pragma unroll
    for (int g = 0; g < NG; ++g)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        uint32_t yh[BW][NT][2];
#pragma unroll
        for (int fb = 0; fb < BW; ++fb)
#pragma unroll
          for (int nt = 0; nt < NT; ++nt)
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2)
              yh[fb][nt][s2] = pk_rne(acc[g][fb][mt][nt][2 * s2] * YS, acc[g][fb][mt][nt][2 * s2 + 1] * YS);
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          char* yb = region + (8 * mt + 2 * yt + s2) * XS + 4096 * g + 256 * wave;
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) {         // yhalf64(wave, 16 nt + o16, par)
            const int oo = 8 * ((16 * nt + (ml & 15)) ^ ox);
            *reinterpret_cast<uint2*>(yb + oo) = make_uint2(yh[0][nt][s2], yh[2][nt][s2]);
            *reinterpret_cast<uint2*>(yb + 2048 + oo) = make_uint2(yh[1][nt][s2], yh[3][nt][s2]);
          }
        }
      }
#pragma unroll
    for (int g = 0; g < NG; ++g)
#pragma unroll
      for (int fb = 0; fb < BW; ++fb)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) acc[g][fb][mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  };

  // ---- stage 3 (token slot tl of a region, group g of the workgroup's, reference exponent rref):
  // bcfft_dm64.hip's stage 3; tok < 0 stores nothing (the stores are still issued, with an empty
  // range)
  auto stage3 = [&](char* region, int tl, int gi, int rref, int64_t tok) {
    if constexpr ((ABL & 8) != 0) {                 // keep the VMEM count: 4 empty-range stores
      const __amdgpu_buffer_rsrc_t zr = __builtin_amdgcn_make_buffer_rsrc(yv, 0, 0, 0x00020000);
#pragma unroll
      for (int q = 0; q < 4; ++q) __builtin_amdgcn_raw_buffer_store_b128(u32x4{0u, 0u, 0u, 0u}, zr, 0, 0, 0);
      return;
    }
    const int l = opaque(lane);
    const int o16 = l & 15, g = l >> 4;
    char* slot = region + tl * XS + 4096 * gi;
    const int grp_o = NG * sgrp + gi;
    float ysc[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) ysc[nt] = __builtin_ldexpf(reinterpret_cast<const float*>(lds + OS_OFF)[32 * gi + 16 * nt + o16], 30 - rref);
    uint4 yf[2][NT];
#pragma unroll
    for (int pr = 0; pr < 2; ++pr)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const int o = 16 * nt + o16;
        const uint2 lo = *reinterpret_cast<const uint2*>(slot + yhalf64(2 * g, o, pr));
        const uint2 hi = *reinterpret_cast<const uint2*>(slot + yhalf64(2 * g + 1, o, pr));
        yf[pr][nt] = make_uint4(lo.x, lo.y, hi.x, hi.y);
      }
    f16x8 gt[2][2];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        const int t = 16 * mt + o16;
        gt[mt][pr] = *reinterpret_cast<const f16x8*>(lds + F_OFF + 128 * t + 16 * ((4 * pr + g) ^ fsw64(t)));
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // Y is in registers: the slot is free
    const bool tok_ok = tok >= 0 && tok < n_tokens && (ABL & 32) == 0;
    const int nvalid = n_out - grp_o * NOG;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      f32x4 E[NT], O[NT];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        E[nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(gt[mt][0], __builtin_bit_cast(f16x8, yf[0][nt]), f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        O[nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(gt[mt][1], __builtin_bit_cast(f16x8, yf[1][nt]), f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      }
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const int o = 16 * nt + o16;
        float os[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) os[r] = O[nt][r] * ysc[nt];
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = hf ? fmaf(E[nt][r], ysc[nt], -os[r]) : fmaf(E[nt][r], ysc[nt], os[r]);
          if (HB) {                                 // .to(x dtype) :266, + bias :270-271
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = round_to(v[r], XT);
            if (o < nvalid) {
              const int64_t cc = (int64_t)(grp_o * NOG + o) * B + 16 * mt + 4 * g + 32 * hf;
#pragma unroll
              for (int r = 0; r < 4; ++r) v[r] += load_scalar(bias, cc + r, bias_dt);
            }
          }
          *reinterpret_cast<uint2*>(slot + 128 * o + 8 * ((4 * mt + g + 8 * hf) ^ o16)) =
              make_uint2(pack16<XT>(v[0], v[1]), pack16<XT>(v[2], v[3]));
        }
      }
    }
    constexpr int RB = B * ESY;
    const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
        (char*)yv + (tok_ok ? tok : 0) * M * ESY + (int64_t)grp_o * NOG * RB, 0,
        tok_ok ? (int)((M - (int64_t)grp_o * NOG * B) * ESY) : 0, 0x00020000);
    const int w = l & 7, lr = l >> 3;
    const int vofs = lr * RB + 16 * w;
    uint4 d[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int rr = 8 * q + lr;
      uint4 v = *reinterpret_cast<const uint4*>(slot + 128 * rr + 16 * (w ^ ((rr & 15) >> 1)));
      if (lr & 1) v = make_uint4(v.z, v.w, v.x, v.y);
      d[q] = v;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, d[q]), yrs, vofs + q * 1024, 0, BCFFT_YAUX);
  };

  // Pipeline: one step per (M-tile m of 16 tokens, chunk c), two barriers per step (rsel: the
  // region holding chunk c's x; the other holds the previous chunk's X or, at c = 0, the
  // previous tile's Y units):
  //   c = 0   stage 3 of the previous tile's tokens w, w + 8 from the other region (8 stores)
  //           x(m, c) landed; stage 1, per token slot issuing the x DMA of the next step's
  //           chunk into the other region (zeros past the last tile)                         | Ba |
  //           stage 2 on B(c) (loaded in the previous step), loading the next step's B      | Bb |
  //   c last  Y of the tile into this region                                                 | Be |
  // VMEM younger than x(m, c) when it is waited for: B(c) 16 (the previous step's stage 2) and,
  // at c = 0, the NST stores (the first step's x and B were waited for up front); NG = 2: B(c) is
  // both groups' fragments (group 1 of this step and group 0 of the next, 2 FRAGS).
  u32x4 breg[BW][KC][NT];
#pragma unroll
  for (int fb = 0; fb < BW; ++fb)
#pragma unroll
    for (int j = 0; j < KC; ++j) {
      load_b1(0, 0, fb, j, 0, breg, true);
      load_b1(0, 0, fb, j, 1, breg, true);
    }
  wait_vmcnt<0>();
  int rsel = 0;
  int64_t mprev = -1;
  int64_t m = wg_in_grp;
  int c = 0;
  // stamps build: slots 8 c + phase for the steps of the workgroup's second tile
  [[maybe_unused]] int tcount = 0;
#define DST(o) do { if (tcount == 1 && c < 7) STAMP(8 * c + (o)); } while (0)
  while (m < n_mtiles) {
    char* region = lds + rsel * REGION;
    char* other = lds + (rsel ^ 1) * REGION;
    const bool tile0 = c == 0;
    DST(0);
    if (tile0) {
#pragma unroll
      for (int t2 = 0; t2 < TPW; ++t2)
#pragma unroll
        for (int g = 0; g < NG; ++g)
          stage3(other, wave + 8 * t2, g, wrr[wave + 8 * t2], mprev >= 0 ? mprev * TT + wave + 8 * t2 : -1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the slots' staging reads are done
    }
    DST(1);
    const bool last = c + 1 == nch;
    const int64_t mn = last ? m + gstride : m;
    const int cn = last ? 0 : c + 1;
    DST(2);
    // x(m, c) landed: younger VMEM is B(c) (the previous step's stage 2) and, at c = 0, the stores
    if (tile0) wait_vmcnt<NG * FRAGS + NST>();
    else wait_vmcnt<NG * FRAGS>();
    DST(3);
    stage1(region, [&](int t2) { dma_tok(mn, cn, other, t2); });
    DST(4);
    lds_barrier();                                  // Ba: X units and quarter scales complete
    DST(5);
    stage2(region, breg, c, mn < n_mtiles ? cn : -1, tile0, tile0);
    DST(6);
    lds_barrier();                                  // Bb: every read of this chunk's X done
    DST(7);
    if (last) {
      ywrite(region);
      lds_barrier();                                // Be: Y units and reference exponents
      mprev = m;
      ++tcount;
    }
    rsel ^= 1;
    m = mn;
    c = cn;
  }
  char* yreg = lds + (rsel ^ 1) * REGION;
#pragma unroll
  for (int t2 = 0; t2 < TPW; ++t2)
#pragma unroll
    for (int g = 0; g < NG; ++g)
      stage3(yreg, wave + 8 * t2, g, wrr[wave + 8 * t2], mprev >= 0 ? mprev * TT + wave + 8 * t2 : -1);
  // the last step's empty-range B loads: waited for with the fragments as operands, so that their
  // registers stay reserved (not reused by ywrite / stage 3) until the loads have returned
  wait_b(std::integral_constant<int, 0>{}, breg);
}

#undef DST

#ifndef BCFFT_DM64K_PAIRS
#define BCFFT_DM64K_PAIRS 1
#endif
bool dm64k_pairs(int groups) { return BCFFT_DM64K_PAIRS != 0 && groups % 2 == 0; }

bool dm64k_eligible(int n_in, int b, int xdt, bool yf32) {
  return dm64k_geometry(n_in, b) && xdt == BCFFT_BF16 && !yf32;
}

void launch_forward_dm64k(const void* x, int64_t n, int n_in, int n_out, const void* spec, const void* bias,
                          int bias_dt, void* y, hipStream_t s) {
  const int groups = (n_out + dm64k::NOG - 1) / dm64k::NOG;
  const SpecLayout sl = spec_layout(n_out, n_in, 64);
  const uint32_t* stat = reinterpret_cast<const uint32_t*>(spec) + sl.stat_off_u32;
  const float* osc = reinterpret_cast<const float*>(spec) + sl.osc_off_u32;
  const int cus = device_cu_count();
  // an even group count: two groups per workgroup (stage 1 once for both)
  if (dm64k_pairs(groups)) {
    const int64_t total = group_grid(cus, groups / 2, (n + dm64k::Geo<2>::TT - 1) / dm64k::Geo<2>::TT);
    if (bias_dt != BCFFT_NONE)
      hipLaunchKernelGGL((bc_forward_dm64k_kernel<true, 2>), dim3((unsigned)total), dim3(512), 0, s, x, n, n_in, n_out,
                         stat, osc, bias, bias_dt, y);
    else
      hipLaunchKernelGGL((bc_forward_dm64k_kernel<false, 2>), dim3((unsigned)total), dim3(512), 0, s, x, n, n_in, n_out,
                         stat, osc, bias, bias_dt, y);
    return;
  }
  const int64_t total = group_grid(cus, groups, (n + dm64k::Geo<1>::TT - 1) / dm64k::Geo<1>::TT);
  if (bias_dt != BCFFT_NONE)
    hipLaunchKernelGGL((bc_forward_dm64k_kernel<true, 1>), dim3((unsigned)total), dim3(512), 0, s, x, n, n_in, n_out,
                       stat, osc, bias, bias_dt, y);
  else
    hipLaunchKernelGGL((bc_forward_dm64k_kernel<false, 1>), dim3((unsigned)total), dim3(512), 0, s, x, n, n_in, n_out,
                       stat, osc, bias, bias_dt, y);
}

}  // namespace bcfft

BCFFT_STAMPS_SETTER(dm64k)
