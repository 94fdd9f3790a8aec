// bcfft_dmm.hip — the fused BC-MLP on the matrix cores (gfx950):
//   y = BC_down( silu(BC_gate(x)) * BC_up(x) )   in ONE launch, bf16 I/O, b = 128,
// hidden 4096 (32 blocks), intermediate 32 < n_h <= 127 blocks (LLaMA-7B: 11008 = 86 blocks).
//
// The reference times this unit as `bc_down(F.silu(bc_gate(x)) * bc_up(x))`
// (src/microbench_dense_vs_bc.py:183-188, `--bench_mlp`; the MLP of the patched model,
// patch_llama_fft.py:343-394). The two-launch form (bcfft_dmg.hip's gate/up + SwiGLU, then
// bcfft_dmk.hip's down projection) writes h (n x 11008 bf16, 180 MB at 8192 tokens) to HBM and
// reads it back. Here h never leaves the CU: one workgroup owns an 8-token tile for the whole MLP.
//
//  * Gate/up stage 1 once per tile (wave w: token w), X units in region XR (bcfft_dmg.hip's).
//  * Per gate/up group g (16 gate + 16 up output blocks = 16 h blocks = the down projection's
//    16-block K-chunk g):
//      - gate/up stage 2 against g's B fragments, streamed from L2; A fragments read from XR per
//        K-step (they stay in LDS, not in VGPRs: the down accumulators need those registers);
//        Y units into region WR;
//      - gate/up stage 3 of token w with SiLU and the product, the 16 h rows staged in WR's slot w
//        in exactly the layout bcfft_dmk.hip's x DMA gives a 16-block chunk;
//      - down stage 1 of token w on that chunk (bcfft_dmk.hip's: per-(token, chunk) power-of-two
//        scale with 2^HEAD headroom), in place;
//      - down stage 2 of chunk g for all 8 tokens on the wave's 8 bins, accumulating over the
//        chunks in 64 VGPRs (the reference-exponent alignment of bcfft_dmk.hip).
//  * Tile end: the down accumulators as Y units into WR; their stage 3 (token w) and y stores run
//    beside the next tile's gate/up stage 1.
//
// One 64-register buffer carries every B fragment, in the order they are consumed: gate/up
// K-step 0 of group g, K-step 1 of g, down chunk g, gate/up K-step 0 of g + 1, ... Each fragment
// is refilled right after its last use with the next one (compiler-visible buffer loads: the
// compiler places the waits), so a whole stage covers the L2 latency of every load but the
// K-step-1 ones (7 bins of cover). The next tile's x streams into XR by LDS-DMA from the last
// group's stage 3 on.
//
// Numerics: every rounding of the two-launch path at 8-token tiles (bcfft_dmg.hip<GLU> then
// bcfft_dmk.hip<8>) in the same order: h is rounded to bf16 where the two-launch path stores it,
// so the fused output is bit-identical to it (tests/test_gpu_mlp.py checks this).
//
// LDS (149,760 B): XR and WR, each 8 token slots of 8,256 B (64 B off the 256-B bank period, as
// in bcfft_dm8.hip), the DFT table, the scale exponents, the inverse weight scales.
#ifndef BCFFT_STREAM_POLICY
#define BCFFT_STREAM_POLICY 1                       // nt x / sc1 y: the weight fragments stay in L2 (bcfft_device.h)
#endif
#include "bcfft_device.h"
#include "bcfft_dm_table.h"
#include "bcfft_dm_common.h"

namespace bcfft {

namespace dmm {
// wave priority falling through gate/up stage 2 (1), down stage 2 (2), gate/up stage 3 and
// down stage 1 (4): set_prio
constexpr int PRIO = 7;
using namespace dmh;
constexpr int B = 128, NI = 32, KS = 2, NOG = 32, TT = 8, NW = 8;
constexpr int BW = 8, NT = 2;                       // bins per wave, 16-wide N-tiles
constexpr int OPG = 16;                             // h blocks per gate/up group = down chunk
constexpr int K = NI * B;
constexpr int SLOT = 8192 + 64;                     // one token
constexpr int REGION = TT * SLOT;
constexpr int XR_OFF = 0, WR_OFF = REGION;
constexpr int F_OFF = 2 * REGION;                   // DFT table image, 64 rows x 256 B
constexpr int GSC_OFF = F_OFF + 16384;              // gate/up stage-1 exponents [8 token][2 half]
constexpr int DSC_OFF = GSC_OFF + 64;               // down stage-1 exponents [8 token]
constexpr int RR_OFF = DSC_OFF + 32;                // down reference exponents [8 token]
constexpr int MAXG = 8;                             // n_h <= 127 blocks
constexpr int GOS_OFF = RR_OFF + 32;                // gate/up inverse weight scales [MAXG][32]
constexpr int DOS_OFF = GOS_OFF + MAXG * NOG * 4;   // down inverse weight scales [32]
constexpr int LDS_BYTES = DOS_OFF + NOG * 4;
constexpr int NPIECE = BW * KS * NT;                // gate/up B fragments per wave and group
constexpr int DFRAGS = BW * NT;                     // down B fragments per wave and chunk
constexpr int NDMA = K * 2 / 1024;                  // 1-KiB LDS-DMA pieces per token (bf16 x)
constexpr int HEAD = 4;                             // bcfft_dmk.hip's chunk headroom
static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
static_assert(F_OFF % 256 == 0 && SLOT % 256 == 64, "bank map");
__device__ __forceinline__ uint32_t f16_pow2_neg(int d) {
  return d <= 14 ? (uint32_t)(15 - d) << 10 : (d <= 24 ? 1u << (24 - d) : 0u);
}
}  // namespace dmm

// SPL (short grids, dmm_ksplit): the gate/up groups (= the down projection's K-chunks) are split
// into kz slices; workgroup b takes slice b % kz of exactly one 8-token tile and writes its partial
// y in fp32 to ws[slice][token][column]; launch_partials_finish sums the slices and rounds.
template <bool SPL>
__global__ __launch_bounds__(512, 2) void bc_mlp_dmm_kernel(
    const void* __restrict__ xv, int64_t n_tokens, int n_h, const uint32_t* __restrict__ gstat,
    const float* __restrict__ gosc, const uint32_t* __restrict__ dstat, const float* __restrict__ dosc,
    void* __restrict__ yv, int kz, float* __restrict__ ws) {
  using namespace dmm;
  constexpr int XT = BCFFT_BF16;
  constexpr int ES = 2;

  __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];
  int* gsc = reinterpret_cast<int*>(lds + GSC_OFF);
  int* dsc = reinterpret_cast<int*>(lds + DSC_OFF);
  int* wrr = reinterpret_cast<int*>(lds + RR_OFF);
  const float* gos = reinterpret_cast<const float*>(lds + GOS_OFF);
  const float* dos = reinterpret_cast<const float*>(lds + DOS_OFF);
  char* const xr = lds + XR_OFF;
  char* const wr = lds + WR_OFF;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n_groups = (n_h + OPG - 1) / OPG;       // gate/up groups = down K-chunks
  constexpr int64_t M = (int64_t)NOG * B;           // y row: 4096
  const int64_t n_mtiles = (n_tokens + TT - 1) / TT;
  // gate/up group range [g0, g1) of this workgroup; unsplit: all groups, persistent over tiles
  int g0 = 0, g1 = n_groups, slice = 0;
  int64_t m0 = blockIdx.x, gstride = gridDim.x;
  if constexpr (SPL) {
    slice = blockIdx.x % kz;
    m0 = blockIdx.x / kz;
    gstride = n_mtiles;                             // one tile per workgroup
    const int gps = (n_groups + kz - 1) / kz;
    g0 = slice * gps;
    g1 = min(n_groups, g0 + gps);
  }
  const uint32_t lds_base = __builtin_amdgcn_readfirstlane(lds_addr(lds));
  const uint4* gimg = reinterpret_cast<const uint4*>(gstat + 4);
  const uint4* dimg = reinterpret_cast<const uint4*>(dstat + 4);

  // ---- x of token `wave` of M-tile m -> its XR slot by LDS-DMA (bcfft_dmg.hip's)
  auto dma_token = [&](int64_t m) {
    const int64_t tok = m * TT + wave;
    const bool ok = tok < n_tokens;
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<char*>((const char*)xv) + (ok ? tok : 0) * K * ES, 0, ok ? K * ES : 0, 0x00020000);
    const int dl = opaque(lane);
    const uint32_t dst0 = lds_base + XR_OFF + wave * SLOT;
    int vb[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int r = dl >> 4;
      vb[c] = r * 256 + 16 * ((dl & 15) ^ ((4 * c + r) & 15));
    }
#pragma unroll
    for (int q = 0; q < NDMA; ++q) {
      uint32_t keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen" BCFFT_XPOL " lds\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep) : "v"(vb[q & 3]), "s"(xrs), "s"(dst0 + q * 1024), "s"(q * 1024) : "memory");
    }
  };

  // ---- the B-fragment buffer and its three sources (compiler-visible loads, as in bcfft_dmg.hip:
  // the asm x DMA is not counted by the compiler, so its waits can only drain more, never less)
  u32x4 bb[BW][NT];
  auto g_rsrc = [&](int g) {                        // gate/up group g: piece ((fb KS + ks) NT + nt)
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint4*>(gimg + ((int64_t)(g * NW + wave) * NPIECE) * 64), 0,
                                             NPIECE * 1024, 0x00020000);
  };
  auto d_rsrc = [&](int c) {                        // down chunk c: piece fb NT + nt
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint4*>(dimg + ((int64_t)(c * NW + wave) * DFRAGS) * 64), 0,
                                             DFRAGS * 1024, 0x00020000);
  };
  auto load_g = [&](const __amdgpu_buffer_rsrc_t& rs, int vo, int ks, int fb, int nt) {
    bb[fb][nt] = __builtin_amdgcn_raw_buffer_load_b128(rs, vo, ((fb * KS + ks) * NT + nt) * 1024, 0);
  };
  auto load_d = [&](const __amdgpu_buffer_rsrc_t& rs, int vo, int fb, int nt) {
    bb[fb][nt] = __builtin_amdgcn_raw_buffer_load_b128(rs, vo, (fb * NT + nt) * 1024, 0);
  };

  // ---- prologue: the first tile's x, the DFT table, the inverse weight scales, gate/up group g0's
  // K-step 0 fragments
  dma_token(m0);
  {
    const uint4* tab = reinterpret_cast<const uint4*>(kDmF);
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int c = tid + 512 * r;                  // chunk c: row c >> 4, chunk c & 15
      const int t = c >> 4, ch = c & 15;
      *reinterpret_cast<uint4*>(lds + F_OFF + 256 * t + 16 * (ch ^ fsw(t))) = tab[c];
    }
    for (int e = tid; e < n_groups * NOG; e += 512) reinterpret_cast<float*>(lds + GOS_OFF)[e] = gosc[e];
    if (tid < NOG) reinterpret_cast<float*>(lds + DOS_OFF)[tid] = dosc[tid];
  }
  wait_vmcnt<0>();
  {
    const __amdgpu_buffer_rsrc_t rs = g_rsrc(g0);
    const int vo = opaque(lane) * 16;
#pragma unroll
    for (int fb = 0; fb < BW; ++fb)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) load_g(rs, vo, 0, fb, nt);
  }
  lds_barrier();

  // ---- gate/up stage 1 (wave w, XR slot w): x rows -> X units (one fp16 term) in place, per
  // 16-block half (bcfft_dmg.hip's stage 1)
  auto gu_stage1 = [&]() {
    const int l = opaque(lane);
    const int b16 = l & 15, g = l >> 4;
    char* slot = xr + wave * SLOT;
    const int q4 = (l & 15) >> 2, p4 = l & 3;
    const int cx = (p4 >> 1) ^ fsw(8 * g + q4);
    const int trb = F_OFF + 256 * (8 * g + q4) + 8 * (p4 & 1);
    int xwb[2];
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) xwb[pr] = 256 * g + 64 * (pr ^ (g & 1)) + 4 * b16;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      float xv8[2][2][8];
      const char* rowp = slot + (16 * h + b16) * (B * ES);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int pt = 0; pt < 2; ++pt) {
          const int u = 4 * ks + g + 8 * pt;
          const uint4 w = *reinterpret_cast<const uint4*>(rowp + 16 * (u ^ b16));
          const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float2 f = unpack16<XT>(ww[e]);
            xv8[ks][pt][2 * e] = f.x;
            xv8[ks][pt][2 * e + 1] = f.y;
          }
        }
      float m0f = 0.f, m1f = 0.f;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int pt = 0; pt < 2; ++pt)
#pragma unroll
          for (int j = 0; j < 8; j += 4) {
            m0f = amax3(m0f, xv8[ks][pt][j], xv8[ks][pt][j + 1]);
            m1f = amax3(m1f, xv8[ks][pt][j + 2], xv8[ks][pt][j + 3]);
          }
      const float mxf = __builtin_fmaxf(m0f, m1f);
      const int sx = stat_scale_exp(2.f * __uint_as_float(wave_umax(__float_as_uint(mxf))));
      if (l == 0) gsc[wave * 2 + h] = sx - 7;
      const float S = __int_as_float((sx + 127) << 23);
      f32x4 acc[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        uint32_t ah[4], dh[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float u0 = xv8[ks][1][2 * e] * S, u1 = xv8[ks][1][2 * e + 1] * S;
          ah[e] = pk_rne(fmaf(xv8[ks][0][2 * e], S, u0), fmaf(xv8[ks][0][2 * e + 1], S, u1));
          dh[e] = pk_rne(fmaf(xv8[ks][0][2 * e], S, -u0), fmaf(xv8[ks][0][2 * e + 1], S, -u1));
        }
        const f16x8 bah = frag(ah[0], ah[1], ah[2], ah[3]), bdh = frag(dh[0], dh[1], dh[2], dh[3]);
#pragma unroll
        for (int pr = 0; pr < 2; ++pr)
#pragma unroll
          for (int mt = 0; mt < 4; ++mt) {
            const int cb = 16 * ((8 * pr + 2 * mt) ^ cx);
            const char* p0 = lds + trb + 256 * 32 * ks + cb;
            const s16x4 r0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p0));
            const s16x4 r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p0 + 256 * 4));
            const f16x8 af = __builtin_bit_cast(f16x8, __builtin_shufflevector(r0, r1, 0, 1, 2, 3, 4, 5, 6, 7));
            acc[4 * pr + mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, pr ? bdh : bah, acc[4 * pr + mt], 0, 0, 0);
          }
      }
      char* xb = slot + 4096 * h;
#pragma unroll
      for (int pr = 0; pr < 2; ++pr)
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          *reinterpret_cast<uint32_t*>(xb + xwb[pr] + 1024 * mt) = pk_rne(acc[4 * pr + mt][0], acc[4 * pr + mt][1]);
          *reinterpret_cast<uint32_t*>(xb + xwb[pr] + 1024 * mt + 128) = pk_rne(acc[4 * pr + mt][2], acc[4 * pr + mt][3]);
        }
    }
  };

  // gate/up A-row factors of the lane's token (bcfft_dmg.hip's load_a): the halves aligned to the
  // token's smaller exponent, re rows [Xr, Xi], im rows [Xi, -Xr]; bin 0 with the extra 1/2
  uint32_t gmul[KS], gmul0[KS];
  auto gu_factors = [&]() {
    const int ml = opaque(lane);
    const int arow = ml & 15;
    const int a_t = arow >> 1, a_reim = arow & 1;
    int nk[KS];
    nk[0] = gsc[a_t * 2];
    nk[1] = gsc[a_t * 2 + 1];
    const int nmin = min(nk[0], nk[1]);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const uint32_t hh = f16_pow2_neg(nk[ks] - nmin);
      const uint32_t h0 = f16_pow2_neg(nk[ks] - nmin + 1);
      gmul[ks] = a_reim ? (hh | ((hh | 0x8000u) << 16)) : (hh | (hh << 16));
      gmul0[ks] = a_reim ? (h0 << 16) : h0;
    }
  };

  // ---- gate/up stage 2 of group g (all waves; bins 8 wave + fb, all 8 tokens), K-step-major:
  // K-step 0 consumes bb and refills it with K-step 1's fragments, K-step 1 refills it with down
  // chunk g's. The per-(bin, N-tile) MFMA order is bcfft_dmg.hip's (K-step 0, then 1).
  auto gu_stage2 = [&](int g) {
    constexpr float YS = 1.f / 2097152.f;            // 2^-21: |Y| < 2^14 in fp16
    const int ml = opaque(lane);
    const int arow = ml & 15, kb = ml >> 4;
    const int a_t = arow >> 1, a_reim = arow & 1;
    const uint32_t a_sel = a_reim ? 0x01000302u : 0x03020100u;
    const int yt = ml >> 4;
    const char* ab = xr + a_t * SLOT + 512 * wave + 16 * kb;
    const __amdgpu_buffer_rsrc_t grs = g_rsrc(g), drs = d_rsrc(g);
    const int vo = opaque(lane) * 16;
    f32x4 acc[BW][NT];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int fb = 0; fb < BW; ++fb) {
        if constexpr ((PRIO & 1) != 0) set_prio(3 - 4 * (ks * BW + fb) / (KS * BW));
        uint4 raw = *reinterpret_cast<const uint4*>(ab + 4096 * ks + 64 * (fb ^ ((fb >> 2) & 1)));
        if (wave == 0 && fb == 0) {
          raw.x = pkmul(raw.x, gmul0[ks]); raw.y = pkmul(raw.y, gmul0[ks]);
          raw.z = pkmul(raw.z, gmul0[ks]); raw.w = pkmul(raw.w, gmul0[ks]);
        } else {
          raw.x = pkmul(__builtin_amdgcn_perm(raw.x, raw.x, a_sel), gmul[ks]);
          raw.y = pkmul(__builtin_amdgcn_perm(raw.y, raw.y, a_sel), gmul[ks]);
          raw.z = pkmul(__builtin_amdgcn_perm(raw.z, raw.z, a_sel), gmul[ks]);
          raw.w = pkmul(__builtin_amdgcn_perm(raw.w, raw.w, a_sel), gmul[ks]);
        }
        const f16x8 a = __builtin_bit_cast(f16x8, raw);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const f16x8 bf = __builtin_bit_cast(f16x8, bb[fb][nt]);
          acc[fb][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, bf, ks == 0 ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[fb][nt],
                                                               0, 0, 0);
        }
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          if (ks == 0) load_g(grs, vo, 1, fb, nt);
          else load_d(drs, vo, fb, nt);
        }
      }
    // Y units into WR (bcfft_dmg.hip's stage-2 store: rows 4 yt + r = token 2 yt + (r >> 1))
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      char* yb = wr + (2 * yt + s2) * SLOT + 512 * wave + 16 * (ml & 15);
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        uint32_t u[BW];
#pragma unroll
        for (int fb = 0; fb < BW; ++fb) u[fb] = pk_rne(acc[fb][nt][2 * s2] * YS, acc[fb][nt][2 * s2 + 1] * YS);
        *reinterpret_cast<uint4*>(yb + 256 * nt) = make_uint4(u[0], u[2], u[4], u[6]);
        *reinterpret_cast<uint4*>(yb + 4096 + 256 * nt) = make_uint4(u[1], u[3], u[5], u[7]);
      }
    }
  };

  // ---- gate/up stage 3 of group g (wave w, WR slot w): Y -> gate, up -> h = silu(gate) * up with
  // torch's roundings (bcfft_dmg.hip's GLU epilogue), the 16 h rows written over the slot's first
  // 4 KiB as bcfft_dmk.hip's x chunk: element e of block row r in unit e >> 3, stored at unit
  // (e >> 3) ^ r. Rows past n_h are zero (the two-launch path's DMA reads zeros there).
  auto gu_stage3 = [&](int g) {
    if constexpr ((PRIO & 4) != 0) set_prio(3);
    const int l = opaque(lane);
    const int o16 = l & 15, gq = l >> 4;
    char* slot = wr + wave * SLOT;
    const int nmin = min(gsc[wave * 2], gsc[wave * 2 + 1]);
    float ysc[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) ysc[nt] = __builtin_ldexpf(gos[g * NOG + 16 * nt + o16], 30 - nmin);
    uint4 yf[KS][2][NT];
    const char* yb = slot + 512 * gq + 16 * o16;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int pr = 0; pr < 2; ++pr)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          yf[ks][pr][nt] = *reinterpret_cast<const uint4*>(yb + 4096 * pr + 2048 * ks + 256 * nt);
    const int gx = gq ^ fsw(o16);
    const char* gb = lds + F_OFF + 256 * o16;
    auto gload = [&](int mt, f16x8 (&gf)[KS][2]) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int pr = 0; pr < 2; ++pr)
          gf[ks][pr] = *reinterpret_cast<const f16x8*>(gb + 4096 * mt + 16 * ((8 * pr + 4 * ks) ^ gx));
    };
    f16x8 gcur[KS][2];
    gload(0, gcur);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // Y is in registers: the slot is free
    const bool row_ok = g * OPG + o16 < n_h;
    char* hrow = slot + 256 * o16 + 8 * (gq & 1);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      f32x4 E[NT], O[NT];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        E[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
        O[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          E[nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(gcur[ks][0], __builtin_bit_cast(f16x8, yf[ks][0][nt]), E[nt], 0, 0, 0);
          O[nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(gcur[ks][1], __builtin_bit_cast(f16x8, yf[ks][1][nt]), O[nt], 0, 0, 0);
        }
      if (mt < 3) gload(mt + 1, gcur);
      float gu[NT][2][4];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int hf = 0; hf < 2; ++hf)
#pragma unroll
          for (int r = 0; r < 4; ++r)               // gate / up rounded to x's dtype (:266)
            gu[nt][hf][r] = round_to(hf ? fmaf(E[nt][r], ysc[nt], -O[nt][r] * ysc[nt]) : fmaf(E[nt][r], ysc[nt], O[nt][r] * ysc[nt]), XT);
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r)                 // torch: silu rounded, then the product rounded
          v[r] = round_to(round_to(silu(gu[0][hf][r]), XT) * gu[1][hf][r], XT);
        // elements 16 mt + 4 gq + 64 hf + r: unit 2 mt + (gq >> 1) + 8 hf, byte 8 (gq & 1)
        const int u = 2 * mt + (gq >> 1) + 8 * hf;
        const uint2 pv = row_ok ? make_uint2(pack16<XT>(v[0], v[1]), pack16<XT>(v[2], v[3])) : make_uint2(0u, 0u);
        *reinterpret_cast<uint2*>(hrow + 16 * (u ^ o16)) = pv;
      }
    }
  };

  // ---- down stage 1 (wave w, WR slot w): the h chunk -> X units in place (bcfft_dmk.hip's
  // stage 1: per-(token, chunk) exponent with HEAD headroom)
  auto dn_stage1 = [&]() {
    if constexpr ((PRIO & 4) != 0) set_prio(1);
    const int l = opaque(lane);
    const int b16 = l & 15, g = l >> 4;
    const int q4 = (l & 15) >> 2, p4 = l & 3;
    const int cx = (p4 >> 1) ^ fsw(8 * g + q4);
    const int trb = F_OFF + 256 * (8 * g + q4) + 8 * (p4 & 1);
    char* slot = wr + wave * SLOT;
    const char* rowp = slot + b16 * (B * ES);
    uint32_t xw[2][2][4];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int pt = 0; pt < 2; ++pt) {
        const uint4 w = *reinterpret_cast<const uint4*>(rowp + 16 * ((4 * ks + g + 8 * pt) ^ b16));
        xw[ks][pt][0] = w.x; xw[ks][pt][1] = w.y; xw[ks][pt][2] = w.z; xw[ks][pt][3] = w.w;
      }
    float m0 = 0.f, m1 = 0.f;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int pt = 0; pt < 2; ++pt)
#pragma unroll
        for (int e = 0; e < 4; e += 2) {
          const float2 f0 = unpack16<XT>(xw[ks][pt][e]), f1 = unpack16<XT>(xw[ks][pt][e + 1]);
          m0 = amax3(m0, f0.x, f0.y);
          m1 = amax3(m1, f1.x, f1.y);
        }
    const float mxf = __builtin_fmaxf(m0, m1);
    const int sx = stat_scale_exp(2.f * __uint_as_float(wave_umax(__float_as_uint(mxf)))) - HEAD;
    if (l == 0) dsc[wave] = sx - 7;
    const float S = __int_as_float((sx + 127) << 23);
    uint32_t ah[2][4], dh[2][4];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float2 lo = unpack16<XT>(xw[ks][0][e]), hi = unpack16<XT>(xw[ks][1][e]);
        const float u0 = hi.x * S, u1 = hi.y * S;
        ah[ks][e] = pk_rne(fmaf(lo.x, S, u0), fmaf(lo.y, S, u1));
        dh[ks][e] = pk_rne(fmaf(lo.x, S, -u0), fmaf(lo.y, S, -u1));
      }
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
      f32x4 acc4[4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) acc4[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const f16x8 bx = pr ? frag(dh[ks][0], dh[ks][1], dh[ks][2], dh[ks][3])
                            : frag(ah[ks][0], ah[ks][1], ah[ks][2], ah[ks][3]);
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          const int cb = 16 * ((8 * pr + 2 * mt) ^ cx);
          const char* p0 = lds + trb + 256 * 32 * ks + cb;
          const s16x4 r0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p0));
          const s16x4 r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p0 + 256 * 4));
          const f16x8 af = __builtin_bit_cast(f16x8, __builtin_shufflevector(r0, r1, 0, 1, 2, 3, 4, 5, 6, 7));
          acc4[mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bx, acc4[mt], 0, 0, 0);
        }
      }
      const int xwb = 256 * g + 64 * (pr ^ (g & 1)) + 4 * b16;
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        *reinterpret_cast<uint32_t*>(slot + xwb + 1024 * mt) = pk_rne(acc4[mt][0], acc4[mt][1]);
        *reinterpret_cast<uint32_t*>(slot + xwb + 1024 * mt + 128) = pk_rne(acc4[mt][2], acc4[mt][3]);
      }
    }
  };

  // down accumulators of the tile: [bin of the wave][N-tile], rows 4 yt + r = token 2 yt + (r >> 1),
  // re/im r & 1; reference exponents of the lane's A-row token and accumulator-row tokens
  f32x4 dacc[BW][NT];
  int ra = 0, rc[2] = {0, 0};

  // ---- down stage 2 of chunk c (all waves; bcfft_dmk.hip's stage 2 at 8-token tiles): consumes bb
  // (chunk c's fragments) and refills it with gate/up group gnext's K-step-0 fragments (gnext < 0:
  // none, the launch's last chunk)
  auto dn_stage2 = [&](auto first_tag, int gnext) {
    constexpr bool FIRST = decltype(first_tag)::value;
    const int ml = opaque(lane);
    const int arow = ml & 15, kb = ml >> 4;
    const int a_tl = arow >> 1, a_reim = arow & 1;
    const uint32_t a_sel = a_reim ? 0x01000302u : 0x03020100u;
    const int yt = ml >> 4;
    const int nka = dsc[a_tl];
    if constexpr (FIRST) {
      ra = nka;
      rc[0] = dsc[2 * yt];
      rc[1] = dsc[2 * yt + 1];
    } else {
      ra = min(ra, nka + HEAD);
      float fct[2];
      bool need = false;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int nn = dsc[2 * yt + s] + HEAD;
        const int d = rc[s] - nn;
        fct[s] = d > 0 ? __builtin_ldexpf(1.f, -d) : 1.f;
        need |= d > 0;
        rc[s] = min(rc[s], nn);
      }
      if (__builtin_amdgcn_ballot_w64(need)) {
#pragma unroll
        for (int fb = 0; fb < BW; ++fb)
#pragma unroll
          for (int nt = 0; nt < NT; ++nt)
#pragma unroll
            for (int r = 0; r < 4; ++r) dacc[fb][nt][r] *= fct[r >> 1];
      }
    }
    const int d = nka - ra;                         // >= -HEAD: factor 2^-d <= 2^HEAD
    const uint32_t hh = f16_pow2_neg(d);
    const uint32_t h0 = f16_pow2_neg(d + 1);        // bin 0: the inverse's 1/b vs 2/b
    const uint32_t amul = a_reim ? (hh | ((hh | 0x8000u) << 16)) : (hh | (hh << 16));
    const uint32_t amul0 = a_reim ? (h0 << 16) : h0;
    const char* ab = wr + a_tl * SLOT + 512 * wave + 16 * kb;
    const __amdgpu_buffer_rsrc_t grs = g_rsrc(gnext < 0 ? 0 : gnext);
    const int vo = opaque(lane) * 16;
#pragma unroll
    for (int fb = 0; fb < BW; ++fb) {
      if constexpr ((PRIO & 2) != 0) set_prio(3 - 4 * fb / BW);
      uint4 raw = *reinterpret_cast<const uint4*>(ab + 64 * (fb ^ ((fb >> 2) & 1)));
      if (wave == 0 && fb == 0) {
        raw.x = pkmul(raw.x, amul0); raw.y = pkmul(raw.y, amul0);
        raw.z = pkmul(raw.z, amul0); raw.w = pkmul(raw.w, amul0);
      } else {
        raw.x = pkmul(__builtin_amdgcn_perm(raw.x, raw.x, a_sel), amul);
        raw.y = pkmul(__builtin_amdgcn_perm(raw.y, raw.y, a_sel), amul);
        raw.z = pkmul(__builtin_amdgcn_perm(raw.z, raw.z, a_sel), amul);
        raw.w = pkmul(__builtin_amdgcn_perm(raw.w, raw.w, a_sel), amul);
      }
      const f16x8 a = __builtin_bit_cast(f16x8, raw);
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const f16x8 bf = __builtin_bit_cast(f16x8, bb[fb][nt]);
        if constexpr (FIRST)
          dacc[fb][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, bf, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        else
          dacc[fb][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, bf, dacc[fb][nt], 0, 0, 0);
      }
      if (gnext >= 0) {
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) load_g(grs, vo, 0, fb, nt);
      }
    }
  };

  // ---- the tile's down Y as fp16 units into WR (bcfft_dmk.hip's ywrite) and the reference
  // exponents of its tokens
  auto dn_ywrite = [&]() {
    const int ml = opaque(lane);
    const int yt = ml >> 4;
    constexpr float YS = 1.f / 2097152.f;            // 2^-21: |Y| <= n_h 2^9 < 65504 (n_h <= 127)
    if (wave == 0 && (ml & 15) == 0) {
      wrr[2 * yt] = rc[0];
      wrr[2 * yt + 1] = rc[1];
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      char* yb = wr + (2 * yt + s2) * SLOT + 512 * wave + 16 * (ml & 15);
#pragma unroll
      for (int par = 0; par < 2; ++par)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          uint32_t u[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const f32x4 a = dacc[par + 2 * j][nt];
            u[j] = pk_rne(a[2 * s2] * YS, a[2 * s2 + 1] * YS);
          }
          *reinterpret_cast<uint4*>(yb + 4096 * par + 256 * nt) = make_uint4(u[0], u[1], u[2], u[3]);
        }
    }
  };

  // ---- down stage 3 (wave w, WR slot w): Y -> y rows staged in the slot, 1 KiB stores
  // (bcfft_dmk.hip's stage 3 without bias: LLaMA's down projection has none)
  auto dn_stage3 = [&](int64_t tok) {
    const int l = opaque(lane);
    const int o16 = l & 15, g = l >> 4;
    char* slot = wr + wave * SLOT;
    float* wsp = SPL ? ws + ((int64_t)slice * n_tokens + (tok < n_tokens ? tok : 0)) * M : nullptr;
    const int rref = wrr[wave];
    float ysc[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) ysc[nt] = __builtin_ldexpf(dos[16 * nt + o16], 30 - rref);
    uint4 yf[2][2][NT];
    const char* yb = slot + 512 * g + 16 * o16;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int pr = 0; pr < 2; ++pr)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          yf[ks][pr][nt] = *reinterpret_cast<const uint4*>(yb + 4096 * pr + 2048 * ks + 256 * nt);
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
    const bool tok_ok = tok < n_tokens;
    int swb[4];
    {
      const int sg = ((o16 & 7) << 1) | (o16 >> 3);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) swb[mt] = 256 * o16 + 8 * ((4 * mt + g) ^ sg);
    }
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      f32x4 E[NT], O[NT];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        E[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
        O[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          E[nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(gcur[ks][0], __builtin_bit_cast(f16x8, yf[ks][0][nt]), E[nt], 0, 0, 0);
          O[nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(gcur[ks][1], __builtin_bit_cast(f16x8, yf[ks][1][nt]), O[nt], 0, 0, 0);
        }
      if (mt < 3) gload(mt + 1, gcur);
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        float os[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) os[r] = O[nt][r] * ysc[nt];
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = hf ? fmaf(E[nt][r], ysc[nt], -os[r]) : fmaf(E[nt][r], ysc[nt], os[r]);
          if constexpr (SPL) {                      // fp32 partial, 4 consecutive columns
            if (tok_ok)
              *reinterpret_cast<float4*>(wsp + (16 * nt + o16) * B + 16 * mt + 4 * g + 64 * hf) =
                  make_float4(v[0], v[1], v[2], v[3]);
          } else {
            *reinterpret_cast<uint2*>(slot + 4096 * nt + swb[mt] + 128 * hf) =
                make_uint2(pack16<XT>(v[0], v[1]), pack16<XT>(v[2], v[3]));
          }
        }
      }
    }
    if constexpr (SPL) return;
    constexpr int RB = B * ES;
    const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
        (char*)yv + (tok_ok ? tok : 0) * M * ES, 0, tok_ok ? (int)(M * ES) : 0, 0x00020000);
    const int w = l & 15, lr = l >> 4;
    const int vofs = lr * RB + 16 * w;
    int rdb[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) rdb[c] = lr * RB + 16 * ((w ^ lr) ^ (4 * c));
    uint4 dv[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      uint4 v = *reinterpret_cast<const uint4*>(slot + 1024 * q + rdb[q & 1]);
      if (q & 2) v = make_uint4(v.z, v.w, v.x, v.y);   // rows with bit 3: 8-B halves swapped
      dv[q] = v;
    }
#pragma unroll
    for (int q = 0; q < 8; ++q)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, dv[q]), yrs, vofs + q * 1024, 0, BCFFT_YAUX);
  };

  // Per 8-token tile m (x(m) in XR):
  //   stage 1 of token w                                                               | Ba |
  //   per group g: gate/up stage 2 (A from XR; bb: K-step 0 -> 1 -> down chunk g)       | Bb |
  //                [last group: LDS-DMA of x(m + stride) into XR]
  //                gate/up stage 3 of token w (h chunk into WR slot w); down stage 1    | Bd |
  //                down stage 2 of chunk g (bb -> gate/up K-step 0 of the next group)   | Be |
  //   down Y units into WR                                                             | Bf |
  // and the tile's down stage 3 (token w, y stores) runs beside the NEXT tile's stage 1: they
  // touch different regions (WR / XR), and that tile's Ba orders WR's reuse (bcfft_dmk.hip's
  // deferred stage 3)
  int64_t mprev = -1;
  for (int64_t m = m0; m < n_mtiles; m += gstride) {
    const bool more_tiles = m + gstride < n_mtiles;
    wait_vmcnt<0>();                                // x(m), and the first group's fragments
    gu_stage1();
    if (mprev >= 0) dn_stage3(mprev * TT + wave);
    lds_barrier();                                  // Ba: X units and exponents complete
    gu_factors();
    for (int g = g0; g < g1; ++g) {
      gu_stage2(g);
      lds_barrier();                                // Bb: Y units complete, XR reads done
      if (g + 1 == g1 && more_tiles) dma_token(m + gstride);
      gu_stage3(g);
      dn_stage1();
      lds_barrier();                                // Bd: the chunk's X units and exponents
      const int gnext = g + 1 < g1 ? g + 1 : (more_tiles ? g0 : -1);
      if (g == g0) dn_stage2(std::true_type{}, gnext);
      else dn_stage2(std::false_type{}, gnext);
      lds_barrier();                                // Be: the chunk's X-unit reads done
    }
    dn_ywrite();
    lds_barrier();                                  // Bf: Y units and reference exponents
    mprev = m;
  }
  dn_stage3(mprev * TT + wave);                     // the last tile's (every workgroup has one)
}

bool dmm_eligible(int n_in, int b, int xdt, int n_h, int n_out) {
  return b == 128 && n_in == dmm::NI && xdt == BCFFT_BF16 && n_out == dmm::NOG && dmk_geometry(n_h, b) &&
         (n_h + dmm::OPG - 1) / dmm::OPG <= dmm::MAXG;
}

// spec_gu: bcfft_spectra of glu_weights(c_gate, c_up) (32 ceil(n_h / 16) blocks x 32 inputs);
// spec_dn: bcfft_spectra of c_down (32 outputs x n_h inputs, the streamed-weight image)
void launch_mlp_dmm(const void* x, int64_t n, int n_h, const void* spec_gu, const void* spec_dn, void* y,
                    hipStream_t s) {
  const int groups = (n_h + dmm::OPG - 1) / dmm::OPG;
  const SpecLayout sg = spec_layout(32 * groups, dmm::NI, 128);
  const SpecLayout sd = spec_layout(dmm::NOG, n_h, 128);
  const int64_t n_mtiles = (n + dmm::TT - 1) / dmm::TT;
  int64_t total = device_cu_count();
  if (total > n_mtiles) total = n_mtiles;
  hipLaunchKernelGGL(bc_mlp_dmm_kernel<false>, dim3((unsigned)total), dim3(512), 0, s, x, n, n_h,
                     reinterpret_cast<const uint32_t*>(spec_gu) + sg.stat_off_u32,
                     reinterpret_cast<const float*>(spec_gu) + sg.osc_off_u32,
                     reinterpret_cast<const uint32_t*>(spec_dn) + sd.stat_off_u32,
                     reinterpret_cast<const float*>(spec_dn) + sd.osc_off_u32, y, 1, nullptr);
}

// group slices of the split form: where the one-launch kernel's tiles would fill at most half the
// CUs, as many slices as fill them, >= 1 group each
int dmm_ksplit(int64_t n, int n_h) {
  const int64_t tiles = (n + dmm::TT - 1) / dmm::TT, cus = device_cu_count();
  const int groups = (n_h + dmm::OPG - 1) / dmm::OPG;
  if (n <= 0 || tiles * 2 > cus) return 1;
  const int kz = (int)(cus / tiles < groups ? cus / tiles : groups);
  if (kz < 2) return 1;
  const int gps = (groups + kz - 1) / kz;
  return (groups + gps - 1) / gps;                  // every slice non-empty
}

void launch_mlp_dmm_split(const void* x, int64_t n, int n_h, const void* spec_gu, const void* spec_dn, void* y,
                          float* ws, int kz, hipStream_t s) {
  const int groups = (n_h + dmm::OPG - 1) / dmm::OPG;
  const SpecLayout sg = spec_layout(32 * groups, dmm::NI, 128);
  const SpecLayout sd = spec_layout(dmm::NOG, n_h, 128);
  const int64_t n_mtiles = (n + dmm::TT - 1) / dmm::TT;
  hipLaunchKernelGGL(bc_mlp_dmm_kernel<true>, dim3((unsigned)(kz * n_mtiles)), dim3(512), 0, s, x, n, n_h,
                     reinterpret_cast<const uint32_t*>(spec_gu) + sg.stat_off_u32,
                     reinterpret_cast<const float*>(spec_gu) + sg.osc_off_u32,
                     reinterpret_cast<const uint32_t*>(spec_dn) + sd.stat_off_u32,
                     reinterpret_cast<const float*>(spec_dn) + sd.osc_off_u32, y, kz, ws);
  launch_partials_finish(ws, kz, n, (int64_t)dmm::NOG * dmm::B, nullptr, BCFFT_NONE, y, s);
}

}  // namespace bcfft
