// bcfft_dm64g.hip — the b = 64 DFT-on-MFMA forward for layers with several output groups
// (gfx950): bf16 I/O, b = 64, K = 4096, M > 4096 (three or more output groups) — the block-size sweep's b = 64 gate / up
// projections 4096 -> 11008 (6 output groups) and their fused gate/up + SwiGLU (11 groups).
//
// Same operator as the other DFT kernels (BlockCirculantLinear.forward, patch_llama_fft.py:
// 226-275; per block src/fft_utils.py:3-34). bcfft_dm64.hip keeps ONE output group's weights in
// VGPRs, so G groups run G workgroups per token tile, each repeating stage 1 on the same x tile;
// at b = 64 stage 1 is the dominant stage (profiles/r03_ab_dm64k_ablation.log). Here one
// workgroup owns a token tile for ALL its groups (bcfft_dmg.hip's scheme on the b = 64 stages):
//
//  * stage 1 once per 8-token tile (wave w: token w, four 16-block quarters), X units in LDS as in
//    bcfft_dm64.hip;
//  * every wave takes the A fragments of its 4 bins x 4 K-steps for all 8 tokens into VGPRs (64),
//    with the per-quarter exponent alignment and the im-row transform applied once;
//  * per output group g: stage 2 against g's B fragments (the STAT image), streamed from L2 in
//    four passes of 8 (2 K-steps x 4 bins of one N-tile), double-buffered in 64 VGPRs through
//    compiler-visible buffer loads; Y half-units into the tile's slots; stage 3 of token w
//    (bcfft_dm64.hip's: 32 rows x 128 B staged, 4 x 1 KiB stores; GLU: 16 h rows);
//  * the next tile's x streams into the other LDS region from the start of the tile.
//
// Numerics are bcfft_dm64.hip's, in the same order: the output is bit-identical to running the
// per-group kernel on each group (tests/test_gpu_dm64g.py).
//
// LDS (144,640 B): two regions x 8 token slots of 8,256 B, the 4 KiB DFT table, the scale
// exponents, the inverse weight scales of up to 64 groups.
#ifndef BCFFT_STREAM_POLICY
#define BCFFT_STREAM_POLICY 1                       // nt x / sc1 y: the weight fragments stay in L2 (bcfft_device.h)
#endif
#include "bcfft_device.h"
#include "bcfft_dm_table.h"
#include "bcfft_dm_common.h"

namespace bcfft {

namespace dm64g {
using namespace dmh;

constexpr int B = 64, NI = 64, KS = 4, NOG = 32, TT = 8, NW = 8;
constexpr int BW = 4, NT = 2;                       // bins per wave, 16-wide N-tiles per group
constexpr int K = NI * B;
constexpr int SLOT = 8192 + 64;                     // one token
constexpr int REGION = TT * SLOT;
constexpr int F_OFF = 2 * REGION;                   // DFT table image, 32 rows x 128 B
constexpr int SC_OFF = F_OFF + 4096;                // scale exponents [2 parity][8 token][4 quarter]
constexpr int OS_OFF = SC_OFF + 256;                // inverse weight scales [MAXG][32]
constexpr int MAXG = 64;
constexpr int LDS_BYTES = OS_OFF + MAXG * NOG * 4;
constexpr int NPIECE = BW * KS * NT;                // B fragments per wave and group (STAT image)
constexpr int NDMA = K * 2 / 1024;                  // 1-KiB LDS-DMA pieces per token (bf16 x)
constexpr int PF = 8;                               // fragments per stage-2 pass
static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");

__device__ __forceinline__ int fsw64(int t) { return (((t >> 1) & 1) << 1) | (((t >> 3) & 1) << 2); }
__device__ __forceinline__ int yhalf64(int w, int o, int par) { return 2048 * par + 256 * w + 8 * (o ^ (16 * ((w >> 1) & 1))); }
// pass p (N-tile major: one N-tile's accumulators live at a time): N-tile p >> 1, K-steps
// 2 (p & 1) and 2 (p & 1) + 1; its fragment j = 2 fb + (ks & 1) is STAT piece (fb KS + ks) NT + nt
__host__ __device__ constexpr int pass_nt(int p) { return p >> 1; }
__host__ __device__ constexpr int pass_ks(int p, int j) { return 2 * (p & 1) + (j & 1); }
}  // namespace dm64g

// HB: a bias is added (the runtime bias_dt then names its dtype); without one the store path is
// straight-line (a runtime test per stored quad split stage 3 into hundreds of basic blocks)
template <bool GLU, bool HB>
__global__ __launch_bounds__(512, 2) void bc_forward_dm64g_kernel(
    const void* __restrict__ xv, int64_t n_tokens, int n_out, const uint32_t* __restrict__ stat,
    const float* __restrict__ osc, const void* __restrict__ bias, int bias_dt, void* __restrict__ yv) {
  using namespace dm64g;
  constexpr int XT = BCFFT_BF16;
  constexpr int ES = 2, ESY = 2;

  __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];
  int* wsc = reinterpret_cast<int*>(lds + SC_OFF);
  const float* osl = reinterpret_cast<const float*>(lds + OS_OFF);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // GLU (fused gate/up + SwiGLU): n_out counts h blocks; group g holds gate blocks [16g, 16g+16)
  // in N-tile 0 and the matching up blocks in N-tile 1, and stores 16 h rows
  constexpr int OPG = GLU ? NOG / 2 : NOG;
  const int n_groups = (n_out + OPG - 1) / OPG;
  const int64_t M = (int64_t)n_out * B;
  const int64_t n_mtiles = (n_tokens + TT - 1) / TT;
  const int64_t gstride = gridDim.x;
  const uint32_t lds_base = __builtin_amdgcn_readfirstlane(lds_addr(lds));
  const uint4* bimg = reinterpret_cast<const uint4*>(stat + 4);

  // ---- x of token `wave` of M-tile m -> its slot by LDS-DMA (bcfft_dm64.hip's: piece q = rows
  // 8q + (lane >> 3), 128 B each; unit u of row r at u ^ (r & 7); zeros past n_tokens)
  auto dma_token = [&](int64_t m, char* region) {
    const int64_t tok = m * TT + wave;
    const bool ok = tok < n_tokens;
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<char*>((const char*)xv) + (ok ? tok : 0) * K * ES, 0, ok ? K * ES : 0, 0x00020000);
    const int dl = opaque(lane);
    const uint32_t dst0 = lds_base + (uint32_t)(region - lds) + wave * SLOT;
    const int r = dl >> 3;
    const int vb = r * 128 + 16 * ((dl & 7) ^ r);
#pragma unroll
    for (int q = 0; q < NDMA; ++q) {
      uint32_t keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen" BCFFT_XPOL " lds\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep) : "v"(vb), "s"(xrs), "s"(dst0 + q * 1024), "s"(q * 1024) : "memory");
    }
  };

  // ---- B fragments of group g, pass p, from L2: compiler-visible buffer loads (bcfft_dmg.hip's
  // reasoning: the compiler's waits can only cover more operations than needed, never fewer)
  typedef u32x4 Breg[PF];
  auto b_rsrc = [&](int g) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint4*>(bimg + ((int64_t)(g * NW + wave) * NPIECE) * 64), 0,
                                             NPIECE * 1024, 0x00020000);
  };
  auto load_b1 = [&](const __amdgpu_buffer_rsrc_t& brs, int vo, int p, int j, Breg& br) {
    const int fb = j >> 1;
    br[j] = __builtin_amdgcn_raw_buffer_load_b128(brs, vo, ((fb * KS + pass_ks(p, j)) * NT + pass_nt(p)) * 1024, 0);
  };
  auto load_pass = [&](int g, int p, Breg& br) {
    const __amdgpu_buffer_rsrc_t brs = b_rsrc(g);
    const int vo = opaque(lane) * 16;
#pragma unroll
    for (int j = 0; j < PF; ++j) load_b1(brs, vo, p, j, br);
  };

  // ---- prologue: the first tile's x, the DFT table, every group's inverse weight scales, the
  // first group's first B pass
  Breg breg[2];
  const int64_t m0 = blockIdx.x;
  dma_token(m0, lds);
  if (tid < 256) {                                  // chunk c: row c >> 3, chunk c & 7
    const uint4* tab = reinterpret_cast<const uint4*>(kDmF64);
    const int t = tid >> 3, ch = tid & 7;
    *reinterpret_cast<uint4*>(lds + F_OFF + 128 * t + 16 * (ch ^ fsw64(t))) = tab[tid];
  }
  for (int e = tid; e < n_groups * NOG; e += 512) reinterpret_cast<float*>(lds + OS_OFF)[e] = osc[e];
  wait_vmcnt<0>();
  load_pass(0, 0, breg[0]);
  lds_barrier();

  // ---- stage 1 (wave w, token slot w): bcfft_dm64.hip's, per quarter
  auto stage1 = [&](char* region, int par) {
    const int l = opaque(lane);
    const int b16 = l & 15, g = l >> 4;
    char* slot = region + wave * SLOT;
    const int q4 = (l & 15) >> 2, p4 = l & 3;
    const int r0 = 8 * g + q4, r1 = r0 + 4;
    const int trb0 = F_OFF + 128 * r0 + 8 * (p4 & 1), trb1 = F_OFF + 128 * r1 + 8 * (p4 & 1);
    const int cx0 = (p4 >> 1) ^ fsw64(r0), cx1 = (p4 >> 1) ^ fsw64(r1);
    int xwb[2];
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) xwb[pr] = 256 * g + 64 * (pr ^ (g & 1)) + 4 * b16;
    // A = F^T (16 bin-reals x 32 t) fragments, read once for the four quarters (the X stores
    // between quarters kept the compiler from reusing them: 32 -> 8 transposed reads per token)
    f16x8 afr[2][2];
#pragma unroll
    for (int pr = 0; pr < 2; ++pr)
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const int c = 4 * pr + 2 * mt;
        const s16x4 ra = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4*)(lds + trb0 + 16 * (c ^ cx0)));
        const s16x4 rb = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4*)(lds + trb1 + 16 * (c ^ cx1)));
        afr[pr][mt] = __builtin_bit_cast(f16x8, __builtin_shufflevector(ra, rb, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      float xq[2][8];
      const char* rowp = slot + (16 * h + b16) * (B * ES);
#pragma unroll
      for (int pt = 0; pt < 2; ++pt) {
        const uint4 w = *reinterpret_cast<const uint4*>(rowp + 16 * ((g + 4 * pt) ^ (b16 & 7)));
        const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float2 f = unpack16<XT>(ww[e]);
          xq[pt][2 * e] = f.x;
          xq[pt][2 * e + 1] = f.y;
        }
      }
      float m0f = 0.f, m1f = 0.f;
#pragma unroll
      for (int pt = 0; pt < 2; ++pt)
#pragma unroll
        for (int j = 0; j < 8; j += 4) {
          m0f = amax3(m0f, xq[pt][j], xq[pt][j + 1]);
          m1f = amax3(m1f, xq[pt][j + 2], xq[pt][j + 3]);
        }
      const float mxf = __builtin_fmaxf(m0f, m1f);
      const int sx = stat_scale_exp(2.f * __uint_as_float(wave_umax(__float_as_uint(mxf))));
      if (l == 0) wsc[par * 32 + wave * 4 + h] = sx - 7;    // X = D 2^-(sx - 7): the table's 2^-7
      const float S = __int_as_float((sx + 127) << 23);
      uint32_t ah[4], dh[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float u0 = xq[1][2 * e] * S, u1 = xq[1][2 * e + 1] * S;
        ah[e] = pk_rne(fmaf(xq[0][2 * e], S, u0), fmaf(xq[0][2 * e + 1], S, u1));
        dh[e] = pk_rne(fmaf(xq[0][2 * e], S, -u0), fmaf(xq[0][2 * e + 1], S, -u1));
      }
      const f16x8 bah = frag(ah[0], ah[1], ah[2], ah[3]), bdh = frag(dh[0], dh[1], dh[2], dh[3]);
      f32x4 acc4[4];
#pragma unroll
      for (int pr = 0; pr < 2; ++pr)
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
          const f16x8 af = afr[pr][mt];
          acc4[2 * pr + mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, pr ? bdh : bah, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        }
      char* xb = slot + 2048 * h;
#pragma unroll
      for (int pr = 0; pr < 2; ++pr)
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
          *reinterpret_cast<uint32_t*>(xb + xwb[pr] + 1024 * mt) = pk_rne(acc4[2 * pr + mt][0], acc4[2 * pr + mt][1]);
          *reinterpret_cast<uint32_t*>(xb + xwb[pr] + 1024 * mt + 128) = pk_rne(acc4[2 * pr + mt][2], acc4[2 * pr + mt][3]);
        }
    }
  };

  // ---- A fragments of the wave's bins f = 4 wave + fb for all 8 tokens and 4 K-steps, read once
  // per tile (bcfft_dm64.hip's stage-2 operand: re rows [Xr, Xi], im rows [Xi, -Xr] by v_perm +
  // v_pk_mul_f16, which also brings the token's quarters to its smallest exponent; bin 0 with
  // the extra 1/2)
  f16x8 areg[BW][KS];
  auto load_a = [&](char* region, int par) {
    const int ml = opaque(lane);
    const int arow = ml & 15, kb = ml >> 4;
    const int a_t = arow >> 1, a_reim = arow & 1;
    const uint32_t a_sel = a_reim ? 0x01000302u : 0x03020100u;
    const int* sc = wsc + par * 32 + a_t * 4;
    int nk[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) nk[ks] = sc[ks];
    const int nmin = min(min(nk[0], nk[1]), min(nk[2], nk[3]));
    uint32_t amul[KS], amul0[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int d = nk[ks] - nmin;
      const uint32_t hh = d <= 14 ? (uint32_t)(15 - d) << 10 : (d <= 24 ? 1u << (24 - d) : 0u);
      const int d0 = d + 1;                          // bin 0: the inverse's 1/b vs 2/b
      const uint32_t h0 = d0 <= 14 ? (uint32_t)(15 - d0) << 10 : (d0 <= 24 ? 1u << (24 - d0) : 0u);
      amul[ks] = a_reim ? (hh | ((hh | 0x8000u) << 16)) : (hh | (hh << 16));
      amul0[ks] = a_reim ? (h0 << 16) : h0;
    }
    const int sw = 64 * (wave & 1);
    const char* ab_e = region + a_t * SLOT + 256 * wave + 16 * kb + sw;   // even fb: +64 fb
    const char* ab_o = region + a_t * SLOT + 256 * wave + 16 * kb - sw;   // odd fb
#pragma unroll
    for (int fb = 0; fb < BW; ++fb) {
      const int f = wave * BW + fb;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        uint4 raw = *reinterpret_cast<const uint4*>((fb & 1 ? ab_o : ab_e) + 64 * fb + 2048 * ks);
        if (f == 0) {
          raw.x = pkmul(raw.x, amul0[ks]); raw.y = pkmul(raw.y, amul0[ks]);
          raw.z = pkmul(raw.z, amul0[ks]); raw.w = pkmul(raw.w, amul0[ks]);
        } else {
          raw.x = pkmul(__builtin_amdgcn_perm(raw.x, raw.x, a_sel), amul[ks]);
          raw.y = pkmul(__builtin_amdgcn_perm(raw.y, raw.y, a_sel), amul[ks]);
          raw.z = pkmul(__builtin_amdgcn_perm(raw.z, raw.z, a_sel), amul[ks]);
          raw.w = pkmul(__builtin_amdgcn_perm(raw.w, raw.w, a_sel), amul[ks]);
        }
        areg[fb][ks] = __builtin_bit_cast(f16x8, raw);
      }
    }
  };

  // ---- stage 2 of group g (all waves, bins 4 wave + fb, all 8 tokens): four passes over the
  // double-buffered B registers. Pass p consumes breg[p & 1] and refills it fragment by fragment
  // with pass p + 2's; passes 0 and 1 are in flight on entry. Y half-units go over the tile's X
  // units (the X reads are done): bcfft_dm64.hip's map.
  auto stage2 = [&](char* region, int g) {
    constexpr float YS = 1.f / 2097152.f;            // 2^-21
    const int ml = opaque(lane);
    const int yt = ml >> 4;
    f32x4 acc[BW];
    uint32_t yh[BW][NT][2];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      Breg& br = breg[p & 1];
      const __amdgpu_buffer_rsrc_t brs = b_rsrc(g);
      const int vo = opaque(lane) * 16;
      const int nt = pass_nt(p);
#pragma unroll
      for (int j = 0; j < PF; ++j) {
        const int fb = j >> 1, ks = pass_ks(p, j);
        const f16x8 bf = __builtin_bit_cast(f16x8, br[j]);
        if (ks == 0)
          acc[fb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(areg[fb][0], bf, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        else
          acc[fb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(areg[fb][ks], bf, acc[fb], 0, 0, 0);
        if (p < 2) load_b1(brs, vo, p + 2, j, br);  // pass p + 2 into the same register
      }
      if ((p & 1) == 1) {                             // N-tile nt done: rows 4 yt + r are token
#pragma unroll                                        // 2 yt + (r >> 1), re/im r & 1
        for (int fb = 0; fb < BW; ++fb)
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) yh[fb][nt][s2] = pk_rne(acc[fb][2 * s2] * YS, acc[fb][2 * s2 + 1] * YS);
      }
    }
    const int ox = 16 * ((wave >> 1) & 1);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      char* yb = region + (2 * yt + s2) * SLOT + 256 * wave;
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {             // yhalf64(wave, 16 nt + o16, par)
        const int oo = 8 * ((16 * nt + (ml & 15)) ^ ox);
        *reinterpret_cast<uint2*>(yb + oo) = make_uint2(yh[0][nt][s2], yh[2][nt][s2]);
        *reinterpret_cast<uint2*>(yb + 2048 + oo) = make_uint2(yh[1][nt][s2], yh[3][nt][s2]);
      }
    }
  };

  // ---- stage 3 of group g (wave w, token slot w of this tile): bcfft_dm64.hip's
  auto stage3 = [&](char* region, int par, int64_t m, int g, auto&& before_stores) {
    const int l = opaque(lane);
    const int o16 = l & 15, gq = l >> 4;
    char* slot = region + wave * SLOT;
    const int* sc = wsc + par * 32 + wave * 4;
    const int nmin = min(min(sc[0], sc[1]), min(sc[2], sc[3]));
    float ysc[NT];                                  // output block o = 16 nt + o16: 1 / s_o
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) ysc[nt] = __builtin_ldexpf(osl[g * NOG + 16 * nt + o16], 30 - nmin);
    uint4 yf[2][NT];
#pragma unroll
    for (int pr = 0; pr < 2; ++pr)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const int o = 16 * nt + o16;
        const uint2 lo = *reinterpret_cast<const uint2*>(slot + yhalf64(2 * gq, o, pr));
        const uint2 hi = *reinterpret_cast<const uint2*>(slot + yhalf64(2 * gq + 1, o, pr));
        yf[pr][nt] = make_uint4(lo.x, lo.y, hi.x, hi.y);
      }
    f16x8 gt[2][2];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        const int t = 16 * mt + o16;
        gt[mt][pr] = *reinterpret_cast<const f16x8*>(lds + F_OFF + 128 * t + 16 * ((4 * pr + gq) ^ fsw64(t)));
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // Y is in registers: the slot is free
    const int64_t tok = m * TT + wave;
    const bool tok_ok = tok < n_tokens;
    const int nvalid = n_out - g * OPG;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      f32x4 E[NT], O[NT];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        E[nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(gt[mt][0], __builtin_bit_cast(f16x8, yf[0][nt]), f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        O[nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(gt[mt][1], __builtin_bit_cast(f16x8, yf[1][nt]), f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      }
      if constexpr (GLU) {                          // h = silu(gate) * up of block o16
        float gu[NT][2][4];
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
          for (int hf = 0; hf < 2; ++hf)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              gu[nt][hf][r] = round_to(hf ? fmaf(E[nt][r], ysc[nt], -O[nt][r] * ysc[nt]) : fmaf(E[nt][r], ysc[nt], O[nt][r] * ysc[nt]), XT);
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = round_to(round_to(silu(gu[0][hf][r]), XT) * gu[1][hf][r], XT);
          *reinterpret_cast<uint2*>(slot + 128 * o16 + 8 * ((4 * mt + gq + 8 * hf) ^ o16)) =
              make_uint2(pack16<XT>(v[0], v[1]), pack16<XT>(v[2], v[3]));
        }
      } else {
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
            if (HB) {                               // .to(x dtype) :266, + bias :270-271
#pragma unroll
              for (int r = 0; r < 4; ++r) v[r] = round_to(v[r], XT);
              if (o < nvalid) {
                const int64_t cc = (int64_t)(g * NOG + o) * B + 16 * mt + 4 * gq + 32 * hf;
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] += load_scalar(bias, cc + r, bias_dt);
              }
            }
            *reinterpret_cast<uint2*>(slot + 128 * o + 8 * ((4 * mt + gq + 8 * hf) ^ o16)) =
                make_uint2(pack16<XT>(v[0], v[1]), pack16<XT>(v[2], v[3]));
          }
        }
      }
    }
    before_stores();
    constexpr int RB = B * ESY;
    constexpr int NQ = GLU ? 2 : 4;
    const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
        (char*)yv + (tok_ok ? tok : 0) * M * ESY + (int64_t)g * OPG * RB, 0,
        tok_ok ? (int)((M - (int64_t)g * OPG * B) * ESY) : 0, 0x00020000);
    const int w = l & 7, lr = l >> 3;
    const int vofs = lr * RB + 16 * w;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int rr = 8 * q + lr;
      uint4 v = *reinterpret_cast<const uint4*>(slot + 128 * rr + 16 * (w ^ ((rr & 15) >> 1)));
      if (lr & 1) v = make_uint4(v.z, v.w, v.x, v.y);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), yrs, vofs + q * 1024, 0, BCFFT_YAUX);
    }
  };

  // Pipeline per 8-token tile m (bcfft_dmg.hip's; region R = it & 1 holds its x, R' is free):
  //   LDS-DMA of x(m + stride) into R'; stage 1 of token w in R                       | Ba |
  //   A fragments of the wave's bins -> VGPRs; B pass 1 of group 0                     | Bx |
  //   per group g: stage 2 (B passes streamed; Y half-units into R)                    | Bb |
  //                B pass 0 of the next group (or of the next tile's group 0); stage 3
  //                of token w, B pass 1 of the next group, stores                      | Bc |
  int it = 0;
  for (int64_t m = m0; m < n_mtiles; m += gstride, ++it) {
    char* region = lds + (it & 1) * REGION;
    char* other = lds + ((it + 1) & 1) * REGION;
    const int par = it & 1;
    const bool dma = m + gstride < n_mtiles;
    if (dma) dma_token(m + gstride, other);         // R' was released by the previous tile's Bc
    stage1(region, par);
    lds_barrier();                                  // Ba: X units and scales complete
    load_a(region, par);
    load_pass(0, 1, breg[1]);
    lds_barrier();                                  // Bx: every wave holds its A fragments
    for (int g = 0; g < n_groups; ++g) {
      stage2(region, g);
      lds_barrier();                                // Bb: Y units complete
      const bool more = g + 1 < n_groups;
      if (more) load_pass(g + 1, 0, breg[0]);
      else if (dma) load_pass(0, 0, breg[0]);       // the next tile's group 0 (consumed there)
      stage3(region, par, m, g, [&] {
        if (more) load_pass(g + 1, 1, breg[1]);
      });
      lds_barrier();                                // Bc: staging reads done (slots reusable)
    }
  }
}

}  // namespace bcfft

namespace {
template <bool GLU, bool HB>
void launch_dm64g(const void* x, int64_t n, int n_out, const void* spec, const void* bias, int bias_dt, void* y,
                  hipStream_t s) {
  const int groups = GLU ? (n_out + 15) / 16 : (n_out + 31) / 32;
  const bcfft::SpecLayout sl = bcfft::spec_layout(GLU ? 32 * groups : n_out, 64, 64);
  const int64_t n_mtiles = (n + 7) / 8;
  int64_t total = bcfft::device_cu_count();
  if (total > n_mtiles) total = n_mtiles;
  const uint32_t* stat = reinterpret_cast<const uint32_t*>(spec) + sl.stat_off_u32;
  const float* osc = reinterpret_cast<const float*>(spec) + sl.osc_off_u32;
  hipLaunchKernelGGL((bcfft::bc_forward_dm64g_kernel<GLU, HB>), dim3((unsigned)total), dim3(512), 0, s, x, n, n_out,
                     stat, osc, bias, bias_dt, y);
}
}  // namespace

namespace bcfft {
// b = 64, K = 4096, bf16 x and y, three or more output groups (GLU: groups of 16 gate + 16 up
// blocks), at most dm64g::MAXG groups. With two groups the per-group kernel is 4 % faster
// (4096^2: 50.0 vs 52.0 us, profiles/r03_ab_dm64g.log); from three the shared stage 1 wins
// (4096 -> 11008: 137 -> 113 us; fused gate/up: 262 -> 194 us).
bool dm64g_eligible(int n_in, int b, int xdt, bool yf32, int n_out, bool glu) {
  const int groups = glu ? (n_out + 15) / 16 : (n_out + 31) / 32;
  return dm64_eligible(n_in, b, xdt, yf32) && groups >= 3 && groups <= dm64g::MAXG;
}

void launch_forward_dm64g(const void* x, int64_t n, int n_out, const void* spec, const void* bias, int bias_dt,
                          void* y, bool glu, hipStream_t s) {
  if (glu) launch_dm64g<true, false>(x, n, n_out, spec, nullptr, BCFFT_NONE, y, s);
  else if (bias_dt != BCFFT_NONE) launch_dm64g<false, true>(x, n, n_out, spec, bias, bias_dt, y, s);
  else launch_dm64g<false, false>(x, n, n_out, spec, bias, bias_dt, y, s);
}
}  // namespace bcfft
