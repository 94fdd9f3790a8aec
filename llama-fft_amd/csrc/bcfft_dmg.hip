// bcfft_dmg.hip — the DFT-on-MFMA block-circulant forward for layers with several output groups
// (gfx950): bf16 I/O, b = 128, K = 4096, M > 4096 — the LLaMA gate / up projections 4096 -> 11008
// (BASELINE config 2) and their fused gate/up + SwiGLU.
//
// Same operator as the other DFT kernels (BlockCirculantLinear.forward, patch_llama_fft.py:
// 226-275; per block src/fft_utils.py:3-34) and the same three matrix-core stages as
// bcfft_dm8.hip: forward block DFT (stage 1), per-bin complex MAC (stage 2), inverse block DFT
// (stage 3). bcfft_dm8.hip keeps ONE output group's weight spectra in VGPRs, so a layer with G
// groups runs G workgroups per token tile and each of them repeats stage 1 on the same x tile
// (and reads x from HBM again unless the XCD map lines the groups up). Here one workgroup owns a
// token tile for ALL its groups:
//
//  * stage 1 runs once per 8-token tile (wave w: token w), X units in LDS as in bcfft_dm8.hip;
//  * every wave then takes the A fragments of its 8 bins for all 8 tokens into VGPRs (64), with
//    the per-token exponent alignment and the im-row transform applied once for all groups;
//  * per output group g: stage 2 against g's fp16 B fragments (the STAT image), streamed from
//    L2 in four passes of 8 (K-step, N-tile) fragments, double-buffered in 64 VGPRs; the Y units
//    go into the tile's LDS slots (the X units are in registers by then); stage 3 of token w
//    (y staged in the slot, 1 KiB stores of group g's 32 rows);
//  * the next tile's x streams into the other LDS region from the start of the tile (LDS-DMA).
//
// So stage 1 and the x read happen once per tile instead of once per group, and the weight
// stream from L2 is 256 KiB per group per 8-token tile (32 KiB per token and group).
//
// Numerics: bcfft_dm8.hip's (a, d, X and Y one RNE fp16 term each, C and the table one term each,
// per-output-block weight scales, fp32 accumulation; tests/dm_model.py, single_x).
//
// LDS (156,800 B): two regions x 8 token slots of 8,256 B (x -> X units -> Y units -> y staging),
// the DFT table, the scale exponents, the inverse weight scales of up to 64 groups. In-slot
// layouts are bcfft_dm8.hip's (checked conflict-free by tools/lds_banks_dm.py).
#ifndef BCFFT_STREAM_POLICY
#define BCFFT_STREAM_POLICY 1                       // nt x / sc1 y: the weight fragments stay in L2 (bcfft_device.h)
#endif
#include "bcfft_device.h"
#include "bcfft_dm_table.h"
#include "bcfft_dm_common.h"

namespace bcfft {

namespace dmg {
using namespace dmh;
// analysis builds only (results are WRONG when set): 1 no B loads, 2 no stage-1 arithmetic, 4 no
// stage-2 MFMAs, 8 no stage 3, 16 no x DMA, 32 no y stores
#ifdef BCFFT_DMG_ABL
constexpr int ABL = BCFFT_DMG_ABL;
#else
constexpr int ABL = 0;
#endif

constexpr int B = 128, NI = 32, KS = 2, NOG = 32, TT = 8, NW = 8;
constexpr int BW = 8, NT = 2;                       // bins per wave, 16-wide N-tiles per group
constexpr int K = NI * B;
constexpr int SLOT = 8192 + 64;                     // one token
constexpr int REGION = TT * SLOT;
constexpr int F_OFF = 2 * REGION;                   // DFT table image, 64 rows x 256 B
constexpr int SC_OFF = F_OFF + 16384;               // scale exponents [2 parity][8 token][2 half]
constexpr int OS_OFF = SC_OFF + 128;                // inverse weight scales [MAXG][32]
constexpr int MAXG = 64;
constexpr int LDS_BYTES = OS_OFF + MAXG * NOG * 4;
constexpr int NPIECE = BW * KS * NT;                // B fragments per wave and group (STAT image)
constexpr int NDMA = K * 2 / 1024;                  // 1-KiB LDS-DMA pieces per token (bf16 x)
static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
static_assert(F_OFF % 256 == 0, "table rows on the bank period");

// (K-step, N-tile) pass p of stage 2, N-tile-major (one N-tile's accumulators live at a time):
// its fragment of bin fb sits at STAT piece (fb KS + ks) NT + nt
__host__ __device__ constexpr int pass_ks(int p) { return p & 1; }
__host__ __device__ constexpr int pass_nt(int p) { return p >> 1; }
}  // namespace dmg

// HB: a bias is added (the runtime bias_dt then names its dtype); without one the store path is
// straight-line (a runtime test per stored quad split stage 3 into hundreds of basic blocks)
template <bool GLU, bool HB>
__global__ __launch_bounds__(512, 2) void bc_forward_dmg_kernel(
    const void* __restrict__ xv, int64_t n_tokens, int n_out, const uint32_t* __restrict__ stat,
    const float* __restrict__ osc, const void* __restrict__ bias, int bias_dt, void* __restrict__ yv) {
  using namespace dmg;
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
  ANALYSIS_INIT;
  const uint4* bimg = reinterpret_cast<const uint4*>(stat + 4);

  // ---- x of token `wave` of M-tile m -> its slot by LDS-DMA (bcfft_dm8.hip's: the buffer range
  // zero-fills tokens past n_tokens; the slot's unit swizzle is applied to the source offsets)
  auto dma_token = [&](int64_t m, char* region, int sl) {   // token slot sl of tile m
    if constexpr ((ABL & 16) != 0) return;
    const int64_t tok = m * TT + sl;
    const bool ok = tok < n_tokens;
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<char*>((const char*)xv) + (ok ? tok : 0) * K * ES, 0, ok ? K * ES : 0, 0x00020000);
    const int dl = opaque(lane);
    const uint32_t dst0 = lds_base + (uint32_t)(region - lds) + sl * SLOT;
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

  // ---- B fragments of group g, pass p (K-step, N-tile) for the wave's 8 bins, from L2. These
  // are compiler-visible buffer loads: the compiler places the waits before their uses. It does
  // not count the asm x DMA, so a wait it computes can only cover MORE operations than needed
  // (the x DMA issued between two B passes is then drained early), never fewer. (Asm loads with
  // hand-counted waits were wrong here: the register allocator copied in-flight results.)
  typedef u32x4 Breg[BW];
  auto b_rsrc = [&](int g) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint4*>(bimg + ((int64_t)(g * NW + wave) * NPIECE) * 64), 0,
                                             NPIECE * 1024, 0x00020000);
  };
  auto load_b1 = [&](const __amdgpu_buffer_rsrc_t& brs, int vo, int p, int fb, Breg& br) {
    if constexpr ((ABL & 1) != 0) br[fb] = u32x4{(uint32_t)vo, (uint32_t)p, (uint32_t)fb, 0u};
    else br[fb] = __builtin_amdgcn_raw_buffer_load_b128(brs, vo, ((fb * KS + pass_ks(p)) * NT + pass_nt(p)) * 1024, 0);
  };
  auto load_pass = [&](int g, int p, Breg& br) {
    const __amdgpu_buffer_rsrc_t brs = b_rsrc(g);
    const int vo = opaque(lane) * 16;
#pragma unroll
    for (int fb = 0; fb < BW; ++fb) load_b1(brs, vo, p, fb, br);
  };

  // ---- prologue: the first tile's x, the DFT table, every group's inverse weight scales, the
  // first group's first B pass
  Breg breg[2];
  const int64_t m0 = blockIdx.x;
  dma_token(m0, lds, wave);
  {
    const uint4* tab = reinterpret_cast<const uint4*>(kDmF);
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int c = tid + 512 * r;                  // chunk c: row c >> 4, chunk c & 15
      const int t = c >> 4, ch = c & 15;
      *reinterpret_cast<uint4*>(lds + F_OFF + 256 * t + 16 * (ch ^ fsw(t))) = tab[c];
    }
    for (int e = tid; e < n_groups * NOG; e += 512) reinterpret_cast<float*>(lds + OS_OFF)[e] = osc[e];
  }
  wait_vmcnt<0>();
  load_pass(0, 0, breg[0]);
  lds_barrier();

  // ---- stage 1 (wave w, token slot w): x rows -> X units (one fp16 term), in place, per half
  // (bcfft_dm8.hip's stage 1)
  auto stage1 = [&](char* region, int par) {
    if constexpr ((ABL & 2) != 0) {
      if (lane < 2) wsc[par * 16 + wave * 2 + lane] = 0;
      return;
    }
    const int l = opaque(lane);
    const int b16 = l & 15, g = l >> 4;
    char* slot = region + wave * SLOT;
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
      float m0f = 0.f, m1f = 0.f;                   // max |x|: two v_max3_f32 chains
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
      const int sx = stat_scale_exp(2.f * __uint_as_float(wave_umax(__float_as_uint(mxf))));   // |a|, |d| <= 2 max|x|
      if (l == 0) wsc[par * 16 + wave * 2 + h] = sx - 7;    // X = D 2^-(sx - 7): the table's 2^-7
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

  // ---- A fragments of the wave's bins f = 8 wave + fb for all 8 tokens, read once per tile: A
  // rows (token t = row >> 1, re/im): re rows [Xr, Xi] per block, im rows [Xi, -Xr] (v_perm +
  // v_pk_mul_f16, which also brings the token's two halves to its smaller exponent); bin 0
  // (X0, X64) with the extra 1/2 (bcfft_dm8.hip's stage-2 operand)
  f16x8 areg[BW][KS];
  auto load_a = [&](char* region, int par) {
    const int ml = opaque(lane);
    const int arow = ml & 15, kb = ml >> 4;
    const int a_t = arow >> 1, a_reim = arow & 1;
    const uint32_t a_sel = a_reim ? 0x01000302u : 0x03020100u;
    const int* sc = wsc + par * 16;
    int nk[KS];
    nk[0] = sc[a_t * 2];
    nk[1] = sc[a_t * 2 + 1];
    const int nmin = min(nk[0], nk[1]);
    uint32_t amul[KS], amul0[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int d = nk[ks] - nmin;                  // factor 2^-d (fp16; subnormal / 0 far down)
      const uint32_t hh = d <= 14 ? (uint32_t)(15 - d) << 10 : (d <= 24 ? 1u << (24 - d) : 0u);
      const int d0 = d + 1;                          // bin 0: the inverse's 1/b vs 2/b
      const uint32_t h0 = d0 <= 14 ? (uint32_t)(15 - d0) << 10 : (d0 <= 24 ? 1u << (24 - d0) : 0u);
      amul[ks] = a_reim ? (hh | ((hh | 0x8000u) << 16)) : (hh | (hh << 16));
      amul0[ks] = a_reim ? (h0 << 16) : h0;
    }
    const char* ab = region + a_t * SLOT + 512 * wave + 16 * kb;
#pragma unroll
    for (int fb = 0; fb < BW; ++fb) {
      const int f = wave * BW + fb;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {               // xunit8(ks, 8 wave + fb, kb) - 512 wave
        uint4 raw = *reinterpret_cast<const uint4*>(ab + 4096 * ks + 64 * (fb ^ ((fb >> 2) & 1)));
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

  // ---- stage 2 of group g (all waves, bins 8 wave + fb, all 8 tokens): four passes (K-step,
  // N-tile) over the double-buffered B registers. Pass p consumes breg[p & 1] and refills it bin
  // by bin with pass p + 2's fragments; passes 0 and 1 are in flight on entry. Y units go over the
  // tile's X units (the X reads are done).
  auto stage2 = [&](char* region, int g) {
    constexpr float YS = 1.f / 2097152.f;            // 2^-21: |Y| < 2^14 in fp16
    const int ml = opaque(lane);
    const int yt = ml >> 4;
    f32x4 acc[BW];
    uint32_t yh[BW][NT][2];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      Breg& br = breg[p & 1];
      const __amdgpu_buffer_rsrc_t brs = b_rsrc(g);
      const int vo = opaque(lane) * 16;
      const int ks = pass_ks(p), nt = pass_nt(p);
#pragma unroll
      for (int fb = 0; fb < BW; ++fb) {
        const f16x8 bf = __builtin_bit_cast(f16x8, br[fb]);
        if constexpr ((ABL & 4) != 0)
          acc[fb] = ks == 0 ? f32x4{bf[0], bf[1], areg[fb][0][0], 0.f} : acc[fb] + f32x4{bf[0], bf[1], areg[fb][1][0], 0.f};
        else if (ks == 0)
          acc[fb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(areg[fb][0], bf, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        else
          acc[fb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(areg[fb][1], bf, acc[fb], 0, 0, 0);
        if (p < 2) load_b1(brs, vo, p + 2, fb, br);  // pass p + 2 into the same register
      }
      if (ks == 1) {                                  // N-tile nt done: rows 4 yt + r are token
#pragma unroll                                        // 2 yt + (r >> 1), re/im r & 1
        for (int fb = 0; fb < BW; ++fb)
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) yh[fb][nt][s2] = pk_rne(acc[fb][2 * s2] * YS, acc[fb][2 * s2 + 1] * YS);
      }
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      char* yb = region + (2 * yt + s2) * SLOT + 512 * wave + 16 * (ml & 15);
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {             // yunit8(wave, 16 nt + o16, par)
        *reinterpret_cast<uint4*>(yb + 256 * nt) = make_uint4(yh[0][nt][s2], yh[2][nt][s2], yh[4][nt][s2], yh[6][nt][s2]);
        *reinterpret_cast<uint4*>(yb + 4096 + 256 * nt) = make_uint4(yh[1][nt][s2], yh[3][nt][s2], yh[5][nt][s2], yh[7][nt][s2]);
      }
    }
  };

  // ---- stage 3 of group g (wave w, token slot w of this tile): Y -> y rows staged in the slot
  // (32 rows x 256 B; GLU: 16 h rows) and stored as 1 KiB buffer stores (bcfft_dm8.hip's).
  auto stage3 = [&](char* region, int par, int64_t m, int g, auto&& before_stores) {
    if constexpr ((ABL & 8) != 0) {
      before_stores();
      return;
    }
    const int l = opaque(lane);
    const int o16 = l & 15, gq = l >> 4;
    char* slot = region + wave * SLOT;
    const int* sc = wsc + par * 16 + wave * 2;
    const int nmin = min(sc[0], sc[1]);
    float ysc[NT];                                  // output block o = 16 nt + o16: 1 / s_o
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) ysc[nt] = __builtin_ldexpf(osl[g * NOG + 16 * nt + o16], 30 - nmin);
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
    const int64_t tok = m * TT + wave;
    const bool tok_ok = tok < n_tokens;
    const int nvalid = n_out - g * OPG;
    int swb[4];
    {
      const int sg = ((o16 & 7) << 1) | (o16 >> 3);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) swb[mt] = 256 * o16 + 8 * ((4 * mt + gq) ^ sg);
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
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          E[nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(gcur[ks][0], __builtin_bit_cast(f16x8, yf[ks][0][nt]), E[nt], 0, 0, 0);
          O[nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(gcur[ks][1], __builtin_bit_cast(f16x8, yf[ks][1][nt]), O[nt], 0, 0, 0);
        }
      if (mt < 3) gload(mt + 1, gcur);
      if constexpr (GLU) {                          // h = silu(gate) * up of block o16
        float gu[NT][2][4];
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
          for (int hf = 0; hf < 2; ++hf)
#pragma unroll
            for (int r = 0; r < 4; ++r)             // gate / up rounded to x's dtype (:266)
              gu[nt][hf][r] = round_to(hf ? fmaf(E[nt][r], ysc[nt], -O[nt][r] * ysc[nt]) : fmaf(E[nt][r], ysc[nt], O[nt][r] * ysc[nt]), XT);
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r)               // torch: silu rounded, then the product rounded
            v[r] = round_to(round_to(silu(gu[0][hf][r]), XT) * gu[1][hf][r], XT);
          *reinterpret_cast<uint2*>(slot + swb[mt] + 128 * hf) = make_uint2(pack16<XT>(v[0], v[1]), pack16<XT>(v[2], v[3]));
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
                const int64_t cc = (int64_t)(g * NOG + o) * B + 16 * mt + 4 * gq + 64 * hf;
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] += load_scalar(bias, cc + r, bias_dt);
              }
            }
            *reinterpret_cast<uint2*>(slot + 4096 * nt + swb[mt] + 128 * hf) =
                make_uint2(pack16<XT>(v[0], v[1]), pack16<XT>(v[2], v[3]));
          }
        }
      }
    }
    before_stores();
    // staged rows -> global: each instruction stores 1 KiB = 4 whole rows (16 lanes per row); the
    // group's y rows start the buffer (rows past nvalid fall outside it and are dropped)
    constexpr int RB = B * ESY;
    constexpr int NQ = GLU ? 4 : 8;
    const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
        (char*)yv + (tok_ok ? tok : 0) * M * ESY + (int64_t)g * OPG * RB, 0,
        tok_ok ? (int)((M - (int64_t)g * OPG * B) * ESY) : 0, 0x00020000);
    const int w = l & 15, lr = l >> 4;
    const int vofs = lr * RB + 16 * w;
    int rdb[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) rdb[c] = lr * RB + 16 * ((w ^ lr) ^ (4 * c));
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      uint4 v = *reinterpret_cast<const uint4*>(slot + 1024 * q + rdb[q & 1]);
      if (q & 2) v = make_uint4(v.z, v.w, v.x, v.y);   // rows with bit 3: 8-B halves swapped
      if constexpr ((ABL & 32) != 0) {
        if (v.x == 0x7fc00001u && tok < 0) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), yrs, vofs, 0, BCFFT_YAUX);
      } else {
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), yrs, vofs + q * 1024, 0, BCFFT_YAUX);
      }
    }
  };

  // Pipeline per 8-token tile m (region R = it & 1 holds its x; R' is free):
  //   LDS-DMA of x(m + stride) into R'; stage 1 of token w in R                       | Ba |
  //   A fragments of the wave's bins -> VGPRs; B pass 1 of group 0                     | Bx |
  //   per group g: stage 2 (B passes streamed; Y units into R)                         | Bb |
  //                B pass 0 of the next group (or of the next tile's group 0); stage 3
  //                of token w (y staged in slot w), B pass 1 of the next group (not of
  //                the next tile: its registers stay free through stage 1), stores     | Bc |
  // Per wave, waiting for a B pass drains every older VMEM operation, so the x DMA of tile
  // m + stride is complete after group 0's pass 1 of tile m, at the latest.
  constexpr int NST = GLU ? 4 : 8;                  // y stores per wave and group
  int it = 0;
  // stamps build (tools/timeline_dmg.py): slots of the workgroup's second tile, 0 top | 1 DMA
  // issued | 2 stage 1 | 3 Ba | 4 A fragments | 5 Bx | per group g < 4: 6 + 4g stage 2 | 7 + 4g
  // Bb | 8 + 4g stage 3 | 9 + 4g Bc
#define DGS(o) do { if (it == 1) STAMP(o); } while (0)
  for (int64_t m = m0; m < n_mtiles; m += gstride, ++it) {
    char* region = lds + (it & 1) * REGION;
    char* other = lds + ((it + 1) & 1) * REGION;
    const int par = it & 1;
    const bool dma = m + gstride < n_mtiles;
    DGS(0);
    if (dma) dma_token(m + gstride, other, wave);   // R' was released by the previous tile's Bc
    DGS(1);
    stage1(region, par);
    DGS(2);
    lds_barrier();                                  // Ba: X units and scales complete
    DGS(3);
    load_a(region, par);
    load_pass(0, 1, breg[1]);
    DGS(4);
    lds_barrier();                                  // Bx: every wave holds its A fragments
    DGS(5);
    for (int g = 0; g < n_groups; ++g) {
      // group 0: [pass 0, (previous group's stores), (x DMA), pass 1]; later groups: [pass 0,
      // pass 1, previous group's stores]
      stage2(region, g);
      if (g < 4) DGS(6 + 4 * g);
      lds_barrier();                                // Bb: Y units complete
      if (g < 4) DGS(7 + 4 * g);
      const bool more = g + 1 < n_groups;
      if (more) load_pass(g + 1, 0, breg[0]);
      else if (dma) load_pass(0, 0, breg[0]);       // the next tile's group 0 (consumed there)
      stage3(region, par, m, g, [&] {
        if (more) load_pass(g + 1, 1, breg[1]);
      });
      if (g < 4) DGS(8 + 4 * g);
      lds_barrier();                                // Bc: staging reads done (slots reusable)
      if (g < 4) DGS(9 + 4 * g);
    }
  }
#undef DGS
}

}  // namespace bcfft

namespace {
template <bool GLU, bool HB>
void launch_dmg(const void* x, int64_t n, int n_out, const void* spec, const void* bias, int bias_dt, void* y,
                hipStream_t s) {
  const int groups = GLU ? (n_out + 15) / 16 : (n_out + 31) / 32;
  const bcfft::SpecLayout sl = bcfft::spec_layout(GLU ? 32 * groups : n_out, 32, 128);
  const int64_t n_mtiles = (n + 7) / 8;
  int64_t total = bcfft::device_cu_count();
  if (total > n_mtiles) total = n_mtiles;
  const uint32_t* stat = reinterpret_cast<const uint32_t*>(spec) + sl.stat_off_u32;
  const float* osc = reinterpret_cast<const float*>(spec) + sl.osc_off_u32;
  hipLaunchKernelGGL((bcfft::bc_forward_dmg_kernel<GLU, HB>), dim3((unsigned)total), dim3(512), 0, s, x, n, n_out, stat,
                     osc, bias, bias_dt, y);
}
}  // namespace

namespace bcfft {
// bf16 x and bf16 y (no bias or a bf16 bias), b = 128, K = 4096, two or more output groups (GLU:
// two or more groups of 16 gate + 16 up blocks), at most dmg::MAXG groups
bool dmg_eligible(int n_in, int b, int xdt, bool yf32, int n_out, bool glu) {
  const int groups = glu ? (n_out + 15) / 16 : (n_out + 31) / 32;
  return dm8_eligible(n_in, b, xdt, yf32) && groups >= 2 && groups <= dmg::MAXG;
}

void launch_forward_dmg(const void* x, int64_t n, int n_out, const void* spec, const void* bias, int bias_dt, void* y,
                        bool glu, hipStream_t s) {
  if (glu) launch_dmg<true, false>(x, n, n_out, spec, nullptr, BCFFT_NONE, y, s);
  else if (bias_dt != BCFFT_NONE) launch_dmg<false, true>(x, n, n_out, spec, bias, bias_dt, y, s);
  else launch_dmg<false, false>(x, n, n_out, spec, bias, bias_dt, y, s);
}
}  // namespace bcfft

BCFFT_STAMPS_SETTER(dmg)
