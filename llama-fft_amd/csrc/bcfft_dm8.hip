// bcfft_dm8.hip — the DFT-on-MFMA block-circulant forward for bf16 I/O, 8 tokens per M-tile
// (gfx950).
//
// Same operator and the same three matrix-core stages as bc_forward_dm_kernel (bcfft_dm.hip:
// BlockCirculantLinear.forward, patch_llama_fft.py:226-275; b = 128, K = 4096). With bf16
// outputs the output rounding (2^-9 relative) is far above the transforms' fp16 noise, so the
// per-bin spectra X are ONE fp16 term here instead of hi + lo. That frees the stage-2 MFMA rows
// the lo terms took: a tile carries 8 tokens x (re, im) = 16 rows, which halves the stage-2
// work per token. bf16 x is 8 KiB per token, so 8 tokens still fit two 64 KiB LDS regions.
//
//  * Wave roles per M-tile: wave w does stage 1 (x -> X) of token w of this tile, then stage 3
//    (Y -> y, 1 KiB stores) of token w of the previous tile, then streams the next tile's x for
//    token w into the slot it just emptied (LDS-DMA). Every slot has one owner, so no barrier
//    or counter is shared between waves for x. All 8 waves then run the per-bin complex MAC
//    (stage 2) on their 8 bins. Two workgroup barriers per M-tile.
//  * Numerics: per-(token, half) power-of-two scales; a, d, X, Y one RNE fp16 term each, C and
//    the table one term each, fp32 accumulation: ~5e-4 relative before the bf16 output rounding
//    (tests/dm_model.py, `single_x`).
//
// LDS (148,608 B): two regions x 8 token slots of 8,256 B (x -> X units -> Y units -> y
// staging), the DFT table, the scales. The slot stride is 64 B off the 256-B bank period so
// that stage 2's reads of eight tokens at once are conflict-free (tools/lds_banks_dm.py checks
// every access).
#include "bcfft_device.h"
#include "bcfft_dm_table.h"
#include "bcfft_dm_common.h"

namespace bcfft {

namespace dm8 {
using namespace dmh;

constexpr int B = 128, NI = 32, KS = 2, NOG = 32, TT = 8, NW = 8;
constexpr int BW = 8, NT = 2;                       // bins per wave, 16-wide N-tiles per group
constexpr int K = NI * B;
constexpr int SLOT = 8192 + 64;                     // one token
constexpr int REGION = TT * SLOT;
constexpr int F_OFF = 2 * REGION;                   // DFT table image, 64 rows x 256 B
constexpr int SC_OFF = F_OFF + 16384;               // scale exponents [2 parity][8 token][2 half]
constexpr int OS_OFF = SC_OFF + 128;                // the group's 32 inverse weight scales
constexpr int LDS_BYTES = OS_OFF + 128;
static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
static_assert(F_OFF % 256 == 0, "table rows on the bank period");

// X unit (16 B: 4 input blocks 4q..4q+3 x (re, im) fp16 of bin f) of K-step ks in a token slot;
// bins 4 apart swap their 64-B blocks by bin bit 2 (stage-1 writes of two such bins at once)
__device__ __forceinline__ int xunit8(int ks, int f, int q) { return 4096 * ks + 64 * (f ^ ((f >> 2) & 1)) + 16 * q; }
// Y unit (16 B = 4 bins of parity par of wave w x (re, im) fp16) of output block o; lies over
// the K-step-par X units of wave w's bins
__device__ __forceinline__ int yunit8(int w, int o, int par) { return 4096 * par + 512 * w + 16 * o; }
}  // namespace dm8

// HB: a bias is added (the runtime bias_dt then names its dtype); without one the store path is
// straight-line (a runtime test per stored quad split stage 3 into ~300 basic blocks)
template <bool GLU, bool HB>
__global__ __launch_bounds__(512, 2) void bc_forward_dm8_kernel(
    const void* __restrict__ xv, int64_t n_tokens, int n_out, const uint32_t* __restrict__ stat,
    const float* __restrict__ osc, const void* __restrict__ bias, int bias_dt, void* __restrict__ yv) {
  using namespace dm8;
  constexpr int XT = BCFFT_BF16;
  constexpr int ES = 2, ESY = 2;
  constexpr int NPIECE = BW * KS * NT;
  constexpr int NDMA = K * ES / 1024;               // 1-KiB LDS-DMA pieces per token

  __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];
  int* wsc = reinterpret_cast<int*>(lds + SC_OFF);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // GLU (fused gate/up + SwiGLU): n_out counts h blocks; group g holds gate blocks [16g, 16g+16)
  // in N-tile 0 and the matching up blocks in N-tile 1, and stores 16 h rows
  constexpr int OPG = GLU ? NOG / 2 : NOG;
  const int n_groups = (n_out + OPG - 1) / OPG;
  const GroupMap gm = group_map(n_groups);          // XCD-aware when the grid allows it
  const int grp_o = gm.grp, wg_in_grp = gm.lane;
  const int64_t M = (int64_t)n_out * B;
  const int64_t n_mtiles = (n_tokens + TT - 1) / TT;
  const int gstride = gm.stride;
  const uint32_t lds_base = __builtin_amdgcn_readfirstlane(lds_addr(lds));
  ANALYSIS_INIT;
  STAMP(62);                                        // kernel entry (stamps builds: the prologue's length)

  // ---- x of token `wave` of M-tile m -> its slot by LDS-DMA (the buffer range zero-fills
  // tokens past n_tokens); piece q = rows 4q + (lane >> 4), 256 B each, with the slot's unit
  // swizzle (unit u of block row r at u ^ (r & 15)) applied to the global source offsets
  auto dma_token = [&](int64_t m, char* region, int sl) {
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

  // ---- prologue: first tile's x, the DFT table, the stationary B fragments
  if (wg_in_grp < n_mtiles) dma_token(wg_in_grp, lds, wave);
  {
    const uint4* tab = reinterpret_cast<const uint4*>(kDmF);
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int c = tid + 512 * r;                  // chunk c: row c >> 4, chunk c & 15
      const int t = c >> 4, ch = c & 15;
      *reinterpret_cast<uint4*>(lds + F_OFF + 256 * t + 16 * (ch ^ fsw(t))) = tab[c];
    }
  }
  f16x8 creg[BW][KS][NT];
  {
    const uint4* img = reinterpret_cast<const uint4*>(stat + 4) + ((int64_t)(grp_o * NW + wave) * NPIECE) * 64 + lane;
#pragma unroll
    for (int fb = 0; fb < BW; ++fb)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          creg[fb][ks][nt] = __builtin_bit_cast(f16x8, img[((fb * KS + ks) * NT + nt) * 64]);
    // pin the loads here (hipcc would otherwise sink them into the tile loop)
#pragma unroll
    for (int fb = 0; fb < BW; ++fb)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) asm volatile("" : "+v"(creg[fb][ks][nt]));
  }
  // the group's inverse weight scales 1 / s_o (per output block) -> LDS (after the weight loads: its wait must not hold them back)
  if (tid < 32) reinterpret_cast<float*>(lds + OS_OFF)[tid] = osc[grp_o * 32 + tid];
  wait_vmcnt<0>();
  lds_barrier();

  // ---- stage 1 (wave w, token slot w): x rows -> X units (one fp16 term), in place, per half.
  // xwait: this wave's x DMA of the token is in flight (pieces 0-3 = half 0, behind its older y
  // stores): wait for half 0 alone, then for half 1 after half 0's transform
  // XOFF: VMEM operations issued after the x DMA this wave waits for (the stage-3-first order
  // below has issued its 8 y stores and the next tile's 8 DMA pieces by then)
  auto stage1 = [&](char* region, int par, int sl, bool xwait, auto xoff_c) {
    constexpr int XOFF = decltype(xoff_c)::value;
    const int l = opaque(lane);
    const int b16 = l & 15, g = l >> 4;
    char* slot = region + sl * SLOT;
    // transposed-read lane address of the table: row 8g + q (+ 32 ks + 4 sec), chunk
    // (8 par + 2 mt + (p >> 1)) ^ fsw(row) = (8 par + 2 mt) ^ cx
    const int q4 = (l & 15) >> 2, p4 = l & 3;
    const int cx = (p4 >> 1) ^ fsw(8 * g + q4);
    const int trb = F_OFF + 256 * (8 * g + q4) + 8 * (p4 & 1);
    // X write lane bases: D^T row 4g + r is bin 16 mt + 4 g + pr (+ 2 for r >= 2), column block
    // b16 (unit quad b16 >> 2, 4 B at 4 (b16 & 3)); bin bit 2 = g & 1 swaps the 64-B blocks
    int xwb[2];
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) xwb[pr] = 256 * g + 64 * (pr ^ (g & 1)) + 4 * b16;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (xwait) {
        if (h == 0) wait_vmcnt<NDMA / 2 + XOFF>();
        else wait_vmcnt<XOFF>();
      }
      // x of blocks 16h + b16: t = 32 ks + 8 g + j and t + 64 (j < 8); the half's x rows are
      // exactly the bytes its X units replace
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
      float m0 = 0.f, m1 = 0.f;                     // max |x|: two v_max3_f32 chains
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int pt = 0; pt < 2; ++pt)
#pragma unroll
          for (int j = 0; j < 8; j += 4) {
            m0 = amax3(m0, xv8[ks][pt][j], xv8[ks][pt][j + 1]);
            m1 = amax3(m1, xv8[ks][pt][j + 2], xv8[ks][pt][j + 3]);
          }
      const float mxf = __builtin_fmaxf(m0, m1);
      const int sx = stat_scale_exp(2.f * __uint_as_float(wave_umax(__float_as_uint(mxf))));   // |a|, |d| <= 2 max|x|
      if (l == 0) wsc[par * 16 + sl * 2 + h] = sx - 7;      // X = D 2^-(sx - 7): the table's 2^-7
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
            // A = F^T (16 bins-reals x 32 t): two transposed reads of 4 rows each
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

  // ---- stage 2 (all waves): per-bin complex MAC on bins f = 8 wave + fb for all 8 tokens.
  // A rows (token t = row >> 1, re/im): re rows [Xr, Xi] per block, im rows [Xi, -Xr] (v_perm
  // + v_pk_mul_f16, which also brings the token's two halves to its smaller exponent); bin 0
  // (X0, X64) with the extra 1/2. Y units over the wave's own X units (in-order DS per wave).
  auto stage2 = [&](char* region, int par) {
    const int ml = opaque(lane);
    const int arow = ml & 15, kb = ml >> 4;
    const int a_t = arow >> 1, a_reim = arow & 1;
    const uint32_t a_sel = a_reim ? 0x01000302u : 0x03020100u;
    const int yt = ml >> 4;
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
    uint4 araw[BW][KS];
#pragma unroll
    for (int fb = 0; fb < BW; ++fb)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)               // xunit8(ks, 8 wave + fb, kb) - 512 wave
        araw[fb][ks] = *reinterpret_cast<const uint4*>(ab + 4096 * ks + 64 * (fb ^ ((fb >> 2) & 1)));
    uint32_t yh[BW][NT][2];
#pragma unroll
    for (int fb = 0; fb < BW; ++fb) {
      const int f = wave * BW + fb;
      f32x4 acc[NT];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        uint4 raw = araw[fb][ks];
        if (f == 0) {
          raw.x = pkmul(raw.x, amul0[ks]); raw.y = pkmul(raw.y, amul0[ks]);
          raw.z = pkmul(raw.z, amul0[ks]); raw.w = pkmul(raw.w, amul0[ks]);
        } else {
          raw.x = pkmul(__builtin_amdgcn_perm(raw.x, raw.x, a_sel), amul[ks]);
          raw.y = pkmul(__builtin_amdgcn_perm(raw.y, raw.y, a_sel), amul[ks]);
          raw.z = pkmul(__builtin_amdgcn_perm(raw.z, raw.z, a_sel), amul[ks]);
          raw.w = pkmul(__builtin_amdgcn_perm(raw.w, raw.w, a_sel), amul[ks]);
        }
        const f16x8 a = __builtin_bit_cast(f16x8, raw);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, creg[fb][ks][nt], acc[nt], 0, 0, 0);
      }
      constexpr float YS = 1.f / 2097152.f;          // 2^-21: |Y| < 2^14 in fp16
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)                // rows 4 yt + r: token 2 yt + (r >> 1), re/im r & 1
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) yh[fb][nt][s2] = pk_rne(acc[nt][2 * s2] * YS, acc[nt][2 * s2 + 1] * YS);
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

  // ---- stage 3 (wave w, token slot w of the previous tile): Y -> y rows staged in the slot
  // (32 rows x 256 B; GLU: 16 h rows) and stored as 1 KiB buffer stores. The slot's Y units are
  // read into registers first.
  auto stage3 = [&](char* region, int par, int64_t mp, int sl) {
    const int l = opaque(lane);
    const int o16 = l & 15, g = l >> 4;
    char* slot = region + sl * SLOT;
    const int* sc = wsc + par * 16 + sl * 2;
    const int nmin = min(sc[0], sc[1]);
    float ysc[NT];                                  // output block o = 16 nt + o16: 1 / s_o
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) ysc[nt] = __builtin_ldexpf(reinterpret_cast<const float*>(lds + OS_OFF)[16 * nt + o16], 30 - nmin);
    // all Y fragments of the token: B[k = 8 g + j][o] = yunit8(wave 4 ks + g, o, parity)
    uint4 yf[KS][2][NT];
    const char* yb = slot + 512 * g + 16 * o16;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int pr = 0; pr < 2; ++pr)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          yf[ks][pr][nt] = *reinterpret_cast<const uint4*>(yb + 4096 * pr + 2048 * ks + 256 * nt);
    // table row reads: row 16 mt + o16, chunk (8 par + 4 ks + g) ^ fsw(o16)
    const int gx = g ^ fsw(o16);
    const char* gb = lds + F_OFF + 256 * o16;
    auto gload = [&](int mt, f16x8 (&gf)[KS][2]) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int pr = 0; pr < 2; ++pr)
          gf[ks][pr] = *reinterpret_cast<const f16x8*>(gb + 4096 * mt + 16 * ((8 * pr + 4 * ks) ^ gx));
    };
    f16x8 gcur[KS][2], gnxt[KS][2];
    gload(0, gcur);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // Y is in registers: the slot is free
    const int64_t tok = mp * TT + sl;
    const bool tok_ok = tok < n_tokens;
    const int nvalid = n_out - grp_o * OPG;
    // staging write bases: row o = 16 nt + o16, 8-B unit (4 mt + g + 16 hf) ^ sg
    int swb[4];
    {
      const int sg = ((o16 & 7) << 1) | (o16 >> 3);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) swb[mt] = 256 * o16 + 8 * ((4 * mt + g) ^ sg);
    }
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      if (mt < 3) gload(mt + 1, gnxt);
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
      // rows t = 16 mt + 4 g + r (and t + 64), column o = 16 nt + o16
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
                const int64_t cc = (int64_t)(grp_o * NOG + o) * B + 16 * mt + 4 * g + 64 * hf;
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] += load_scalar(bias, cc + r, bias_dt);
              }
            }
            *reinterpret_cast<uint2*>(slot + 4096 * nt + swb[mt] + 128 * hf) =
                make_uint2(pack16<XT>(v[0], v[1]), pack16<XT>(v[2], v[3]));
          }
        }
      }
      if (mt < 3) {
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
#pragma unroll
          for (int pr = 0; pr < 2; ++pr) gcur[ks][pr] = gnxt[ks][pr];
      }
    }
    // staged rows -> global: each instruction stores 1 KiB = 4 whole rows (16 lanes per row); the
    // group's y rows start the buffer (rows past nvalid fall outside it and are dropped). LDS row
    // rr = 4 q + lr, unit w ^ (rr & 7) = (w ^ lr) ^ 4 (q & 1)
    constexpr int RB = B * ESY;
    constexpr int NQ = GLU ? 4 : 8;
    const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
        (char*)yv + (tok_ok ? tok : 0) * M * ESY + (int64_t)grp_o * OPG * RB, 0,
        tok_ok ? (int)((M - (int64_t)grp_o * OPG * B) * ESY) : 0, 0x00020000);
    const int w = l & 15, lr = l >> 4;
    const int vofs = lr * RB + 16 * w;
    int rdb[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) rdb[c] = lr * RB + 16 * ((w ^ lr) ^ (4 * c));
    uint4 d[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      uint4 v = *reinterpret_cast<const uint4*>(slot + 1024 * q + rdb[q & 1]);
      if (q & 2) v = make_uint4(v.z, v.w, v.x, v.y);   // rows with bit 3: 8-B halves swapped
      d[q] = v;
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, d[q]), yrs, vofs + q * 1024, 0, BCFFT_YAUX);
  };

  // Pipeline, two workgroup barriers per M-tile. Iteration it (region R = it & 1 holds tile m,
  // the other R' tile m - gstride); every wave w:
  //   P1  waits for its own x DMA, stage 1 of token w of tile m in R; stage 3 of token w of tile
  //       m - gstride from R' (stores issued); LDS-DMA of x(m + gstride, token w) into that
  //       slot of R' (its staging reads have completed)                               | Ba |
  //   P2  stage 2 of tile m in R                                                       | Bb |
  int64_t m = wg_in_grp;
  STAMP(0);
  for (int it = 0; m < n_mtiles || it > 0; ++it, m += gstride) {
    char* region = lds + (it & 1) * REGION;
    char* other = lds + ((it + 1) & 1) * REGION;
    const int par = it & 1;
    const bool have = m < n_mtiles;
    const int sb = 1 + 6 * (it < 9 ? it : 9);       // stamp slots: iterations 0-8, then the latest
    STAMP(sb);
    // waves 0-3 run stage 3 and the next tile's x DMA before their stage 1, waves 4-7 after it:
    // each SIMD then pairs a memory-heavy wave with a transform-heavy one, and the 64 DMA pieces
    // of the CU issue in two bursts half a phase apart instead of one
    if (wave < 4 && it > 0 && have) {
      STAMP(sb + 1);
      stage3(other, par ^ 1, m - gstride, wave);
      STAMP(sb + 2);
      if (m + gstride < n_mtiles) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the slot's staging reads are done
        dma_token(m + gstride, other, wave);
        stage1(region, par, wave, true, std::integral_constant<int, (GLU ? 4 : 8) + NDMA>{});   // stores, DMA
      } else {
        stage1(region, par, wave, true, std::integral_constant<int, GLU ? 4 : 8>{});          // stores
      }
    } else {
      if (have) {
        STAMP(sb + 1);
        // YPRIO: the transform-first waves (the younger of each SIMD pair) issue ahead of their
        // partner's stage 3: their stage 1 was the tile's critical path (6.1 k cycles against 2.6 k,
        // profiles/r05f4_timeline_dm8.txt); with it both waves finish at ~8.1 k and the kernel
        // reads 36.3 -> 35.9 us (profiles/r05ab_ab_dm8_yprio.log)
        __builtin_amdgcn_s_setprio(1);
        stage1(region, par, wave, true, std::integral_constant<int, 0>{});   // waits per half for this wave's x (and its older y stores)
        __builtin_amdgcn_s_setprio(0);
      }
      STAMP(sb + 2);
      if (it > 0) stage3(other, par ^ 1, m - gstride, wave);
      if (m + gstride < n_mtiles) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the slot's staging reads are done
        dma_token(m + gstride, other, wave);
      }
    }
    STAMP(sb + 3);
    if (!have) break;
    lds_barrier();                                  // Ba: X units and scales complete
    STAMP(sb + 4);
    stage2(region, par);
    lds_barrier();                                  // Bb: Y units complete
    STAMP(sb + 5);
  }
  STAMP(63);
}

}  // namespace bcfft

namespace {
template <bool GLU, bool HB>
void launch_dm8(const void* x, int64_t n, int n_out, const void* spec, const void* bias, int bias_dt, void* y,
                hipStream_t s) {
  const int groups = GLU ? (n_out + 15) / 16 : (n_out + 31) / 32;
  const bcfft::SpecLayout sl = bcfft::spec_layout(GLU ? 32 * groups : n_out, 32, 128);
  const int64_t n_mtiles = (n + 7) / 8;
  const int64_t total = bcfft::group_grid(bcfft::device_cu_count(), groups, n_mtiles);
  const uint32_t* stat = reinterpret_cast<const uint32_t*>(spec) + sl.stat_off_u32;
  const float* osc = reinterpret_cast<const float*>(spec) + sl.osc_off_u32;
  hipLaunchKernelGGL((bcfft::bc_forward_dm8_kernel<GLU, HB>), dim3((unsigned)total), dim3(512), 0, s, x, n, n_out, stat,
                     osc, bias, bias_dt, y);
}
}  // namespace

namespace bcfft {
// bf16 x and bf16 y (no bias or a bf16 bias), the default (non-exact) DFT variant
bool dm8_eligible(int n_in, int b, int xdt, bool yf32) { return dm_eligible(n_in, b) && xdt == BCFFT_BF16 && !yf32; }

void launch_forward_dm8(const void* x, int64_t n, int n_out, const void* spec, const void* bias, int bias_dt, void* y,
                        bool glu, hipStream_t s) {
  if (glu) launch_dm8<true, false>(x, n, n_out, spec, nullptr, BCFFT_NONE, y, s);
  else if (bias_dt != BCFFT_NONE) launch_dm8<false, true>(x, n, n_out, spec, bias, bias_dt, y, s);
  else launch_dm8<false, false>(x, n, n_out, spec, bias, bias_dt, y, s);
}
}  // namespace bcfft

// analysis build only: stamp buffer of bc_forward_dm8_kernel (this TU's copy). Slots per wave: 0
// start | per iteration it < 9 (base 1 + 6 it, then the latest): +0 top, +1 own x landed, +2
// stage 1 done, +3 stage 3 + DMA issued, +4 after Ba, +5 stage 2 + Bb done | 63 end
BCFFT_STAMPS_SETTER(dm8)
