// bcfft_dm64.hip — the DFT-on-MFMA block-circulant forward at b = 64 (K = 4096) for bf16 I/O,
// 8 tokens per M-tile (gfx950).
//
// bc_forward_dm8_kernel (bcfft_dm8.hip) restated for 64-point blocks. BlockCirculantLinear.forward
// (patch_llama_fft.py:226-275) with 64 input blocks per token and H = 32 packed bins:
//  * even/odd split a_t = x_t + x_{t+32}, d_t = x_t - x_{t+32} (t < 32): X = [a Fe | d Fo] with
//    two 32 x 32 fp16 matrices (bcfft_dm_table.h kDmF64, times 2^-7); one 32-deep MFMA K-step
//    per 16-block quarter; the inverse is the transpose, y_t = E_t + O_t, y_{t+32} = E_t - O_t.
//  * the same stationary weights (the STAT image at b = 64: 4 bins x 4 K-steps x 2 N-tiles of
//    B fragments per wave, 128 VGPRs) and the same roles: wave w owns token slot w (stage 1,
//    stage 3, its x DMA), all waves run stage 2 on their 4 bins for all 8 tokens.
//  * numerics: per-(token, quarter) power-of-two scales; a, d, X, Y one RNE fp16 term each.
//
// LDS (136,448 B): two regions x 8 token slots of 8,256 B (bf16 x: 64 rows x 128 B -> X units
// -> Y units -> y staging, 32 rows x 128 B), the 4 KiB DFT table, the scales. Every access is
// checked conflict-free by tools/lds_banks_dm.py.
#include "bcfft_device.h"
#include "bcfft_dm_table.h"
#include "bcfft_dm_common.h"

namespace bcfft {

namespace dm64 {
using namespace dmh;

constexpr int B = 64, NI = 64, KS = 4, NOG = 32, TT = 8, NW = 8;
constexpr int BW = 4, NT = 2;                       // bins per wave, 16-wide N-tiles per group
constexpr int K = NI * B;
constexpr int SLOT = 8192 + 64;                     // one token
constexpr int REGION = TT * SLOT;
constexpr int F_OFF = 2 * REGION;                   // DFT table image, 32 rows x 128 B
constexpr int SC_OFF = F_OFF + 4096;                // scale exponents [2 parity][8 token][4 quarter]
constexpr int OS_OFF = SC_OFF + 256;                // the group's 32 inverse weight scales
constexpr int LDS_BYTES = OS_OFF + 128;
static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
static_assert(F_OFF % 256 == 0, "table rows on the bank period");

// table image: row t (128 B = 8 chunks), chunk ch stored at ch ^ fsw64(t) (conflict-free for the
// stage-1 transposed reads of rows 8g + q and the stage-3 row reads)
__device__ __forceinline__ int fsw64(int t) { return (((t >> 1) & 1) << 1) | (((t >> 3) & 1) << 2); }
// X unit (16 B: 4 input blocks 4q..4q+3 x (re, im) fp16 of bin f) of K-step (quarter) ks
__device__ __forceinline__ int xunit64(int ks, int f, int q) { return 2048 * ks + 64 * (f ^ ((f >> 2) & 1)) + 16 * q; }
// Y half-unit (8 B: the 2 bins of parity par of wave w x (re, im)) of output block o, in wave w's
// K-step-par X area; the output index flips bit 4 for odd wave pairs (stage-3 reads of two pairs)
__device__ __forceinline__ int yhalf64(int w, int o, int par) { return 2048 * par + 256 * w + 8 * (o ^ (16 * ((w >> 1) & 1))); }
}  // namespace dm64

// HB: a bias is added (the runtime bias_dt then names its dtype); without one the store path is
// straight-line (a runtime test per stored quad split stage 3 into hundreds of basic blocks)
template <bool GLU, bool HB>
__global__ __launch_bounds__(512, 2) void bc_forward_dm64_kernel(
    const void* __restrict__ xv, int64_t n_tokens, int n_out, const uint32_t* __restrict__ stat,
    const float* __restrict__ osc, const void* __restrict__ bias, int bias_dt, void* __restrict__ yv) {
  using namespace dm64;
  constexpr int XT = BCFFT_BF16;
  constexpr int ES = 2, ESY = 2;
  constexpr int NPIECE = BW * KS * NT;
  constexpr int NDMA = K * ES / 1024;               // 1-KiB LDS-DMA pieces per token

  __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];
  int* wsc = reinterpret_cast<int*>(lds + SC_OFF);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  constexpr int OPG = GLU ? NOG / 2 : NOG;          // output blocks stored per group
  const int n_groups = (n_out + OPG - 1) / OPG;
  const GroupMap gm = group_map(n_groups);          // XCD-aware when the grid allows it
  const int grp_o = gm.grp, wg_in_grp = gm.lane;
  const int64_t M = (int64_t)n_out * B;
  const int64_t n_mtiles = (n_tokens + TT - 1) / TT;
  const int gstride = gm.stride;
  const uint32_t lds_base = __builtin_amdgcn_readfirstlane(lds_addr(lds));

  // ---- x of token `wave` of M-tile m -> its slot by LDS-DMA: piece q = rows 8q + (lane >> 3),
  // 128 B each; unit u of block row r at u ^ (r & 7), applied to the global source offsets
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

  // ---- prologue: first tile's x, the DFT table, the stationary B fragments
  if (wg_in_grp < n_mtiles) dma_token(wg_in_grp, lds);
  if (tid < 256) {                                  // chunk c: row c >> 3, chunk c & 7
    const uint4* tab = reinterpret_cast<const uint4*>(kDmF64);
    const int t = tid >> 3, ch = tid & 7;
    *reinterpret_cast<uint4*>(lds + F_OFF + 128 * t + 16 * (ch ^ fsw64(t))) = tab[tid];
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

  // ---- stage 1 (wave w, token slot w): x rows -> X units (one fp16 term), in place, per quarter
  auto stage1 = [&](char* region, int par) {
    const int l = opaque(lane);
    const int b16 = l & 15, g = l >> 4;
    char* slot = region + wave * SLOT;
    // transposed-read lane address of the table: rows 8g + q4 (and + 4), cols 16 (2 pr + mt) +
    // 4 p4 .. +3 = chunk (4 pr + 2 mt + (p4 >> 1)), byte 8 (p4 & 1)
    const int q4 = (l & 15) >> 2, p4 = l & 3;
    const int r0 = 8 * g + q4, r1 = r0 + 4;
    const int trb0 = F_OFF + 128 * r0 + 8 * (p4 & 1), trb1 = F_OFF + 128 * r1 + 8 * (p4 & 1);
    const int cx0 = (p4 >> 1) ^ fsw64(r0), cx1 = (p4 >> 1) ^ fsw64(r1);
    // X write lane bases: D^T row 4g + r is bin 16 mt + 4 g + pr (+ 2 for r >= 2), column block b16
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
      // x of block 16h + b16: t = 8 g + j (unit g) and t + 32 (unit g + 4), j < 8
      float xv[2][8];
      const char* rowp = slot + (16 * h + b16) * (B * ES);
#pragma unroll
      for (int pt = 0; pt < 2; ++pt) {
        const uint4 w = *reinterpret_cast<const uint4*>(rowp + 16 * ((g + 4 * pt) ^ (b16 & 7)));
        const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float2 f = unpack16<XT>(ww[e]);
          xv[pt][2 * e] = f.x;
          xv[pt][2 * e + 1] = f.y;
        }
      }
      float m0 = 0.f, m1 = 0.f;
#pragma unroll
      for (int pt = 0; pt < 2; ++pt)
#pragma unroll
        for (int j = 0; j < 8; j += 4) {
          m0 = amax3(m0, xv[pt][j], xv[pt][j + 1]);
          m1 = amax3(m1, xv[pt][j + 2], xv[pt][j + 3]);
        }
      const float mxf = __builtin_fmaxf(m0, m1);
      const int sx = stat_scale_exp(2.f * __uint_as_float(wave_umax(__float_as_uint(mxf))));
      if (l == 0) wsc[par * 32 + wave * 4 + h] = sx - 7;    // X = D 2^-(sx - 7): the table's 2^-7
      const float S = __int_as_float((sx + 127) << 23);
      uint32_t ah[4], dh[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float u0 = xv[1][2 * e] * S, u1 = xv[1][2 * e + 1] * S;
        ah[e] = pk_rne(fmaf(xv[0][2 * e], S, u0), fmaf(xv[0][2 * e + 1], S, u1));
        dh[e] = pk_rne(fmaf(xv[0][2 * e], S, -u0), fmaf(xv[0][2 * e + 1], S, -u1));
      }
      const f16x8 bah = frag(ah[0], ah[1], ah[2], ah[3]), bdh = frag(dh[0], dh[1], dh[2], dh[3]);
      f32x4 acc[4];
#pragma unroll
      for (int pr = 0; pr < 2; ++pr)
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
          const f16x8 af = afr[pr][mt];
          acc[2 * pr + mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, pr ? bdh : bah, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        }
      char* xb = slot + 2048 * h;
#pragma unroll
      for (int pr = 0; pr < 2; ++pr)
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
          *reinterpret_cast<uint32_t*>(xb + xwb[pr] + 1024 * mt) = pk_rne(acc[2 * pr + mt][0], acc[2 * pr + mt][1]);
          *reinterpret_cast<uint32_t*>(xb + xwb[pr] + 1024 * mt + 128) = pk_rne(acc[2 * pr + mt][2], acc[2 * pr + mt][3]);
        }
    }
  };

  // ---- stage 2 (all waves): per-bin complex MAC on bins f = 4 wave + fb for all 8 tokens (rows
  // token t = row >> 1, re/im); Y half-units over the wave's own X units (in-order DS per wave)
  auto stage2 = [&](char* region, int par) {
    const int ml = opaque(lane);
    const int arow = ml & 15, kb = ml >> 4;
    const int a_t = arow >> 1, a_reim = arow & 1;
    const uint32_t a_sel = a_reim ? 0x01000302u : 0x03020100u;
    const int yt = ml >> 4;
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
    // unit of bin 4 wave + fb: 256 wave + 64 (fb ^ (wave & 1)) + 2048 ks + 16 kb
    const int sw = 64 * (wave & 1);
    const char* ab_e = region + a_t * SLOT + 256 * wave + 16 * kb + sw;   // even fb: +64 fb
    const char* ab_o = region + a_t * SLOT + 256 * wave + 16 * kb - sw;   // odd fb
    uint4 araw[BW][KS];
#pragma unroll
    for (int fb = 0; fb < BW; ++fb)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        araw[fb][ks] = *reinterpret_cast<const uint4*>((fb & 1 ? ab_o : ab_e) + 64 * fb + 2048 * ks);
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
      constexpr float YS = 1.f / 2097152.f;          // 2^-21
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) yh[fb][nt][s2] = pk_rne(acc[nt][2 * s2] * YS, acc[nt][2 * s2 + 1] * YS);
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

  // ---- stage 3 (wave w, token slot w of the previous tile): Y -> y rows staged in the slot (32
  // rows x 128 B; GLU: 16 h rows), 1 KiB buffer stores
  auto stage3 = [&](char* region, int par, int64_t mp) {
    const int l = opaque(lane);
    const int o16 = l & 15, g = l >> 4;
    char* slot = region + wave * SLOT;
    const int* sc = wsc + par * 32 + wave * 4;
    const int nmin = min(min(sc[0], sc[1]), min(sc[2], sc[3]));
    float ysc[NT];                                  // output block o = 16 nt + o16: 1 / s_o
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) ysc[nt] = __builtin_ldexpf(reinterpret_cast<const float*>(lds + OS_OFF)[16 * nt + o16], 30 - nmin);
    // Y fragments: B[k = 8 g + j][o] = bins 8g + par' + {0, 2} of wave 2g, {4, 6} of wave 2g + 1
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
    // table row reads: row 16 mt + o16, chunk (4 pr + g) ^ fsw64(row)
    f16x8 gt[2][2];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        const int t = 16 * mt + o16;
        gt[mt][pr] = *reinterpret_cast<const f16x8*>(lds + F_OFF + 128 * t + 16 * ((4 * pr + g) ^ fsw64(t)));
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // Y is in registers: the slot is free
    const int64_t tok = mp * TT + wave;
    const bool tok_ok = tok < n_tokens;
    const int nvalid = n_out - grp_o * OPG;
    // staging: row o (128 B = 16 units of 8 B), t = 16 mt + 4 g + 32 hf -> unit (4 mt + g + 8 hf) ^ o16
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
          *reinterpret_cast<uint2*>(slot + 128 * o16 + 8 * ((4 * mt + g + 8 * hf) ^ o16)) =
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
    }
    // staged rows -> global: each instruction stores 1 KiB = 8 whole rows (8 lanes per row); LDS
    // 16-B unit w of row rr holds 8-B units (2w, 2w+1) ^ (rr & 15), i.e. 16-B unit
    // w ^ ((rr & 15) >> 1) with its halves swapped when rr is odd
    constexpr int RB = B * ESY;
    constexpr int NQ = GLU ? 2 : 4;
    const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
        (char*)yv + (tok_ok ? tok : 0) * M * ESY + (int64_t)grp_o * OPG * RB, 0,
        tok_ok ? (int)((M - (int64_t)grp_o * OPG * B) * ESY) : 0, 0x00020000);
    const int w = l & 7, lr = l >> 3;
    const int vofs = lr * RB + 16 * w;
    uint4 d[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int rr = 8 * q + lr;
      uint4 v = *reinterpret_cast<const uint4*>(slot + 128 * rr + 16 * (w ^ ((rr & 15) >> 1)));
      if (lr & 1) v = make_uint4(v.z, v.w, v.x, v.y);
      d[q] = v;
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, d[q]), yrs, vofs + q * 1024, 0, BCFFT_YAUX);
  };

  // Pipeline as bc_forward_dm8_kernel: P1 every wave: stage 1 (own token, this tile), stage 3
  // (own token, previous tile), x DMA (own token, next tile) | Ba | P2 stage 2 | Bb
  int64_t m = wg_in_grp;
  for (int it = 0; m < n_mtiles || it > 0; ++it, m += gstride) {
    char* region = lds + (it & 1) * REGION;
    char* other = lds + ((it + 1) & 1) * REGION;
    const int par = it & 1;
    const bool have = m < n_mtiles;
    // waves 0-3 run stage 3 and the next tile's x DMA before their stage 1 (bcfft_dm8.hip's mixed
    // order: a memory-heavy and a transform-heavy wave per SIMD, two DMA bursts per phase)
    if (wave < 4 && it > 0 && have) {
      constexpr int NST = GLU ? 2 : 4;              // stage 3's stores
      stage3(other, par ^ 1, m - gstride);
      if (m + gstride < n_mtiles) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the slot's staging reads are done
        dma_token(m + gstride, other);
        wait_vmcnt<NST + NDMA>();                   // this wave's x (older than the stores and the DMA)
      } else {
        wait_vmcnt<NST>();
      }
      stage1(region, par);
    } else {
      if (have) {
        wait_vmcnt<0>();                            // this wave's x (and its older y stores)
        // YPRIO: the transform-first (younger) waves issue ahead of their partner's stage 3
        // (bcfft_dm8.hip's finding): 50.3 -> 47.9 us over six interleaved passes
        // (profiles/r05ac_ab_dm64_yprio.log)
        __builtin_amdgcn_s_setprio(1);
        stage1(region, par);
        __builtin_amdgcn_s_setprio(0);
      }
      if (it > 0) stage3(other, par ^ 1, m - gstride);
      if (m + gstride < n_mtiles) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the slot's staging reads are done
        dma_token(m + gstride, other);
      }
    }
    if (!have) break;
    lds_barrier();                                  // Ba: X units and scales complete
    stage2(region, par);
    lds_barrier();                                  // Bb: Y units complete
  }
}

}  // namespace bcfft

namespace {
template <bool GLU, bool HB>
void launch_dm64(const void* x, int64_t n, int n_out, const void* spec, const void* bias, int bias_dt, void* y,
                 hipStream_t s) {
  const int groups = GLU ? (n_out + 15) / 16 : (n_out + 31) / 32;
  const bcfft::SpecLayout sl = bcfft::spec_layout(GLU ? 32 * groups : n_out, 64, 64);
  const int64_t n_mtiles = (n + 7) / 8;
  const int64_t total = bcfft::group_grid(bcfft::device_cu_count(), groups, n_mtiles);
  const uint32_t* stat = reinterpret_cast<const uint32_t*>(spec) + sl.stat_off_u32;
  const float* osc = reinterpret_cast<const float*>(spec) + sl.osc_off_u32;
  hipLaunchKernelGGL((bcfft::bc_forward_dm64_kernel<GLU, HB>), dim3((unsigned)total), dim3(512), 0, s, x, n, n_out, stat,
                     osc, bias, bias_dt, y);
}
}  // namespace

namespace bcfft {
// b = 64 with K = 4096, bf16 x and bf16 y (no bias or a bf16 bias)
bool dm64_eligible(int n_in, int b, int xdt, bool yf32) { return b == 64 && n_in == 64 && xdt == BCFFT_BF16 && !yf32; }

void launch_forward_dm64(const void* x, int64_t n, int n_out, const void* spec, const void* bias, int bias_dt,
                         void* y, bool glu, hipStream_t s) {
  if (dm64g_eligible(64, 64, BCFFT_BF16, false, n_out, glu) && multigroup_pays(n, glu ? 5 : 4)) {   // x transformed once
    launch_forward_dm64g(x, n, n_out, spec, bias, bias_dt, y, glu, s);
    return;
  }
  if (glu) launch_dm64<true, false>(x, n, n_out, spec, nullptr, BCFFT_NONE, y, s);
  else if (bias_dt != BCFFT_NONE) launch_dm64<false, true>(x, n, n_out, spec, bias, bias_dt, y, s);
  else launch_dm64<false, false>(x, n, n_out, spec, bias, bias_dt, y, s);
}
}  // namespace bcfft
