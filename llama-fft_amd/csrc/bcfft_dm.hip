// bcfft_dm.hip — block-circulant forward with all three stages on the matrix cores (gfx950).
//
// Same operator as bc_forward_stat_kernel (BlockCirculantLinear.forward,
// patch_llama_fft.py:226-275) and the same stationary weights: one persistent 512-thread
// workgroup per CU keeps its output group's conj(C) s_C spectra (the STAT image, fp16 B
// fragments) in 128 VGPRs per lane and streams tokens in tiles of 4. What changes is the
// transforms: the real DFT of every 128-point x row and the inverse DFT of every output row are
// dense fp16 GEMMs on v_mfma_f32_16x16x32_f16 instead of VALU FFTs.
//
//  * Even/odd split (half of a 128 x 128 DFT): a_t = x_t + x_{t+64}, d_t = x_t - x_{t+64}
//    (t < 64). The even packed bins are a 64-point real DFT of a, the odd ones the DFT of d
//    against e^{-2 pi i (2j+1) t / 128}: X = [a Fe | d Fo] with two 64 x 64 matrices (the fp16
//    table bcfft_dm_table.h, times 2^-7). The inverse is the transpose: E = Fe Y_even,
//    O = Fo Y_odd, y_t = E_t + O_t, y_{t+64} = E_t - O_t; its weights (1/b, 2/b) are the bin-0
//    factor 1/2 in the MAC and the per-token output scale.
//  * Wave roles per M-tile: waves 0-3 (F) transform token w's x rows (stage 1) while waves 4-7
//    (I) inverse-transform token w-4 of the previous tile (stage 3) and stream the next x in by
//    LDS-DMA; then all 8 waves run the per-bin complex MAC (stage 2) on their 8 bins, exactly as
//    the stationary kernel. Two workgroup barriers per M-tile, two 64 KiB LDS regions.
//  * Numerics: per-(token, 16-block half) power-of-two scales; X split into fp16 hi + lo; C and
//    the table one fp16 term each; fp32 accumulation everywhere. a, d and the per-bin products Y
//    (a fixed 2^-21 keeps Y in range) are one RNE fp16 term each (~4e-4 relative on the layer
//    output; the default) or, in the exact variant EX (BCFFT_ALGO_DFTX, and always for fp16
//    outputs, whose ulp is close to that noise), hi + lo (~2.8e-4, linear in x to ~1e-6)
//    (tests/dm_model.py restates both; north star: 1e-3).
//
// Geometry: b = 128 with K = 4096 (32 input blocks: two K-steps of 16), any M (output groups of
// 32 blocks), x fp32 / fp16 / bf16, y = promote(x, bias). LDS and register maps below; every
// LDS access pattern is checked conflict-free by tools/lds_banks_dm.py.
#include "bcfft_device.h"
#include "bcfft_dm_table.h"
#include "bcfft_dm_common.h"


namespace bcfft {

namespace dmk {
using namespace dmh;

constexpr int B = 128, NI = 32, KS = 2, NOG = 32, TT = 4, NW = 8;
constexpr int BW = 8, NT = 2;                       // bins per wave, 16-wide N-tiles per group
constexpr int K = NI * B;
constexpr int SLOT = 16384;                         // one token of a tile
constexpr int REGION = TT * SLOT;                   // 64 KiB
constexpr int F_OFF = 2 * REGION;                   // DFT table image, 64 rows x 256 B
constexpr int SC_OFF = F_OFF + 16384;               // scale exponents [2 parity][4 token][2 half]
constexpr int OS_OFF = SC_OFF + 64;                  // the group's 32 inverse weight scales
constexpr int LDS_BYTES = OS_OFF + 128;
static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
// precise engine (EP): the e4m3 table residual, pair-packed (rows 2p, 2p + 1 of a column in one
// 16-bit element), 32 pair-rows at a 288-B stride (a 32-lane half's 8 pair-rows fall on distinct
// 8-bank groups for both the stage-1 transposed reads and the stage-3 16-B row reads)
constexpr int FL_OFF = LDS_BYTES, FL_STRIDE = 288;
constexpr int LDS_BYTES_EP = FL_OFF + 32 * FL_STRIDE;
static_assert(LDS_BYTES_EP <= 160 * 1024, "LDS budget (EP)");

// X unit (16 B = 4 input blocks x (re, im) fp16 of bin f, precision p, block quad q) of the
// token in slot tok, K-step ks; swizzle: the precision bit flips with bin bit 2, the quad with
// the token pair
__device__ __forceinline__ int xunit(int ks, int f, int p, int q, int tok) {
  return ks * 8192 + 128 * f + 16 * ((4 * (p ^ ((f >> 2) & 1))) + (q ^ (3 * (tok >> 1))));
}
// Y unit (16 B = 4 bins of parity par of wave w x (re, im) fp16) of output block o; lies over
// the K-step-0 X units of wave w's bins in the same token slot
__device__ __forceinline__ int yunit(int w, int o, int par) { return w * 1024 + 16 * (32 * par + o); }

}  // namespace dmk

// bf8 (e5m2) of eight fp16 values: the high byte of each (fp16 and e5m2 share sign and exponent
// fields, so this is the value truncated to 2 mantissa bits). (w0, w1, w2, w3) hold the values in
// order, two per word; the result keeps that order, one byte each (an fp8 MFMA operand).
__device__ __forceinline__ long bf8x8(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3) {
  const uint32_t lo = __builtin_amdgcn_perm(w1, w0, 0x07050301u), hi = __builtin_amdgcn_perm(w3, w2, 0x07050301u);
  return (long)(((uint64_t)hi << 32) | lo);
}

// e4m3 (round to nearest even) of eight fp16 values times 2^-6, in order, one byte each (an fp8
// MFMA operand): |X| < 2^14 in the A rows keeps v 2^-6 within e4m3's 448; the product is scaled
// back by 2^6 where the residual accumulator joins the main one. v_cvt_scalef32_pk_fp8_f16 converts
// two fp16 values to e4m3(v / scale) with RNE (tools/probe/cvt_fp8.hip, profiles/r06_probe_cvt_fp8.txt)
typedef _Float16 f16x2v __attribute__((ext_vector_type(2)));
typedef short s16x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ long e4m3x8_s6(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3) {
  s16x2v lo = {0, 0}, hi = {0, 0};
  lo = __builtin_amdgcn_cvt_scalef32_pk_fp8_f16(lo, __builtin_bit_cast(f16x2v, w0), 64.f, false);
  lo = __builtin_amdgcn_cvt_scalef32_pk_fp8_f16(lo, __builtin_bit_cast(f16x2v, w1), 64.f, true);
  hi = __builtin_amdgcn_cvt_scalef32_pk_fp8_f16(hi, __builtin_bit_cast(f16x2v, w2), 64.f, false);
  hi = __builtin_amdgcn_cvt_scalef32_pk_fp8_f16(hi, __builtin_bit_cast(f16x2v, w3), 64.f, true);
  return (long)(((uint64_t)__builtin_bit_cast(uint32_t, hi) << 32) | __builtin_bit_cast(uint32_t, lo));
}

// An MFMA that reads as SrcC the result of an MFMA of ANOTHER opcode (here f16 <-> fp8_bf8) issued
// fewer than ~6 instructions before it reads a stale C on gfx950 (every lane; tools/probe/srcc.hip:
// wrong at 0-3 independent VALU between them, right at 6, profiles/r06j_mfma_srcc_chain_probe.txt).
// hipcc forwards same-opcode accumulation chains back to back, correctly, and inserts no wait
// states for the cross-opcode pair either. xdl_gap sits between the two MFMAs of such a pair: it
// names the accumulator, so the compiler cannot move either MFMA across it, and its 8 wait states
// plus the instruction give the distance (tools/mfma_audit.py checks every kernel for the pair).
__device__ __forceinline__ void xdl_gap(f32x4& acc) { asm volatile("s_nop 7" : "+v"(acc)); }

// EP (precise engine, BCFFT_ALGO_DFTP; bit 1: stage-1 table residual, 2: weight residual, 4:
// stage-3 table residual; 0 = the dft / dftx kernel): every fp16 single term of the dftx kernel
// gets its rounding residual back through an fp8 MFMA into the same fp32 accumulator:
//   * the table is F 2^8 in fp16 (kDmFp) and a is scaled 2^15 lower, so D's scale is unchanged;
//     the residual F 2^8 - kDmFp (|.| <= 2^-3) is e4m3 (kDmFl8) and multiplies a bf8 copy of the
//     data's fp16 hi term (the high byte: same value range), in the same fp32 accumulator;
//   * stage 2 adds A x e4m3(conj(C) s_o - fp16(conj(C) s_o)) (the lo8 image, streamed from L2
//     by every wave for its bins, four bins ahead): A as e4m3 (RNE) of the fp16 A rows times 2^-6
//     into an accumulator of its own, joined to the fp16 product's times 2^6 (worst
//     structured token 2.4e-4, tools/precision_terms.py; A as bf8, the fp16 value's high byte,
//     gave 9.0e-4: profiles/r06_precise_probe.txt);
//   * stage 3 adds e4m3 table residual x bf8(Y hi).
// The F waves' x DMA (asm, invisible to the compiler's counters) is issued after Ba, once the
// first lo8 loads of stage 2 have been waited for. Numpy mirror: tests/dm_model.py
// (precise=True); error ~1e-5 relative (north star 1e-3), per token ~1e-5 x its cancellation.
// BM: bias handling, -1 = by the runtime bias_dt (dft / dftx); 0 = none, 1 = fp32 bias, 2 = 16-bit
// bias, its 4 consecutive values per lane read by one buffer load (the precise engine: the general
// per-element path's address registers do not fit beside its residual operands)
template <int XT, bool YF32, bool EX, bool GLU, int EP = 0, int BM = -1>
__global__ __launch_bounds__(512, 2) void bc_forward_dm_kernel(
    const void* __restrict__ xv, int64_t n_tokens, int n_out, const uint32_t* __restrict__ stat,
    const float* __restrict__ osc, const void* __restrict__ bias, int bias_dt, void* __restrict__ yv,
    const uint4* __restrict__ lo8) {
  using namespace dmk;
  static_assert(EP == 0 || EX, "the precise engine extends the exact (hi + lo) variant");
  constexpr int ES = XTraits<XT>::ES;
  constexpr bool Y32 = YF32 || XT == BCFFT_F32;
  constexpr int ESY = Y32 ? 4 : 2;
  constexpr int NPIECE = BW * KS * NT;
  constexpr int NDMA = K * ES / 1024;               // 1-KiB LDS-DMA pieces per token
  // LATE_W: the weight fragments are waited for after the first stage 1; EARLY_X: in iteration 0
  // the I waves stream the next tile's x at once (both measured wins)
  constexpr bool LATE_W = true;
  constexpr bool EARLY_X = true;
  // FILL_SPLIT / DRAIN_SPLIT: the pipeline's first P1 has no stage 3 and its last no stage 1, so
  // half the waves would idle through them: the first stage 1 runs one half of each token on its
  // F wave and the other on its I wave (fp32 x: the halves are in place independently; the
  // prologue's x DMA is split the same way), and the last stage 3 one N-tile on each
  // (the precise engine: the drain split only, and not with an fp32 bias; its residual operands
  // leave no registers for the fill split, and those two spill 20 B per lane: DESIGN.md section 8b)
  constexpr bool FILL_SPLIT = LATE_W && ES == 4 && EP == 0;
  constexpr bool DRAIN_SPLIT = !GLU && (EP == 0 || BM != 1);
  // (round 4 measured and rejected other x-DMA placements and role splits: docs/HISTORY.md section 8c,
  // item 8, with their A/B logs; their switches are in the git history of this file)

  ANALYSIS_INIT;
  bool sub_on = false;                              // sub-phase stamps (analysis builds: iteration 4)
  __shared__ __attribute__((aligned(16))) char lds[EP ? LDS_BYTES_EP : LDS_BYTES];
  int* wsc = reinterpret_cast<int*>(lds + SC_OFF);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool fwave = wave < 4;                      // F waves: stage 1 of token slot `wave`
  const int tslot = wave & 3;                       // I waves: stage 3 of token slot wave - 4
  // GLU (fused gate/up + SwiGLU): n_out counts h blocks; group g holds gate blocks [16g, 16g+16)
  // in N-tile 0 and the matching up blocks in N-tile 1, and stores 16 h rows
  constexpr int OPG = GLU ? NOG / 2 : NOG;          // output blocks stored per group
  const int n_groups = (n_out + OPG - 1) / OPG;
  const GroupMap gm = group_map(n_groups);          // XCD-aware when the grid allows it
  const int grp_o = gm.grp, wg_in_grp = gm.lane;
  const int64_t M = (int64_t)n_out * B;
  const int64_t n_mtiles = (n_tokens + TT - 1) / TT;
  const int gstride = gm.stride;
  const uint32_t lds_base = __builtin_amdgcn_readfirstlane(lds_addr(lds));

  // ---- x of one token -> its slot by LDS-DMA (I waves; the buffer range zero-fills tokens past
  // n_tokens). LDS is lane-linear per piece, so the slot's unit swizzle (logical 16-B unit u of
  // block row r at physical u ^ (r & 15)) is applied to the global source offsets.
  auto dma_token = [&](int64_t m, char* region, int q0, int q1) {   // pieces [q0, q1)
#ifdef BCFFT_DM_NOMEM                               // analysis build: compute only (no x, no y)
    return;
#endif
    const int64_t tok = m * TT + tslot;
    const bool ok = tok < n_tokens;
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<char*>((const char*)xv) + (ok ? tok : 0) * K * ES, 0, ok ? K * ES : 0, 0x00020000);
    const int dl = opaque(lane);
    const uint32_t dst0 = lds_base + (uint32_t)(region - lds) + tslot * SLOT;
    if constexpr (ES == 4) {                        // piece q: rows 2q + (lane >> 5), 512 B each
      int vb[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const int h = dl >> 5;
        vb[c] = h * 512 + 16 * ((dl & 31) ^ ((2 * c + h) & 15));
      }
#pragma unroll
      for (int q = q0; q < q1; ++q) {
        uint32_t keep;
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen" BCFFT_XPOL " lds\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(vb[q & 7]), "s"(xrs), "s"(dst0 + q * 1024), "s"(q * 1024) : "memory");
      }
    } else {                                        // piece q: rows 4q + (lane >> 4), 256 B each
      int vb[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int r = dl >> 4;
        vb[c] = r * 256 + 16 * ((dl & 15) ^ ((4 * c + r) & 15));
      }
#pragma unroll
      for (int q = q0; q < q1; ++q) {
        uint32_t keep;
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen" BCFFT_XPOL " lds\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(vb[q & 3]), "s"(xrs), "s"(dst0 + q * 1024), "s"(q * 1024) : "memory");
      }
    }
  };

  // ---- prologue: first tile's x (I waves), the DFT table, the stationary B fragments
  // (with the fill split below, each wave of a slot streams the half of tile 0's x it transforms)
  if (wg_in_grp < n_mtiles) {
    if (FILL_SPLIT) dma_token(wg_in_grp, lds, fwave ? 0 : NDMA / 2, fwave ? NDMA / 2 : NDMA);
    else if (fwave) dma_token(wg_in_grp, lds, 0, NDMA);
  }
  {
    const uint4* tab = reinterpret_cast<const uint4*>(EP ? kDmFp : kDmF);
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int c = tid + 512 * r;                  // chunk c: row c >> 4, chunk c & 15
      const int t = c >> 4, ch = c & 15;
      *reinterpret_cast<uint4*>(lds + F_OFF + 256 * t + 16 * (ch ^ fsw(t))) = tab[c];
    }
    if constexpr (EP != 0) {                        // residual image: pair-row tid >> 4, 16-B piece tid & 15
      *reinterpret_cast<uint4*>(lds + FL_OFF + FL_STRIDE * (tid >> 4) + 16 * (tid & 15)) =
          reinterpret_cast<const uint4*>(kDmFl8)[tid];
    }
  }
  // the group's inverse weight scales 1 / s_o (per output block) -> LDS
  if (tid < 32) reinterpret_cast<float*>(lds + OS_OFF)[tid] = osc[grp_o * 32 + tid];
  f16x8 creg[BW][KS][NT];
  // LATE_W: the weight fragments (256 KiB per workgroup, ~4k cycles of L2 reads) stay in flight
  // through the first P1 (stage 1 of tile 0 on the F waves) and are waited for at a tie at the
  // end of each P1: only the y stores of stage 3 are younger there, so the compiler's counted wait
  // lets those fly. They are the last loads issued, so the F waves' first x DMA is waited for
  // with vmcnt(NPIECE).
  auto creg_tie = [&]() {
#pragma unroll
    for (int fb = 0; fb < BW; ++fb)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) asm volatile("" : "+v"(creg[fb][ks][nt]));
  };
  {
    const uint4* img = reinterpret_cast<const uint4*>(stat + 4) + ((int64_t)(grp_o * NW + wave) * NPIECE) * 64 + lane;
#pragma unroll
    for (int fb = 0; fb < BW; ++fb)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          creg[fb][ks][nt] = __builtin_bit_cast(f16x8, img[((fb * KS + ks) * NT + nt) * 64]);
    // without LATE_W, pin the loads here: without a use, hipcc keeps counting them up to their
    // first use inside the tile loop (vmcnt(29..0) before each stage-2 MFMA), which then waits
    // for every in-flight x DMA and y store of the iteration
    if constexpr (!LATE_W) creg_tie();
  }
  if constexpr (!LATE_W) wait_vmcnt<0>();
  lds_barrier();

  // ---- stage 1 (token slot tslot): x rows -> X hi/lo units, in place, per half (hmask: the
  // halves this wave does; both for the F wave of a steady-state tile)
  // xwait (fp32 x, steady state): this wave's x DMA of the tile is in flight, pieces 0-7 = half 0
  // first; wait for half 0 alone, then for half 1 after half 0's transform
  auto stage1 = [&](char* region, int par, int hmask, bool xwait = false) {
#if defined(BCFFT_DM_MEMONLY) || (defined(BCFFT_DM_ABL) && (BCFFT_DM_ABL & 1))   // analysis builds
    if (lane < 2 && ((hmask >> lane) & 1)) wsc[par * 8 + tslot * 2 + lane] = 0;
    return;
#endif
    const int l = opaque(lane);
    const int b16 = l & 15, g = l >> 4;
    char* slot = region + tslot * SLOT;
    // transposed-read lane address of the table: row 8g + q (+ 32 ks + 4 sec), chunk
    // (8 par + 2 mt + (p >> 1)) ^ fsw(row) = (8 par + 2 mt) ^ cx
    const int q4 = (l & 15) >> 2, p4 = l & 3;
    const int cx = (p4 >> 1) ^ fsw(8 * g + q4);
    const int trb = F_OFF + 256 * (8 * g + q4) + 8 * (p4 & 1);
    // EP: residual A fragments, one transposed read each: lane 4 q4 + p4 of group g supplies
    // pair-row 4 g + q4 (t = 8 g + 2 q4, + 1), columns 4 p4 .. 4 p4 + 3 of the tile's 16
    const int flb = FL_OFF + FL_STRIDE * (4 * g + q4) + 8 * p4;
    // X write lane bases: precision p at (4 (p ^ (g & 1)) + (q ^ phi)) units
    const int xq = (b16 >> 2) ^ (3 * (tslot >> 1));
    const int xw0 = 128 * 4 * g + 16 * (4 * (g & 1) + xq) + 4 * (b16 & 3);
    const int xw1 = 128 * 4 * g + 16 * (4 * ((g & 1) ^ 1) + xq) + 4 * (b16 & 3);
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      // 16-bit x sits in the slot's first 8 KiB: half 1 (bytes 4-8 KiB) goes first, so that the
      // in-place X writes of half 1 (8-16 KiB) and then half 0 (0-8 KiB) clobber nothing unread
      const int h = ES == 4 ? hh : 1 - hh;
      if (!((hmask >> h) & 1)) continue;
      if constexpr (ES == 4) {
        if (xwait) {
          if (hh == 0) wait_vmcnt<NDMA / 2>();
          else wait_vmcnt<0>();
        }
      }
      // x of blocks 16h + b16: t = 32 ks + 8 g + j and t + 64 (j < 8)
      float xv8[2][2][8];
      const char* rowp = slot + (16 * h + b16) * (B * ES);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int pt = 0; pt < 2; ++pt) {
          if constexpr (ES == 4) {
            const int u = 8 * ks + 2 * g + 16 * pt;
            const float4 v0 = *reinterpret_cast<const float4*>(rowp + 16 * (u ^ b16));
            const float4 v1 = *reinterpret_cast<const float4*>(rowp + 16 * ((u + 1) ^ b16));
            xv8[ks][pt][0] = v0.x; xv8[ks][pt][1] = v0.y; xv8[ks][pt][2] = v0.z; xv8[ks][pt][3] = v0.w;
            xv8[ks][pt][4] = v1.x; xv8[ks][pt][5] = v1.y; xv8[ks][pt][6] = v1.z; xv8[ks][pt][7] = v1.w;
          } else {
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
        }
      SUBSTAMP(55 + 4 * hh);
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
      // across lanes as magnitude bits: no NaN canonicalisation around the DPP moves
      const int sx = stat_scale_exp(2.f * __uint_as_float(wave_umax(__float_as_uint(mxf))));   // |a|, |d| <= 2 max|x|
      if (l == 0) wsc[par * 8 + tslot * 2 + h] = sx - 7;    // X = D 2^-(sx - 7): the table's 2^-7
      // EP: a 2^(sx - 15) against the table 2^8 (the same D); max|x| < 2^125 keeps the scale normal
      const float S = __int_as_float((EP ? max(sx - 15, -126) + 127 : sx + 127) << 23);
      SUBSTAMP(56 + 4 * hh);
      f32x4 acc[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        uint32_t ah[4], al[4], dh[4], dl[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          // a S = x_t S + x_{t+64} S, d S = x_t S - x_{t+64} S: exact power-of-two scale, so the
          // fused forms round like (x_t +- x_{t+64}) S
          const float u0 = xv8[ks][1][2 * e] * S, u1 = xv8[ks][1][2 * e + 1] * S;
          const float a0 = fmaf(xv8[ks][0][2 * e], S, u0), a1 = fmaf(xv8[ks][0][2 * e + 1], S, u1);
          const float d0 = fmaf(xv8[ks][0][2 * e], S, -u0), d1 = fmaf(xv8[ks][0][2 * e + 1], S, -u1);
          if constexpr (EX) {
            split2(a0, a1, ah[e], al[e]);
            split2(d0, d1, dh[e], dl[e]);
          } else {                                  // one RNE fp16 term
            ah[e] = pk_rne(a0, a1);
            dh[e] = pk_rne(d0, d1);
          }
        }
        const f16x8 bah = frag(ah[0], ah[1], ah[2], ah[3]), bdh = frag(dh[0], dh[1], dh[2], dh[3]);
        long b8a = 0, b8d = 0;
        if constexpr ((EP & 1) != 0) {
          b8a = bf8x8(ah[0], ah[1], ah[2], ah[3]);
          b8d = bf8x8(dh[0], dh[1], dh[2], dh[3]);
        }
        // EP: the K-step's eight residual A fragments, read before its MFMAs. (Read in between,
        // hipcc gave a read the registers of an operand that an issued, still queued MFMA had
        // not consumed yet (no wait for it on gfx950): garbage in the accumulators. Hoisted,
        // they land in registers of their own.)
        s16x4 rlv[8];
        if constexpr ((EP & 1) != 0) {
#pragma unroll
          for (int i = 0; i < 8; ++i)
            rlv[i] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (__attribute__((address_space(3))) s16x4*)(lds + flb + FL_STRIDE * 16 * ks + 32 * i));
          __builtin_amdgcn_sched_barrier(0);
        }
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
            if constexpr (EX) {
              const f16x8 bal = frag(al[0], al[1], al[2], al[3]), bdl = frag(dl[0], dl[1], dl[2], dl[3]);
              acc[4 * pr + mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, pr ? bdl : bal, acc[4 * pr + mt], 0, 0, 0);
            }
            if constexpr ((EP & 1) != 0) {          // + e4m3 table residual x bf8(hi), pair-rows 16 ks + 4 g + q
              const s16x4 rl = rlv[4 * pr + mt];
              xdl_gap(acc[4 * pr + mt]);             // f16 -> fp8 on one accumulator (xdl_gap)
              acc[4 * pr + mt] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_bf8(__builtin_bit_cast(long, rl), pr ? b8d : b8a,
                                                                           acc[4 * pr + mt], 0, 0, 0);
              xdl_gap(acc[4 * pr + mt]);             // ... and on to the next K-step's f16 MFMAs
            }
          }
      }
      // D^T tile (pr, mt): rows 4g + r = cols of bins fA = 16 mt + 4 g + pr (r = 0, 1: re, im)
      // and fA + 2 (r = 2, 3); column = input block 16 h + b16. Split and write 4 B per unit.
      SUBSTAMP(57 + 4 * hh);
      char* xb = slot + 8192 * h;
#pragma unroll
      for (int pr = 0; pr < 2; ++pr)
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          uint32_t hA, lA, hB, lB;
          split2(acc[4 * pr + mt][0], acc[4 * pr + mt][1], hA, lA);
          split2(acc[4 * pr + mt][2], acc[4 * pr + mt][3], hB, lB);
          const int fo = 128 * (16 * mt + pr);
          *reinterpret_cast<uint32_t*>(xb + xw0 + fo) = hA;
          *reinterpret_cast<uint32_t*>(xb + xw1 + fo) = lA;
          *reinterpret_cast<uint32_t*>(xb + xw0 + fo + 256) = hB;
          *reinterpret_cast<uint32_t*>(xb + xw1 + fo + 256) = lB;
        }
      SUBSTAMP(58 + 4 * hh);
    }
  };

  // ---- EP: the wave's lo8 fragments (16 B per (bin, K-step): N-tile 0 then 1), a ring of four
  // bins: bins 0-3 are loaded at the end of P1, bin fb + 4 while stage 2 works on bin fb
  // (the ring is a per-iteration array handed to stage 2 / stage 3, so that it is dead outside P1's
  // end .. stage 2 and holds no registers through stage 1)
  // one buffer descriptor per wave over its 16 KiB of fragments: lane offset in one VGPR, the
  // (bin, K-step) piece in the scalar offset
  const __amdgpu_buffer_rsrc_t clrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint4*>(lo8) + ((EP & 2) ? (int64_t)(grp_o * NW + wave) * BW * KS * 64 : 0), 0,
      (EP & 2) ? BW * KS * 1024 : 0, 0x00020000);
  constexpr int RING = 4;                           // bins of lo8 fragments in flight
  typedef u32x4 ClRing[RING][KS];
  auto cl_load = [&](ClRing& clr, int fb) {
    asm volatile("" ::: "memory");                  // keep the loads here: hoisted, they would hold
#pragma unroll                                      // their registers through the phase before
    for (int ks = 0; ks < KS; ++ks)
      clr[fb % RING][ks] = __builtin_amdgcn_raw_buffer_load_b128(clrs, 16 * opaque(lane), (fb * KS + ks) * 1024, 0);
  };

  // ---- stage 2 (all waves): per-bin complex MAC on bins f = 8 wave + fb; Y units over the
  // wave's own K-step-0 X units (the wave's DS operations execute in order)
  auto stage2 = [&](char* region, int par, ClRing& clr) {
#if defined(BCFFT_DM_MEMONLY) || (defined(BCFFT_DM_ABL) && (BCFFT_DM_ABL & 2))
    return;
#endif
    const int ml = opaque(lane);
    const int arow = ml & 15, kb = ml >> 4;
    const int a_t = arow >> 2, a_reim = (arow >> 1) & 1, a_prec = arow & 1;
    const uint32_t a_sel = a_reim ? 0x01000302u : 0x03020100u;
    const int yt = ml >> 4;
    const int* sc = wsc + par * 8;
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
    const int xq = kb ^ (3 * (a_t >> 1));
    const char* ab0 = region + a_t * SLOT + wave * 1024 + 16 * (4 * a_prec + xq);        // bins fb < 4
    const char* ab1 = region + a_t * SLOT + wave * 1024 + 16 * (4 * (a_prec ^ 1) + xq);  // fb >= 4
    // A units: all bins up front (dft / dftx); EP loads each bin's as it goes (its registers
    // hold the lo8 ring instead)
    constexpr int NAR = EP ? 1 : BW;
    uint4 araw[NAR][KS];
    auto a_load = [&](int fb) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        araw[fb % NAR][ks] = *reinterpret_cast<const uint4*>((fb < 4 ? ab0 : ab1) + 128 * fb + 8192 * ks);
    };
    if constexpr (!EP) {
#pragma unroll
      for (int fb = 0; fb < BW; ++fb) a_load(fb);
    }
    uint32_t yh[BW][NT], yl[BW][NT];
#pragma unroll
    for (int fb = 0; fb < BW; ++fb) {
      const int f = wave * BW + fb;
      if constexpr (EP != 0) a_load(fb);
      f32x4 acc[NT], racc[NT];                      // racc: the weight residual's products
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[nt] = racc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        uint4 raw = araw[fb % NAR][ks];
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
        if constexpr ((EP & 2) != 0) {              // + A x e4m3 weight residual
          const u32x4 c8 = clr[fb % RING][ks];
          const long b0 = (long)(((uint64_t)c8.y << 32) | c8.x), b1 = (long)(((uint64_t)c8.w << 32) | c8.z);
          const long a8 = e4m3x8_s6(raw.x, raw.y, raw.z, raw.w);
          racc[0] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(a8, b0, racc[0], 0, 0, 0);
          racc[1] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(a8, b1, racc[1], 0, 0, 0);
        }
      }
      constexpr float YS = 1.f / 2097152.f;          // 2^-21: |Y| < 2^14 in fp16
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)                // rows 4 yt + {re hi, re lo, im hi, im lo}
      {
        float yr = acc[nt][0] + acc[nt][1], yi = acc[nt][2] + acc[nt][3];
        if constexpr ((EP & 2) != 0) {
          yr = fmaf(racc[nt][0] + racc[nt][1], 64.f, yr);
          yi = fmaf(racc[nt][2] + racc[nt][3], 64.f, yi);
        }
        yr *= YS;
        yi *= YS;
        if constexpr (EX) split2(yr, yi, yh[fb][nt], yl[fb][nt]);
        else yh[fb][nt] = pk_rne(yr, yi);
      }
      // EP: refill the ring slot only now that the bin's accumulators have been read, i.e. its
      // MFMAs have finished with the slot's registers (a load issued right after them can
      // overwrite an operand a queued MFMA has not read yet, as in stage 1)
      if constexpr ((EP & 2) != 0) {
        __builtin_amdgcn_sched_barrier(0);
        if (fb + RING < BW) cl_load(clr, fb + RING);
        __builtin_amdgcn_sched_barrier(0);          // one bin at a time: the overlapped schedule spills
      }
    }
    char* yb = region + yt * SLOT + wave * 1024 + 16 * (ml & 15);
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      *reinterpret_cast<uint4*>(yb + 16 * 16 * nt) = make_uint4(yh[0][nt], yh[2][nt], yh[4][nt], yh[6][nt]);
      *reinterpret_cast<uint4*>(yb + 16 * (32 + 16 * nt)) = make_uint4(yh[1][nt], yh[3][nt], yh[5][nt], yh[7][nt]);
      if constexpr (EX) {                           // lo terms over the K-step-1 X units of these bins
        *reinterpret_cast<uint4*>(yb + 8192 + 16 * 16 * nt) = make_uint4(yl[0][nt], yl[2][nt], yl[4][nt], yl[6][nt]);
        *reinterpret_cast<uint4*>(yb + 8192 + 16 * (32 + 16 * nt)) = make_uint4(yl[1][nt], yl[3][nt], yl[5][nt], yl[7][nt]);
      }
    }
  };

  // ---- stage 3 (I wave, token slot j = wave - 4 of the previous tile): Y -> y rows staged in
  // the slot and stored as 1 KiB contiguous buffer stores. The slot's Y units are read into
  // registers first. 16-bit y: 32 rows x 256 B in the second 8 KiB; fp32 y: N-tile 0's 16 rows
  // in the second 8 KiB, N-tile 1's in the first. (The next tile's x arrives in P2.)
  // ntm: the N-tiles this wave does (3: both, the I wave of a steady-state tile; the last pass
  // splits them between the slot's F and I waves, which then meet at a barrier between their Y
  // reads and staging writes: the staging of one N-tile overlays the Y units of both)
  // (a compile-time mask: a runtime one split the stage into ~30 basic blocks, one per N-tile's
  // MFMAs and staging writes, which the scheduler could not interleave)
  auto stage3 = [&](char* region, int par, int64_t mp, auto ntm_c) {
    constexpr int ntm = decltype(ntm_c)::value;
    const int l = opaque(lane);
    const int o16 = l & 15, g = l >> 4;
    char* slot = region + tslot * SLOT;
    const int* sc = wsc + par * 8 + tslot * 2;
    const int nmin = min(sc[0], sc[1]);
    float ysc[NT];                                  // output block o = 16 nt + o16: 1 / s_o (EP: the table's 2^8)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
      ysc[nt] = __builtin_ldexpf(reinterpret_cast<const float*>(lds + OS_OFF)[16 * nt + o16], (EP ? 15 : 30) - nmin);
    // EP: residual A fragments of table row t = 16 mt + o16: the 16-B pairs of columns
    // 64 pr + 32 ks + 8 g .. + 7 in pair-row t >> 1, the byte of row parity t & 1 picked by perm
    const int fl3 = FL_OFF + FL_STRIDE * (o16 >> 1) + 16 * g;
    const uint32_t flsel = (o16 & 1) ? 0x07050301u : 0x06040200u;
    // all Y fragments of the token: B[k = 8 g + j][o] = unit(wave 4 ks + g, o, parity)
    constexpr int NYP = EX ? 2 : 1;                 // Y precision terms (hi; lo 8 KiB further)
    constexpr bool YSP_PREF_OFF = EX;               // the lo terms take the table prefetch's VGPRs
    uint4 yf[NYP][KS][2][NT];
    const char* yb = slot + g * 1024 + 16 * o16;
#pragma unroll
    for (int yp = 0; yp < NYP; ++yp)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int pr = 0; pr < 2; ++pr)
#pragma unroll
          for (int nt = 0; nt < NT; ++nt)
            if ((ntm >> nt) & 1)
              yf[yp][ks][pr][nt] = *reinterpret_cast<const uint4*>(yb + 8192 * yp + 4096 * ks + 16 * (32 * pr + 16 * nt));
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
    if constexpr (ntm != 3) lds_barrier();          // ... for both waves of the slot
    SUBSTAMP(55);
    SUBSTAMP(56);
    const int64_t tok = mp * TT + tslot;
    const bool tok_ok = tok < n_tokens;
    const int nvalid = n_out - grp_o * OPG;
    // staging write bases (lane part of the XOR-swizzled address; the rest are immediates).
    // fp32: (4 mt + g) ^ s = 4 mt + (g ^ (s & 3)) +- 4 (s >> 2) by the parity of mt (s = o16 & 7);
    // 16-bit: (4 mt + g) ^ sg for each mt (sg = ((o16 & 7) << 1) | (o16 >> 3))
    int swb[Y32 ? 2 : 4];
    if constexpr (Y32) {
      const int s7 = o16 & 7;
      const int b0 = 512 * o16 + 16 * (g ^ (s7 & 3));
      swb[0] = b0 + 64 * (s7 >> 2);
      swb[1] = b0 - 64 * (s7 >> 2);
    } else {
      const int sg = ((o16 & 7) << 1) | (o16 >> 3);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) swb[mt] = 256 * o16 + 8 * ((4 * mt + g) ^ sg);
    }
#if !defined(BCFFT_DM_MEMONLY) && !(defined(BCFFT_DM_ABL) && (BCFFT_DM_ABL & 4))
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      if (!YSP_PREF_OFF && mt < 3) gload(mt + 1, gnxt);
      f32x4 E[NT], O[NT];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        E[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
        O[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int yp = 0; yp < NYP; ++yp)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) {
            if (!((ntm >> nt) & 1)) continue;
            E[nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(gcur[ks][0], __builtin_bit_cast(f16x8, yf[yp][ks][0][nt]), E[nt], 0, 0, 0);
            O[nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(gcur[ks][1], __builtin_bit_cast(f16x8, yf[yp][ks][1][nt]), O[nt], 0, 0, 0);
          }
      if constexpr ((EP & 4) != 0) {                // + e4m3 table residual x bf8(Y hi)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {           // f16 -> fp8 on one accumulator (xdl_gap)
          if ((ntm >> nt) & 1) {
            xdl_gap(E[nt]);
            xdl_gap(O[nt]);
          }
        }
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
#pragma unroll
          for (int pr = 0; pr < 2; ++pr) {
            asm volatile("" ::: "memory");          // one residual fragment at a time (registers)
            const uint4 w = *reinterpret_cast<const uint4*>(lds + fl3 + 2304 * mt + 128 * pr + 64 * ks);
            const long fl = (long)(((uint64_t)__builtin_amdgcn_perm(w.w, w.z, flsel) << 32) |
                                   __builtin_amdgcn_perm(w.y, w.x, flsel));
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
              if (!((ntm >> nt) & 1)) continue;
              const uint4 v = yf[0][ks][pr][nt];
              f32x4& acc3 = pr ? O[nt] : E[nt];
              acc3 = __builtin_amdgcn_mfma_f32_16x16x32_fp8_bf8(fl, bf8x8(v.x, v.y, v.z, v.w), acc3, 0, 0, 0);
            }
          }
      }
      // rows t = 16 mt + 4 g + r (and t + 64), column o = 16 nt + o16
      if constexpr (GLU) {                          // h = silu(gate) * up of block o16
        float gu[NT][2][4];
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
#pragma unroll
          for (int hf = 0; hf < 2; ++hf)
#pragma unroll
            for (int r = 0; r < 4; ++r)             // gate / up rounded to x's dtype (:266)
              gu[nt][hf][r] = round_to(hf ? fmaf(E[nt][r], ysc[nt], -O[nt][r] * ysc[nt]) : fmaf(E[nt][r], ysc[nt], O[nt][r] * ysc[nt]), XT);
        }
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r)               // torch: silu rounded, then the product rounded
            v[r] = round_to(round_to(silu(gu[0][hf][r]), XT) * gu[1][hf][r], XT);
          if constexpr (Y32) {
            *reinterpret_cast<float4*>(slot + 8192 + swb[mt & 1] + 64 * mt + 256 * hf) = make_float4(v[0], v[1], v[2], v[3]);
          } else {
            *reinterpret_cast<uint2*>(slot + 8192 + swb[mt] + 128 * hf) =
                make_uint2(pack16<XT>(v[0], v[1]), pack16<XT>(v[2], v[3]));
          }
        }
      } else
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        if (!((ntm >> nt) & 1)) continue;
        const int o = 16 * nt + o16;
        float os[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) os[r] = O[nt][r] * ysc[nt];
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = hf ? fmaf(E[nt][r], ysc[nt], -os[r]) : fmaf(E[nt][r], ysc[nt], os[r]);
          // the precise engine (BM >= 0, fp32 outputs) adds its bias to the staged rows at the store
          // phase instead (the same value: v is already in its fp32 form), where registers are free
          const bool has_bias = BM < 0 && bias_dt != BCFFT_NONE;
          if (Y32 || has_bias) {                    // .to(x dtype) :266, + bias :270-271
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = round_to(v[r], XT);
            if (has_bias && o < nvalid) {
              const int64_t cc = (int64_t)(grp_o * NOG + o) * B + 16 * mt + 4 * g + 64 * hf;
#pragma unroll
              for (int r = 0; r < 4; ++r) v[r] += load_scalar(bias, cc + r, bias_dt);
            }
          }
          if constexpr (Y32) {                      // N-tile nt's 16 rows: unit (4 mt + g + 16 hf) ^ (o16 & 7)
            *reinterpret_cast<float4*>(slot + (nt ? 0 : 8192) + swb[mt & 1] + 64 * mt + 256 * hf) =
                make_float4(v[0], v[1], v[2], v[3]);
          } else {                                  // row o of the 32: 8-B unit (4 mt + g + 16 hf) ^ sg
            *reinterpret_cast<uint2*>(slot + 8192 + 4096 * nt + swb[mt] + 128 * hf) =
                make_uint2(pack16<XT>(v[0], v[1]), pack16<XT>(v[2], v[3]));
          }
        }
      }
      if constexpr ((EP & 4) != 0) __builtin_amdgcn_sched_barrier(0);   // one mt at a time (registers)
      if (mt < 3) {
        if (YSP_PREF_OFF) {
          gload(mt + 1, gcur);                      // no prefetch: registers for the Y lo terms
        } else {
#pragma unroll
          for (int ks = 0; ks < KS; ++ks)
#pragma unroll
            for (int pr = 0; pr < 2; ++pr) gcur[ks][pr] = gnxt[ks][pr];
        }
      }
    }
#endif
    SUBSTAMP(57);
    // staged rows -> global: each instruction stores 1 KiB = RPI whole y rows of the group. The
    // y rows of the group start the buffer (rows past nvalid fall outside it and are dropped);
    // lane offsets are two or four bases plus immediates.
    constexpr int RB = B * ESY, RPI = 1024 / RB, LPR = 64 / RPI;   // row bytes, rows/store, lanes/row
    const int w = l & (LPR - 1), lr = (int)((unsigned)l / LPR);
    const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
        (char*)yv + (tok_ok ? tok : 0) * M * ESY + (int64_t)grp_o * OPG * RB, 0,
        tok_ok ? (int)((M - (int64_t)grp_o * OPG * B) * ESY) : 0, 0x00020000);
    constexpr int NQ = GLU && !Y32 ? 4 : 8;         // store instructions per half (GLU 16-bit: 16 rows)

    const int vofs = lr * RB + 16 * w;
    // LDS read bases: fp32 row s16 = 2 q + lr, unit w ^ (s16 & 7) = (w ^ lr) ^ 2 (q & 3);
    // 16-bit row rr = 4 q + lr, unit w ^ (rr & 7) = (w ^ lr) ^ 4 (q & 1)
    int rdb[Y32 ? 4 : 2];
#pragma unroll
    for (int c = 0; c < (Y32 ? 4 : 2); ++c)
      rdb[c] = lr * RB + 16 * ((w ^ lr) ^ (Y32 ? 2 * c : 4 * c));
#pragma unroll
    for (int half = 0; half < (Y32 && !GLU ? 2 : 1); ++half) {   // 8 store instructions at a time
      if (Y32 && !GLU && !((ntm >> half) & 1)) continue;
      uint4 d[8];
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        if constexpr (Y32) {                        // rows 16 half + 2 q + lr: N-tile half's staging
          d[q] = *reinterpret_cast<const uint4*>(slot + (half ? 0 : 8192) + 1024 * q + rdb[q & 3]);
          if constexpr (BM >= 1) {                  // + bias of output row 16 half + 2 q + lr, t = 4 w .. 4 w + 3
            static_assert(!GLU, "no bias on the fused gate/up");
            const int bes = BM == 1 ? 4 : 2;
            const __amdgpu_buffer_rsrc_t brs = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<char*>((const char*)bias) + (int64_t)grp_o * NOG * B * bes, 0,
                (int)((M - (int64_t)grp_o * NOG * B) * bes), 0x00020000);
            const int boff = (lr * B + 4 * w) * bes, bimm = ((16 * half + 2 * q) * B) * bes;
            float4 bv;
            if constexpr (BM == 1) {
              bv = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(brs, boff, bimm, 0));
            } else {
              const u32x2 bw = __builtin_amdgcn_raw_buffer_load_b64(brs, boff, bimm, 0);
              bv = bias_dt == BCFFT_BF16
                       ? make_float4(bf16_to_f32(bw.x & 0xffffu), bf16_to_f32(bw.x >> 16), bf16_to_f32(bw.y & 0xffffu),
                                     bf16_to_f32(bw.y >> 16))
                       : make_float4(f16_to_f32(bw.x & 0xffffu), f16_to_f32(bw.x >> 16), f16_to_f32(bw.y & 0xffffu),
                                     f16_to_f32(bw.y >> 16));
            }
            d[q] = make_uint4(__float_as_uint(__uint_as_float(d[q].x) + bv.x), __float_as_uint(__uint_as_float(d[q].y) + bv.y),
                              __float_as_uint(__uint_as_float(d[q].z) + bv.z), __float_as_uint(__uint_as_float(d[q].w) + bv.w));
          }
        } else {
          uint4 v = *reinterpret_cast<const uint4*>(slot + 8192 + 1024 * q + rdb[q & 1]);
          if (q & 2) v = make_uint4(v.z, v.w, v.x, v.y);   // rows with bit 3: 8-B halves swapped
          d[q] = v;
        }
      }
#ifdef BCFFT_DM_NOMEM
      if (tok < 0)                                  // never (analysis build): keeps the staging reads
#endif
#pragma unroll
      for (int q = 0; q < NQ; ++q)                  // byte offset of row 8 RPI half + RPI q + lr
        if (Y32 || GLU || ((ntm >> (q >> 2)) & 1))  // 16-bit: rows of N-tile q >> 2
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, d[q]), yrs,
                                                 vofs + (8 * half + q) * 1024, 0, BCFFT_YAUX);
    }
    SUBSTAMP(58);
  };

  // Pipeline, two workgroup barriers per M-tile. Iteration it (region R = it & 1 holds tile m,
  // the other R' tile m - gstride):
  //   P1  F waves: wait for their own x DMA, stage 1 of tile m in R.  I waves: stage 3 of tile
  //       m - gstride from R' (Y read, y staged in the slot, 1 KiB stores)          | Ba |
  //   P2  F waves: LDS-DMA of x(m + gstride) into their slot of R'; all waves: stage 2 of
  //       tile m in R                                                               | Bb |
  // so the tile's HBM traffic is split between the phases: y stores in P1, x loads in P2.
  int64_t m = wg_in_grp;
  STAMP(0);
  for (int it = 0; m < n_mtiles || it > 0; ++it, m += gstride) {
    char* region = lds + (it & 1) * REGION;
    char* other = lds + ((it + 1) & 1) * REGION;
    const int par = it & 1;
    const bool have_f = m < n_mtiles;
    const int sb = 1 + 6 * (it < 8 ? it : 8);       // stamp slots: iterations 0-7, then the latest
    sub_on = it == 4;
    STAMP(sb);
    // EARLY_X: in iteration 0 the I waves have no stage 3, and region R' is free: they stream
    // tile m + gstride's x into it at once (slot wave - 4, the slot of the F wave that would
    // otherwise issue it after Ba), so HBM is not idle through the first stage 1; they wait for
    // it before Bb. FILL_SPLIT / DRAIN_SPLIT: see the kernel's top.
    const bool early = EARLY_X && it == 0 && !fwave && m + gstride < n_mtiles;
    if (early) dma_token(m + gstride, other, 0, NDMA);
    // stage 1 has ONE call site: the fill (each wave of a slot one half) runs the same code as the
    // steady state, so its instruction fetch warms the F waves' stage 1 of iteration 1 (with two
    // inlined copies, the first steady-state stage 1 of every CU missed the instruction cache
    // together: ~5 k cycles, profiles/r05y_timeline_dm_nofd.txt)
    const bool fill = FILL_SPLIT && it == 0;
    constexpr bool XW = ES == 4 && EP == 0;         // steady-state stage 1 waits for each half of x on its own
    if (have_f && (fill || fwave)) {
      if (fill) {                                   // fill: both waves of a slot, one half each
        if (!fwave && early) wait_vmcnt<NPIECE + NDMA>();   // own half of tile 0's x (prologue)
        else wait_vmcnt<NPIECE>();
      } else {
        if (LATE_W && it == 0) wait_vmcnt<NPIECE>();   // tile 0's x, not the weight loads behind it
        else if (!XW) wait_vmcnt<0>();              // this wave's own x DMA (issued a phase ahead)
      }
      stage1(region, par, fill ? (fwave ? 1 : 2) : 3, !fill && XW && it > 0);
    } else if (fwave) {
      if (!have_f && DRAIN_SPLIT)                   // drain: the last tile's stage 3, N-tile 1
        stage3(other, par ^ 1, m - gstride, std::integral_constant<int, 2>{});
    } else if (it > 0) {
      if (DRAIN_SPLIT && !have_f) stage3(other, par ^ 1, m - gstride, std::integral_constant<int, 1>{});
      else stage3(other, par ^ 1, m - gstride, std::integral_constant<int, 3>{});
    }
    if constexpr (LATE_W) creg_tie();               // the weights, first needed by stage 2
    STAMP(sb + 1);
    if (!have_f) break;
    // EP: the first lo8 bins of stage 2, issued by every wave here (one definition point: the
    // ring holds no registers through stage 1 or stage 3) and waited for after Ba, before the F
    // waves' x DMA: the compiler counts none of the asm DMA, so a wait behind it would drain it
    ClRing clr;
    if constexpr ((EP & 2) != 0) {
#pragma unroll
      for (int i = 0; i < RING; ++i) cl_load(clr, i);
    }
    lds_barrier();                                  // Ba: X units and scales complete
    if constexpr ((EP & 2) != 0) {
#pragma unroll
      for (int i = 0; i < RING; ++i) asm volatile("" : "+v"(clr[i][0]), "+v"(clr[i][1]));
    }
    STAMP(sb + 2);
    // F wave j streams the next tile's x for its slot j of the other region in one burst: stage 3
    // has read that slot's Y and staged y (each wave's LDS reads completed before Ba)
    // (EP: after stage 2 instead. Loads return in order, so a wait for a lo8 refill issued behind
    // the DMA waits for the DMA too: DESIGN.md section 6c)
    const bool dma_now = fwave && m + gstride < n_mtiles && !(EARLY_X && it == 0);
    if (dma_now && (EP & 2) == 0) dma_token(m + gstride, other, 0, NDMA);
    STAMP(sb + 3);
    stage2(region, par, clr);
    if constexpr ((EP & 2) != 0) {
      if (dma_now) dma_token(m + gstride, other, 0, NDMA);
    }
    if (EARLY_X && it == 0 && !fwave) wait_vmcnt<0>();   // the next tile's x (issued by this I wave) has landed
    STAMP(sb + 4);
    lds_barrier();                                  // Bb: Y units complete
    STAMP(sb + 5);
  }
  STAMP(63);
}

}  // namespace bcfft

namespace {
template <int XT, bool YF32, bool EX, bool GLU = false, int EP = 0, int BM = -1>
void launch_dm(const void* x, int64_t n, int n_out, const void* spec, const void* bias, int bias_dt, void* y,
               hipStream_t s) {
  const int groups = GLU ? (n_out + 15) / 16 : (n_out + 31) / 32;
  const bcfft::SpecLayout sl = bcfft::spec_layout(GLU ? 32 * groups : n_out, 32, 128);
  const int64_t n_mtiles = (n + 3) / 4;
  const int64_t total = bcfft::group_grid(bcfft::device_cu_count(), groups, n_mtiles);
  const uint32_t* stat = reinterpret_cast<const uint32_t*>(spec) + sl.stat_off_u32;
  const float* osc = reinterpret_cast<const float*>(spec) + sl.osc_off_u32;
  const uint4* lo8 = reinterpret_cast<const uint4*>(reinterpret_cast<const uint32_t*>(spec) + sl.lo8_off_u32);
  hipLaunchKernelGGL((bcfft::bc_forward_dm_kernel<XT, YF32, EX, GLU, EP, BM>), dim3((unsigned)total), dim3(512), 0, s, x,
                     n, n_out, stat, osc, bias, bias_dt, y, lo8);
}
}  // namespace

// analysis builds only: stamp buffer of bc_forward_dm_kernel (this TU's copy). Slots per wave:
// 0 start | per M-tile it (base 1 + 6 min(it, 8)): +0 loop top, +1 stage 1 / stage 3 done,
// +2 after Ba, +3 DMA issued (F waves), +4 stage 2 done, +5 after Bb | 55-62 sub-phases of
// iteration 4 (F waves, per half: x read, scale, MFMAs, X written; I waves: Y read, DMA issued,
// per N-tile computed + stored, DMA 2 issued) | 63 end
BCFFT_STAMPS_SETTER(dm)

namespace bcfft {
bool dm_eligible(int n_in, int b) { return b == 128 && n_in == 32; }
// the precise engine's forms (launch_forward_dm): fp32 outputs; a 16-bit bias with fp32 x only
bool dftp_serves(int xdt, bool yf32, int bias_dt) {
  return yf32 && (bias_dt == BCFFT_NONE || bias_dt == BCFFT_F32 || xdt == BCFFT_F32);
}

// mode 0: dft; 1 (exact): Y as hi + lo (BCFFT_ALGO_DFTX), which fp16 outputs always take; 2: the
// precise engine (BCFFT_ALGO_DFTP) for fp32 outputs: fp32 x with no, an fp32 or a 16-bit bias, and
// 16-bit x with no or an fp32 bias (the reference rounds 16-bit x's output to x's dtype before the
// bias, :266-271; the kernel does the same). 16-bit outputs run DFTX, whose error already sits far
// below their rounding. (Round 6: the 16-bit-x and 16-bit-bias instantiations had computed wrong
// values because the residual MFMAs accumulated into the fp16 MFMAs' accumulators, an SrcC chain
// across opcodes that gfx950 does not forward: DESIGN.md section 6b.)
bool launch_forward_dm(int b, int n_in, int xdt, bool yf32, int mode, const void* x, int64_t n, int n_out,
                       const void* spec, const void* bias, int bias_dt, void* y, hipStream_t s) {
  if (!dm_eligible(n_in, b)) return false;
  const bool exact = mode >= 1;
  if (mode == 2 && dftp_serves(xdt, yf32, bias_dt)) {
    constexpr int P = 7;                            // all three residual terms
    if (xdt == BCFFT_F32) {
      if (bias_dt == BCFFT_NONE) launch_dm<BCFFT_F32, true, true, false, P, 0>(x, n, n_out, spec, bias, bias_dt, y, s);
      else if (bias_dt == BCFFT_F32) launch_dm<BCFFT_F32, true, true, false, P, 1>(x, n, n_out, spec, bias, bias_dt, y, s);
      else launch_dm<BCFFT_F32, true, true, false, P, 2>(x, n, n_out, spec, bias, bias_dt, y, s);
    } else if (xdt == BCFFT_BF16) {
      if (bias_dt == BCFFT_NONE) launch_dm<BCFFT_BF16, true, true, false, P, 0>(x, n, n_out, spec, bias, bias_dt, y, s);
      else launch_dm<BCFFT_BF16, true, true, false, P, 1>(x, n, n_out, spec, bias, bias_dt, y, s);
    } else {
      if (bias_dt == BCFFT_NONE) launch_dm<BCFFT_F16, true, true, false, P, 0>(x, n, n_out, spec, bias, bias_dt, y, s);
      else launch_dm<BCFFT_F16, true, true, false, P, 1>(x, n, n_out, spec, bias, bias_dt, y, s);
    }
    return true;
  }
  // fp32 outputs with a bias add it at the store phase (BM = 1 / 2: one buffer load per 4 values);
  // the per-element path of BM = -1 costs ~50 % at the north star's size
  const int bm = bias_dt == BCFFT_NONE ? 0 : bias_dt == BCFFT_F32 ? 1 : 2;
#define BCFFT_DM_LAUNCH_EX(XT, EXV)                                                                       \
  (!yf32            ? launch_dm<XT, true, EXV>(x, n, n_out, spec, bias, bias_dt, y, s)                  \
   : bm == 0        ? launch_dm<XT, true, EXV, false, 0, 0>(x, n, n_out, spec, bias, bias_dt, y, s)     \
   : bm == 1        ? launch_dm<XT, true, EXV, false, 0, 1>(x, n, n_out, spec, bias, bias_dt, y, s)     \
                    : launch_dm<XT, true, EXV, false, 0, 2>(x, n, n_out, spec, bias, bias_dt, y, s))
#define BCFFT_DM_LAUNCH(XT, YF)                                                                           \
  (YF ? (exact ? BCFFT_DM_LAUNCH_EX(XT, true) : BCFFT_DM_LAUNCH_EX(XT, false))                             \
      : (exact ? launch_dm<XT, YF, true>(x, n, n_out, spec, bias, bias_dt, y, s)                          \
               : launch_dm<XT, YF, false>(x, n, n_out, spec, bias, bias_dt, y, s)))
  if (!exact && dm8_eligible(n_in, b, xdt, yf32)) {  // bf16 I/O: 8 tokens per tile
    if (dmg_eligible(n_in, b, xdt, yf32, n_out, false) && multigroup_pays(n, 3)) {   // x transformed once (bcfft_dmg.hip)
      launch_forward_dmg(x, n, n_out, spec, bias, bias_dt, y, false, s);
      return true;
    }
    launch_forward_dm8(x, n, n_out, spec, bias, bias_dt, y, false, s);   // bcfft_dm8.hip
    return true;
  }
  if (xdt == BCFFT_F32) BCFFT_DM_LAUNCH(BCFFT_F32, true);
  else if (xdt == BCFFT_F16 && yf32) BCFFT_DM_LAUNCH(BCFFT_F16, true);
  else if (xdt == BCFFT_F16) launch_dm<BCFFT_F16, false, true>(x, n, n_out, spec, bias, bias_dt, y, s);
  else if (yf32) BCFFT_DM_LAUNCH(BCFFT_BF16, true);
  else BCFFT_DM_LAUNCH(BCFFT_BF16, false);
#undef BCFFT_DM_LAUNCH
#undef BCFFT_DM_LAUNCH_EX
  return true;
}

// fused gate/up + SwiGLU (bcfft_forward_glu): h has x's dtype, no bias; fp16 takes the exact variant
bool launch_forward_dm_glu(int b, int n_in, int xdt, int mode, const void* x, int64_t n, int n_gate,
                           const void* spec, void* h, hipStream_t s) {
  if (!dm_eligible(n_in, b)) return false;
  const bool exact = mode >= 1;
  if (mode == 2 && xdt == BCFFT_F32) {             // precise engine: fp32 h only (16-bit h: DFTX)
    launch_dm<BCFFT_F32, true, true, true, 7, 0>(x, n, n_gate, spec, nullptr, BCFFT_NONE, h, s);
    return true;
  }
  if (xdt == BCFFT_F32) {
    if (exact) launch_dm<BCFFT_F32, true, true, true>(x, n, n_gate, spec, nullptr, BCFFT_NONE, h, s);
    else launch_dm<BCFFT_F32, true, false, true>(x, n, n_gate, spec, nullptr, BCFFT_NONE, h, s);
  } else if (xdt == BCFFT_F16) {
    launch_dm<BCFFT_F16, false, true, true>(x, n, n_gate, spec, nullptr, BCFFT_NONE, h, s);
  } else {
    if (exact) launch_dm<BCFFT_BF16, false, true, true>(x, n, n_gate, spec, nullptr, BCFFT_NONE, h, s);
    else if (dmg_eligible(n_in, b, xdt, false, n_gate, true) && multigroup_pays(n, 5))
      launch_forward_dmg(x, n, n_gate, spec, nullptr, BCFFT_NONE, h, true, s);   // x transformed once per tile
    else launch_forward_dm8(x, n, n_gate, spec, nullptr, BCFFT_NONE, h, true, s);   // 8 tokens per tile
  }
  return true;
}
}  // namespace bcfft
