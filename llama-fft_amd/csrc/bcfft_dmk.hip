// bcfft_dmk.hip — the DFT-on-MFMA block-circulant forward for K > 4096 at b = 128, bf16 I/O
// (gfx950): the LLaMA down projection 11008 -> 4096 and every other wide-input layer.
//
// Same operator as the other DFT kernels (BlockCirculantLinear.forward, patch_llama_fft.py:
// 226-275; per block src/fft_utils.py:3-34) and the same three matrix-core stages: forward
// block DFT (stage 1), per-bin complex MAC (stage 2), inverse block DFT (stage 3). What changes
// is where the weights live. An output group's fp16 spectra at K = 11008 are 704 KiB: more than
// the register file and the LDS together, so they cannot stay resident as in bcfft_dm8.hip.
// Instead the K axis is cut into 16-block chunks and each chunk's B fragments are streamed from
// L2 into VGPRs once per M-tile (TT = 8 or 16 tokens), while the per-bin products accumulate in
// registers over all chunks.
//
//  * Workgroup: 8 waves (two per SIMD), persistent, one per CU. Wave w owns the 8 bins
//    8w .. 8w + 7 and keeps Y of the tile's TT tokens for them: 8 bins x TT/8 M-tiles (8 tokens
//    x re/im) x 2 N-tiles (16 output blocks) of fp32 accumulators (64 or 128 registers).
//  * Per chunk step: wave w streams x of its TT/8 tokens (16 blocks, 4 KiB of bf16 each) into
//    LDS one step ahead (LDS-DMA) and runs stage 1 of them; barrier; stage 2 of all TT tokens on
//    its bins against the chunk's 16 B fragments (64 VGPRs), loading the next chunk's fragments
//    bin by bin as each bin is done; barrier. Each fragment serves TT tokens: the L2 -> CU weight
//    stream is 96 or 48 KiB per token.
//  * Tile end: Y as fp16 units into the last chunk's region, 8 tokens at a time, with stage 3 of
//    token w (y staged in LDS, 1 KiB stores); the last 8 tokens' stage 3 runs at the start of
//    the next tile, beside its first stage 1.
//  * The launcher takes 16-token tiles once every CU gets one, else 8 (a tile is a serial chain
//    of chunk steps, so small N wants more, shorter tiles).
//  * Numerics: per-(token, chunk) power-of-two scales from stage 1, which keeps |X| < 2^(14 -
//    HEAD). Stage 2 aligns each chunk to the token's reference exponent (the first chunk's,
//    lowered when a chunk is more than 2^HEAD louder): A rows are multiplied by 2^-d, d >= -HEAD
//    (exact, below fp16's max), and a lowered reference scales the token's accumulator rows
//    down once. a, d, X and Y are one RNE fp16 term each, C and the table one term each, fp32
//    accumulation (tests/dm_model.py, head = 4, mirrors it).
//
// LDS (TT = 16: 149,632 B; TT = 8: 148,608 B): two regions of x-chunk slots of 4,160 B, each also
// holding 8 Y / y-staging slots of 8,256 B at the tile end, the DFT table, the scales. Slot
// strides are 64 B off the 256-B bank period, as in bcfft_dm8.hip, so the stage-2 reads of eight
// tokens at once are conflict-free; all in-slot offsets are bcfft_dm8.hip's.
#ifndef BCFFT_STREAM_POLICY
#define BCFFT_STREAM_POLICY 3                       // write-through y stores: 4-5 % faster here, nt x loads slower (profiles/r04_ab_stream_policy_split.log)
#endif
#include "bcfft_device.h"
#include "bcfft_dm_table.h"
#include "bcfft_dm_common.h"
#include <algorithm>

namespace bcfft {

namespace dmk {
using namespace dmh;
// analysis builds only (tools/ab_dmk.sh; results are WRONG when set): 1 no B loads, 2 no stage-1
// arithmetic, 4 no stage-2 MFMAs, 8 no stage 3, 16 no x DMA
#ifdef BCFFT_DMK_ABL
constexpr int ABL = BCFFT_DMK_ABL;
#else
constexpr int ABL = 0;
#endif
// wave priority falling through stage 1 (1) and stage 2 (2): set_prio, bcfft_dm64k.hip's finding
constexpr int PRIO = 3;

constexpr int B = 128, NW = 8, BPW = 8, NT = 2, NOG = 32;
constexpr int XSLOT = 4096 + 64;                    // one token's 16-block x chunk -> X units
constexpr int YSLOT = 8192 + 64;                    // one token's Y units -> y staging
static_assert(XSLOT % 256 == 64 && YSLOT % 256 == 64, "slot strides 64 B off the bank period");
constexpr int FRAGS = BPW * NT;                     // B fragments per wave and chunk
// per tile size TT (8 or 16 tokens): M-tiles, x DMA pieces per wave and chunk, LDS map
template <int TT>
struct Geo {
  static constexpr int MT = TT / 8;
  static constexpr int TPW = TT / NW;               // tokens per wave (x DMA, stage 1)
  static constexpr int NDMA = TPW * 4;              // 1-KiB x DMA pieces per wave and chunk
  static constexpr int REGION = TT * XSLOT > 8 * YSLOT ? TT * XSLOT : 8 * YSLOT;   // x, or Y of 8 tokens
  static constexpr int F_OFF = 2 * REGION;          // DFT table image, 64 rows x 256 B
  static constexpr int SC_OFF = F_OFF + 16384;      // chunk scale exponents [TT]
  static constexpr int RR_OFF = SC_OFF + 64;        // per-token reference exponents [TT]
  static constexpr int OS_OFF = RR_OFF + 64;       // the group's 32 inverse weight scales
  static constexpr int LDS_BYTES = OS_OFF + 128;
  static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
  static_assert(F_OFF % 256 == 0, "table rows on the bank period");
};

// chunk alignment headroom: stage 1 keeps |X| below 2^(14 - HEAD), so stage 2 can raise a chunk
// up to 2^HEAD louder than the token's reference exponent without an fp16 overflow, and the
// accumulator rescale runs only for chunks beyond that (never for chunk maxima that differ by
// less than 16x, i.e. practically never for activations without outliers)
constexpr int HEAD = 4;
// fp16 factor 2^-d (d >= -15) as a (lo, hi) pair: subnormal below 2^-14, zero below 2^-24
__device__ __forceinline__ uint32_t f16_pow2_neg(int d) {
  return d <= 14 ? (uint32_t)(15 - d) << 10 : (d <= 24 ? 1u << (24 - d) : 0u);
}
}  // namespace dmk

// SPL (decode / short-prefill sizes, bc_dmk_finish_kernel): the K-chunks are split into kz slices;
// workgroup b takes slice b % kz of exactly one (group, tile) and writes its partial y in fp32 to
// ws[slice][token][column] (no rounding, no bias), and a finishing pass sums the slices.
// HB: a bias is added (the runtime bias_dt then names its dtype); without one the store path is
// straight-line (a runtime test per stored quad split stage 3 into hundreds of basic blocks)
template <int TT, bool SPL = false, bool HB = false>
__global__ __launch_bounds__(512, 2) void bc_forward_dmk_kernel(
    const void* __restrict__ xv, int64_t n_tokens, int n_in, int n_out, const uint32_t* __restrict__ stat,
    const float* __restrict__ osc, const void* __restrict__ bias, int bias_dt, void* __restrict__ yv,
    int kz, float* __restrict__ ws) {
  using namespace dmk;
  using G = Geo<TT>;
  constexpr int MT = G::MT, TPW = G::TPW, NDMA = G::NDMA, REGION = G::REGION, F_OFF = G::F_OFF;
  constexpr int XT = BCFFT_BF16;
  constexpr int ES = 2, ESY = 2;

  __shared__ __attribute__((aligned(16))) char lds[G::LDS_BYTES];
  int* wsc = reinterpret_cast<int*>(lds + G::SC_OFF);
  int* wrr = reinterpret_cast<int*>(lds + G::RR_OFF);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n_groups = (n_out + NOG - 1) / NOG;
  const int64_t K = (int64_t)n_in * B;
  const int64_t M = (int64_t)n_out * B;
  const int nch = (n_in + 15) / 16;
  const int64_t n_mtiles = (n_tokens + TT - 1) / TT;
  // chunk range [c0, c1) of this workgroup; unsplit: all chunks, persistent over tiles
  int grp_o, wg_in_grp, gstride, c0 = 0, c1 = nch, slice = 0;
  if constexpr (SPL) {                              // grid = kz x groups x tiles, one tile each
    slice = blockIdx.x % kz;
    const int rest = blockIdx.x / kz;
    grp_o = rest % n_groups;
    wg_in_grp = rest / n_groups;
    gstride = (int)n_mtiles;
    const int cps = (nch + kz - 1) / kz;
    c0 = slice * cps;
    c1 = min(nch, c0 + cps);
  } else {
    const GroupMap gm = group_map(n_groups);        // XCD-aware when the grid allows it
    grp_o = gm.grp;
    wg_in_grp = gm.lane;
    gstride = gm.stride;
  }
  const uint32_t lds_base = __builtin_amdgcn_readfirstlane(lds_addr(lds));
  const uint4* bimg = reinterpret_cast<const uint4*>(stat + 4);
  ANALYSIS_INIT;

  // ---- x chunk c of token `wave` of M-tile m -> their slots by LDS-DMA. The
  // buffer range ends at the token's row end (a partial last chunk reads zeros) and is empty
  // for tokens past n_tokens or tiles past the end, which then land as zeros. Piece q of a
  // token = block rows 4q + (lane >> 4), with the slot's unit swizzle (unit u of block row r at
  // u ^ r) applied to the global source offsets.
  auto dma_chunk = [&](int64_t m, int c, char* region) {
    if constexpr ((ABL & 16) != 0) return;
    const int dl = opaque(lane);
    int vb[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = dl >> 4;
      vb[q] = r * 256 + 16 * ((dl & 15) ^ ((4 * q + r) & 15));
    }
#pragma unroll
    for (int t2 = 0; t2 < TPW; ++t2) {
      const int64_t tok = m * TT + TPW * wave + t2;
      const bool ok = m < n_mtiles && tok < n_tokens;
      const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<char*>((const char*)xv) + (ok ? tok * K * ES + (int64_t)c * 4096 : 0), 0,
          ok ? (int)(K * ES - (int64_t)c * 4096) : 0, 0x00020000);
      const uint32_t dst0 = lds_base + (uint32_t)(region - lds) + (TPW * wave + t2) * XSLOT;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        uint32_t keep;
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen" BCFFT_XPOL " lds\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(vb[q]), "s"(xrs), "s"(dst0 + q * 1024), "s"(q * 1024) : "memory");
      }
    }
  };

  // ---- the wave's B fragments of chunk c for N-tile nt (bins 8 wave + fb), from L2. Asm
  // buffer loads like the x DMA: the compiler does not count them, so its own waits never
  // drain the x DMA issued after them; wait_b (below) is the one wait on them, with the exact
  // number of younger VMEM operations, and it redefines the registers it waited for, so no use
  // can be scheduled above it.
  // The dependency the compiler cannot see: between load_b1 and wait_b the destination registers
  // are being written by the memory system, but hipcc treats them as holding their value. It must
  // not copy, spill or reuse them there. Round 5's late-DMA schedule (-DBCFFT_DMK_LATE_DMA, kept as
  // the negative control of tests/test_vmem_audit.py) made hipcc rotate all 64 fragment registers
  // with v_mov copies across the chunk loop: wrong tokens at N = 4090 on the GPU
  // (profiles/r06_dmk_late_dma_repro.txt). tools/vmem_audit.py checks every
  // build's ISA for that; wait_b's `; bcfft-wait <regs>` comment names the registers for it.
  auto b_rsrc = [&](int c) {
    return __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint4*>(bimg + ((int64_t)(grp_o * nch + (c < 0 ? 0 : c)) * NW + wave) * FRAGS * 64), 0,
        FRAGS * 1024, 0x00020000);
  };
  // fragment (fb, nt); no memory clobber: the asm only writes its register, so LDS reads may
  // be scheduled across it (both asm statements are volatile, so load and wait keep their order)
  auto load_b1 = [&](const __amdgpu_buffer_rsrc_t& brs, int vo, int fb, int nt, u32x4 (&breg)[BPW][NT]) {
    if constexpr ((ABL & 1) != 0) breg[fb][nt] = u32x4{(uint32_t)vo, (uint32_t)vo, (uint32_t)vo, (uint32_t)vo};
    else asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen"
                      : "=v"(breg[fb][nt]) : "v"(vo), "s"(brs), "s"((fb * NT + nt) * 1024));
  };
  auto load_b = [&](int c, int nt, u32x4 (&breg)[BPW][NT]) {
    const __amdgpu_buffer_rsrc_t brs = b_rsrc(c);
    const int vo = opaque(lane) * 16;
#pragma unroll
    for (int fb = 0; fb < BPW; ++fb) load_b1(brs, vo, fb, nt, breg);
  };
  // wait until at most N VMEM operations younger than N-tile nt's fragments are outstanding:
  // those fragments have then landed
  auto wait_b = [&](auto n_tag, int nt, u32x4 (&breg)[BPW][NT]) {
    constexpr int N = decltype(n_tag)::value;
    static_assert(N >= 0 && N < 64, "vmcnt");
    asm volatile("s_waitcnt vmcnt(%8) ; bcfft-wait %0 %1 %2 %3 %4 %5 %6 %7"
                 : "+v"(breg[0][nt]), "+v"(breg[1][nt]), "+v"(breg[2][nt]), "+v"(breg[3][nt]),
                   "+v"(breg[4][nt]), "+v"(breg[5][nt]), "+v"(breg[6][nt]), "+v"(breg[7][nt])
                 : "n"(N) : "memory");
  };
  static_assert(BPW == 8, "wait_b names eight fragments");

  // ---- stage 1 (wave w, tokens 2w, 2w + 1): x rows -> X units (one fp16 term), in place;
  // bcfft_dm8.hip's stage 1 on one 16-block half, with the x rows kept packed and the two
  // output parities in turn (the wave's 128 accumulators and 64 B registers stay live)
  auto stage1 = [&](char* region) {
    if constexpr ((ABL & 2) != 0) {
      if (lane < TPW) wsc[TPW * wave + lane] = 0;
      return;
    }
    const int l = opaque(lane);
    const int b16 = l & 15, g = l >> 4;
    const int q4 = (l & 15) >> 2, p4 = l & 3;
    const int cx = (p4 >> 1) ^ fsw(8 * g + q4);
    const int trb = F_OFF + 256 * (8 * g + q4) + 8 * (p4 & 1);
    if constexpr ((PRIO & 1) != 0) set_prio(2);
#pragma unroll 1
    for (int t2 = 0; t2 < TPW; ++t2) {
      char* slot = region + (TPW * wave + t2) * XSLOT;
      // x of block b16: t = 32 ks + 8 g + j and t + 64 (j < 8)
      const char* rowp = slot + b16 * (B * ES);
      uint32_t xr[2][2][4];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int pt = 0; pt < 2; ++pt) {
          const uint4 w = *reinterpret_cast<const uint4*>(rowp + 16 * ((4 * ks + g + 8 * pt) ^ b16));
          xr[ks][pt][0] = w.x; xr[ks][pt][1] = w.y; xr[ks][pt][2] = w.z; xr[ks][pt][3] = w.w;
        }
      float m0 = 0.f, m1 = 0.f;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int pt = 0; pt < 2; ++pt)
#pragma unroll
          for (int e = 0; e < 4; e += 2) {
            const float2 f0 = unpack16<XT>(xr[ks][pt][e]), f1 = unpack16<XT>(xr[ks][pt][e + 1]);
            m0 = amax3(m0, f0.x, f0.y);
            m1 = amax3(m1, f1.x, f1.y);
          }
      const float mxf = __builtin_fmaxf(m0, m1);
      // |a|, |d| <= 2 max|x| < 2^(15 - HEAD): stage 2 may raise a chunk by up to 2^HEAD
      const int sx = stat_scale_exp(2.f * __uint_as_float(wave_umax(__float_as_uint(mxf)))) - HEAD;
      if (l == 0) wsc[TPW * wave + t2] = sx - 7;      // X = D 2^-(sx - 7): the table's 2^-7
      const float S = __int_as_float((sx + 127) << 23);
      uint32_t ah[2][4], dh[2][4];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float2 lo = unpack16<XT>(xr[ks][0][e]), hi = unpack16<XT>(xr[ks][1][e]);
          const float u0 = hi.x * S, u1 = hi.y * S;
          ah[ks][e] = pk_rne(fmaf(lo.x, S, u0), fmaf(lo.y, S, u1));
          dh[ks][e] = pk_rne(fmaf(lo.x, S, -u0), fmaf(lo.y, S, -u1));
        }
      // X write lane bases: D^T row 4g + r is bin 16 mt + 4 g + pr (+ 2 for r >= 2), column
      // block b16; bin bit 2 = g & 1 swaps the 64-B blocks
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
            // A = F^T (16 bins-reals x 32 t): two transposed reads of 4 rows each
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
      if constexpr ((PRIO & 1) != 0) set_prio(1);
    }
  };

  // accumulators of the tile: [bin of the wave][M-tile][N-tile], rows 4 yt + r = token
  // 8 mt + 2 yt + (r >> 1), re/im r & 1; and the reference exponents of the lane's tokens
  f32x4 acc[BPW][MT][NT];
  int ra[MT];                                       // A-row token 8 mt + (lane & 15) / 2
  int rc[MT][2];                                    // accumulator-row tokens 8 mt + 2 yt + s

  // ---- stage 2 (all waves): per-bin complex MAC of chunk c on bins 16 wave + fb for all 8
  // tokens. A rows (token, re/im): re rows [Xr, Xi] per block, im rows [Xi, -Xr] (v_perm +
  // v_pk_mul_f16, which also aligns the chunk to the token's reference exponent); bin 0 (X0,
  // X64) with the extra 1/2.
  auto stage2 = [&](char* region, u32x4 (&breg)[BPW][NT], int cn, auto first_tag) {
    constexpr bool FIRST = decltype(first_tag)::value;
    const int ml = opaque(lane);
    const int arow = ml & 15, kb = ml >> 4;
    const int a_tl = arow >> 1, a_reim = arow & 1;
    const uint32_t a_sel = a_reim ? 0x01000302u : 0x03020100u;
    const int yt = ml >> 4;
    int nka[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      nka[mt] = wsc[8 * mt + a_tl];
      const int n0 = wsc[8 * mt + 2 * yt], n1 = wsc[8 * mt + 2 * yt + 1];
      if constexpr (FIRST) {
        ra[mt] = nka[mt];
        rc[mt][0] = n0;
        rc[mt][1] = n1;
      } else {
        ra[mt] = min(ra[mt], nka[mt] + HEAD);
      }
    }
    if constexpr (!FIRST) {
      // a chunk more than 2^HEAD louder than the token's reference: the reference drops to the
      // chunk's exponent + HEAD and the token's accumulator rows scale down once
      float fct[MT][2];
      bool need = false;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int nn = wsc[8 * mt + 2 * yt + s] + HEAD;
          const int d = rc[mt][s] - nn;
          fct[mt][s] = d > 0 ? __builtin_ldexpf(1.f, -d) : 1.f;
          need |= d > 0;
          rc[mt][s] = min(rc[mt][s], nn);
        }
      if (__builtin_amdgcn_ballot_w64(need)) {
#pragma unroll
        for (int fb = 0; fb < BPW; ++fb)
#pragma unroll
          for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
#pragma unroll
              for (int r = 0; r < 4; ++r) acc[fb][mt][nt][r] *= fct[mt][r >> 1];
      }
    }
    uint32_t amul[MT], amul0[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int d = nka[mt] - ra[mt];               // >= -HEAD: factor 2^-d <= 2^HEAD
      const uint32_t hh = f16_pow2_neg(d);
      const uint32_t h0 = f16_pow2_neg(d + 1);      // bin 0: the inverse's 1/b vs 2/b
      amul[mt] = a_reim ? (hh | ((hh | 0x8000u) << 16)) : (hh | (hh << 16));
      amul0[mt] = a_reim ? (h0 << 16) : h0;
    }
    const char* ab = region + a_tl * XSLOT + 512 * wave + 16 * kb;
    // B of this chunk (prefetched bin by bin in the previous step): younger VMEM is, outside
    // step 0, the next chunk's x DMA (NDMA)
    if constexpr (FIRST) {                          // younger: 8 stage-3 stores and x(1)
      wait_b(std::integral_constant<int, 8 + NDMA>{}, 0, breg);
      wait_b(std::integral_constant<int, 8 + NDMA>{}, 1, breg);
    } else {
      wait_b(std::integral_constant<int, NDMA>{}, 0, breg);
      wait_b(std::integral_constant<int, NDMA>{}, 1, breg);
    }
    const __amdgpu_buffer_rsrc_t nbrs = b_rsrc(cn);
    const int vo = opaque(lane) * 16;
    // A rows of bin fb for the MT M-tiles; the next bin's are read while this bin's are scaled and
    // multiplied (issued above the per-bin load branch, so the LDS latency is off the chain)
    auto a_off = [&](int fb, int mt) { return 8 * XSLOT * mt + 64 * (fb ^ ((fb >> 2) & 1)); };
    uint4 araw[2][MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) araw[0][mt] = *reinterpret_cast<const uint4*>(ab + a_off(0, mt));
    const bool bin0 = wave == 0;                    // bin 0 (wave 0, fb 0): (X_0, X_64), no swap
#pragma unroll
    for (int fb = 0; fb < BPW; ++fb) {
      if constexpr ((PRIO & 2) != 0) set_prio(3 - 4 * fb / BPW);
      if (fb + 1 < BPW) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) araw[(fb + 1) & 1][mt] = *reinterpret_cast<const uint4*>(ab + a_off(fb + 1, mt));
      }
      const uint32_t sel = (fb == 0 && bin0) ? 0x03020100u : a_sel;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const uint32_t mul = (fb == 0 && bin0) ? amul0[mt] : amul[mt];
        uint4 raw = araw[fb & 1][mt];
        raw.x = pkmul(__builtin_amdgcn_perm(raw.x, raw.x, sel), mul);
        raw.y = pkmul(__builtin_amdgcn_perm(raw.y, raw.y, sel), mul);
        raw.z = pkmul(__builtin_amdgcn_perm(raw.z, raw.z, sel), mul);
        raw.w = pkmul(__builtin_amdgcn_perm(raw.w, raw.w, sel), mul);
        const f16x8 a = __builtin_bit_cast(f16x8, raw);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const f16x8 bf = __builtin_bit_cast(f16x8, breg[fb][nt]);
          if constexpr ((ABL & 4) != 0)
            acc[fb][mt][nt] = FIRST ? f32x4{a[0], a[1], bf[0], bf[1]} : acc[fb][mt][nt] + f32x4{a[0], a[1], bf[0], bf[1]};
          else if constexpr (FIRST)
            acc[fb][mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, bf, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
          else
            acc[fb][mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, bf, acc[fb][mt][nt], 0, 0, 0);
        }
      }
      // this bin's fragments of the next chunk into the same registers, a whole step ahead of
      // their use; spread over the bins, not one burst. None after the last chunk: an asm load
      // whose result is never read leaves its registers free to the allocator while the load
      // is still in flight
      if (cn >= 0) {
        load_b1(nbrs, vo, fb, 0, breg);
        load_b1(nbrs, vo, fb, 1, breg);
      }
    }
  };

  // ---- Y of the tile's 8 tokens (M-tile MTI) as fp16 units into the region's 8 Y slots:
  // bcfft_dm8.hip's Y units
  auto ywrite = [&](char* region, auto mt_tag) {
    constexpr int MTI = decltype(mt_tag)::value;
    const int ml = opaque(lane);
    const int yt = ml >> 4;
    constexpr float YS = 1.f / 2097152.f;            // 2^-21: |Y| <= n_in 2^9 < 65504 (n_in <= 127)
    if (wave == 0 && (ml & 15) == 0) {
      wrr[8 * MTI + 2 * yt] = rc[MTI][0];
      wrr[8 * MTI + 2 * yt + 1] = rc[MTI][1];
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      char* yb = region + (2 * yt + s2) * YSLOT + 512 * wave + 16 * (ml & 15);
#pragma unroll
      for (int par = 0; par < 2; ++par)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          uint32_t u[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const f32x4 a = acc[par + 2 * j][MTI][nt];
            u[j] = pk_rne(a[2 * s2] * YS, a[2 * s2 + 1] * YS);
          }
          *reinterpret_cast<uint4*>(yb + 4096 * par + 256 * nt) = make_uint4(u[0], u[1], u[2], u[3]);
        }
    }
  };

  // ---- stage 3 (wave w, Y slot tl of a region): Y -> y rows staged in the slot and
  // stored as 1 KiB buffer stores; bcfft_dm8.hip's stage 3. tok < 0: nothing is stored.
  auto stage3 = [&](char* region, int tl, int rref, int64_t tok) {
    if constexpr ((ABL & 8) != 0) return;
    // SPL: a real token's partial y goes to ws in fp32 straight from registers (4 consecutive
    // columns per lane and store); tok < 0 keeps the staged path (8 dropped stores), whose count
    // the first stage 2's hand-counted wait relies on
    const bool part = SPL && tok >= 0;
    float* wsp = SPL ? ws + ((int64_t)slice * n_tokens + (tok >= 0 ? tok : 0)) * M + (int64_t)grp_o * NOG * B : nullptr;
    const int l = opaque(lane);
    const int o16 = l & 15, g = l >> 4;
    char* slot = region + tl * YSLOT;
    float ysc[NT];                                  // output block o = 16 nt + o16: 1 / s_o
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) ysc[nt] = __builtin_ldexpf(reinterpret_cast<const float*>(lds + G::OS_OFF)[16 * nt + o16], 30 - rref);
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
    f16x8 gcur[2][2], gnxt[2][2];
    gload(0, gcur);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // Y is in registers: the slot is free
    const bool tok_ok = tok >= 0 && tok < n_tokens;
    const int nvalid = n_out - grp_o * NOG;
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
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          E[nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(gcur[ks][0], __builtin_bit_cast(f16x8, yf[ks][0][nt]), E[nt], 0, 0, 0);
          O[nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(gcur[ks][1], __builtin_bit_cast(f16x8, yf[ks][1][nt]), O[nt], 0, 0, 0);
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
          if (part) {
            if (tok_ok && o < nvalid)
              *reinterpret_cast<float4*>(wsp + o * B + 16 * mt + 4 * g + 64 * hf) = make_float4(v[0], v[1], v[2], v[3]);
            continue;
          }
          if (HB) {                                 // .to(x dtype) :266, + bias :270-271
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
      if (mt < 3) {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int pr = 0; pr < 2; ++pr) gcur[ks][pr] = gnxt[ks][pr];
      }
    }
    if (part) return;
    constexpr int RB = B * ESY;
    const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
        (char*)yv + (tok_ok ? tok : 0) * M * ESY + (int64_t)grp_o * NOG * RB, 0,
        tok_ok ? (int)((M - (int64_t)grp_o * NOG * B) * ESY) : 0, 0x00020000);
    const int w = l & 15, lr = l >> 4;
    const int vofs = lr * RB + 16 * w;
    int rdb[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) rdb[c] = lr * RB + 16 * ((w ^ lr) ^ (4 * c));
    uint4 d[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      uint4 v = *reinterpret_cast<const uint4*>(slot + 1024 * q + rdb[q & 1]);
      if (q & 2) v = make_uint4(v.z, v.w, v.x, v.y);
      d[q] = v;
    }
#pragma unroll
    for (int q = 0; q < 8; ++q)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, d[q]), yrs, vofs + q * 1024, 0, BCFFT_YAUX);
  };

  // ---- prologue: the first tile's chunk 0, the DFT table
  u32x4 breg[BPW][NT];
  dma_chunk(wg_in_grp, c0, lds);
  {
    const uint4* tab = reinterpret_cast<const uint4*>(kDmF);
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int c = tid + 512 * r;                  // chunk c: row c >> 4, chunk c & 15
      const int t = c >> 4, ch = c & 15;
      *reinterpret_cast<uint4*>(lds + F_OFF + 256 * t + 16 * (ch ^ fsw(t))) = tab[c];
    }
  }
  // the group's inverse weight scales 1 / s_o (per output block) -> LDS
  if (tid < 32) reinterpret_cast<float*>(lds + G::OS_OFF)[tid] = osc[grp_o * 32 + tid];
  wait_vmcnt<0>();
  lds_barrier();
  STAMP(0);

  // Pipeline per M-tile m of 16 tokens (region r holds its chunk 0; the other region the
  // previous tile's Y units of tokens 8-15), two barriers per chunk step:
  //   step 0   B(0); stage 1; stage 3 of the previous tile's deferred token         | Ba |
  //            DMA x(1) into the other region; stage 2 on B(0), loading B(1)        | Bb |
  //   step c   DMA x(c + 1) (or the next tile's chunk 0) into the other region,
  //            stage 1                                                              | Ba |
  //            stage 2 on B(c), loading B(c + 1) unless c is the last chunk         | Bb |
  //   end      Y(tokens 0-7) into the last region | Bc | stage 3 of token w           | Bd |
  //            Y(tokens 8-15)                                                       | Be |
  // Every wave streams and transforms its own two tokens, so x needs no barrier of its own.
  // VMEM order is x DMA of step c, then the B loads for step c + 1, so the compiler's waits on
  // B (it does not see the asm DMA) drain at most that one DMA, a stage 1 after its issue.
  int rsel = 0;
  int64_t mprev = -1;
  constexpr int LH = MT - 1;                        // the half tile whose stage 3 is deferred
  int tix = 0;                                      // stamps builds: tiles 0 and 1 are timed
  for (int64_t m = wg_in_grp; m < n_mtiles; m += gstride, ++tix) {
    const int sb = 1 + 30 * tix;
#define DSTAMP(o) do { if (tix < 2) STAMP(sb + (o)); } while (0)
    // ---- step 0
    {
      char* region = lds + rsel * REGION;
      char* other = lds + (rsel ^ 1) * REGION;
      DSTAMP(0);
      load_b(c0, 0, breg);                          // B(c0): issued here, not carried across the
      load_b(c0, 1, breg);                          // tile end (the accumulators are dead now)
      wait_vmcnt<16 + 8 * (MT - 1)>();              // x(0): older than B(0) and a half tile's stores
      // stage 1 of this tile and the deferred stage 3 of the previous one touch different
      // regions: one barrier for both, and the scheduler may interleave them
      stage1(region);
      DSTAMP(1);
      stage3(other, wave, wrr[8 * LH + wave], mprev >= 0 ? mprev * TT + 8 * LH + wave : -1);
      DSTAMP(3);
      lds_barrier();                                // B0 + Ba: X(0) complete, the other region free
      DSTAMP(4);
      if (c0 + 1 < c1) dma_chunk(m, c0 + 1, other);
      else dma_chunk(m + gstride, c0, other);       // one chunk: the next tile's first (or nothing)
      stage2(region, breg, c0 + 1 < c1 ? c0 + 1 : -1, std::true_type{});
      DSTAMP(5);
      lds_barrier();                                // Bb
      DSTAMP(6);
      rsel ^= 1;
    }
    // ---- steps 1 .. nch - 1
    for (int c = c0 + 1; c < c1; ++c) {
      char* region = lds + rsel * REGION;
      char* other = lds + (rsel ^ 1) * REGION;
      wait_vmcnt<16>();                             // x(c) (older than B(c))
#ifdef BCFFT_DMK_LATE_DMA
      // analysis build: the younger waves 4-7 issue this step's x DMA after
      // their stage 1 instead of before it (round 5's failing variant, re-created)
      const bool late = wave >= 4;
      if (!late) {
        if (c + 1 < c1) dma_chunk(m, c + 1, other);
        else dma_chunk(m + gstride, c0, other);
      }
      stage1(region);
      if (late) {
        if (c + 1 < c1) dma_chunk(m, c + 1, other);
        else dma_chunk(m + gstride, c0, other);
#if BCFFT_DMK_LATE_DMA == 2
        wait_vmcnt<0>();                            // bisection: the late DMA landed before Ba
#endif
      }
#else
      if (c + 1 < c1) dma_chunk(m, c + 1, other);
      else dma_chunk(m + gstride, c0, other);       // zero-filled past the last tile
      stage1(region);
#endif
      if (c <= 5) DSTAMP(7 + 3 * (c - 1));
      lds_barrier();                                // Ba
      if (c <= 5) DSTAMP(8 + 3 * (c - 1));
      stage2(region, breg, c + 1 < c1 ? c + 1 : -1, std::false_type{});
      lds_barrier();                                // Bb
      if (c <= 5) DSTAMP(9 + 3 * (c - 1));
      rsel ^= 1;
    }
    // ---- tile end: the last chunk's region takes the Y units, 8 tokens at a time
    char* last = lds + (rsel ^ 1) * REGION;
    if constexpr (MT == 2) {
      ywrite(last, std::integral_constant<int, 0>{});
      lds_barrier();                                // Bc
      DSTAMP(22);
      stage3(last, wave, wrr[wave], m * TT + wave);
      DSTAMP(23);
      lds_barrier();                                // Bd: staging reads of tokens 0-7 done
      DSTAMP(24);
    }
    ywrite(last, std::integral_constant<int, LH>{});
    lds_barrier();                                  // Be
    DSTAMP(25);
#undef DSTAMP
    mprev = m;
  }
  // ---- epilogue: the last tile's deferred half
  stage3(lds + (rsel ^ 1) * REGION, wave, wrr[8 * LH + wave], mprev * TT + 8 * LH + wave);
  STAMP(63);
}

// one thread per (group, chunk, wave, bin, N-tile, lane) 16-B fragment: 4 input blocks x
// (re, im) fp16 of conj(S) * s_o (bin 0: (S_0, S_H) * s_o), zero outside the operator
__global__ void bc_dmk_image_kernel(int n_out, int n_in, float2* __restrict__ spec) {
  using namespace dmk;
  constexpr int H = B / 2;
  const SpecLayout sl = spec_layout(n_out, n_in, B);
  const int nch = (n_in + 15) / 16;
  const int64_t total = (int64_t)sl.stat_groups * sl.stat_pieces * 64;
  uint32_t* hdr = reinterpret_cast<uint32_t*>(spec) + sl.stat_off_u32;
  uint4* img = reinterpret_cast<uint4*>(hdr + 4);
  const uint32_t* osc = reinterpret_cast<const uint32_t*>(spec) + sl.osc_off_u32;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int lane = (int)(idx & 63);
    const int64_t rest = idx >> 6;
    const int nt = (int)(rest % NT);
    const int fb = (int)((rest / NT) % BPW);
    const int w = (int)((rest / FRAGS) % NW);
    const int c = (int)((rest / (FRAGS * NW)) % nch);
    const int gq = (int)(rest / (FRAGS * NW) / nch);
    const int f = w * BPW + fb;
    const int o = gq * NOG + nt * 16 + (lane & 15);
    const float sc = __uint_as_float((254u << 23) - osc[o]);   // s_o = 1 / osc[o] (powers of two)
    const int i0 = c * 16 + 4 * (lane >> 4);
    uint32_t d[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int i = i0 + e;
      float2 cv = make_float2(0.f, 0.f);
      if (o < n_out && i < n_in) {
        cv = spec[((int64_t)o * n_in + i) * H + f];
        if (f != 0) cv.y = -cv.y;
      }
      const f16x2 h = {(_Float16)(cv.x * sc), (_Float16)(cv.y * sc)};
      d[e] = __builtin_bit_cast(uint32_t, h);
    }
    img[idx] = make_uint4(d[0], d[1], d[2], d[3]);
  }
}

bool dmk_eligible(int n_in, int b, int xdt, bool yf32) {
  // dmk_geometry caps n_in at 127: Y = acc 2^-21 stays below fp16's max (n_in 2^30 2^-21 < 65504)
  return dmk_geometry(n_in, b) && xdt == BCFFT_BF16 && !yf32;
}

void launch_forward_dmk(const void* x, int64_t n, int n_in, int n_out, const void* spec, const void* bias,
                        int bias_dt, void* y, hipStream_t s) {
  const int groups = (n_out + dmk::NOG - 1) / dmk::NOG;
  const SpecLayout sl = spec_layout(n_out, n_in, 128);
  const int64_t cus = device_cu_count();
  const uint32_t* stat = reinterpret_cast<const uint32_t*>(spec) + sl.stat_off_u32;
  const float* osc = reinterpret_cast<const float*>(spec) + sl.osc_off_u32;
  // A tile is a serial chain of chunk steps: the launch takes about (tiles per CU, rounded up)
  // x the tile time, ~21.7 us for 8 tokens and ~39.7 us for 16 at nI = 86 (16-token tiles
  // halve the weight stream per token). The smaller makespan wins; this model picks the faster
  // size at every measured N (profiles/r02_ab_dmk_tile_switch.log: 16 at N = 3000 and 4096, 8
  // at 5000 and 6144, 16 at 8192, 8 at 1700).
  const int64_t waves8 = (groups * ((n + 7) / 8) + cus - 1) / cus;
  const int64_t waves16 = (groups * ((n + 15) / 16) + cus - 1) / cus;
  const bool t16 = waves16 * 40 < waves8 * 22;
  const int64_t n_mtiles = t16 ? (n + 15) / 16 : (n + 7) / 8;
  const int64_t total = group_grid(cus, groups, n_mtiles);
  const bool hb = bias_dt != BCFFT_NONE;
  if (t16 && hb)
    hipLaunchKernelGGL((bc_forward_dmk_kernel<16, false, true>), dim3((unsigned)total), dim3(512), 0, s, x, n, n_in,
                       n_out, stat, osc, bias, bias_dt, y, 1, nullptr);
  else if (t16)
    hipLaunchKernelGGL((bc_forward_dmk_kernel<16, false, false>), dim3((unsigned)total), dim3(512), 0, s, x, n, n_in,
                       n_out, stat, osc, bias, bias_dt, y, 1, nullptr);
  else if (hb)
    hipLaunchKernelGGL((bc_forward_dmk_kernel<8, false, true>), dim3((unsigned)total), dim3(512), 0, s, x, n, n_in,
                       n_out, stat, osc, bias, bias_dt, y, 1, nullptr);
  else
    hipLaunchKernelGGL((bc_forward_dmk_kernel<8, false, false>), dim3((unsigned)total), dim3(512), 0, s, x, n, n_in,
                       n_out, stat, osc, bias, bias_dt, y, 1, nullptr);
}

// the split form's finishing pass: y = (sum over the kz slices in order, rounded to bf16) + bias,
// rounded (the unsplit kernel's epilogue: .to(x dtype) :266, + bias :270-271); 4 columns a thread
__global__ void bc_dmk_finish_kernel(const float* __restrict__ ws, int kz, int64_t n_tokens, int64_t M,
                                     const void* __restrict__ bias, int bias_dt, uint16_t* __restrict__ y) {
  const int64_t quads = n_tokens * M / 4;
  const int64_t slab = n_tokens * M;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < quads; q += (int64_t)gridDim.x * blockDim.x) {
    float4 a = reinterpret_cast<const float4*>(ws)[q];
    for (int z = 1; z < kz; ++z) {
      const float4 b = reinterpret_cast<const float4*>(ws + z * slab)[q];
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
    float v[4] = {a.x, a.y, a.z, a.w};
    if (bias_dt != BCFFT_NONE) {
      const int64_t col = (q * 4) % M;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = round_to(v[r], BCFFT_BF16) + load_scalar(bias, col + r, bias_dt);
    }
    reinterpret_cast<uint2*>(y)[q] = make_uint2(pack16<BCFFT_BF16>(v[0], v[1]), pack16<BCFFT_BF16>(v[2], v[3]));
  }
}

// K-chunk slices of the split form: only where the unsplit grid leaves almost every CU idle (at
// most 1/16 of the CUs' worth of (group, 8-token tile) pairs), as many slices as fill the CUs,
// >= 1 chunk each. Measured at 11008 -> 4096 (profiles/r03l_dmk_split.log, 256 CUs): N = 1 11.9 vs
// 20.9 us unsplit, N = 20 15.2 vs 21.1, N = 128 20.2 vs 21.4; N = 256 24.6 vs 21.7 (the fp32
// partials and the finishing pass grow with N)
int dmk_ksplit(int64_t n, int n_in, int n_out) {
  const int64_t units = (n + 7) / 8 * ((n_out + dmk::NOG - 1) / dmk::NOG);
  const int64_t cus = device_cu_count();
  const int nch = (n_in + 15) / 16;
  if (n <= 0 || units * 16 > cus) return 1;
  int kz = (int)std::min<int64_t>(nch, cus / units);
  if (kz < 2) return 1;
  const int cps = (nch + kz - 1) / kz;
  return (nch + cps - 1) / cps;                     // every slice non-empty
}

void launch_forward_dmk_split(const void* x, int64_t n, int n_in, int n_out, const void* spec, const void* bias,
                              int bias_dt, void* y, float* ws, int kz, hipStream_t s) {
  const int groups = (n_out + dmk::NOG - 1) / dmk::NOG;
  const SpecLayout sl = spec_layout(n_out, n_in, 128);
  const uint32_t* stat = reinterpret_cast<const uint32_t*>(spec) + sl.stat_off_u32;
  const float* osc = reinterpret_cast<const float*>(spec) + sl.osc_off_u32;
  const int64_t total = (int64_t)kz * groups * ((n + 7) / 8);
  hipLaunchKernelGGL((bc_forward_dmk_kernel<8, true>), dim3((unsigned)total), dim3(512), 0, s, x, n, n_in, n_out, stat,
                     osc, nullptr, BCFFT_NONE, y, kz, ws);
  launch_partials_finish(ws, kz, n, (int64_t)n_out * 128, bias, bias_dt, y, s);
}

void launch_partials_finish(const float* ws, int kz, int64_t n, int64_t M, const void* bias, int bias_dt, void* y,
                            hipStream_t s) {
  const int64_t quads = n * M / 4;
  const unsigned blocks = (unsigned)((quads + 255) / 256 < 4096 ? (quads + 255) / 256 : 4096);
  hipLaunchKernelGGL(bc_dmk_finish_kernel, dim3(blocks), dim3(256), 0, s, ws, kz, n, M, bias, bias_dt, (uint16_t*)y);
}

void launch_dmk_image(int n_out, int n_in, void* spec, hipStream_t s) {
  const SpecLayout sl = spec_layout(n_out, n_in, 128);
  const int64_t total = (int64_t)sl.stat_groups * sl.stat_pieces * 64;
  const unsigned blocks = (unsigned)((total + 255) / 256 < 65535 ? (total + 255) / 256 : 65535);
  hipLaunchKernelGGL(bc_dmk_image_kernel, dim3(blocks), dim3(256), 0, s, n_out, n_in, (float2*)spec);
}

}  // namespace bcfft

// analysis build only: stamp buffer of bc_forward_dmk_kernel (this TU's copy). Slots per wave: 0
// start | per tile t < 2 (base 1 + 30 t): +0 step 0 top, +1 stage 3 done, +2 after B0, +3 stage 1
// done, +4 after Ba, +5 stage 2 done, +6 after Bb; step c in 1..5: +7 + 3 (c - 1) stage 1 done,
// +8 ... after Ba, +9 ... after Bb | 16-token tiles: +22 after Bc, +23 stage 3 done, +24 after Bd |
// +25 after Be | 63 end (tools/timeline_dmk.py)
BCFFT_STAMPS_SETTER(dmk)
