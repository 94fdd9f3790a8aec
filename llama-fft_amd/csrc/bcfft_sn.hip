// bcfft_sn.hip — the block-circulant forward for short token counts (decode steps, small
// batches; BASELINE config 1: 4096 -> 4096, b = 64, N = 128, fp32) on the matrix cores (gfx950).
//
// BlockCirculantLinear.forward (patch_llama_fft.py:226-275) with the DFT-on-MFMA arithmetic of
// bc_forward_dm_kernel (b = 128) / bc_forward_dm64_kernel (b = 64): even/odd split
// a_t = x_t + x_{t+b/2}, d_t = x_t - x_{t+b/2}; X = [a Fe | d Fo] with the fp16 table
// (bcfft_dm_table.h, times 2^-7); the per-bin complex MAC against the STAT image's fp16
// conj(C) s_o fragments; the inverse as the transposed table product, y_t = E_t + O_t,
// y_{t+b/2} = E_t - O_t. Numerics are the exact (dftx) variant for every dtype: a, d, X and Y
// are fp16 hi + lo, fp32 accumulation, per-(token, 16-block chunk) power-of-two scales aligned to
// the token's smallest exponent in the MAC, one scale per output block (tests/dm_model.py,
// exact=True, restates it).
//
// What differs is the work split. The persistent kernels hold an output group's weights in VGPRs
// and stream token tiles through one workgroup per CU, so a launch of N tokens fills only
// ceil(N / 4) x groups CUs and runs the three stages of one tile back to back: config 1's
// stationary kernel used 64 of 256 CUs for a ~13 k-cycle chain. Here one workgroup takes ONE
// tile of TT tokens and ONE 16-wide N-tile of output blocks (half a STAT group), loads that
// N-tile's fragments once (64 VGPRs per lane: the weights are used by TT tokens only, so nothing
// is kept across tiles), and exits: ceil(N / TT) x ceil(n_out / 16) workgroups, each a short
// chain (x LDS-DMA and fragment loads in flight together; stage 1 over all 8 waves; barrier;
// stage 2; barrier; stage 3 with direct stores).
//
// LDS: x rows (TT tokens, DMA'd with a per-row unit swizzle) whose space the Y image reuses after
// stage 1, the X image (hi/lo units, token stride padded by 128 B so the stage-2 reads of 4
// tokens are conflict-free), the table image (as the dm kernels lay it out), the scales.
#include "bcfft_device.h"
#include "bcfft_dm_table.h"
#include "bcfft_dm_common.h"

namespace bcfft {

namespace sn {
using namespace dmh;
constexpr int NW = 8;

template <int B, int KS, int TT, int ES>
struct Geo {
  static constexpr int H = B / 2;                  // packed bins
  static constexpr int TQ = B / 2;                 // a / d length
  static constexpr int TK = TQ / 32;               // stage-1 K-steps over t; stage-3 K-steps per parity
  static constexpr int MT = TQ / 16;               // stage-1 M-tiles per parity; stage-3 t-tiles
  static constexpr int BW = H / NW;                // stage-2 bins per wave
  static constexpr int NI = 16 * KS;               // input blocks
  static constexpr int K = NI * B;
  static constexpr int RB = B * ES;                // x row bytes
  static constexpr int UPR = RB / 16;              // 16-B units per x row
  static constexpr int SWM = (UPR < 16 ? UPR : 16) - 1;   // x unit swizzle mask
  static constexpr int RPP = 1024 / RB;            // x rows per 1-KiB DMA piece
  static constexpr int PT = K * ES / 1024;         // DMA pieces per token
  static constexpr int XTOK = KS * H * 128;        // X image bytes per token: (chunk, bin, prec, quad) x 16 B
  static constexpr int TSX = XTOK + 128;           // ... padded (bank shift for odd tokens)
  static constexpr int JG = H / 8;                 // 4-bin groups per parity
  static constexpr int TSY = 2 * 2 * JG * 16 * 16; // Y image bytes per token: (prec, parity, group, o) x 16 B
  static constexpr int XS_BYTES = TT * K * ES > TT * TSY ? TT * K * ES : TT * TSY;
  static constexpr int XS_OFF = 0;                 // x rows, later the Y image
  static constexpr int XI_OFF = XS_BYTES;
  static constexpr int F_OFF = XI_OFF + TT * TSX;  // table image (256-B aligned below)
  static constexpr int TROW = 2 * B;               // table row bytes: [even TQ | odd TQ] fp16
  static constexpr int SC_OFF = F_OFF + TQ * TROW; // scale exponents [TT][KS]
  static constexpr int OS_OFF = SC_OFF + TT * KS * 4;   // the N-tile's 16 inverse weight scales
  static constexpr int LDS_BYTES = OS_OFF + 64;
  static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
  static_assert(XI_OFF % 256 == 0 && F_OFF % 256 == 0, "bank-period alignment");
  static_assert(PT * TT % NW == 0, "whole DMA pieces per wave");
  static constexpr int NFRAG = BW * KS;            // 16-B weight fragment loads per lane
  static_assert(NFRAG < 64, "vmcnt range");
  static constexpr int UPW1 = (TT * KS + NW - 1) / NW;   // stage-1 units per wave (TT = 2: some waves idle)
  static constexpr int UPW3 = (TT * MT + NW - 1) / NW;   // stage-3 units per wave
};
}  // namespace sn

// One workgroup: token tile `tile` (TT tokens from tile * TT), output N-tile `og` (blocks
// 16 og .. 16 og + 15 = STAT group og / 2, N-tile og % 2). XT: x dtype; y = promote(x, bias).
template <int B, int KS, int TT, int XT, bool YF32>
__global__ __launch_bounds__(512, 2) void bc_forward_sn_kernel(
    const void* __restrict__ xv, int64_t n_tokens, int n_out, const uint32_t* __restrict__ stat,
    const float* __restrict__ osc, const void* __restrict__ bias, int bias_dt, void* __restrict__ yv) {
  using namespace sn;
  constexpr int ES = XTraits<XT>::ES;
  using G = Geo<B, KS, TT, ES>;
  constexpr int H = G::H, TQ = G::TQ, TK = G::TK, MT = G::MT, BW = G::BW, K = G::K, RB = G::RB;
  constexpr bool Y32 = YF32 || XT == BCFFT_F32;
  constexpr int ESY = Y32 ? 4 : 2;
  ANALYSIS_INIT;
  STAMP(0);
  __shared__ __attribute__((aligned(16))) char lds[G::LDS_BYTES];
  int* wsc = reinterpret_cast<int*>(lds + G::SC_OFF);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n_og = (n_out + 15) >> 4;
  const int og = (int)(blockIdx.x % (unsigned)n_og);
  const int64_t tile = blockIdx.x / (unsigned)n_og;
  const int grp = og >> 1, nt = og & 1;
  const int64_t tok0 = tile * TT;
  const int64_t M = (int64_t)n_out * B;
  const uint32_t lds_base = __builtin_amdgcn_readfirstlane(lds_addr(lds));

  // ---- x rows of the tile -> LDS by LDS-DMA (1-KiB pieces, PT per token; tokens past n_tokens
  // read as zeros through an empty buffer range). A piece's LDS bytes are lane-linear, so the
  // unit swizzle (source unit u of row r at LDS unit u ^ (r & SWM)) goes into the source offsets.
  {
    constexpr int PPW = G::PT * TT / NW;
    const int dl = opaque(lane);
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int pc = wave * PPW + i;                // piece of the tile
      const int tk = pc / G::PT, pq = pc % G::PT;
      const int64_t tok = tok0 + tk;
      const bool ok = tok < n_tokens;
      // wave-uniform by construction; readfirstlane keeps the descriptor in SGPRs in every build
      const uint64_t base = (uint64_t)(uintptr_t)((const char*)xv + (ok ? tok : 0) * K * ES);
      const uint32_t blo = __builtin_amdgcn_readfirstlane((uint32_t)base), bhi = __builtin_amdgcn_readfirstlane((uint32_t)(base >> 32));
      const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(uintptr_t)(((uint64_t)bhi << 32) | blo), 0, __builtin_amdgcn_readfirstlane(ok ? K * ES : 0), 0x00020000);
      const int r = pq * G::RPP + dl / G::UPR, p = dl % G::UPR;
      const int voff = r * RB + 16 * (p ^ (r & G::SWM));
      const uint32_t dst = __builtin_amdgcn_readfirstlane(lds_base + G::XS_OFF + tk * K * ES + pq * 1024);
      uint32_t keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep) : "v"(voff), "s"(xrs), "s"(dst) : "memory");
    }
  }
  STAMP(1);
  // ---- the DFT table image (the dm kernels' swizzle), the N-tile's inverse weight scales
  if constexpr (B == 128) {
    const uint4* tab = reinterpret_cast<const uint4*>(kDmF);
#pragma unroll
    for (int r = 0; r < 2; ++r) {                   // chunk c: row c >> 4, chunk c & 15
      const int c = tid + 512 * r, t = c >> 4, ch = c & 15;
      *reinterpret_cast<uint4*>(lds + G::F_OFF + 256 * t + 16 * (ch ^ fsw(t))) = tab[c];
    }
  } else {
    if (tid < 256) {                                // chunk c: row c >> 3, chunk c & 7
      const uint4* tab = reinterpret_cast<const uint4*>(kDmF64);
      const int t = tid >> 3, ch = tid & 7;
      const int sw = (((t >> 1) & 1) << 1) | (((t >> 3) & 1) << 2);
      *reinterpret_cast<uint4*>(lds + G::F_OFF + 128 * t + 16 * (ch ^ sw)) = tab[tid];
    }
  }
  if (tid < 16) reinterpret_cast<float*>(lds + G::OS_OFF)[tid] = osc[grp * 32 + 16 * nt + tid];
  // the weight fragments are issued last and first needed in stage 2: their L2 / HBM latency runs
  // under stage 1. The table's LDS writes above waited for its loads, i.e. (in issue order) for the
  // x DMA too; the explicit wait covers the tokens whose table share the compiler did not count.
  // ---- the N-tile's weight fragments: wave w's bins w BW .. + BW - 1, all chunks (64 VGPRs)
  f16x8 creg[BW][KS];
  {
    constexpr int NPIECE = BW * KS * 2;
    const uint4* img = reinterpret_cast<const uint4*>(stat + 4) + ((int64_t)(grp * NW + wave) * NPIECE) * 64 + lane;
#pragma unroll
    for (int fb = 0; fb < BW; ++fb)
#pragma unroll
      for (int c = 0; c < KS; ++c) creg[fb][c] = __builtin_bit_cast(f16x8, img[((fb * KS + c) * 2 + nt) * 64]);
  }
  STAMP(2);
  wait_vmcnt<G::NFRAG>();                           // x DMA and table loads (not the fragments)
  STAMP(3);
  lds_barrier();
  STAMP(4);

  // ---- stage 1: units (token tk, chunk c of 16 input blocks); x -> X hi / lo units
#pragma unroll
  for (int iu = 0; iu < G::UPW1; ++iu) {
    const int u = wave + NW * iu;
    if (u >= TT * KS) break;                        // wave-uniform
    const int tk = u / KS, c = u % KS;
    const int l = opaque(lane);
    const int b16 = l & 15, g = l >> 4;
    const int r = 16 * c + b16;                     // the lane's input block (B operand column)
    const char* row = lds + G::XS_OFF + tk * K * ES + r * RB;
    // x_t and x_{t+TQ} for t = 32 k + 8 g + j (j < 8) of each t-step k
    float xa[TK][2][8];
#pragma unroll
    for (int k = 0; k < TK; ++k)
#pragma unroll
      for (int pt = 0; pt < 2; ++pt) {
        const int t0 = 32 * k + 8 * g + TQ * pt;
        if constexpr (ES == 4) {
          const int us = t0 / 4;
          const float4 v0 = *reinterpret_cast<const float4*>(row + 16 * (us ^ (r & G::SWM)));
          const float4 v1 = *reinterpret_cast<const float4*>(row + 16 * ((us + 1) ^ (r & G::SWM)));
          xa[k][pt][0] = v0.x; xa[k][pt][1] = v0.y; xa[k][pt][2] = v0.z; xa[k][pt][3] = v0.w;
          xa[k][pt][4] = v1.x; xa[k][pt][5] = v1.y; xa[k][pt][6] = v1.z; xa[k][pt][7] = v1.w;
        } else {
          const int us = t0 / 8;
          const uint4 w = *reinterpret_cast<const uint4*>(row + 16 * (us ^ (r & G::SWM)));
          const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float2 f = unpack16<XT>(ww[e]);
            xa[k][pt][2 * e] = f.x;
            xa[k][pt][2 * e + 1] = f.y;
          }
        }
      }
    float m0 = 0.f, m1 = 0.f;
#pragma unroll
    for (int k = 0; k < TK; ++k)
#pragma unroll
      for (int pt = 0; pt < 2; ++pt)
#pragma unroll
        for (int j = 0; j < 8; j += 4) {
          m0 = amax3(m0, xa[k][pt][j], xa[k][pt][j + 1]);
          m1 = amax3(m1, xa[k][pt][j + 2], xa[k][pt][j + 3]);
        }
    const int sx = stat_scale_exp(2.f * __uint_as_float(wave_umax(__float_as_uint(__builtin_fmaxf(m0, m1)))));
    if (l == 0) wsc[tk * KS + c] = sx - 7;           // X = D 2^-(sx - 7): the table's 2^-7
    const float S = __int_as_float((sx + 127) << 23);
    // transposed table reads (A = F^T: 16 bin-reals x 32 t), the dm / dm64 kernels' addressing
    const int q4 = (l & 15) >> 2, p4 = l & 3;
    f32x4 acc[2 * MT];
#pragma unroll
    for (int i = 0; i < 2 * MT; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < TK; ++k) {
      uint32_t ah[4], al[4], dh[4], dlo[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float u0 = xa[k][1][2 * e] * S, u1 = xa[k][1][2 * e + 1] * S;
        split2(fmaf(xa[k][0][2 * e], S, u0), fmaf(xa[k][0][2 * e + 1], S, u1), ah[e], al[e]);
        split2(fmaf(xa[k][0][2 * e], S, -u0), fmaf(xa[k][0][2 * e + 1], S, -u1), dh[e], dlo[e]);
      }
      const f16x8 bah = frag(ah[0], ah[1], ah[2], ah[3]), bal = frag(al[0], al[1], al[2], al[3]);
      const f16x8 bdh = frag(dh[0], dh[1], dh[2], dh[3]), bdl = frag(dlo[0], dlo[1], dlo[2], dlo[3]);
#pragma unroll
      for (int pr = 0; pr < 2; ++pr)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          f16x8 af;
          if constexpr (B == 128) {
            const int cx = (p4 >> 1) ^ fsw(8 * g + q4);
            const char* p0 = lds + G::F_OFF + 256 * (8 * g + q4) + 8 * (p4 & 1) + 256 * 32 * k + 16 * ((8 * pr + 2 * mt) ^ cx);
            const s16x4 r0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p0));
            const s16x4 r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p0 + 256 * 4));
            af = __builtin_bit_cast(f16x8, __builtin_shufflevector(r0, r1, 0, 1, 2, 3, 4, 5, 6, 7));
          } else {
            const int r0 = 8 * g + q4, r1 = r0 + 4;
            const int sw0 = (((r0 >> 1) & 1) << 1) | (((r0 >> 3) & 1) << 2);
            const int sw1 = (((r1 >> 1) & 1) << 1) | (((r1 >> 3) & 1) << 2);
            const int cc = 4 * pr + 2 * mt;
            const s16x4 ra = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(
                lds + G::F_OFF + 128 * r0 + 8 * (p4 & 1) + 16 * (cc ^ ((p4 >> 1) ^ sw0))));
            const s16x4 rb = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(
                lds + G::F_OFF + 128 * r1 + 8 * (p4 & 1) + 16 * (cc ^ ((p4 >> 1) ^ sw1))));
            af = __builtin_bit_cast(f16x8, __builtin_shufflevector(ra, rb, 0, 1, 2, 3, 4, 5, 6, 7));
          }
          acc[MT * pr + mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, pr ? bdh : bah, acc[MT * pr + mt], 0, 0, 0);
          acc[MT * pr + mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, pr ? bdl : bal, acc[MT * pr + mt], 0, 0, 0);
        }
    }
    // D^T tile (pr, mt): lane rows 4 g + r are the (re, im) of bins fA = 16 mt + 4 g + pr (r < 2)
    // and fA + 2 (r >= 2) of block b16: X unit ((c H + f) 2 + prec) x 64 B + 16 (b16 >> 2), 4 B at b16 & 3
    char* xi = lds + G::XI_OFF + tk * G::TSX + 4 * b16;
#pragma unroll
    for (int pr = 0; pr < 2; ++pr)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int fA = 16 * mt + 4 * g + pr;
        uint32_t hA, lA, hB, lB;
        split2(acc[MT * pr + mt][0], acc[MT * pr + mt][1], hA, lA);
        split2(acc[MT * pr + mt][2], acc[MT * pr + mt][3], hB, lB);
        char* ua = xi + ((c * H + fA) * 2) * 64;
        char* ub = xi + ((c * H + fA + 2) * 2) * 64;
        *reinterpret_cast<uint32_t*>(ua) = hA;
        *reinterpret_cast<uint32_t*>(ua + 64) = lA;
        *reinterpret_cast<uint32_t*>(ub) = hB;
        *reinterpret_cast<uint32_t*>(ub + 64) = lB;
      }
  }
  STAMP(5);
  lds_barrier();                                    // X units and scales complete; x rows free
  STAMP(6);

  // ---- stage 2 (wave w: bins w BW .. + BW - 1): MFMA rows (token, re/im, hi/lo), K = 16 blocks
  // x (re, im) per chunk, one N-tile; Y hi / lo into the Y image over the x rows
  {
    const int ml = opaque(lane);
    const int arow = ml & 15, kb = ml >> 4;
    const int a_t = arow >> 2, a_reim = (arow >> 1) & 1, a_prec = arow & 1;
    const int at = a_t < TT ? a_t : TT - 1;          // TT = 2: rows of tokens 2, 3 repeat token 1 (discarded)
    const uint32_t a_sel = a_reim ? 0x01000302u : 0x03020100u;
    int nk[KS];
#pragma unroll
    for (int c = 0; c < KS; ++c) nk[c] = wsc[at * KS + c];
    int nmin = nk[0];
#pragma unroll
    for (int c = 1; c < KS; ++c) nmin = min(nmin, nk[c]);
    uint32_t amul[KS], amul0[KS];
#pragma unroll
    for (int c = 0; c < KS; ++c) {
      const int d = nk[c] - nmin;                   // factor 2^-d (fp16; subnormal / 0 far down)
      const uint32_t hh = d <= 14 ? (uint32_t)(15 - d) << 10 : (d <= 24 ? 1u << (24 - d) : 0u);
      const int d0 = d + 1;                          // bin 0: the inverse's 1/b vs 2/b
      const uint32_t h0 = d0 <= 14 ? (uint32_t)(15 - d0) << 10 : (d0 <= 24 ? 1u << (24 - d0) : 0u);
      amul[c] = a_reim ? (hh | ((hh | 0x8000u) << 16)) : (hh | (hh << 16));
      amul0[c] = a_reim ? (h0 << 16) : h0;
    }
    const char* ab = lds + G::XI_OFF + at * G::TSX + a_prec * 64 + 16 * kb;
    const int yt = ml >> 4, o16 = ml & 15;
    char* yb = lds + G::XS_OFF + yt * G::TSY + 16 * o16;
    // the Y stores after the bin loop: a store between two bins kept the compiler from issuing
    // the next bin's A reads early (their LDS latency then sat on each bin's chain)
    uint32_t yhs[BW], yls[BW];
#pragma unroll
    for (int fb = 0; fb < BW; ++fb) {
      const int f = wave * BW + fb;
      uint4 raw[KS];
#pragma unroll
      for (int c = 0; c < KS; ++c) raw[c] = *reinterpret_cast<const uint4*>(ab + (c * H + f) * 128);
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < KS; ++c) {
        uint4 rw = raw[c];
        if (f == 0) {
          rw.x = pkmul(rw.x, amul0[c]); rw.y = pkmul(rw.y, amul0[c]);
          rw.z = pkmul(rw.z, amul0[c]); rw.w = pkmul(rw.w, amul0[c]);
        } else {
          rw.x = pkmul(__builtin_amdgcn_perm(rw.x, rw.x, a_sel), amul[c]);
          rw.y = pkmul(__builtin_amdgcn_perm(rw.y, rw.y, a_sel), amul[c]);
          rw.z = pkmul(__builtin_amdgcn_perm(rw.z, rw.z, a_sel), amul[c]);
          rw.w = pkmul(__builtin_amdgcn_perm(rw.w, rw.w, a_sel), amul[c]);
        }
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, rw), creg[fb][c], acc, 0, 0, 0);
      }
      constexpr float YS = 1.f / 2097152.f;          // 2^-21: |Y| < 2^14 in fp16
      // rows 4 yt + {re hi, re lo, im hi, im lo}
      split2((acc[0] + acc[1]) * YS, (acc[2] + acc[3]) * YS, yhs[fb], yls[fb]);
    }
    if (yt < TT) {                                   // Y unit (prec, parity, 4-bin group, o) + 4 B per bin
#pragma unroll
      for (int fb = 0; fb < BW; ++fb) {
        const int f = wave * BW + fb;
        const int j = f >> 1, pr = f & 1;
        char* w0 = yb + (((0 * 2 + pr) * G::JG + (j >> 2)) * 16) * 16 + 4 * (j & 3);
        char* w1 = yb + (((1 * 2 + pr) * G::JG + (j >> 2)) * 16) * 16 + 4 * (j & 3);
        *reinterpret_cast<uint32_t*>(w0) = yhs[fb];
        *reinterpret_cast<uint32_t*>(w1) = yls[fb];
      }
    }
  }
  STAMP(7);
  lds_barrier();                                    // Y units complete
  STAMP(8);

  // ---- stage 3: units (token tk, t-tile mt): E = Fe Y_even, O = Fo Y_odd on 16 t x 16 output
  // blocks; y_t = (E + O) / s_o 2^(30 - nmin), y_{t+TQ} = (E - O) ...; the reference's roundings
  // (.to(x dtype) :266, + bias :270-271) and direct 16-B (fp32) / 8-B stores
#pragma unroll
  for (int iu = 0; iu < G::UPW3; ++iu) {
    const int u = wave + NW * iu;
    if (u >= TT * MT) break;                        // wave-uniform
    const int tk = u / MT, mt = u % MT;
    const int l = opaque(lane);
    const int o16 = l & 15, g = l >> 4;
    const int t = 16 * mt + o16;                    // the lane's table row (A operand)
    const int tsw = B == 128 ? fsw(t) : ((((t >> 1) & 1) << 1) | (((t >> 3) & 1) << 2));
    f32x4 E = {0.f, 0.f, 0.f, 0.f}, O = {0.f, 0.f, 0.f, 0.f};
    const char* yb = lds + G::XS_OFF + tk * G::TSY + 16 * o16;
#pragma unroll
    for (int k = 0; k < TK; ++k)
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        const f16x8 gf = *reinterpret_cast<const f16x8*>(lds + G::F_OFF + G::TROW * t + 16 * ((TQ / 8 * pr + 4 * k + g) ^ tsw));
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const uint4 yv = *reinterpret_cast<const uint4*>(yb + (((p * 2 + pr) * G::JG + 4 * k + g) * 16) * 16);
          if (pr == 0) E = __builtin_amdgcn_mfma_f32_16x16x32_f16(gf, __builtin_bit_cast(f16x8, yv), E, 0, 0, 0);
          else O = __builtin_amdgcn_mfma_f32_16x16x32_f16(gf, __builtin_bit_cast(f16x8, yv), O, 0, 0, 0);
        }
      }
    const int* sc = wsc + tk * KS;
    int nmin = sc[0];
#pragma unroll
    for (int c = 1; c < KS; ++c) nmin = min(nmin, sc[c]);
    const int64_t tok = tok0 + tk;
    const int o = 16 * og + o16;                    // output block
    if (tok < n_tokens && o < n_out) {
      const float ysc = __builtin_ldexpf(reinterpret_cast<const float*>(lds + G::OS_OFF)[o16], 30 - nmin);
      // rows t = 16 mt + 4 g + r (and + TQ) of output block o
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = hf ? fmaf(E[r], ysc, -O[r] * ysc) : fmaf(E[r], ysc, O[r] * ysc);
        const int64_t col = (int64_t)o * B + 16 * mt + 4 * g + TQ * hf;
        store4<XT, YF32>(make_float4(v[0], v[1], v[2], v[3]), yv, tok * M + col, bias, col, bias_dt);
      }
    }
  }
  STAMP(9);
  (void)ESY;
}

}  // namespace bcfft

// analysis builds only: stamp buffer of bc_forward_sn_kernel (this TU's copy). Slots per wave: 0
// start | 1 x DMA issued | 2 table + scales written, fragments issued | 3 x and table landed |
// 4 after the prologue barrier | 5 stage 1 done | 6 after its barrier | 7 stage 2 done | 8 after
// its barrier | 9 stage 3 + stores issued
BCFFT_STAMPS_SETTER(sn)

namespace {
template <int B, int KS, int TT, int XT, bool YF32>
void launch_sn(const void* x, int64_t n, int n_out, const void* spec, const void* bias, int bias_dt, void* y,
               hipStream_t s) {
  const bcfft::SpecLayout sl = bcfft::spec_layout(n_out, 16 * KS, B);
  const int64_t tiles = (n + TT - 1) / TT;
  const int64_t total = tiles * ((n_out + 15) / 16);
  const uint32_t* stat = reinterpret_cast<const uint32_t*>(spec) + sl.stat_off_u32;
  const float* osc = reinterpret_cast<const float*>(spec) + sl.osc_off_u32;
  hipLaunchKernelGGL((bcfft::bc_forward_sn_kernel<B, KS, TT, XT, YF32>), dim3((unsigned)total), dim3(512), 0, s, x, n,
                     n_out, stat, osc, bias, bias_dt, y);
}

template <int B, int KS, int TT>
bool launch_sn_dt(int xdt, bool yf32, const void* x, int64_t n, int n_out, const void* spec, const void* bias,
                  int bias_dt, void* y, hipStream_t s) {
  if (xdt == BCFFT_F32) launch_sn<B, KS, TT, BCFFT_F32, true>(x, n, n_out, spec, bias, bias_dt, y, s);
  else if (xdt == BCFFT_BF16 && yf32) launch_sn<B, KS, TT, BCFFT_BF16, true>(x, n, n_out, spec, bias, bias_dt, y, s);
  else if (xdt == BCFFT_BF16) launch_sn<B, KS, TT, BCFFT_BF16, false>(x, n, n_out, spec, bias, bias_dt, y, s);
  else if (yf32) launch_sn<B, KS, TT, BCFFT_F16, true>(x, n, n_out, spec, bias, bias_dt, y, s);
  else launch_sn<B, KS, TT, BCFFT_F16, false>(x, n, n_out, spec, bias, bias_dt, y, s);
  return true;
}
}  // namespace

namespace bcfft {
// the short-N kernel serves the STAT image's geometries (b = 128 with K = 4096; b = 64 with
// K = 2048 or 4096), every x dtype and bias
bool sn_eligible(int n_in, int b) { return stat_eligible(n_in, b); }

bool launch_forward_sn(int b, int n_in, int xdt, bool yf32, const void* x, int64_t n, int n_out, const void* spec,
                       const void* bias, int bias_dt, void* y, hipStream_t s) {
  if (!sn_eligible(n_in, b)) return false;
  // 2-token tiles where they still fit one round of workgroups: twice the workgroups, each with
  // half the x and half the stage-1 / stage-3 work (the weight fragments per workgroup are the same)
  const bool t2 = sn_tt2(n, n_out);
  if (b == 128)
    return t2 ? launch_sn_dt<128, 2, 2>(xdt, yf32, x, n, n_out, spec, bias, bias_dt, y, s)
              : launch_sn_dt<128, 2, 4>(xdt, yf32, x, n, n_out, spec, bias, bias_dt, y, s);
  if (n_in == 64)
    return t2 ? launch_sn_dt<64, 4, 2>(xdt, yf32, x, n, n_out, spec, bias, bias_dt, y, s)
              : launch_sn_dt<64, 4, 4>(xdt, yf32, x, n, n_out, spec, bias, bias_dt, y, s);
  return t2 ? launch_sn_dt<64, 2, 2>(xdt, yf32, x, n, n_out, spec, bias, bias_dt, y, s)
            : launch_sn_dt<64, 2, 4>(xdt, yf32, x, n, n_out, spec, bias, bias_dt, y, s);
}
}  // namespace bcfft
