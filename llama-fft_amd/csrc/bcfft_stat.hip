// bcfft_stat.hip — stationary-weight block-circulant forward for gfx950 (MI355X).
//
// Same operator as bc_forward_mfma_kernel (BlockCirculantLinear.forward,
// patch_llama_fft.py:226-275), organised the other way round: the WEIGHTS stay in registers
// and the TOKENS stream.
//
//  * One persistent 512-thread workgroup per CU (8 waves, 2 per SIMD, <= 256 VGPRs). Each
//    workgroup owns one output group of 32 blocks (= 4096 outputs at b = 128). It loads that
//    group's packed weight spectra ONCE, as fp16 MFMA B fragments scaled by a power of two
//    s_C: K/32 = 128 VGPRs per lane. Wave w keeps bins [w*BW, (w+1)*BW).
//  * Tokens go through in M-tiles of 4, two 64 KiB LDS regions alternating, each cut into
//    8 KiB slots. Slot w is wave w's: its x rows arrive there by LDS-DMA (issued by wave w a
//    whole tile ahead), its forward replaces them in place by its A fragments, and after the
//    MFMAs the slot holds the Y units of the inverse rows wave w transforms and stores. Two
//    workgroup barriers per M-tile:
//      P1  inverse of the previous tile, its y stores, the next tile's DMA, then the forward:
//          one row (token, input block) per L = b/32 lanes, 16 complex points per lane: an
//          in-register 16-point DFT, the four-step twiddle, an L-point DFT across the lanes
//          (DPP), the real-FFT untangle (partner bin by DPP). The wave's rows are one token's
//          K-step(s), so the wave's own max |X'| sets a power-of-two scale; X' is split into
//          fp16 hi + lo A fragments.                                           | barrier |
//      P2  per bin: v_mfma_f32_16x16x32_f16 with rows (token, re/im, hi/lo) x 16 output
//          blocks, K = 16 input blocks x (re, im); B = stationary conj(C) fragments. A token's
//          K-steps are brought to one exponent by exact fp16 power-of-two factors folded into
//          the im-row transform; the per-bin results go to the Y units.          | barrier |
//      The inverse: the real-FFT pre-process from LDS, a 16-point DFT, twiddle, L-point DFT
//      across the lanes, scale 1/(s_t s_C), cast/bias/cast, staged in the slot and stored as
//      1 KiB buffer stores. Each lane ends up holding 32 contiguous outputs.
//  * Numerics: X is split into two fp16 terms (~2^-21). C is one fp16 term (~2^-11 relative
//    per bin, ~3e-4 relative on the layer output). Accumulation is fp32. This is inside the
//    north star's 1e-3. bc_forward_mfma_kernel (bf16 hi/lo on both operands, ~1e-5) and
//    bc_forward_valu_kernel (fp32) remain for callers that want more.
//
// Geometries (stat_eligible): b = 128 with K = 4096, and b = 64 with K = 2048 or 4096; any M.
// DESIGN.md has the layouts, swizzles and the roofline accounting.
#include "bcfft_device.h"

#include <atomic>

namespace bcfft {

typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(2))) _Float16 f16x2;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

template <int B>
struct GeoS {
  static constexpr int H = B / 2;            // packed bins
  static constexpr int L = H / 16;           // lanes per transform (16 points per lane)
  static constexpr int BW = H / 8;           // bins per wave
  static constexpr int NT = 2;               // 16-wide N-tiles per output group
  static constexpr int NOG = STAT_OUT_BLOCKS;
  static constexpr int TT = 4;               // tokens per M-tile (MFMA rows: 4 x re/im x hi/lo)
  static constexpr int NW = 8, NTHR = 512;
  static constexpr int REGION = 65536;       // x tile / A image / Y image
  static constexpr int LOG2_2B = B == 128 ? 8 : 7;
  // LDS tables behind the two regions
  // lane-position tables use a 17-entry stride: the 4 (or 2) positions read by one instruction
  // then sit in different banks
  static constexpr int TS = 17;
  static constexpr int TWF_OFF = 2 * REGION;                 // [L][TS] float2  W_H^(g k2)
  static constexpr int TWI_OFF = TWF_OFF + L * TS * 8;       // [L][TS] float2  W_H^(-g k2)
  static constexpr int UCO_OFF = TWI_OFF + L * TS * 8;       // [L][TS] float4  untangle
  static constexpr int TWB_OFF = UCO_OFF + L * TS * 16;      // [B] float2      W_b^k
  static constexpr int SLOT_OFF = TWB_OFF + B * 8;           // [2][4] uint     token max |x|
  static constexpr int BIAS_OFF = SLOT_OFF + 32;             // [NOG * B] float  group's bias
  static constexpr int OS_OFF = BIAS_OFF + NOG * B * 4;      // [NOG] float      1 / s_o
  static constexpr int LDS_BYTES = OS_OFF + NOG * 4;
  static_assert(L == 2 || L == 4, "16 points per lane over 2 or 4 lanes");
  static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
};

// lane position j of a transform -> k1 of the bins it owns after the cross-lane DFT
template <int L>
__device__ __forceinline__ int k1_of(int j) { return L == 4 ? ((j == 1) ? 2 : (j == 2) ? 1 : j) : j; }


// L-point DFT across the L lanes of a transform, for each of the 16 registers (four-step
// step 3). Radix-2 DPP stages with lane-constant coefficients; lane j ends with bins
// k1 = k1_of(j), stored as D_j^-1 (true) with D from stat_decode (signs / one rotation).
template <int L, bool INV>
__device__ __forceinline__ void lane_dft(float2 (&v)[16], int g) {
  if constexpr (L == 2) {
    const float s = g ? -1.f : 1.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const float px = dpp<DPP_XOR1>(v[k].x), py = dpp<DPP_XOR1>(v[k].y);
      v[k].x = fmaf(s, px, v[k].x);
      v[k].y = fmaf(s, py, v[k].y);
    }
  } else {
    const float sa = g < 2 ? 1.f : -1.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) {            // stage A: partner g ^ 2
      const float px = dpp<DPP_XOR2>(v[k].x), py = dpp<DPP_XOR2>(v[k].y);
      v[k].x = fmaf(sa, px, v[k].x);
      v[k].y = fmaf(sa, py, v[k].y);
    }
    // stage B: partner g ^ 1; lanes 2,3 combine with -/+ i (forward / inverse)
    const float al = g == 0 ? 1.f : (g == 1 ? -1.f : 0.f);
    const float be = g < 2 ? 0.f : (INV ? -1.f : 1.f);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const float px = dpp<DPP_XOR1>(v[k].x), py = dpp<DPP_XOR1>(v[k].y);
      const float nx = fmaf(be, py, fmaf(al, px, v[k].x));
      const float ny = fmaf(-be, px, fmaf(al, py, v[k].y));
      v[k].x = nx;
      v[k].y = ny;
    }
  }
}

// lane_dft with the cross-lane operand read through DPP inside v_fmac_f32 (hipcc emits a separate
// v_mov_b32_dpp per operand and never folds it): stage A 2, stage B 5 instructions per complex
// instead of 4 and 6. Same operations in the same order: bit-identical to the C++ form. The
// s_nop 1 at each end covers the VALU-write -> DPP-read hazard (2 wait states) on the inputs and
// for the caller's next DPP read; inside, every DPP read is of a register last written >= 2
// instructions earlier.
template <int L, bool INV>
__device__ __forceinline__ void lane_dft_dpp(float2 (&v)[16], int g) {
  if constexpr (L == 2) {
    const float s = g ? -1.f : 1.f;
    asm volatile("s_nop 1\n\t"
        "v_fmac_f32_dpp %0, %0, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %1, %1, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %2, %2, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %3, %3, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %4, %4, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %5, %5, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %6, %6, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %7, %7, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %8, %8, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %9, %9, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %10, %10, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %11, %11, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %12, %12, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %13, %13, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %14, %14, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %15, %15, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %16, %16, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %17, %17, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %18, %18, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %19, %19, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %20, %20, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %21, %21, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %22, %22, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %23, %23, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %24, %24, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %25, %25, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %26, %26, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %27, %27, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %28, %28, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %29, %29, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %30, %30, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %31, %31, %32 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1"
        : "+v"(v[0].x), "+v"(v[0].y), "+v"(v[1].x), "+v"(v[1].y), "+v"(v[2].x), "+v"(v[2].y), "+v"(v[3].x), "+v"(v[3].y), "+v"(v[4].x), "+v"(v[4].y), "+v"(v[5].x), "+v"(v[5].y), "+v"(v[6].x), "+v"(v[6].y), "+v"(v[7].x), "+v"(v[7].y), "+v"(v[8].x), "+v"(v[8].y), "+v"(v[9].x), "+v"(v[9].y), "+v"(v[10].x), "+v"(v[10].y), "+v"(v[11].x), "+v"(v[11].y), "+v"(v[12].x), "+v"(v[12].y), "+v"(v[13].x), "+v"(v[13].y), "+v"(v[14].x), "+v"(v[14].y), "+v"(v[15].x), "+v"(v[15].y)
        : "v"(s));
  } else {
    const float sa = g < 2 ? 1.f : -1.f;
    const float al = g == 0 ? 1.f : (g == 1 ? -1.f : 0.f);
    const float be = g < 2 ? 0.f : (INV ? -1.f : 1.f);
    const float mbe = -be;
    float t;
    asm volatile("s_nop 1\n\t"
        "v_fmac_f32_dpp %0, %0, %33 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %1, %1, %33 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %2, %2, %33 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %3, %3, %33 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %4, %4, %33 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %5, %5, %33 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %6, %6, %33 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %7, %7, %33 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %8, %8, %33 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %9, %9, %33 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %10, %10, %33 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %11, %11, %33 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %12, %12, %33 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %13, %13, %33 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %14, %14, %33 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %15, %15, %33 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %16, %16, %33 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %17, %17, %33 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %18, %18, %33 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %19, %19, %33 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %20, %20, %33 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %21, %21, %33 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %22, %22, %33 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %23, %23, %33 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %24, %24, %33 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %25, %25, %33 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %26, %26, %33 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %27, %27, %33 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %28, %28, %33 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %29, %29, %33 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %30, %30, %33 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %31, %31, %33 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "v_mov_b32_dpp %32, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %1, %1, %34 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %1, %0, %36 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %0, %0, %34 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32 %0, %32, %35\n\t"
        "v_mov_b32_dpp %32, %3 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %3, %3, %34 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %3, %2, %36 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %2, %2, %34 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32 %2, %32, %35\n\t"
        "v_mov_b32_dpp %32, %5 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %5, %5, %34 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %5, %4, %36 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %4, %4, %34 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32 %4, %32, %35\n\t"
        "v_mov_b32_dpp %32, %7 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %7, %7, %34 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %7, %6, %36 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %6, %6, %34 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32 %6, %32, %35\n\t"
        "v_mov_b32_dpp %32, %9 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %9, %9, %34 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %9, %8, %36 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %8, %8, %34 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32 %8, %32, %35\n\t"
        "v_mov_b32_dpp %32, %11 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %11, %11, %34 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %11, %10, %36 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %10, %10, %34 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32 %10, %32, %35\n\t"
        "v_mov_b32_dpp %32, %13 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %13, %13, %34 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %13, %12, %36 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %12, %12, %34 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32 %12, %32, %35\n\t"
        "v_mov_b32_dpp %32, %15 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %15, %15, %34 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %15, %14, %36 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %14, %14, %34 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32 %14, %32, %35\n\t"
        "v_mov_b32_dpp %32, %17 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %17, %17, %34 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %17, %16, %36 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %16, %16, %34 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32 %16, %32, %35\n\t"
        "v_mov_b32_dpp %32, %19 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %19, %19, %34 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %19, %18, %36 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %18, %18, %34 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32 %18, %32, %35\n\t"
        "v_mov_b32_dpp %32, %21 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %21, %21, %34 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %21, %20, %36 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %20, %20, %34 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32 %20, %32, %35\n\t"
        "v_mov_b32_dpp %32, %23 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %23, %23, %34 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %23, %22, %36 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %22, %22, %34 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32 %22, %32, %35\n\t"
        "v_mov_b32_dpp %32, %25 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %25, %25, %34 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %25, %24, %36 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %24, %24, %34 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32 %24, %32, %35\n\t"
        "v_mov_b32_dpp %32, %27 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %27, %27, %34 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %27, %26, %36 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %26, %26, %34 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32 %26, %32, %35\n\t"
        "v_mov_b32_dpp %32, %29 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %29, %29, %34 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %29, %28, %36 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %28, %28, %34 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32 %28, %32, %35\n\t"
        "v_mov_b32_dpp %32, %31 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %31, %31, %34 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %31, %30, %36 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32_dpp %30, %30, %34 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f32 %30, %32, %35\n\t"
        "s_nop 1"
        : "+v"(v[0].x), "+v"(v[0].y), "+v"(v[1].x), "+v"(v[1].y), "+v"(v[2].x), "+v"(v[2].y), "+v"(v[3].x), "+v"(v[3].y), "+v"(v[4].x), "+v"(v[4].y), "+v"(v[5].x), "+v"(v[5].y), "+v"(v[6].x), "+v"(v[6].y), "+v"(v[7].x), "+v"(v[7].y), "+v"(v[8].x), "+v"(v[8].y), "+v"(v[9].x), "+v"(v[9].y), "+v"(v[10].x), "+v"(v[10].y), "+v"(v[11].x), "+v"(v[11].y), "+v"(v[12].x), "+v"(v[12].y), "+v"(v[13].x), "+v"(v[13].y), "+v"(v[14].x), "+v"(v[14].y), "+v"(v[15].x), "+v"(v[15].y), "=&v"(t)
        : "v"(sa), "v"(al), "v"(be), "v"(mbe));
  }
}

// decode matrix D_j (true = D * stored) after lane_dft, row-major {d00, d01, d10, d11}
template <int L, bool INV>
__host__ __device__ inline void stat_decode(int j, double d[4]) {
  d[0] = 1; d[1] = 0; d[2] = 0; d[3] = 1;
  if (L == 2) {
    if (j == 1) { d[0] = -1; d[3] = -1; }
  } else {
    if (j == 1 || j == 2) { d[0] = -1; d[3] = -1; }
    if (j == 3) {                                   // stored = i X (fwd) / -i X (inv)
      d[0] = 0; d[3] = 0;
      d[1] = INV ? -1 : 1;
      d[2] = INV ? 1 : -1;
    }
  }
}


// the forward storage of stat_decode<L, false> as a complex factor: true = sigma_j * stored
template <int L>
__host__ __device__ inline void stat_sigma(int j, double sg[2]) {
  sg[0] = 1; sg[1] = 0;
  if (j == 1 || (L == 4 && j == 2)) sg[0] = -1;
  if (L == 4 && j == 3) { sg[0] = 0; sg[1] = -1; }
}



// x staging swizzle (16-B units of a row) that keeps the forward DPP-group reads conflict-free
template <int L, int ES>
__device__ __forceinline__ int swz_x(int r) {
  return ES == 4 ? (L == 4 ? 2 * (r & 7) : (r & 15)) : (r & 7);
}

template <int B, int KS, int XT, bool YF32, bool GLU>
__global__ __launch_bounds__(512, 2) void bc_forward_stat_kernel(
    const void* __restrict__ xv, int64_t n_tokens, int n_out, const uint32_t* __restrict__ stat,
    const float* __restrict__ osc, const void* __restrict__ bias, int bias_dt, void* __restrict__ yv) {
  using G = GeoS<B>;
  constexpr int H = G::H, L = G::L, BW = G::BW, NT = G::NT, TT = G::TT, NW = G::NW;
  constexpr int NI = 16 * KS, K = NI * B;
  constexpr int ES = XTraits<XT>::ES;
  constexpr int RB = B * ES;                       // x row bytes
  constexpr int XTILE = TT * K * ES;
  constexpr int RPWF = 64 / L;                     // forward rows per wave
  constexpr int NDMA = RPWF * RB / 1024;           // LDS-DMA pieces per loading wave per M-tile
  constexpr bool Y32 = YF32 || XT == BCFFT_F32;
  constexpr int ESY = Y32 ? 4 : 2;
  constexpr int NST = 32 * ESY / 16;               // 16-B stores per lane per M-tile
  constexpr int NPIECE = BW * KS * NT;
  constexpr int FWD_ROWS = TT * NI, INV_ROWS = TT * G::NOG;
  static_assert(NDMA * 1024 == RPWF * RB && XTILE <= G::REGION, "x tile / DMA split");
  static_assert(FWD_ROWS * L <= 512 && INV_ROWS * L <= 512, "one pass per phase");
  static_assert(H * 32 * NI <= G::REGION && INV_ROWS * 8 * H <= G::REGION, "LDS images");
  static_assert(NI / 4 >= 8, "A image swizzle needs >= 8 block quads per row");

  ANALYSIS_INIT;
  __shared__ __attribute__((aligned(16))) char lds[G::LDS_BYTES];
  float2* twf = reinterpret_cast<float2*>(lds + G::TWF_OFF);
  float2* twi = reinterpret_cast<float2*>(lds + G::TWI_OFF);
  float4* uco = reinterpret_cast<float4*>(lds + G::UCO_OFF);
  float2* twb = reinterpret_cast<float2*>(lds + G::TWB_OFF);
  uint32_t* slots = reinterpret_cast<uint32_t*>(lds + G::SLOT_OFF);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // 1-D grid, one workgroup per CU: workgroup i serves output group i % groups and, with the
  // other workgroups of that group, strides over the M-tiles
  // GLU: n_out counts gate blocks; group g holds gate blocks [16g, 16g+16) and the matching up
  // blocks as its 32 output blocks, and h = silu(gate) * up has n_out blocks
  constexpr int OPG = GLU ? G::NOG / 2 : G::NOG;   // output blocks stored per group
  const int n_groups = (n_out + OPG - 1) / OPG;
  const int grp_o = blockIdx.x % n_groups;         // output group
  const int wg_in_grp = blockIdx.x / n_groups;
  const int64_t M = (int64_t)n_out * B;
  const int64_t n_mtiles = (n_tokens + TT - 1) / TT;
  const int gstride = (gridDim.x - grp_o + n_groups - 1) / n_groups;   // workgroups of this group

  // ---- LDS region layout: NWF slots of 8 KiB. Slot s belongs to forward wave s: that wave's
  // x rows land there (LDS-DMA), its forward replaces them in place by its A fragments (no other
  // wave reads or writes the slot in that phase), and after the MFMAs slot s holds the Y units of
  // the inverse rows [s RPWI, (s+1) RPWI), which inverse wave s reads, replaces by its staged y
  // rows and stores. Bank proofs of every access: tools/lds_banks.py.
  constexpr int SLOT = 8192;
  constexpr int NQ = RPWF / 4;                     // block quads per slot
  constexpr int NWF = FWD_ROWS / RPWF;             // forward waves = A slots
  constexpr int RPWI = 64 / L;                     // inverse rows per wave
  constexpr int NWI = INV_ROWS / RPWI;             // inverse waves = Y slots
  constexpr int SA = L == 4 ? 1 : 2;               // A swizzle shift: log2(8 / L)
  constexpr int SWM = L / 2 - 1;                   // Y swizzle mask
  static_assert(RPWF * H * 8 == SLOT && RPWI * (H / 2) * 16 == SLOT, "slot = A rows = Y rows");
  static_assert(RPWF * RB <= SLOT && NWF * SLOT <= G::REGION && NWI <= NWF, "slots");
  static_assert(NI % RPWF == 0 || RPWF % NI == 0, "a forward wave's rows are one token");
  int* wsc = reinterpret_cast<int*>(slots);        // per forward wave: its scale exponent

  // ---- x M-tile -> region by LDS-DMA: forward wave w loads its own RPWF rows (NDMA 1-KiB
  // pieces) into slot w, so its own vmcnt wait is all it needs before reading them. The tile's
  // 4 token rows are one contiguous span of x: a lane's source offset is its row byte with the
  // row's unit swizzle (swz_x) XORed in; the buffer range check zero-fills rows past n_tokens
  // (those tokens are never stored).
  const uint32_t lds_base = __builtin_amdgcn_readfirstlane(lds_addr(lds));
  auto dma_tile = [&](int64_t m, char* region) {
    if (wave >= NWF) return;
    const int64_t tok0 = m * TT;
    const int64_t ntok = n_tokens - tok0 < TT ? n_tokens - tok0 : TT;
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<char*>((const char*)xv) + tok0 * K * ES, 0, (int)(ntok * K * ES), 0x00020000);
    const int dlane = opaque(lane);
    // piece q's source offset = (wave NDMA + q) KiB + lane's 16 B, with the row's unit swizzle
    // XORed in. The swizzle sees row & 15 only and the wave's first row is a multiple of 16, so
    // it repeats with period DP in q: DP lane bases, q KiB in soffset. (Not the instruction
    // offset: on an LDS-DMA load that offset moves the LDS destination too. soffset is outside
    // the range check, which stays right: a wave's rows are whole tokens, so its lane base
    // alone is in or out of the tile's token range.)
    constexpr int RPK = 1024 / RB;                 // x rows per KiB
    constexpr int DP = 16 / RPK < NDMA ? 16 / RPK : NDMA;
    int vb[DP];
#pragma unroll
    for (int c = 0; c < DP; ++c)
      vb[c] = wave * NDMA * 1024 + ((dlane * 16) ^ (swz_x<L, ES>(c * RPK + (dlane * 16) / RB) << 4));
    // LDS byte address of the slot from the array's base: plain scalar adds, no generic-to-LDS
    // conversion (and its null check) per piece
    const uint32_t dst0 = lds_base + (uint32_t)(region - lds) + wave * SLOT;
#pragma unroll
    for (int q = 0; q < NDMA; ++q) {
      const uint32_t dst = dst0 + q * 1024;
      uint32_t keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen" BCFFT_XPOL " lds\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep) : "v"(vb[q % DP]), "s"(xrs), "s"(dst), "s"(q * 1024) : "memory");
    }
  };
  // the first M-tile's x goes out before anything else: it lands under the tables and the
  // 256 KiB of stationary weight loads
  if (wg_in_grp < n_mtiles && !ABLATE(16)) dma_tile(wg_in_grp, lds);


  // ---- tables (fp64 trig, once per workgroup)
  for (int e = tid; e < L * 16; e += G::NTHR) {
    const int g = e / 16, k2 = e % 16;
    double sn, cs;
    sincospi(2.0 * (double)((g * k2) % H) / (double)H, &sn, &cs);
    twf[g * G::TS + k2] = make_float2((float)cs, (float)-sn);
    twi[g * G::TS + k2] = make_float2((float)cs, (float)sn);
    // forward untangle X'[k] = alpha Z[k] + beta conj(Z[H-k]) with alpha = (1+wi) - i wr,
    // beta = (1-wi) + i wr (W^k = wr + i wi); bin 0: (2(a+b), 2(a-b)) = (2+2i) conj(Z0).
    // Folded in: the lane_dft storage of this lane (sigma_g) and of the partner (sigma_gp).
    const int k = k2 + 16 * k1_of<L>(g);
    double ws, wc;
    sincospi(2.0 * (double)k / (double)B, &ws, &wc);
    const double wr = wc, wi = -ws;
    double ar = 1 + wi, ai = -wr, br = 1 - wi, bi = wr;
    if (k == 0) { ar = 0; ai = 0; br = 2; bi = 2; }
    int gp;                                        // partner lane of bin H - k
    if (k2 == 0) gp = (L == 4) ? (g < 2 ? g : g ^ 1) : g;
    else gp = (L == 4) ? (g ^ 3) : (g ^ 1);
    double sg[2], sp[2];                           // true = sigma * stored
    stat_sigma<L>(g, sg);
    stat_sigma<L>(gp, sp);
    uco[g * G::TS + k2] = make_float4((float)(ar * sg[0] - ai * sg[1]), (float)(ar * sg[1] + ai * sg[0]),   // alpha sigma_g
                         (float)(br * sp[0] + bi * sp[1]), (float)(bi * sp[0] - br * sp[1]));  // beta conj(sigma_gp)
  }
  for (int k = tid; k < B; k += G::NTHR) {
    double sn, cs;
    sincospi(2.0 * (double)k / (double)B, &sn, &cs);
    twb[k] = make_float2((float)cs, (float)-sn);
  }
  if (tid < 8) slots[tid] = 0u;
  lds_barrier();                                   // tables before the weight loads (pressure)

  // ---- stationary B fragments: conj(C) * s_o as fp16, K/32 VGPRs per lane
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
  }
  // the group's bias as fp32 in LDS, so no VMEM load sits in the loop: a waited load would
  // also drain every older y store and x DMA (vmcnt retires in order). Read after the weight
  // loads are issued, so its waits overlap theirs and the first DMA's.
  float* bias_l = reinterpret_cast<float*>(lds + G::BIAS_OFF);
  if (bias_dt != BCFFT_NONE) {
    for (int e = tid; e < G::NOG * B; e += G::NTHR) {
      const int64_t col = (int64_t)grp_o * G::NOG * B + e;
      bias_l[e] = col < (int64_t)n_out * B ? load_scalar(bias, col, bias_dt) : 0.f;
    }
  }
  float* osc_l = reinterpret_cast<float*>(lds + G::OS_OFF);    // the group's 1 / s_o
  if (tid < G::NOG) osc_l[tid] = osc[grp_o * G::NOG + tid];


  // A fragment unit (16 B: 4 blocks x (re, im) fp16 of bin f, precision prec, block quad lq)
  // within slot s; the XOR keeps the lanes of the forward's writes and of the MFMA reads on
  // distinct banks and never leaves bin f
  auto aunit = [](int f, int prec, int lq, int s) {
    const int tsw = s / (NWF / 2);
    return 16 * ((f * 2 * NQ + prec * NQ + lq) ^ (((f >> 4) ^ tsw) << SA));
  };
  // Y unit (bins 2p, 2p+1) of inverse row r of slot w; the units of bins (2p, 2p+1) of every
  // row of the slot are exactly the A units of those two bins there (an MFMA wave overwrites
  // only what it alone has read). The swizzle bit p & SWM is lane-constant in the inverse's reads.
  auto yunit = [](int p, int r) { return 16 * (p * RPWI + (r ^ (p & SWM))); };
  // inverse group gi (within its wave) -> row r. L = 4: half-wave -> bit 0, group bits
  // (0, 1, 2) -> (2, 1, 3); L = 2: identity
  auto inv_row = [](int gi) {
    if constexpr (L == 4)
      return ((gi & 1) << 2) | (gi & 2) | ((gi & 4) << 1) | ((gi >> 3) & 1);
    else
      return gi;
  };
  // output row R = 32 t + o (token t of the tile, block o of the group) <-> (slot, row r). Plain:
  // slot R / RPWI. GLU at b = 128: slot 2t + ((o >> 3) & 1) holds o in 8 half + [0, 8) as
  // r = o & 7 and o + 16 as r + 8, so a wave owns both the gate and the up row of its outputs
  // (at b = 64 a slot is a whole token already: gate r < 16, up r + 16)
  auto slot_of_row = [](int R, int& r) {
    if constexpr (GLU && RPWI == 16) {
      const int o = R & 31;
      r = (o & 7) + 8 * (o >> 4);
      return 2 * (R >> 5) + ((o >> 3) & 1);
    } else {
      r = R % RPWI;
      return R / RPWI;
    }
  };
  auto row_of_slot = [](int w, int r) {
    if constexpr (GLU && RPWI == 16)
      return 32 * (w >> 1) + 8 * (w & 1) + (r & 7) + 16 * (r >> 3);
    else
      return w * RPWI + r;
  };
  // y staging: 16-B piece pc of row r goes to unit pc of row r ^ hmap(pc) (same slot), which
  // spreads one store instruction's pieces over the banks; hmap is linear in the bits of pc
  constexpr int NQL = 32 * ESY / 16;               // 16-B pieces of y per lane
  constexpr int NPR = B * ESY / 16;                // 16-B pieces per y row
  constexpr int RPI = 64 / NPR;                    // rows per store instruction
  auto hmap = [](int pc) {
    constexpr int C128F[5] = {5, 8, 0, 1, 2}, C128H[5] = {0, 2, 5, 10, 0};
    constexpr int C64F[5] = {1, 2, 4, 12, 0}, C64H[5] = {1, 4, 12, 0, 0};
    const int* c = B == 128 ? (ESY == 4 ? C128F : C128H) : (ESY == 4 ? C64F : C64H);
    int r = 0;
#pragma unroll
    for (int i = 0; i < 5; ++i)
      if ((pc >> i) & 1) r ^= c[i];
    return r;
  };


  // the inverse wave stores the rows it staged, in global order, RPI whole rows (1 KiB) per
  // instruction: rows r0 + q RPI of its slot, r0 = lane / NPR
  auto store_tile = [&](int64_t mt, const char* regn) {
    if (wave >= NWI) return;
    const int64_t stok0 = mt * TT;
    const int64_t ntok = n_tokens - stok0 < TT ? n_tokens - stok0 : TT;
    const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
        (char*)yv + stok0 * M * ESY, 0, (int)(ntok * M * ESY), 0x00020000);
    const int slane = opaque(lane);
    const int pc = slane & (NPR - 1);
    const int r0 = (int)((unsigned)slane / NPR);
    const int src0 = wave * SLOT + yunit(pc, r0 ^ hmap(pc));   // row r0 + q RPI = r0 ^ q RPI
    const int rho0 = wave * RPWI + r0;                          // y row: token rho >> 5, block rho & 31
    const int o0 = rho0 & (G::NOG - 1);
    const int yoff0 = (int)((((int64_t)(rho0 >> 5) * M) + (int64_t)(grp_o * G::NOG + o0) * B) * ESY) + 16 * pc;
    const int nvalid = n_out - grp_o * G::NOG;      // output blocks of this group that exist
    uint4 d[NST];                                   // all staged reads first: one LDS latency
#pragma unroll
    for (int q = 0; q < NST; ++q) d[q] = *reinterpret_cast<const uint4*>(regn + (src0 ^ (16 * q * RPI)));
    __builtin_amdgcn_sched_barrier(0);
    if (ABLATE(2)) return;
    if (nvalid >= G::NOG) {                         // uniform: every row of the group exists
#pragma unroll
      for (int q = 0; q < NST; ++q)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, d[q]), yrs, yoff0 + q * RPI * B * ESY, 0, BCFFT_YAUX);
    } else {
#pragma unroll
      for (int q = 0; q < NST; ++q) {
        const int yoff = o0 + q * RPI < nvalid ? yoff0 + q * RPI * B * ESY : 0x7fff0000;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, d[q]), yrs, yoff, 0, BCFFT_YAUX);
      }
    }
  };

  // GLU epilogue: the wave's RPWI/2 h rows, h = silu(g) * u from its staged gate row r and up
  // row r + RPWI/2, with torch's roundings for 16-bit tensors (silu(g) rounded to the dtype,
  // then the product rounded). Same global order and 1 KiB instructions as store_tile.
  auto glu_store = [&](int64_t mt, const char* regn) {
    if constexpr (GLU) {
      if (wave >= NWI) return;
      constexpr int NSTG = NST / 2;
      const int64_t stok0 = mt * TT;
      const int64_t ntok = n_tokens - stok0 < TT ? n_tokens - stok0 : TT;
      const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
          (char*)yv + stok0 * M * ESY, 0, (int)(ntok * M * ESY), 0x00020000);
      const int slane = opaque(lane);
      const int pc = slane & (NPR - 1);
      const int r0 = (int)((unsigned)slane / NPR);
      const int src0 = wave * SLOT + yunit(pc, r0 ^ hmap(pc));
      const int rho0 = row_of_slot(wave, r0);       // gate row: token rho >> 5, block rho & 15
      const int j0 = rho0 & 15;
      const int yoff0 = (int)((((int64_t)(rho0 >> 5) * M) + (int64_t)(grp_o * OPG + j0) * B) * ESY) + 16 * pc;
      const int nvalid = n_out - grp_o * OPG;
      uint4 gq[NSTG], uq[NSTG];
#pragma unroll
      for (int q = 0; q < NSTG; ++q) {
        gq[q] = *reinterpret_cast<const uint4*>(regn + (src0 ^ (16 * q * RPI)));
        uq[q] = *reinterpret_cast<const uint4*>(regn + (src0 ^ (16 * q * RPI) ^ (16 * RPWI / 2)));
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int q = 0; q < NSTG; ++q) {
        uint4 hq;
        if constexpr (Y32) {
          const float4 gv = __builtin_bit_cast(float4, gq[q]), uv = __builtin_bit_cast(float4, uq[q]);
          hq = __builtin_bit_cast(uint4, make_float4(silu(gv.x) * uv.x, silu(gv.y) * uv.y,
                                                     silu(gv.z) * uv.z, silu(gv.w) * uv.w));
        } else {
          const uint32_t* gw = reinterpret_cast<const uint32_t*>(&gq[q]);
          const uint32_t* uw = reinterpret_cast<const uint32_t*>(&uq[q]);
          uint32_t hw[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float2 g2 = unpack16<XT>(gw[e]), u2 = unpack16<XT>(uw[e]);
            const float2 s2 = round_pair<XT>(silu(g2.x), silu(g2.y));
            hw[e] = pack16<XT>(s2.x * u2.x, s2.y * u2.y);
          }
          hq = make_uint4(hw[0], hw[1], hw[2], hw[3]);
        }
        const int yoff = nvalid >= OPG || j0 + q * RPI < nvalid ? yoff0 + q * RPI * B * ESY : 0x7fff0000;
        if (!ABLATE(2)) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, hq), yrs, yoff, 0, BCFFT_YAUX);
      }
    }
  };

  // ---- forward of one M-tile (wave w < NWF, slot w): x rows -> real-FFT bins X' -> scaled
  // fp16 hi/lo A fragments in place. All RPWF rows of the wave are one token's K-step(s): the
  // wave's own max |X'| sets the scale s = 2^(15 - E) (max < 2^E), exponent posted to wsc[w].
  auto forward = [&](char* region, int younger) {
    // this wave's x rows landed: everything but the `younger` VMEM ops issued after them
    constexpr int NSTW = GLU ? NST / 2 : NST;
    if (younger == NSTW + NDMA) wait_vmcnt<NSTW + NDMA>();
    else if (younger == NSTW) wait_vmcnt<NSTW>();
    else if (younger == NDMA) wait_vmcnt<NDMA>();
    else wait_vmcnt<0>();
    MARK(fwd_read);
    const int ptid = opaque(tid);
    const int li = (int)((unsigned)(ptid & 63) / L), g = ptid & (L - 1);
    const int k1 = k1_of<L>(g);
    char* slot = region + wave * SLOT;
    float2 v[16];
    {
      const char* rowp = slot + li * RB;
#pragma unroll
      for (int n2 = 0; n2 < 16; ++n2) {
        const int n = g + L * n2;
        if constexpr (ES == 4) {
          const int off = 8 * n;
          v[n2] = *reinterpret_cast<const float2*>(rowp + (((off >> 4) ^ swz_x<L, ES>(li)) << 4) + (off & 15));
        } else {
          const int off = 4 * n;
          const uint32_t w = *reinterpret_cast<const uint32_t*>(rowp + (((off >> 4) ^ swz_x<L, ES>(li)) << 4) + (off & 15));
          v[n2] = XT == BCFFT_BF16 ? make_float2(bf16_to_f32(w & 0xffffu), bf16_to_f32(w >> 16))
                                   : make_float2(f16_to_f32(w & 0xffffu), f16_to_f32(w >> 16));
        }
      }
    }
    float2 tw[16];                                  // four-step twiddles, issued ahead of the DFT
#pragma unroll
    for (int k2 = 1; k2 < 16; ++k2) tw[k2] = twf[g * G::TS + k2];
    float4 uc[16];
    MARK(fwd_dft);
    if (!ABLATE(4)) {
      dft<16, false>(v);
#pragma unroll
      for (int k2 = 1; k2 < 16; ++k2) v[k2] = cmul(v[k2], tw[k2]);
    }
#pragma unroll
    for (int k2 = 0; k2 < 8; ++k2) uc[k2] = uco[g * G::TS + k2];   // in flight under lane_dft
    __builtin_amdgcn_sched_barrier(0);
    MARK(fwd_lane);
    if (!ABLATE(4)) lane_dft_dpp<L, false>(v, g);
    MARK(untangle);
    // untangle X'[k] = alpha s + beta conj(p), partner bin H - k by DPP
    float2 xs[16];
    float mx = 0.f;
#pragma unroll
    for (int k2 = 0; k2 < 16; ++k2) {
      if (k2 == 4) {                                // second half of the coefficients
#pragma unroll
        for (int kk = 8; kk < 16; ++kk) uc[kk] = uco[g * G::TS + kk];
      }
      const int src = k2 == 0 ? 0 : 16 - k2;
      float px, py;
      if constexpr (L == 4) {
        if (k2 == 0) { px = dpp<DPP_P0>(v[0].x); py = dpp<DPP_P0>(v[0].y); }
        else { px = dpp<DPP_XOR3>(v[src].x); py = dpp<DPP_XOR3>(v[src].y); }
      } else {
        if (k2 == 0) { px = v[0].x; py = v[0].y; }
        else { px = dpp<DPP_XOR1>(v[src].x); py = dpp<DPP_XOR1>(v[src].y); }
      }
      const float4 c = uc[k2];
      xs[k2].x = fmaf(c.x, v[k2].x, fmaf(-c.y, v[k2].y, fmaf(c.z, px, c.w * py)));
      xs[k2].y = fmaf(c.x, v[k2].y, fmaf(c.y, v[k2].x, fmaf(c.w, px, -c.z * py)));
      mx = fmaxf(mx, fmaxf(fabsf(xs[k2].x), fabsf(xs[k2].y)));
    }
    // wave max -> scale exponent nsc: 2^nsc max|X'| < 2^15 (fp16 hi with headroom)
    const int nsc = stat_scale_exp(wave_max(mx));
    if (lane == 0) wsc[wave] = nsc;
    const float s_w = __int_as_float((nsc + 127) << 23);
    MARK(split);
    // hi = fp16(X' s) (round toward zero), lo = fp16(X' s - hi): two fp16 terms ~2^-21
    // aunit's XOR ((f >> 4) ^ tsw) << SA is lane-constant here (f >> 4 = k1) and stays below
    // the bin field, so the 32 writes are two per-lane bases plus immediate bin offsets
    const int ax = (k1 ^ (wave / (NWF / 2))) << SA;
    char* abase0 = slot + 4 * (li & 3) + 16 * ((li >> 2) ^ ax) + k1 * 16 * (32 * NQ);
    char* abase1 = slot + 4 * (li & 3) + 16 * ((NQ + (li >> 2)) ^ ax) + k1 * 16 * (32 * NQ);
#pragma unroll
    for (int k2 = 0; k2 < 16; ++k2) {
      const float ox = xs[k2].x * s_w, oy = xs[k2].y * s_w;
      const f16x2 hi = __builtin_bit_cast(f16x2, __builtin_amdgcn_cvt_pkrtz(ox, oy));
      const f16x2 lo = __builtin_bit_cast(f16x2, __builtin_amdgcn_cvt_pkrtz(ox - (float)hi.x, oy - (float)hi.y));
      *reinterpret_cast<f16x2*>(abase0 + k2 * 16 * (2 * NQ)) = hi;   // = aunit(k2 + 16 k1, 0, li >> 2, wave)
      *reinterpret_cast<f16x2*>(abase1 + k2 * 16 * (2 * NQ)) = lo;
    }
  };

  // ---- per-bin complex MAC on the matrix cores (all waves): wave w's bins f = w BW + fb; the
  // Y pairs overwrite this wave's own A bins.
  auto cmac = [&](char* region) {
    const int mlane = opaque(lane);
    const int arow = mlane & 15, kb = mlane >> 4;   // A row (token, re/im, hi/lo), K quad
    const int a_t = arow >> 2, a_reim = (arow >> 1) & 1, a_prec = arow & 1;
    const uint32_t a_sel = a_reim ? 0x01000302u : 0x03020100u;   // im rows: (re, im) -> (im, re)
    const int yt = mlane >> 4;                      // accumulator rows 4 yt + {re hi, re lo, im hi, im lo}
    // Each K-step was formed at its forward wave's own scale 2^nsc. A token's K-steps are brought
    // to its smallest exponent by an exact power-of-two factor folded into the packed fp16
    // multiply that also applies the im-row sign: (f, f) on re rows, (f, -f) on im rows (after the
    // swap), (f, 0) / (0, f) on bin 0's rows. Same numerics as one scale per token.
    int nmin = 127, nminy = 127;
    int nk[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      nk[ks] = wsc[(a_t * NI + 16 * ks) / RPWF];
      nmin = min(nmin, nk[ks]);
      nminy = min(nminy, wsc[(yt * NI + 16 * ks) / RPWF]);
    }
    uint32_t amul[KS], amul0[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int d = nk[ks] - nmin;                  // factor 2^-d as fp16 (subnormal / 0 far down)
      const uint32_t h = d <= 14 ? (uint32_t)(15 - d) << 10 : (d <= 24 ? 1u << (24 - d) : 0u);
      amul[ks] = a_reim ? (h | ((h | 0x8000u) << 16)) : (h | (h << 16));
      amul0[ks] = a_reim ? (h << 16) : h;
    }
    const float ry = __int_as_float((127 - nminy) << 23);   // 2^-nsc of the accumulator's token
    // A fragment of (bin f, K-step ks) = aunit(f, a_prec, lq, s): the wave's bins share f >> 4,
    // so per K-step one lane base plus an immediate bin offset
    const char* abase[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int row0 = a_t * NI + 16 * ks;
      const int s = row0 / RPWF, lq = (row0 % RPWF) / 4 + kb;
      const int ax = (((wave * BW) >> 4) ^ (s / (NWF / 2))) << SA;
      abase[ks] = region + s * SLOT + 16 * ((a_prec * NQ + lq) ^ ax) + wave * BW * 16 * (2 * NQ);
    }
    uint4 araw[BW][KS];                             // every A fragment of the wave's bins, issued
#pragma unroll                                       // up front in bin order (counted waits)
    for (int fb = 0; fb < BW; ++fb) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        araw[fb][ks] = ABLATE(32) ? make_uint4(a_t, kb, fb, ks)
                                  : *reinterpret_cast<const uint4*>(abase[ks] + fb * 16 * (2 * NQ));
    }
    // a bin pair's Y goes over the wave's own A units of those bins once its MFMAs are done: the
    // wave's DS operations execute in order, so the reads of those units precede the writes and
    // only one pair of results is live
    MARK(mfma);
#pragma unroll
    for (int fp = 0; fp < BW / 2; ++fp) {
      float2 ybuf[2][NT];
      f32x4 acc[2][NT];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int fb = 2 * fp + h;
        const int f = wave * BW + fb;
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[h][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          uint4 raw = araw[fb][ks];
          if (ABLATE(64)) {
          } else if (f == 0) {
            raw.x = pkmul(raw.x, amul0[ks]); raw.y = pkmul(raw.y, amul0[ks]);
            raw.z = pkmul(raw.z, amul0[ks]); raw.w = pkmul(raw.w, amul0[ks]);
          } else {
            raw.x = pkmul(__builtin_amdgcn_perm(raw.x, raw.x, a_sel), amul[ks]);
            raw.y = pkmul(__builtin_amdgcn_perm(raw.y, raw.y, a_sel), amul[ks]);
            raw.z = pkmul(__builtin_amdgcn_perm(raw.z, raw.z, a_sel), amul[ks]);
            raw.w = pkmul(__builtin_amdgcn_perm(raw.w, raw.w, a_sel), amul[ks]);
          }
          const f16x8 a = __builtin_bit_cast(f16x8, raw);
          if (ABLATE(1)) {
            asm volatile("" :: "v"(raw.x));
            continue;
          }
#pragma unroll
          for (int nt = 0; nt < NT; ++nt)
            acc[h][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, creg[fb][ks][nt], acc[h][nt], 0, 0, 0);
        }
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)             // rows 4 yt + {re hi, re lo, im hi, im lo}
          ybuf[h][nt] = make_float2((acc[h][nt][0] + acc[h][nt][1]) * ry, (acc[h][nt][2] + acc[h][nt][3]) * ry);
      }
      const int p = (wave * BW) / 2 + fp;
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        int yr;
        const int ys = slot_of_row(yt * G::NOG + nt * 16 + (mlane & 15), yr);
        *reinterpret_cast<float4*>(region + ys * SLOT + yunit(p, yr)) =
            make_float4(ybuf[0][nt].x, ybuf[0][nt].y, ybuf[1][nt].x, ybuf[1][nt].y);
      }
    }
    MARK(ywrite);
  };

  // ---- inverse of one M-tile (wave w < NWI, slot w): Y rows -> y rows staged in the slot
  auto inverse = [&](char* region) {
    MARK(inv_read);
    const int ptid = opaque(tid);
    const int gi = (int)((unsigned)(ptid & 63) / L), g = ptid & (L - 1);
    const int k1 = k1_of<L>(g);
    const int r = inv_row(gi);
    const int R = row_of_slot(wave, r);             // token R >> 5, output block R & 31
    const int inv_o = R & (G::NOG - 1);
    char* slot = region + wave * SLOT;
    // Y[k], k = g + L n2: unit (g >> 1) + (L/2) n2, half g & 1. Y[H-k] = (H-L-L n2) + (L-g):
    // unit (H-L)/2 - (L/2) n2 + ((L-g) >> 1), half (L-g) & 1 (k = 0 reads past the slot,
    // unused: bin 0 is packed). The swizzle bit p & SWM is lane-constant in both.
    const int gl = L - g;
    const char* ykb = slot + yunit(g >> 1, r) + 8 * (g & 1);
    const char* yhb = slot + yunit(gl >> 1, r) + 8 * (gl & 1);
    float2 v[16];
    float2 yk[16], yh[16], wk[16];
#pragma unroll
    for (int hb = 0; hb < 2; ++hb) {
#pragma unroll
      for (int n2 = 8 * hb; n2 < 8 * hb + 8; ++n2) {
        yk[n2] = *reinterpret_cast<const float2*>(ykb + n2 * (L / 2) * RPWI * 16);
        yh[n2] = *reinterpret_cast<const float2*>(yhb + ((H - L) / 2 - (L / 2) * n2) * RPWI * 16);
        wk[n2] = twb[g + L * n2];
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int n2 = 8 * hb; n2 < 8 * hb + 8; ++n2) {
        const float er = yk[n2].x + yh[n2].x, ei = yk[n2].y - yh[n2].y;   // E = Y[k] + conj(Y[H-k])
        const float dr = yk[n2].x - yh[n2].x, di = yk[n2].y + yh[n2].y;   // D = Y[k] - conj(Y[H-k])
        const float2 w = wk[n2];                                          // Zi = E + i D conj(W^k)
        float2 z;
        z.x = er - (di * w.x - dr * w.y);
        z.y = ei + (dr * w.x + di * w.y);
        if (n2 == 0 && g == 0) z = make_float2(yk[0].x + yk[0].y, yk[0].x - yk[0].y);   // packed bin 0
        v[n2] = z;
      }
    }
    MARK(inv_dft);
    float2 tw[16];
#pragma unroll
    for (int k2 = 1; k2 < 16; ++k2) tw[k2] = twi[g * G::TS + k2];
    if (!ABLATE(8)) {
      dft<16, true>(v);
#pragma unroll
      for (int k2 = 1; k2 < 16; ++k2) v[k2] = cmul(v[k2], tw[k2]);
      lane_dft_dpp<L, true>(v, g);
    }
    MARK(inv_out);
    // y[32 k1 + 2 k2 + {0,1}] = D (R0, R1) / s_o, D = stat_decode<L, true>(g)
    const float sc = osc_l[inv_o];
    const bool rot = L == 4 && g == 3;              // stored = -i z
    const float sd = (g == 1 || g == 2) ? -sc : sc;
    const float c00 = rot ? 0.f : sd, c01 = rot ? -sc : 0.f;
    const float c10 = rot ? sc : 0.f, c11 = rot ? 0.f : sd;
    const float* brow = bias_l + inv_o * B + 32 * k1;
    // piece j of this lane's run (unit k1 NQL + j) goes to row sx ^ hmap(j), sx = r ^ hmap(k1 NQL)
    const int sx = r ^ hmap(k1 * NQL);
    char* stb = slot + 16 * (k1 * NQL * RPWI);
    auto stage = [&](int j) { return stb + 16 * (j * RPWI + (sx ^ hmap(j) ^ (j & SWM))); };
    wave_lds_sync();                                // the wave's Y reads precede its y writes
    // 8 outputs (4 registers) per step: .to(x.dtype) :266, + bias :270-271, .to(y dtype)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float o8[8];
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        const float2 z = v[4 * q + h];
        o8[2 * h] = fmaf(c00, z.x, c01 * z.y);
        o8[2 * h + 1] = fmaf(c10, z.x, c11 * z.y);
      }
      // a 16-bit y without bias is ONE rounding (round_to then the cast is the same value)
      if (Y32 || bias_dt != BCFFT_NONE) {
#pragma unroll
        for (int h = 0; h < 4; ++h) {
          const float2 rr = round_pair<XT>(o8[2 * h], o8[2 * h + 1]);
          o8[2 * h] = rr.x;
          o8[2 * h + 1] = rr.y;
        }
        if (bias_dt != BCFFT_NONE) {
          const float4 b0 = *reinterpret_cast<const float4*>(brow + 8 * q);
          const float4 b1 = *reinterpret_cast<const float4*>(brow + 8 * q + 4);
          o8[0] += b0.x; o8[1] += b0.y; o8[2] += b0.z; o8[3] += b0.w;
          o8[4] += b1.x; o8[5] += b1.y; o8[6] += b1.z; o8[7] += b1.w;
        }
      }
      if constexpr (Y32) {
#pragma unroll
        for (int hq = 0; hq < 2; ++hq)
          *reinterpret_cast<float4*>(stage(2 * q + hq)) =
              make_float4(o8[4 * hq], o8[4 * hq + 1], o8[4 * hq + 2], o8[4 * hq + 3]);
      } else {
        *reinterpret_cast<uint4*>(stage(q)) =
            make_uint4(pack16<XT>(o8[0], o8[1]), pack16<XT>(o8[2], o8[3]), pack16<XT>(o8[4], o8[5]),
                       pack16<XT>(o8[6], o8[7]));
      }
    }
  };

  // Pipeline, two workgroup barriers per M-tile. Iteration it (region R = R[it & 1] holds tile
  // m, R' = the other holds tile m - gstride):
  //   P1  inverse of tile m - gstride (slot w of R' -> y rows staged there), their stores, then
  //       the LDS-DMA of x(m + gstride) into slot w of R' (private to wave w from here on: no
  //       barrier needed, and the DMA gets a whole period of lead), then the forward of tile m
  //       in slot w of R, whose counted vmcnt wait leaves those stores and DMA in flight | Ba |
  //   P2  MFMAs of tile m: A fragments in R -> Y units in R                          | Bb |
  // (Measured alternatives: issuing the stores and DMA inside the forward, after its x reads,
  // and running inverse / forward in opposite orders on SIMD mates were both slower.)
  const bool fwd_active = wave < NWF, inv_active = wave < NWI;
  int64_t m = wg_in_grp;
  STAMP(0);
  for (int it = 0; m < n_mtiles || it > 0; ++it, m += gstride) {
    char* region = lds + (it & 1) * G::REGION;
    char* other = lds + ((it + 1) & 1) * G::REGION;
    const bool have_f = m < n_mtiles;
    const bool st = it > 0 && inv_active;
    const bool dm = m + gstride < n_mtiles && fwd_active && !ABLATE(16);
    constexpr int NSTV = GLU ? NST / 2 : NST;       // VMEM stores issued per wave per tile
    const int sb = 1 + 7 * (it < 7 ? it : 7);       // stamp slots: iterations 0-6, then the latest
    STAMP(sb);
    if (st) inverse(other);
    STAMP(sb + 1);
    MARK(store);
    if (st) {
      if constexpr (GLU) glu_store(m - gstride, other);
      else store_tile(m - gstride, other);
    }
    if (dm) dma_tile(m + gstride, other);
    STAMP(sb + 2);
    if (!have_f) break;
    if (fwd_active) forward(region, (st ? NSTV : 0) + (dm ? NDMA : 0));
    STAMP(sb + 3);
    lds_barrier();                                  // Ba: A fragments and scales complete
    STAMP(sb + 4);
    cmac(region);
    STAMP(sb + 5);
    lds_barrier();                                  // Bb: Y image complete
    STAMP(sb + 6);
  }
  STAMP(63);
}

// ================================================================== weight preparation
// Per output block o (one workgroup each, over the groups' 32 x groups blocks): the weight
// scale s_o = 2^(15 - E_o) with max |S[o][.][.]| < 2^E_o over the block row's packed spectra
// (an all-zero or padded row: s_o = 1). The image holds conj(S) s_o as fp16; the kernels scale
// output block o by osc[o] = 1 / s_o. Header {1, 1, 0, 0} (kept for the layout).
template <int B>
__global__ void bc_stat_scale_kernel(int n_out, int n_in, float2* __restrict__ spec) {
  const SpecLayout sl = spec_layout(n_out, n_in, B);
  const int o = blockIdx.x;
  const float* p = reinterpret_cast<const float*>(spec) + (int64_t)o * n_in * B;   // row o: n_in x B/2 float2
  const int64_t n = o < n_out ? (int64_t)n_in * B : 0;
  float mx = 0.f;
  for (int64_t e = threadIdx.x; e < n; e += blockDim.x) mx = fmaxf(mx, fabsf(p[e]));
  __shared__ float red[256];
  red[threadIdx.x] = mx;
  __syncthreads();
  for (int st = blockDim.x / 2; st > 0; st >>= 1) {
    if ((int)threadIdx.x < st) red[threadIdx.x] = fmaxf(red[threadIdx.x], red[threadIdx.x + st]);
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    int n2 = red[0] > 0.f ? 15 - __builtin_amdgcn_frexp_expf(red[0]) : 0;
    n2 = n2 < -126 ? -126 : (n2 > 126 ? 126 : n2);
    reinterpret_cast<uint32_t*>(spec)[sl.osc_off_u32 + o] = (uint32_t)((127 - n2) << 23);   // 2^-n2
    if (o == 0) {
      uint32_t* hdr = reinterpret_cast<uint32_t*>(spec) + sl.stat_off_u32;
      hdr[0] = 0x3f800000u;
      hdr[1] = 0x3f800000u;
      hdr[2] = 0u;
      hdr[3] = 0u;
    }
  }
}
void launch_stat_scale(int b, int n_out, int n_in, void* spec, hipStream_t s) {
  const SpecLayout sl = spec_layout(n_out, n_in, b);
  const unsigned blocks = (unsigned)(sl.stat_groups * STAT_OUT_BLOCKS);
  if (b == 256) hipLaunchKernelGGL(bc_stat_scale_kernel<256>, dim3(blocks), dim3(256), 0, s, n_out, n_in, (float2*)spec);
  else if (b == 128) hipLaunchKernelGGL(bc_stat_scale_kernel<128>, dim3(blocks), dim3(256), 0, s, n_out, n_in, (float2*)spec);
  else hipLaunchKernelGGL(bc_stat_scale_kernel<64>, dim3(blocks), dim3(256), 0, s, n_out, n_in, (float2*)spec);
}

// one thread per (group, wave, piece, lane) 16-B fragment: 4 input blocks x (re, im) fp16 of
// conj(S) * s_o (bin 0: (S_0, S_H) * s_o), zero outside the operator
template <int B>
__global__ void bc_stat_image_kernel(int n_out, int n_in, float2* __restrict__ spec) {
  constexpr int H = B / 2, BW = H / 8, NT = 2, NW = 8;
  const SpecLayout sl = spec_layout(n_out, n_in, B);
  const int ks_n = (n_in + 15) / 16;
  const int npiece = sl.stat_pieces;
  const int64_t total = (int64_t)sl.stat_groups * NW * npiece * 64;
  uint32_t* hdr = reinterpret_cast<uint32_t*>(spec) + sl.stat_off_u32;
  uint4* img = reinterpret_cast<uint4*>(hdr + 4);
  const uint32_t* osc = reinterpret_cast<const uint32_t*>(spec) + sl.osc_off_u32;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int lane = (int)(idx & 63);
    const int64_t rest = idx >> 6;
    const int p = (int)(rest % npiece);
    const int w = (int)((rest / npiece) % NW);
    const int gq = (int)(rest / npiece / NW);
    const int nt = p % NT, ks = (p / NT) % ks_n, fb = p / NT / ks_n;
    const int f = w * BW + fb;
    const int o = gq * STAT_OUT_BLOCKS + nt * 16 + (lane & 15);
    const float sc = __uint_as_float((254u << 23) - osc[o]);   // s_o = 1 / osc[o] (powers of two)
    const int i0 = ks * 16 + 4 * (lane >> 4);
    uint32_t d[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int i = i0 + e;
      float2 c = make_float2(0.f, 0.f);
      if (o < n_out && i < n_in) {
        c = spec[((int64_t)o * n_in + i) * H + f];
        if (f != 0) c.y = -c.y;
      }
      const f16x2 h = {(_Float16)(c.x * sc), (_Float16)(c.y * sc)};
      d[e] = __builtin_bit_cast(uint32_t, h);
    }
    img[idx] = make_uint4(d[0], d[1], d[2], d[3]);
  }
}

// The precise engine's residual image (SpecLayout::lo8): for every element of the STAT image's B
// fragments of the b = 128, K = 4096 geometry, e4m3(v s_o - fp16(v s_o)), v = conj(C) (fp32 packed
// spectra). 16 B per (group, wave, bin, K-step, lane): N-tile 0's 8 elements, then N-tile 1's, in the
// fragment order of the fp16 image (input block i0 + e, (re, im)).
__global__ void bc_lo8_image_kernel(int n_out, const float2* __restrict__ spec, uint4* __restrict__ lo8,
                                    const uint32_t* __restrict__ osc) {
  constexpr int B = 128, H = 64, BW = 8, NW = 8, N_IN = 32;
  const int groups = (n_out + STAT_OUT_BLOCKS - 1) / STAT_OUT_BLOCKS;
  const int64_t total = (int64_t)groups * NW * BW * 2 * 64;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int lane = (int)(idx & 63);
    const int ks = (int)((idx >> 6) & 1);
    const int fb = (int)((idx >> 7) % BW);
    const int w = (int)((idx >> 7) / BW % NW);
    const int gq = (int)((idx >> 7) / BW / NW);
    const int f = w * BW + fb;
    uint32_t d[4];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      const int o = gq * STAT_OUT_BLOCKS + nt * 16 + (lane & 15);
      const float sc = o < n_out ? __uint_as_float((254u << 23) - osc[o]) : 1.f;
      const int i0 = ks * 16 + 4 * (lane >> 4);
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        float r[4];
#pragma unroll
        for (int e2 = 0; e2 < 2; ++e2) {
          const int i = i0 + 2 * half + e2;
          float2 c = make_float2(0.f, 0.f);
          if (o < n_out && i < N_IN) {
            c = spec[((int64_t)o * N_IN + i) * H + f];
            if (f != 0) c.y = -c.y;
          }
          const float vr = c.x * sc, vi = c.y * sc;
          r[2 * e2] = vr - (float)(_Float16)vr;
          r[2 * e2 + 1] = vi - (float)(_Float16)vi;
        }
        int pk = __builtin_amdgcn_cvt_pk_fp8_f32(r[0], r[1], 0, false);
        pk = __builtin_amdgcn_cvt_pk_fp8_f32(r[2], r[3], pk, true);
        d[2 * nt + half] = (uint32_t)pk;
      }
    }
    lo8[idx] = make_uint4(d[0], d[1], d[2], d[3]);
  }
}

}  // namespace bcfft

namespace {
// CU count of the CURRENT device, cached per device ordinal. Atomic slots: concurrent first
// calls from several threads race only to store the same value (a device's CU count does not
// change), so grid and workspace sizing stay consistent for every caller.
constexpr int kMaxDevices = 64;
std::atomic<int> g_cu_count[kMaxDevices];
int cu_count() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = -1;
  if (dev >= 0 && dev < kMaxDevices) {
    const int c = g_cu_count[dev].load(std::memory_order_relaxed);
    if (c > 0) return c;
  }
  int n = 0;
  if (dev < 0 || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
    n = 256;
  if (dev >= 0 && dev < kMaxDevices) g_cu_count[dev].store(n, std::memory_order_relaxed);
  return n;
}

}  // namespace
int bcfft::device_cu_count() { return cu_count(); }
namespace {

template <int B, int KS, int XT, bool YF32, bool GLU = false>
void launch_stat(const void* x, int64_t n, int n_out, const void* spec, const void* bias, int bias_dt,
                 void* y, hipStream_t s) {
  // GLU: n_out = gate blocks; the spectra hold groups x 32 interleaved gate/up blocks
  const int groups = GLU ? (n_out + 15) / 16 : (n_out + 31) / 32;
  const bcfft::SpecLayout sl = bcfft::spec_layout(GLU ? 32 * groups : n_out, 16 * KS, B);
  // one workgroup per CU (1-D grid, group = index % groups): every group gets cus/groups
  // workgroups, rounded either way, instead of a whole-XCD multiple (11 groups: 253 vs 176)
  const int64_t n_mtiles = (n + 3) / 4;
  int64_t total = cu_count();
  if (total > groups * n_mtiles) total = groups * n_mtiles;
  if (total < groups) total = groups;
  const uint32_t* stat = reinterpret_cast<const uint32_t*>(spec) + sl.stat_off_u32;
  const float* osc = reinterpret_cast<const float*>(spec) + sl.osc_off_u32;
  hipLaunchKernelGGL((bcfft::bc_forward_stat_kernel<B, KS, XT, YF32, GLU>), dim3((unsigned)total), dim3(512), 0, s,
                     x, n, n_out, stat, osc, bias, bias_dt, y);
}

template <int B, int KS>
bool launch_stat_dt(int xdt, bool yf32, const void* x, int64_t n, int n_out, const void* spec,
                    const void* bias, int bias_dt, void* y, hipStream_t s) {
  if (xdt == BCFFT_F32) launch_stat<B, KS, BCFFT_F32, true>(x, n, n_out, spec, bias, bias_dt, y, s);
  else if (xdt == BCFFT_F16 && yf32) launch_stat<B, KS, BCFFT_F16, true>(x, n, n_out, spec, bias, bias_dt, y, s);
  else if (xdt == BCFFT_F16) launch_stat<B, KS, BCFFT_F16, false>(x, n, n_out, spec, bias, bias_dt, y, s);
  else if (yf32) launch_stat<B, KS, BCFFT_BF16, true>(x, n, n_out, spec, bias, bias_dt, y, s);
  else launch_stat<B, KS, BCFFT_BF16, false>(x, n, n_out, spec, bias, bias_dt, y, s);
  return true;
}
template <int B, int KS>
void launch_glu_dt(int xdt, const void* x, int64_t n, int n_gate, const void* spec, void* h, hipStream_t s) {
  if (xdt == BCFFT_F32) launch_stat<B, KS, BCFFT_F32, true, true>(x, n, n_gate, spec, nullptr, BCFFT_NONE, h, s);
  else if (xdt == BCFFT_F16) launch_stat<B, KS, BCFFT_F16, false, true>(x, n, n_gate, spec, nullptr, BCFFT_NONE, h, s);
  else launch_stat<B, KS, BCFFT_BF16, false, true>(x, n, n_gate, spec, nullptr, BCFFT_NONE, h, s);
}
}  // namespace

namespace bcfft {
bool launch_forward_glu(int b, int n_in, int xdt, const void* x, int64_t n, int n_gate, const void* spec,
                        void* h, hipStream_t s) {
  if (!stat_eligible(n_in, b)) return false;
  if (b == 128) launch_glu_dt<128, 2>(xdt, x, n, n_gate, spec, h, s);
  else if (n_in == 64) launch_glu_dt<64, 4>(xdt, x, n, n_gate, spec, h, s);
  else launch_glu_dt<64, 2>(xdt, x, n, n_gate, spec, h, s);
  return true;
}

bool launch_forward_stat(int b, int n_in, int xdt, bool yf32, const void* x, int64_t n, int n_out,
                         const void* spec, const void* bias, int bias_dt, void* y, hipStream_t s) {
  if (!stat_eligible(n_in, b)) return false;
  if (b == 128) return launch_stat_dt<128, 2>(xdt, yf32, x, n, n_out, spec, bias, bias_dt, y, s);
  if (n_in == 64) return launch_stat_dt<64, 4>(xdt, yf32, x, n, n_out, spec, bias, bias_dt, y, s);
  return launch_stat_dt<64, 2>(xdt, yf32, x, n, n_out, spec, bias, bias_dt, y, s);
}

void launch_lo8_image(int n_out, void* spec, hipStream_t s) {
  const SpecLayout sl = spec_layout(n_out, 32, 128);
  if (sl.lo8_u32 == 0) return;
  const int64_t total = sl.lo8_u32 / 4;
  const unsigned blocks = (unsigned)((total + 255) / 256 < 65535 ? (total + 255) / 256 : 65535);
  hipLaunchKernelGGL(bc_lo8_image_kernel, dim3(blocks), dim3(256), 0, s, n_out, (const float2*)spec,
                     reinterpret_cast<uint4*>(reinterpret_cast<uint32_t*>(spec) + sl.lo8_off_u32),
                     reinterpret_cast<const uint32_t*>(spec) + sl.osc_off_u32);
}

void launch_stat_image(int b, int n_out, int n_in, void* spec, hipStream_t s) {
  if (dmk_geometry(n_in, b)) {                      // same scales, streamed per-chunk fragments
    launch_stat_scale(128, n_out, n_in, spec, s);
    launch_dmk_image(n_out, n_in, spec, s);
    return;
  }
  if (!stat_eligible(n_in, b) && !dm256_geometry(n_in, b) && !dm64k_geometry(n_in, b)) return;
  const SpecLayout sl = spec_layout(n_out, n_in, b);
  const int64_t total = (int64_t)sl.stat_groups * 8 * sl.stat_pieces * 64;
  const unsigned blocks = (unsigned)((total + 255) / 256 < 65535 ? (total + 255) / 256 : 65535);
  launch_stat_scale(b, n_out, n_in, spec, s);
  if (b == 256)
    hipLaunchKernelGGL(bc_stat_image_kernel<256>, dim3(blocks), dim3(256), 0, s, n_out, n_in, (float2*)spec);
  else if (b == 128)
    hipLaunchKernelGGL(bc_stat_image_kernel<128>, dim3(blocks), dim3(256), 0, s, n_out, n_in, (float2*)spec);
  else
    hipLaunchKernelGGL(bc_stat_image_kernel<64>, dim3(blocks), dim3(256), 0, s, n_out, n_in, (float2*)spec);
}
}  // namespace bcfft

#ifdef BCFFT_ANALYSIS
// analysis builds only: switches / stamp buffer of bc_forward_stat_kernel (this TU's copies).
// 1 skip MFMAs, 2 skip y stores, 4 skip forward FFT math, 8 skip inverse FFT math, 16 skip x DMA,
// 32 skip A-fragment LDS reads, 64 skip the A im-row transform
extern "C" int bcfft_set_ablation_stat(int flags) {
  return hipMemcpyToSymbol(HIP_SYMBOL(bcfft::g_ablate), &flags, sizeof(int)) == hipSuccess ? 0 : BCFFT_ERR_HIP;
}
// stamp slots per wave: 0 start | per M-tile it (base 1 + 7 (it % 8)): +0 loop top, +1 own x
// landed, +2 after B1, +3 after B2, +4 MFMAs + Y pairs done, +5 after B4, +6 inverse done | 63 end
extern "C" int bcfft_set_stamps_stat(void* buf) {
  unsigned long long* p = (unsigned long long*)buf;
  return hipMemcpyToSymbol(HIP_SYMBOL(bcfft::g_stamps), &p, sizeof(p)) == hipSuccess ? 0 : BCFFT_ERR_HIP;
}
#endif
