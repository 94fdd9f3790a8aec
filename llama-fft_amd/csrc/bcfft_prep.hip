// bcfft_prep.hip — weight preparation: the loss-aware circulant projection of
// BlockCirculantLinear.from_linear (patch_llama_fft.py:180-224, per block
// dense_block_to_circulant_column_loss_aware :82-128) as one launch over every b x b block.
//
// Reference arithmetic, per block W (b x b, dtype DT = the dense weight's dtype):
//   d[t]  = sum_r W[r, (r - t) mod b]           (:116-119, reduction rounded once to DT)
//   c[t]  = mean_r W[r, (r - t) mod b]          (:118)
//   num   = sum_t DT(c[t] * d[t])               (:124)
//   den   = max(DT(b * sum_t DT(c[t]^2)), eps)  (:125)
//   alpha = DT(num / den)                       (:126)
//   out   = DT(alpha * c[t])                    (:128), stored in the fp32 parameter (:219)
// Elementwise results are rounded to DT; reductions accumulate in fp64 (exact for fp16
// operands) and round to fp32 then DT, as oracle/bc_oracle.py:project_loss_aware states the
// reference's torch reductions (float accumulation, one rounding).
//
// Layout: thread t of a b-thread group owns diagonal t of one block; for each row r the
// group reads W[r, (r - t) mod b] over t = the whole row (one coalesced row segment), so every
// weight element is read exactly once. HBM-bound: b^2 * sizeof(DT) read + 4 b written per block.
#include "bcfft_device.h"

namespace bcfft {

template <int B>
__global__ __launch_bounds__(256) void bc_project_kernel(const void* __restrict__ w, int dt, int n_out,
                                                         int n_in, float eps, float* __restrict__ c) {
  constexpr int GPB = 256 / B;                 // blocks per workgroup
  __shared__ double red[2][256];
  __shared__ float alpha_s[GPB];
  const int tid = threadIdx.x, g = tid / B, t = tid % B;
  const int64_t blk = (int64_t)blockIdx.x * GPB + g;
  const bool live = blk < (int64_t)n_out * n_in;
  const int64_t K = (int64_t)n_in * B;
  double s = 0.0;
  if (live) {
    const int j = (int)(blk / n_in), i = (int)(blk % n_in);
    const int64_t base = (int64_t)j * B * K + (int64_t)i * B;
#pragma unroll 8
    for (int r = 0; r < B; ++r) s += (double)load_scalar(w, base + r * K + ((r - t) & (B - 1)), dt);
  }
  const float dsum = round_to((float)s, dt);                                        // :119
  const float cv = dt == BCFFT_F32 ? dsum / (float)B : round_to((float)(s / B), dt);  // :118
  red[0][tid] = (double)round_to(cv * dsum, dt);                                    // c * diag_sums
  red[1][tid] = (double)round_to(cv * cv, dt);                                      // c * c
  __syncthreads();
  if (t == 0) {
    double num = 0.0, cc = 0.0;
    for (int u = 0; u < B; ++u) {                 // fixed order: deterministic
      num += red[0][g * B + u];
      cc += red[1][g * B + u];
    }
    const float numr = round_to((float)num, dt);                                    // :124
    float den = round_to((float)B * round_to((float)cc, dt), dt);                   // :125
    const float e = round_to(eps, dt);
    den = den < e ? e : den;                      // clamp_min; NaN stays NaN like torch
    alpha_s[g] = round_to(numr / den, dt);                                          // :126
  }
  __syncthreads();
  if (live) c[blk * B + t] = round_to(alpha_s[g] * cv, dt);                         // :128
}

bool launch_project(int b, const void* w, int dt, int n_out, int n_in, float eps, float* c, hipStream_t s) {
  const int64_t nblk = (int64_t)n_out * n_in;
  auto go = [&](auto kern, int gpb) {
    hipLaunchKernelGGL(kern, dim3((unsigned)((nblk + gpb - 1) / gpb)), dim3(256), 0, s, w, dt, n_out, n_in, eps, c);
  };
  switch (b) {
    case 32: go(bc_project_kernel<32>, 8); return true;
    case 64: go(bc_project_kernel<64>, 4); return true;
    case 128: go(bc_project_kernel<128>, 2); return true;
    case 256: go(bc_project_kernel<256>, 1); return true;
    default: return false;
  }
}

}  // namespace bcfft
