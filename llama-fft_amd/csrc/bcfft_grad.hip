// bcfft_grad.hip — gradient of the BC forward with respect to the circulant columns c
// (SURVEY.md §8 f3). The reference gets it from torch autograd through
// BlockCirculantLinear.forward (patch_llama_fft.py:246-271: rfft, einsum "oif,nif->nof",
// irfft) when calibrate_bc.py:253-299 trains c; written out:
//   dc[o, i, :] = irfft( sum_n rfft(dy[n, o]) * conj(rfft(x[n, i])) )
//              = circular cross-correlation  sum_n sum_s dy[n, o, (s + t) mod b] x[n, i, s]
//
// Two launches, deterministic (no atomics):
//   bc_grad_c_kernel    grid (o-tile x i-tile, token split). Each workgroup streams its token
//                       range in sub-batches of TT tokens: x rows of its TI input blocks and dy
//                       rows of its TO output blocks -> LDS (fp32), one real FFT per row (the
//                       forward kernels' four-step Fft<B>, untangled in place into packed bins
//                       2X), then per bin f a register tile of SO x SI complex accumulators
//                       += DY' conj(X'). The partial sums go to the caller's workspace.
//   bc_grad_c_finish    per block (o, i): sums the splits in fixed order (fp64), inverse real
//                       DFT in fp64 (twiddle table), x 1/(4b) (the 2 x 2 of the packed bins and
//                       irfft's 1/b), rounded to c's dtype.
// Bound: VALU (complex MACs 8 nO nI (b/2) flop per token, plus the row FFTs); HBM traffic is
// x and dy read (nO/TO and nI/TI times from L2) plus the workspace.
#include "bcfft_device.h"

#ifndef BCFFT_GRAD_ABL
#define BCFFT_GRAD_ABL 0   // analysis builds only: 1 skip MACs, 2 skip FFTs, 4 skip global loads
#endif

namespace bcfft {

template <int B>
struct GeoG {
  using F = Fft<B>;
  static constexpr int H = B / 2, L = F::L, SROW = F::SROW;
  static constexpr int NT = 256;
  static constexpr int PG = NT / H;                       // pair groups (threads per bin)
  static constexpr int PGO = PG >= 8 ? 4 : 2;             // pair groups along outputs
  static constexpr int PGI = PG / PGO;                    // ... along inputs
  static constexpr int SO = 8, SI = 8;                    // accumulator tile per thread
  static constexpr int TO = PGO * SO, TI = PGI * SI;      // blocks per workgroup tile
  static constexpr int TT = B == 256 ? 2 : 4;             // tokens per sub-batch
  static constexpr int RPT = TO + TI;                     // rows per token
  static constexpr int ROWS = RPT * TT;
  static constexpr int NG = NT / L;                       // FFT groups
  static constexpr int TW_FLOATS = 2 * B;
  static constexpr int LDS_FLOATS = TW_FLOATS + ROWS * SROW;
  static_assert(PGO * PGI == PG, "pair groups");
  static_assert(LDS_FLOATS * 4 <= 80 * 1024, "two workgroups per CU");
};

// 8 consecutive elements of a row (16-B aligned; fp32 = two 16-B loads) -> fp32
__device__ __forceinline__ void load8(const void* p, int64_t e, int dt, float (&f)[8]) {
  if (dt == BCFFT_F32) {
    const float4 a = *reinterpret_cast<const float4*>((const float*)p + e);
    const float4 b = *reinterpret_cast<const float4*>((const float*)p + e + 4);
    f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
  } else {
    const uint4 v = *reinterpret_cast<const uint4*>((const uint16_t*)p + e);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float2 u = dt == BCFFT_BF16 ? unpack16<BCFFT_BF16>(w[k]) : unpack16<BCFFT_F16>(w[k]);
      f[2 * k] = u.x;
      f[2 * k + 1] = u.y;
    }
  }
}

template <int B>
__global__ __launch_bounds__(256) void bc_grad_c_kernel(const void* __restrict__ x, int x_dt,
                                                        const void* __restrict__ dy, int dy_dt,
                                                        int64_t n_tokens, int n_in, int n_out,
                                                        int64_t tokens_per_split, int64_t n_splits,
                                                        float2* __restrict__ ws) {
  using G = GeoG<B>;
  using F = Fft<B>;
  constexpr int H = G::H, L = G::L, SROW = G::SROW, TT = G::TT, RPT = G::RPT;
  __shared__ __attribute__((aligned(16))) float lds[G::LDS_FLOATS];
  float2* tw = reinterpret_cast<float2*>(lds);
  float* rows = lds + G::TW_FLOATS;

  const int tid = threadIdx.x;
  const int n_ti = (n_in + G::TI - 1) / G::TI;
  const int n_tiles = ((n_out + G::TO - 1) / G::TO) * n_ti;
  // XCD-aware 1-D grid: blocks b and b + 8 share an XCD (and its L2), so the n_tiles
  // workgroups of one token split are blocks 8 q + xcd of consecutive q: they read the same
  // x / dy rows close in time through one L2 (each row is read by nO/TO resp. nI/TI tiles)
  const int64_t bq = blockIdx.x >> 3;
  const int tile = (int)(bq % n_tiles);
  const int64_t split = (bq / n_tiles) * 8 + (blockIdx.x & 7);
  if (split >= n_splits) return;
  const int o0 = (tile / n_ti) * G::TO, i0 = (tile % n_ti) * G::TI;
  const int64_t nb = split * tokens_per_split;
  const int64_t ne = nb + tokens_per_split < n_tokens ? nb + tokens_per_split : n_tokens;
  const int64_t K = (int64_t)n_in * B, M = (int64_t)n_out * B;

  for (int m = tid; m < B; m += G::NT) {
    double s, c;
    sincospi(2.0 * (double)m / (double)B, &s, &c);
    tw[m] = make_float2((float)c, (float)(-s));
  }

  const int f = tid % H, pg = tid / H;
  const int ol = (pg % G::PGO) * G::SO, il = (pg / G::PGO) * G::SI;
  const bool bin0 = f == 0;
  float2 acc[G::SO][G::SI];
#pragma unroll
  for (int a = 0; a < G::SO; ++a)
#pragma unroll
    for (int b = 0; b < G::SI; ++b) acc[a][b] = make_float2(0.f, 0.f);

  const int g = tid / L, gl = tid % L;
  for (int64_t n0 = nb; n0 < ne; n0 += TT) {
    __syncthreads();
    // rows: token t, then TI x blocks, then TO dy blocks; 8 elements per unit
    for (int u = tid; u < G::ROWS * (B / 8); u += G::NT) {
      const int r = u / (B / 8), v = u % (B / 8);
      const int t = r / RPT, bl = r % RPT;
      const int64_t n = n0 + t;
      float e[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (n < ne && !(BCFFT_GRAD_ABL & 4)) {
        if (bl < G::TI) {
          if (i0 + bl < n_in) load8(x, n * K + (int64_t)(i0 + bl) * B + 8 * v, x_dt, e);
        } else if (o0 + bl - G::TI < n_out) {
          load8(dy, n * M + (int64_t)(o0 + bl - G::TI) * B + 8 * v, dy_dt, e);
        }
      }
      float* d = rows + r * SROW + 8 * v;
      *reinterpret_cast<float4*>(d) = make_float4(e[0], e[1], e[2], e[3]);
      *reinterpret_cast<float4*>(d + 4) = make_float4(e[4], e[5], e[6], e[7]);
    }
    __syncthreads();
    for (int r = g; r < G::ROWS && !(BCFFT_GRAD_ABL & 2); r += G::NG) {   // whole waves: same trip count
      float* row = rows + r * SROW;
      F::template forward<BCFFT_F32>(row, gl, tw);
      // untangle in place: the lane that reads Z[k] and Z[H-k] writes X'[k] and X'[H-k]
      for (int k = gl; k <= H / 2; k += L) {
        const int m = (H - k) & (H - 1);
        const float2 zk = *reinterpret_cast<const float2*>(row + 2 * k);
        const float2 zm = *reinterpret_cast<const float2*>(row + 2 * m);
        auto unt = [&](float2 za, float2 zb, float2 w) {
          const float sr = za.x + zb.x, si = za.y - zb.y, dr = za.x - zb.x, di = za.y + zb.y;
          return make_float2(sr + w.x * di + w.y * dr, si - w.x * dr + w.y * di);
        };
        if (k == 0) {
          *reinterpret_cast<float2*>(row) = make_float2(2.f * (zk.x + zk.y), 2.f * (zk.x - zk.y));
        } else {
          const float2 xk = unt(zk, zm, tw[k]);
          const float2 xm = unt(zm, zk, tw[m]);
          *reinterpret_cast<float2*>(row + 2 * k) = xk;
          if (m != k) *reinterpret_cast<float2*>(row + 2 * m) = xm;
        }
      }
    }
    __syncthreads();
#pragma unroll 1
    for (int t = 0; t < TT && !(BCFFT_GRAD_ABL & 1); ++t) {
      const float* rt = rows + t * RPT * SROW + 2 * f;
      float xr[G::SI], xa[G::SI], xb[G::SI];
#pragma unroll
      for (int b = 0; b < G::SI; ++b) {
        const float2 v = *reinterpret_cast<const float2*>(rt + (il + b) * SROW);
        xr[b] = v.x;
        xa[b] = bin0 ? 0.f : v.y;     // packed bin 0: (X0, X_H) both real
        xb[b] = bin0 ? v.y : v.x;
      }
#pragma unroll
      for (int a = 0; a < G::SO; ++a) {
        const float2 d = *reinterpret_cast<const float2*>(rt + (G::TI + ol + a) * SROW);
#pragma unroll
        for (int b = 0; b < G::SI; ++b) {   // DY conj(X): (d.x xr + d.y xa, d.y xb - d.x xa)
          acc[a][b].x = fmaf(d.x, xr[b], fmaf(d.y, xa[b], acc[a][b].x));
          acc[a][b].y = fmaf(d.y, xb[b], fmaf(-d.x, xa[b], acc[a][b].y));
        }
      }
    }
  }
  const int64_t split_off = split * n_out * n_in;
#pragma unroll
  for (int a = 0; a < G::SO; ++a)
#pragma unroll
    for (int b = 0; b < G::SI; ++b) {
      const int o = o0 + ol + a, i = i0 + il + b;
      if (o < n_out && i < n_in) ws[((split_off + (int64_t)o * n_in + i) * H) + f] = acc[a][b];
    }
}

template <int B>
__global__ __launch_bounds__(256) void bc_grad_c_finish(const float2* __restrict__ ws, int n_splits,
                                                        int n_out, int n_in, int dc_dt, void* __restrict__ dc) {
  // per block (o, i): 256 threads = H bins x SG split groups. Thread (k, sg) sums splits
  // s = sg, sg + SG, ... (coalesced over k, 8 loads in flight); the SG partials are then added
  // in a fixed order (deterministic).
  constexpr int H = B / 2, SG = 256 / H;
  __shared__ double pr[SG][H], pi[SG][H];
  __shared__ double ar[H], ai[H];
  const int64_t blk = blockIdx.x;
  const int tid = threadIdx.x, k = tid % H, sg = tid / H;
  const int64_t stride = (int64_t)n_out * n_in * H;
  const float2* src = ws + blk * H + k;
  double re = 0.0, im = 0.0;
  int s = sg;
  for (; s + 7 * SG < n_splits; s += 8 * SG) {
    float2 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = src[(int64_t)(s + u * SG) * stride];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      re += v[u].x;
      im += v[u].y;
    }
  }
  for (; s < n_splits; s += SG) {
    const float2 v = src[(int64_t)s * stride];
    re += v.x;
    im += v.y;
  }
  pr[sg][k] = re;
  pi[sg][k] = im;
  __syncthreads();
  if (tid < H) {
    double a = 0.0, b = 0.0;
#pragma unroll
    for (int g = 0; g < SG; ++g) {
      a += pr[g][tid];
      b += pi[g][tid];
    }
    ar[tid] = a;
    ai[tid] = b;
  }
  __syncthreads();
  // inverse real DFT of the packed bins, fp64: y[t] = A0 + (-1)^t A_H + 2 sum_k Re(A_k e^{2 pi i k t / B});
  // the per-t twiddle e^{2 pi i t / B} advances by a fp64 complex recurrence (error ~H ulp of fp64)
  for (int t = tid; t < B; t += 256) {
    double st, ct;
    sincospi(2.0 * (double)t / (double)B, &st, &ct);
    double wr = ct, wi = st, acc = 0.0;
    for (int kk = 1; kk < H; ++kk) {
      acc += ar[kk] * wr - ai[kk] * wi;
      const double nr = wr * ct - wi * st;
      wi = wr * st + wi * ct;
      wr = nr;
    }
    const double y = ar[0] + ((t & 1) ? -ai[0] : ai[0]) + 2.0 * acc;
    const float v = (float)(y / (4.0 * B));
    if (dc_dt == BCFFT_F32) ((float*)dc)[blk * B + t] = v;
    else ((uint16_t*)dc)[blk * B + t] = (uint16_t)(dc_dt == BCFFT_BF16 ? f32_to_bf16(v) : f32_to_f16(v));
  }
}

// token split: two workgroups per CU (their LDS / VGPR limit), at least one sub-batch each
template <int B>
GradPlan grad_plan_b(int64_t n, int n_in, int n_out) {
  using G = GeoG<B>;
  GradPlan p;
  p.tiles = (int64_t)((n_out + G::TO - 1) / G::TO) * ((n_in + G::TI - 1) / G::TI);
  int64_t s = (512 + p.tiles - 1) / p.tiles;
  const int64_t sub = (n + G::TT - 1) / G::TT;
  if (s > sub) s = sub;
  if (s < 1) s = 1;
  const int64_t per = (n + s - 1) / s;
  p.tokens_per_split = (per + G::TT - 1) / G::TT * G::TT;
  p.splits = n > 0 ? (n + p.tokens_per_split - 1) / p.tokens_per_split : 0;
  p.workspace_bytes = p.splits * (int64_t)n_out * n_in * (B / 2) * 8;
  return p;
}

GradPlan grad_plan(int b, int64_t n, int n_in, int n_out) {
  switch (b) {
    case 32: return grad_plan_b<32>(n, n_in, n_out);
    case 64: return grad_plan_b<64>(n, n_in, n_out);
    case 128: return grad_plan_b<128>(n, n_in, n_out);
    default: return grad_plan_b<256>(n, n_in, n_out);
  }
}

template <int B>
void launch_grad_c_b(const void* x, int x_dt, const void* dy, int dy_dt, int64_t n, int n_in, int n_out,
                     void* ws, void* dc, int dc_dt, hipStream_t s) {
  const GradPlan p = grad_plan_b<B>(n, n_in, n_out);
  if (p.splits > 0)
    hipLaunchKernelGGL(bc_grad_c_kernel<B>, dim3((unsigned)(p.tiles * ((p.splits + 7) / 8) * 8)), dim3(GeoG<B>::NT),
                       0, s, x, x_dt, dy, dy_dt, n, n_in, n_out, p.tokens_per_split, p.splits, (float2*)ws);
  hipLaunchKernelGGL(bc_grad_c_finish<B>, dim3((unsigned)((int64_t)n_out * n_in)), dim3(256), 0, s,
                     (const float2*)ws, (int)p.splits, n_out, n_in, dc_dt, dc);
}

void launch_grad_c(int b, const void* x, int x_dt, const void* dy, int dy_dt, int64_t n, int n_in, int n_out,
                   void* ws, void* dc, int dc_dt, hipStream_t s) {
  switch (b) {
    case 32: launch_grad_c_b<32>(x, x_dt, dy, dy_dt, n, n_in, n_out, ws, dc, dc_dt, s); break;
    case 64: launch_grad_c_b<64>(x, x_dt, dy, dy_dt, n, n_in, n_out, ws, dc, dc_dt, s); break;
    case 128: launch_grad_c_b<128>(x, x_dt, dy, dy_dt, n, n_in, n_out, ws, dc, dc_dt, s); break;
    default: launch_grad_c_b<256>(x, x_dt, dy, dy_dt, n, n_in, n_out, ws, dc, dc_dt, s); break;
  }
}

}  // namespace bcfft
