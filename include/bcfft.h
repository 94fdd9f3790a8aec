/*
 * bcfft.h — C ABI of the MI355X block-circulant (BC) linear engine (libbcfft.so).
 *
 * This is the drop-in boundary BELOW the reference's Python module API. The reference
 * (Pinguhat/llama-fft) has no FFI of its own: every entry point here replaces a torch call
 * sequence inside its module, cited per function (paths relative to the reference's src/).
 * The Python mirror of the module API (llama-fft_amd/patch_llama_fft.py) binds these with
 * ctypes; INTEGRATION.md shows the binding.
 *
 * Conventions
 *  - Plain pointers and sizes only; every buffer is caller-owned device memory (torch's
 *    allocator in the Python layer). No entry point allocates, frees or synchronises.
 *  - `stream` is a hipStream_t passed as void* (NULL = legacy default stream). Work is
 *    enqueued asynchronously; entry points are reentrant. The only global state is a per-device
 *    cache of the CU count (atomic slots, filled on first use per device ordinal), which sizes
 *    persistent grids and split-K workspaces for the CURRENT device.
 *  - Return value: BCFFT_OK (0) or a BCFFT_ERR_* status. Shape/dtype/alignment problems are
 *    reported before anything is launched. bcfft_status_string() gives a message.
 *  - dtype codes: BCFFT_F32, BCFFT_F16, BCFFT_BF16 (BCFFT_NONE for "no bias").
 *  - Block sizes: 32, 64, 128, 256 (power-of-two b with the 4- or 8-lane four-step FFT).
 */
#ifndef BCFFT_H
#define BCFFT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BCFFT_ABI_VERSION 1

enum bcfft_dtype { BCFFT_NONE = -1, BCFFT_F32 = 0, BCFFT_F16 = 1, BCFFT_BF16 = 2 };

/* Forward algorithms (bcfft_forward_algo). All are single fused launches.
 *  STAT: stationary weights. One persistent workgroup per CU keeps its output group's weight
 *        spectra in VGPRs as fp16 MFMA fragments (scaled by a power of two) for the whole
 *        launch, and streams tokens in tiles of 4. X is split into fp16 hi + lo under a
 *        per-token power-of-two scale, with fp32 accumulation: ~3e-4 relative (the fp16
 *        rounding of the weight spectra), inside the 1e-3 contract.
 *        Geometries: block_size 128 with in_features 4096, block_size 64 with in_features
 *        2048 or 4096; any out_features. BCFFT_ERR_BLOCK for others.
 *  MFMA: per-bin complex MAC on the matrix cores as a bf16 GEMM with hi/lo splitting of both
 *        operands ((Xhi+Xlo)(Chi+Clo), fp32 accumulate; ~1e-5 relative). block_size <= 128.
 *  VALU: per-bin complex MAC in fp32 FMAs (the reference's fp32 arithmetic). Any block size.
 *  DFT:  the STAT weights, with the forward and inverse DFTs of the blocks also on the matrix
 *        cores (dense fp16 GEMMs against a 2^-7-scaled DFT table, even/odd split) instead of
 *        VALU FFTs; ~3.5e-4 relative (fp16 outputs: as DFTX). Geometry: block_size 128 with
 *        in_features 4096; block_size 64 with in_features 4096 and bf16 I/O; and block_size 128
 *        with 4096 < in_features <= 127 * 128 and bf16 I/O, where the weight spectra are
 *        streamed from L2 per 16-block K-chunk (the LLaMA down projection; bcfft_dmk.hip).
 *  DFTX: DFT with the per-bin products also split hi + lo before the inverse transform:
 *        ~2.8e-4 relative and linear in x to ~1e-6, ~6 % slower.
 *  DFTP: the precise engine: DFTX with the rounding residual of every single fp16 term (the DFT
 *        table in both transforms and the weight spectra) added back through fp8 MFMAs (in fp32
 *        accumulators of their own, joined to the fp16 products'): ~2e-5 relative, per token
 *        ~1e-5 times its cancellation (the reference's fp32 arithmetic class). Geometry as DFTX;
 *        fp32 outputs: fp32 x with no, an fp32 or a 16-bit bias, 16-bit x with no or an fp32 bias
 *        (16-bit outputs run DFTX, whose error already sits below the 16-bit rounding the
 *        reference applies to the output, patch_llama_fft.py:266).
 *  AUTO: at block_size 128 with in_features 4096, DFTX for fp32 outputs (linear in x, which the
 *        fp32 backward's dx relies on) and DFT for 16-bit outputs (whose own rounding dominates);
 *        DFT on its other geometries; else STAT where eligible, else MFMA for block_size <= 128,
 *        else VALU. */
enum bcfft_algo { BCFFT_ALGO_AUTO = 0, BCFFT_ALGO_MFMA = 1, BCFFT_ALGO_VALU = 2, BCFFT_ALGO_STAT = 3,
                  BCFFT_ALGO_DFT = 4, BCFFT_ALGO_DFTX = 5, BCFFT_ALGO_DFTP = 6, BCFFT_ALGO_SHORT = 7 };
/* BCFFT_ALGO_SHORT: the short-N DFT kernel (one workgroup per 4-token tile and 16 output blocks,
 * the exact hi + lo arithmetic of DFTX) for the STAT geometries (b = 128 with K = 4096; b = 64 with
 * K = 2048 or 4096). AUTO takes it for those geometries at token counts whose persistent-kernel
 * grid would leave most CUs idle (decode steps, BASELINE config 1). */

enum bcfft_status {
  BCFFT_OK = 0,
  BCFFT_ERR_SHAPE = 1,   /* features not divisible by block_size, non-positive sizes      */
  BCFFT_ERR_BLOCK = 2,   /* unsupported block_size                                          */
  BCFFT_ERR_DTYPE = 3,   /* unsupported dtype code / output dtype != promote(x, bias)       */
  BCFFT_ERR_ALIGN = 4,   /* x / y / spectra not 16-byte aligned                              */
  BCFFT_ERR_HIP = 5,     /* a HIP launch failed (bcfft_last_hip_error() has the text)        */
  BCFFT_ERR_ARG = 6      /* NULL pointer where one is required                               */
};

/* ABI version of the loaded library (== BCFFT_ABI_VERSION it was built with). */
int bcfft_abi_version(void);

/* Human-readable text for a status code. */
const char* bcfft_status_string(int status);

/* Text of the last HIP error seen by this thread (empty if none). */
const char* bcfft_last_hip_error(void);

/* Why the last bcfft_forward* call of this thread returned BCFFT_ERR_BLOCK: the engine that was
 * asked for and the geometry / dtypes it does not serve (empty if the call was not refused). */
const char* bcfft_last_error_detail(void);

/* Bytes of the spectra buffer of an operator with (n_out_blocks x n_in_blocks) b x b
 * circulant blocks: packed fp32 bins (n_out*n_in*b/2 complex64), a b-entry twiddle table,
 * for b <= 128 the split-bf16 image the MFMA kernel streams and, for STAT geometries, the
 * scaled fp16 fragment image the STAT kernel keeps in registers. */
int64_t bcfft_spectra_bytes(int n_out_blocks, int n_in_blocks, int block_size);

/* Packed weight spectra. Replaces `Cf = torch.fft.rfft(self.c.to(float32), dim=-1)`
 * (patch_llama_fft.py:256-257) and the memoised Cf of the cached forward
 * (bench_all_in_one.py:204-216).
 * n_out_blocks / n_in_blocks describe the OPERATOR whose spectra are built:
 *   transpose_conj = 0: the layer itself; c is (n_out_blocks, n_in_blocks, block_size).
 *   transpose_conj = 1: its adjoint (used for dL/dx in the backward pass); c is the layer's
 *                       (n_in_blocks, n_out_blocks, block_size) tensor and the operator's
 *                       block (o, i) is conj(spectrum of c[i, o]).
 *   spectra:  bcfft_spectra_bytes(n_out_blocks, n_in_blocks, block_size) bytes, 16-B aligned;
 *             S[o][i][k] = rfft(c_op[o,i])[k] / (2b) for 0<k<b/2, S[o][i][0] = (X0, X_{b/2})/(2b)
 * Computed in fp64 and rounded once to fp32 (the bf16 image is split from those values). */
int bcfft_spectra(const void* c, int c_dtype, int n_out_blocks, int n_in_blocks, int block_size,
                  int transpose_conj, void* spectra, void* stream);

/* Fused BC forward. Replaces BlockCirculantLinear.forward's body
 * (patch_llama_fft.py:246-271: reshape, .to(fp32), rfft, einsum "oif,nif->nof", irfft,
 * .to(x.dtype), + bias) with ONE kernel launch.
 *   x:  (n_tokens, in_features) row-major, dtype x_dtype, 16-B aligned
 *   y:  (n_tokens, out_features) row-major, y_dtype == promote(x_dtype, bias_dtype)
 *   bias: (out_features,) of bias_dtype, or NULL with bias_dtype = BCFFT_NONE
 * Numerics follow the reference: fp32 spectra math, result rounded to x_dtype, then the
 * bias added in fp32 and the sum rounded to y_dtype. n_tokens == 0 is a no-op. */
int bcfft_forward(const void* x, int x_dtype, int64_t n_tokens, int in_features,
                  int out_features, int block_size, const void* spectra, const void* bias,
                  int bias_dtype, void* y, int y_dtype, void* stream);

/* bcfft_forward with an explicit algorithm (enum bcfft_algo). */
int bcfft_forward_algo(const void* x, int x_dtype, int64_t n_tokens, int in_features,
                       int out_features, int block_size, const void* spectra, const void* bias,
                       int bias_dtype, void* y, int y_dtype, int algo, void* stream);

/* The engine (enum bcfft_algo, AUTO resolved) that bcfft_forward_ws runs for these sizes and I/O
 * dtypes with the workspace bcfft_forward_workspace_bytes_io asks for; < 0 where it would refuse
 * the call. Host logic: nothing is launched. Replaces nothing in the reference (its forward has one
 * code path); benchmarks and tests use it to name what they time. BCFFT_ALGO_DFTP resolves to
 * BCFFT_ALGO_DFTX unless y is fp32 (the precise engine's forms: fp32 x with any bias, 16-bit x with
 * no or an fp32 bias); a 16-bit bias on 16-bit x with an fp32 y, which this query does not see,
 * also runs DFTX. */
int bcfft_forward_resolve(int64_t n_tokens, int in_features, int out_features, int block_size, int algo,
                          int x_dtype, int y_dtype);

/* The kernel symbol (e.g. "bc_forward_dm_kernel") that call runs: each launcher's own choice
 * between its per-group, multi-group and K-split forms for the current device's CU count; ""
 * where the call would be refused. */
const char* bcfft_forward_kernel_name(int64_t n_tokens, int in_features, int out_features, int block_size,
                                      int algo, int x_dtype, int y_dtype);

/* Optional workspace of bcfft_forward_ws, in bytes (0: the forward never uses one; < 0:
 * invalid geometry). Non-zero only where the split-bf16 MFMA kernel or the VALU kernel (algo,
 * AUTO resolved) runs a grid too short to fill the device (MFMA: n_tokens < 8 x CUs) over >= 4
 * chunks of input blocks, e.g.
 * LLaMA's 11008 -> 4096 down projection at prefill and decode sizes: it then splits the input
 * blocks over kz >= 2 workgroup slices (as many as fill two workgroups per CU, >= 2 chunks of 8
 * input blocks each) that write fp32 partial outputs to the workspace (kz x n_tokens x
 * out_features floats), and a finishing pass adds them in a fixed order and applies the
 * epilogue: bit-reproducible, and identical per output block for q/k/v-style concatenations. */
int64_t bcfft_forward_workspace_bytes(int64_t n_tokens, int in_features, int out_features, int block_size,
                                      int algo);

/* The same for known I/O dtypes (y_dtype = promote(x_dtype, bias_dtype)). Besides the MFMA / VALU
 * splits above, this also sizes the K-chunk split of the bf16 streamed-weight DFT kernel (b = 128,
 * K > 4096: the down projection) at decode sizes (at most 1/16 of the CUs' worth of 8-token tiles
 * x output groups): up to 6 slices of its 16-block K-chunks write fp32 partials (kz x n_tokens x
 * out_features floats) that a finishing pass sums in order, rounds and biases. AUTO then resolves
 * exactly as bcfft_forward_ws will, so geometries that run a DFT engine for these dtypes (e.g. the
 * bf16 down projection on the streamed-weight kernel) report 0. < 0 for invalid arguments. */
int64_t bcfft_forward_workspace_bytes_io(int64_t n_tokens, int in_features, int out_features, int block_size,
                                         int algo, int x_dtype, int y_dtype);

/* bcfft_forward_algo with a caller-owned device workspace (16-B aligned), used when
 * workspace_bytes >= bcfft_forward_workspace_bytes(...); NULL / too small runs unsplit. */
int bcfft_forward_ws(const void* x, int x_dtype, int64_t n_tokens, int in_features,
                     int out_features, int block_size, const void* spectra, const void* bias,
                     int bias_dtype, void* y, int y_dtype, int algo, void* workspace,
                     int64_t workspace_bytes, void* stream);

/* Fused gate/up projections + SwiGLU of a LLaMA MLP (the reference MLP
 * computes down(act(gate(x)) * up(x)) with gate/up BC-patched by patch_llama_fft.py:343-394;
 * act = SiLU): h = silu(BC_gate(x)) * BC_up(x) in ONE launch, without writing gate(x) and up(x)
 * to memory. spectra_gu = bcfft_spectra of the interleaved weight c_gu of shape
 * (32 * ceil(gate_blocks / 16), in_blocks, b): group g's 32 blocks are gate blocks [16g, 16g+16)
 * then up blocks [16g, 16g+16), zero past the last gate block (bcfft.ops.glu_weights builds it).
 *   x: (n_tokens, in_features), h: (n_tokens, gate_features), both x_dtype, 16-B aligned
 * Geometries: b = 128 with K = 4096 (the DFT kernels, group g's gate blocks in its first N-tile
 * and up blocks in its second; several groups with bf16 x: the multi-group kernel); b = 64 with
 * K in {2048, 4096} (stationary kernel; bf16 x at K = 4096: the b = 64 DFT kernels); b = 256 with
 * K = 4096 and bf16 x only (the b = 256 multi-group DFT kernel: each group split into 8 gate + 8
 * up columns); else BCFFT_ERR_BLOCK. No bias (LLaMA's gate/up have none). Numerics follow torch
 * on the reference's tensors: gate and up rounded to x_dtype, silu(gate) rounded, the product
 * rounded. */
int bcfft_forward_glu(const void* x, int x_dtype, int64_t n_tokens, int in_features, int gate_features,
                      int block_size, const void* spectra_gu, void* h, void* stream);

/* bcfft_forward_glu with an engine choice: AUTO (bcfft_forward_glu) runs the DFT kernel at b = 128
 * with K = 4096 (DFTX for fp32 x), the b = 64 DFT kernel for bf16 x at b = 64, K = 4096, the b = 256
 * one for bf16 x at b = 256, K = 4096, and the stationary kernel on the other stationary
 * geometries; STAT, DFT and DFTX force one (BCFFT_ERR_BLOCK where it does not serve the
 * geometry; MFMA / VALU: BCFFT_ERR_ARG). */
int bcfft_forward_glu_algo(const void* x, int x_dtype, int64_t n_tokens, int in_features, int gate_features,
                           int block_size, const void* spectra_gu, void* h, int algo, void* stream);

/* Fused BC-MLP: y = BC_down( silu(BC_gate(x)) * BC_up(x) ), the LLaMA MLP of
 * patch_mlp_with_block_circulant (patch_llama_fft.py:343-394) as the reference times it
 * (microbench_dense_vs_bc.py:183-188, `--bench_mlp`: bc_down(F.silu(bc_gate(x)) * bc_up(x))).
 *   x, y: (n_tokens, hidden_features), x_dtype, 16-B aligned
 *   spectra_gu:   bcfft_spectra of the interleaved gate/up weight (as bcfft_forward_glu's)
 *   spectra_down: bcfft_spectra of the down weight (hidden/b x inter/b blocks)
 * Modes:
 *   FUSED: ONE launch (bcfft_dmm.hip). h never leaves the CU: its 180 MB HBM round trip at 8192
 *          LLaMA-7B tokens disappears. Geometry: bf16, block_size 128, hidden 4096,
 *          4096 < intermediate <= 127 * 128 (LLaMA-7B's 11008); else BCFFT_ERR_BLOCK. The output is
 *          bit-identical to SPLIT's where SPLIT runs the 8-token streamed-weight down kernel.
 *   SPLIT: bcfft_forward_glu into the caller's workspace (h), then bcfft_forward (AUTO engines).
 *   AUTO:  on the fused geometry FUSED_SPLITK (below) at short grids, FUSED once its 8-token
 *          tiles fill the CUs (last round >= 3/4 full), else SPLIT.
 * workspace: bcfft_forward_mlp_workspace_bytes(...) bytes (0 for FUSED; may then be NULL). */
enum bcfft_mlp_mode { BCFFT_MLP_AUTO = 0, BCFFT_MLP_FUSED = 1, BCFFT_MLP_SPLIT = 2, BCFFT_MLP_FUSED_SPLITK = 3 };

/* FUSED_SPLITK: the fused kernel with its gate/up groups (= the down projection's K-chunks) split
 * over up to 6 workgroups per 8-token tile, each writing an fp32 partial y to the workspace
 * (kz x n_tokens x hidden floats), plus a finishing pass that sums them in order and rounds: for
 * short grids (decode, short prefill), where the one-launch kernel would leave most CUs idle.
 * Deterministic; not bit-identical to FUSED / SPLIT (each slice has its own down-projection
 * reference exponents). AUTO takes it where the fused geometry applies and FUSED's tiles would
 * fill at most half the CUs (N <= 1024 on 256 CUs: 17-50 us vs 52-57 us one launch), FUSED past
 * that while its tiles fill the CUs. bcfft_forward_mlp_mode returns the mode a call resolves to. */
int bcfft_forward_mlp_mode(int64_t n_tokens, int hidden_features, int inter_features, int block_size, int x_dtype,
                           int mode);

int64_t bcfft_forward_mlp_workspace_bytes(int64_t n_tokens, int hidden_features, int inter_features, int block_size,
                                          int x_dtype, int mode);

int bcfft_forward_mlp(const void* x, int x_dtype, int64_t n_tokens, int hidden_features, int inter_features,
                      int block_size, const void* spectra_gu, const void* spectra_down, void* y, int mode,
                      void* workspace, int64_t workspace_bytes, void* stream);

/* Loss-aware circulant projection of a dense weight. Replaces the per-block
 * Python loop of BlockCirculantLinear.from_linear (patch_llama_fft.py:207-219) over
 * dense_block_to_circulant_column_loss_aware (:82-128) with one launch:
 *   c[j,i,t] = alpha_ji * mean_r W[j*b + r, i*b + (r - t) mod b],
 *   alpha_ji = <W_ji, C(c)> / max(b * sum_t c[t]^2, 1e-12)
 * in the reference's arithmetic: every elementwise result rounded to w_dtype, reductions
 * accumulated wider and rounded once (fp16 weights: bit-identical to the reference's CPU loop
 * on its golden vectors).
 *   w: (out_features, in_features) row-major, w_dtype; c: (out/b, in/b, b) fp32 (the module's
 *   parameter dtype, :219). */
int bcfft_project_circulant(const void* w, int w_dtype, int out_features, int in_features, int block_size,
                            float* c, void* stream);

/* Workspace bytes bcfft_grad_c needs for these sizes (0 when n_tokens == 0). */
int64_t bcfft_grad_c_workspace_bytes(int64_t n_tokens, int in_features, int out_features, int block_size);

/* Gradient of the BC forward with respect to c: what torch autograd computes
 * through patch_llama_fft.py:246-271 for calibrate_bc.py:253-299,
 *   dc[o,i,:] = irfft( sum_n rfft(dy[n,o]) * conj(rfft(x[n,i])) )   (circular cross-correlation)
 * fp32 FFTs and accumulation, splits summed in fp64 in a fixed order (deterministic).
 *   x: (n_tokens, in_features) x_dtype; dy: (n_tokens, out_features) dy_dtype; both 16-B aligned
 *   workspace: bcfft_grad_c_workspace_bytes(...) bytes, 16-B aligned (may be NULL if 0)
 *   dc: (out/b, in/b, b) of dc_dtype (the parameter's dtype), fully overwritten. */
int bcfft_grad_c(const void* x, int x_dtype, const void* dy, int dy_dtype, int64_t n_tokens, int in_features,
                 int out_features, int block_size, void* workspace, void* dc, int dc_dtype, void* stream);

/* Single circulant matvec y = C(c) x, C[i,j] = c[(i-j) mod n], any n >= 1.
 * Replaces fft_utils.circulant_matvec_fft (fft_utils.py:3-34); c, x, y share `dtype`.
 * Direct O(n^2) evaluation accumulated in fp64 (this entry point serves validation-sized
 * vectors; the layer path is bcfft_forward). */
int bcfft_circulant_matvec(const void* c, const void* x, int dtype, int n, void* y, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* BCFFT_H */
