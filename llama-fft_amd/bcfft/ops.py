"""Tensor-level wrappers over the C ABI (torch is plumbing: allocation, streams, autograd).

Every function here enqueues HIP work on the caller's current stream and returns without
synchronising. Shapes/dtypes are validated in Python (for the reference's exception types)
and again in the library (status codes).
"""
from __future__ import annotations

import os
import torch

from . import _lib


def spectra_numel(n_out_blocks: int, n_in_blocks: int, block_size: int) -> int:
    nbytes = _lib.load().bcfft_spectra_bytes(n_out_blocks, n_in_blocks, block_size)
    if nbytes < 0:
        raise ValueError(f"invalid spectra geometry ({n_out_blocks}, {n_in_blocks}, {block_size})")
    return nbytes // 4


def spectra(c: torch.Tensor, transpose_conj: bool = False) -> torch.Tensor:
    """Packed weight spectra of c (nO, nI, b) -> flat float32 device buffer.

    Replaces rfft(c.to(fp32)) (patch_llama_fft.py:256-257). transpose_conj=True gives the
    adjoint operator's spectra (used for dL/dx)."""
    _lib.require_device(c, "bcfft.spectra")
    if c.dim() != 3:
        raise ValueError("c must be (out_blocks, in_blocks, block_size)")
    n_out, n_in, b = c.shape
    if transpose_conj:                       # the adjoint operator has the swapped grid
        n_out, n_in = n_in, n_out
    if b not in _lib.SUPPORTED_BLOCKS:
        raise ValueError(f"block_size {b} not supported (supported: {_lib.SUPPORTED_BLOCKS})")
    c = c.detach().contiguous()
    out = torch.empty(spectra_numel(n_out, n_in, b), dtype=torch.float32, device=c.device)
    lib = _lib.load()
    _lib.check(lib.bcfft_spectra(c.data_ptr(), _lib.dtype_code(c.dtype), n_out, n_in, b,
                                 int(bool(transpose_conj)), out.data_ptr(),
                                 _lib.stream_handle(c.device)), "bcfft_spectra")
    return out


def _check_operand(t: torch.Tensor, device: torch.device, what: str, name: str) -> None:
    """A spectra buffer or bias the kernels read by raw pointer must live on x's device, and a
    spectra buffer must be contiguous (the library indexes it as the flat packed image)."""
    if t.device != device:
        raise ValueError(f"{what}: {name} is on {t.device} but x is on {device}; move it to x's device")
    if name == "spectra" and not t.is_contiguous():
        raise ValueError(f"{what}: the spectra buffer must be contiguous (use bcfft.ops.spectra's output as is)")


def _check_spectra(spec: torch.Tensor, n_out: int, n_in: int, b: int, what: str) -> None:
    """The library cannot see the spectra buffer's size: a buffer built for another geometry
    would be read out of bounds. Checked here, before the launch."""
    if b <= 0 or n_out <= 0 or n_in <= 0:
        raise ValueError(f"{what}: invalid geometry (out_blocks={n_out}, in_blocks={n_in}, block_size={b})")
    need = _lib.load().bcfft_spectra_bytes(n_out, n_in, b)
    if need < 0 or spec.dtype != torch.float32 or spec.numel() * 4 < need:
        raise ValueError(f"{what}: spectra buffer of {spec.numel() * spec.element_size()} B "
                         f"({spec.dtype}) does not hold the ({n_out}, {n_in}, {b}) operator ({need} B)")


def glu_weights(c_gate: torch.Tensor, c_up: torch.Tensor) -> torch.Tensor:
    """Interleave gate/up circulant columns (nO, nI, b) into the (32 G, nI, b) weight of
    bcfft_forward_glu, G = ceil(nO / 16): group g = gate blocks [16g, 16g+16) then up blocks
    [16g, 16g+16), zero blocks past nO. Pure indexing (any device)."""
    if c_gate.shape != c_up.shape or c_gate.dim() != 3:
        raise ValueError("gate and up weights must both be (out_blocks, in_blocks, block_size)")
    n_out, n_in, b = c_gate.shape
    groups = -(-n_out // 16)
    flat = c_gate.new_zeros(groups, 2, 16, n_in, b)
    gpad = torch.zeros(groups * 16, n_in, b, dtype=c_gate.dtype, device=c_gate.device)
    upad = torch.zeros_like(gpad)
    gpad[:n_out] = c_gate.detach()
    upad[:n_out] = c_up.detach()
    flat[:, 0] = gpad.view(groups, 16, n_in, b)
    flat[:, 1] = upad.view(groups, 16, n_in, b)
    return flat.reshape(groups * 32, n_in, b)


def forward_glu(x2d: torch.Tensor, spec_gu: torch.Tensor, block_size: int, gate_features: int,
                algo: str | None = None) -> torch.Tensor:
    """h = silu(BC_gate(x2d)) * BC_up(x2d) in one launch (bcfft_forward_glu_algo); spec_gu =
    spectra(glu_weights(c_gate, c_up)). h has x2d's dtype. algo: None -> BCFFT_ALGO env (auto:
    the DFT kernel at b = 128 with K = 4096, else stationary), or "stationary" / "dft" / "dftx"."""
    algo = default_algo() if algo is None else algo
    if algo == "auto" and x2d.dtype == torch.float32 and precise_mode() and block_size == 128 and x2d.shape[-1] == 4096:
        algo = "dftp"
    if algo not in ("auto", "stationary", "dft", "dftx", "dftp"):
        raise ValueError(f"bcfft.forward_glu: engine {algo!r} has no fused gate/up form "
                         "(auto, stationary, dft, dftx); run gate and up as two forwards instead")
    _lib.require_device(x2d, "bcfft.forward_glu")
    if _lib.native_op():
        return _lib.NATIVE_FORWARD_GLU(x2d, spec_gu, block_size, gate_features, _lib.ALGOS[algo])
    n, k = x2d.shape
    if block_size > 0 and gate_features % block_size == 0 and k % block_size == 0:
        _check_spectra(spec_gu, 32 * (-(-(gate_features // block_size) // 16)), k // block_size, block_size,
                       "bcfft.forward_glu")
    _check_operand(spec_gu, x2d.device, "bcfft.forward_glu", "spectra")
    x2d = x2d.contiguous()
    if x2d.data_ptr() % 16:
        x2d = x2d.clone()
    h = torch.empty((n, gate_features), dtype=x2d.dtype, device=x2d.device)
    if n == 0:
        return h
    lib = _lib.load()
    _lib.check(lib.bcfft_forward_glu_algo(x2d.data_ptr(), _lib.dtype_code(x2d.dtype), n, k, gate_features,
                                          block_size, spec_gu.data_ptr(), h.data_ptr(), _lib.ALGOS[algo],
                                          _lib.stream_handle(x2d.device)), "bcfft_forward_glu")
    return h


def forward_mlp(x2d: torch.Tensor, spec_gu: torch.Tensor, spec_down: torch.Tensor, block_size: int,
                inter_features: int, mode: str = "auto") -> torch.Tensor:
    """y = BC_down(silu(BC_gate(x2d)) * BC_up(x2d)) (bcfft_forward_mlp): the LLaMA
    MLP as microbench_dense_vs_bc.py:183-188 times it. spec_gu = spectra(glu_weights(c_gate,
    c_up)), spec_down = spectra(c_down). mode "fused": one launch, h never written (bf16,
    b = 128, hidden 4096, intermediate 4224..16256); "fused_splitk": the fused kernel with its
    gate/up groups split over more workgroups at short grids (fp32 partials + a finishing pass);
    "split": the gate/up + SwiGLU launch into a workspace, then the down launch; "auto": fused
    where its tiles fill the CUs, fused_splitk at short grids, else split. y has x2d's dtype."""
    if mode not in _lib.MLP_MODES:
        raise ValueError(f"bcfft.forward_mlp: mode {mode!r}, expected one of {sorted(_lib.MLP_MODES)}")
    _lib.require_device(x2d, "bcfft.forward_mlp")
    n, k = x2d.shape
    b = block_size
    if b > 0 and k % b == 0 and inter_features % b == 0:
        _check_spectra(spec_gu, 32 * (-(-(inter_features // b) // 16)), k // b, b, "bcfft.forward_mlp")
        _check_spectra(spec_down, k // b, inter_features // b, b, "bcfft.forward_mlp")
    _check_operand(spec_gu, x2d.device, "bcfft.forward_mlp", "spectra")
    _check_operand(spec_down, x2d.device, "bcfft.forward_mlp", "spectra")
    x2d = x2d.contiguous()
    if x2d.data_ptr() % 16:
        x2d = x2d.clone()
    y = torch.empty((n, k), dtype=x2d.dtype, device=x2d.device)
    lib = _lib.load()
    code = _lib.MLP_MODES[mode]
    ws_bytes = lib.bcfft_forward_mlp_workspace_bytes(n, k, inter_features, b, _lib.dtype_code(x2d.dtype), code)
    ws = torch.empty(max(ws_bytes, 0), dtype=torch.uint8, device=x2d.device) if ws_bytes > 0 else None
    _lib.check(lib.bcfft_forward_mlp(x2d.data_ptr(), _lib.dtype_code(x2d.dtype), n, k, inter_features, b,
                                     spec_gu.data_ptr(), spec_down.data_ptr(), y.data_ptr(), code,
                                     0 if ws is None else ws.data_ptr(), max(ws_bytes, 0),
                                     _lib.stream_handle(x2d.device)), "bcfft_forward_mlp")
    return y


def mlp_fused_eligible(hidden_features: int, inter_features: int, block_size: int,
                       dtype: torch.dtype | None = None) -> bool:
    """Geometries of the one-launch BC-MLP kernel (bcfft_dmm.hip)."""
    return (block_size == 128 and hidden_features == 4096 and inter_features % 128 == 0
            and 32 < inter_features // 128 <= 127 and dtype in (None, torch.bfloat16))


def mlp_auto_is_fused(n_tokens: int, hidden_features: int, inter_features: int, block_size: int,
                      dtype: torch.dtype) -> bool:
    """Whether bcfft_forward_mlp's AUTO mode runs the fused kernel for these sizes (one launch, or
    its group split at short grids) rather than the gate/up launch and the down launch."""
    mode = _lib.load().bcfft_forward_mlp_mode(n_tokens, hidden_features, inter_features, block_size,
                                              _lib.dtype_code(dtype), _lib.MLP_MODES["auto"])
    return mode in (_lib.MLP_MODES["fused"], _lib.MLP_MODES["fused_splitk"])


def glu_eligible(in_features: int, block_size: int, dtype: torch.dtype | None = None, algo: str | None = None,
                 gate_features: int | None = None) -> bool:
    """Whether bcfft_forward_glu_algo serves this geometry with this engine (include/bcfft.h), so
    callers fall back to two launches instead of meeting BCFFT_ERR_BLOCK. Mirrors the C rules:
    b = 256 with K = 4096 only for bf16 x under auto / dft, up to 512 gate blocks (the kernel's
    group limit); otherwise the stationary geometries, where dftx needs b = 128 with K = 4096 and
    dft that or b = 64 with K = 4096 and bf16 x; mfma / valu / short have no fused form. algo None: the
    BCFFT_ALGO environment (default auto)."""
    algo = default_algo() if algo is None else algo
    if algo in ("mfma", "valu", "short") or block_size <= 0 or in_features % block_size:
        return False
    n_in = in_features // block_size
    if block_size == 256 and n_in == 16:
        n_gate = None if gate_features is None else gate_features // block_size
        return (dtype == torch.bfloat16 and algo in ("auto", "dft")
                and (n_gate is None or 2 * (-(-n_gate // 16)) <= 64))
    dm = block_size == 128 and n_in == 32
    dm64 = block_size == 64 and n_in == 64 and dtype == torch.bfloat16
    stat = dm or (block_size == 64 and n_in in (32, 64))
    if algo in ("dftx", "dftp"):
        return dm
    if algo == "dft":
        return dm or dm64
    return stat


def default_algo() -> str:
    """BCFFT_ALGO env var: auto (default) | dft | dftx | dftp | stationary | mfma | valu."""
    a = os.environ.get("BCFFT_ALGO", "auto").lower()
    if a not in _lib.ALGOS:
        raise ValueError(f"BCFFT_ALGO={a!r}: expected one of {sorted(_lib.ALGOS)}")
    return a


def precise_mode() -> bool:
    """BCFFT_PRECISE=1: AUTO picks the fp32-faithful engines for fp32 activations (the reference's
    fp32 arithmetic class, per token): dftp at b = 128 with K = 4096 (~2.8e-5, per token ~1e-5
    times its cancellation), the split-bf16 MFMA kernel (~1e-5) at other b <= 128, fp32 VALU above.
    The default AUTO keeps the faster dftx / stationary engines (~3e-4, per token up to ~6e-3 on
    near-cancelling tokens); 16-bit activations are unaffected (their output rounding dominates)."""
    return os.environ.get("BCFFT_PRECISE", "0") not in ("", "0")


def resolve_algo(algo: str | None, dtype: torch.dtype, block_size: int, in_features: int) -> str:
    """The engine name a call runs before the library's own AUTO rule: algo, else BCFFT_ALGO, with
    BCFFT_PRECISE's choice for fp32 activations (precise_mode)."""
    a = (algo or default_algo()).lower()
    if a != "auto" or dtype != torch.float32 or not precise_mode():
        return a
    if block_size == 128 and in_features == 4096:
        return "dftp"
    return "mfma" if block_size <= 128 else "valu"


def forward(x2d: torch.Tensor, spec: torch.Tensor, bias: torch.Tensor | None, block_size: int,
            out_features: int, algo: str | None = None, split_k: bool = True) -> torch.Tensor:
    """y = BC(x2d) (+ bias) with one fused kernel. x2d: (N, K) device tensor.
    algo: "auto" (at b = 128, K = 4096: dftx for fp32 outputs, dft for 16-bit ones; dft on its
    other geometries; else stationary where eligible, else mfma for b <= 128, else valu), "dft" (block DFTs and MAC on fp16 MFMA, weights in VGPRs, ~3.5e-4), "dftx"
    (dft with the per-bin products split hi + lo: ~2.8e-4, linear to ~1e-6),
    "stationary" (weights in VGPRs, fp16 MFMA, ~3e-4), "mfma" (split-bf16, ~1e-5) or
    "valu" (exact fp32 MAC). See include/bcfft.h. split_k=False withholds the workspace, so short
    grids run unsplit (the split-K forms sum fp32 partials: not bit-identical to the unsplit launch)."""
    _lib.require_device(x2d, "bcfft.forward")
    algo = resolve_algo(algo, x2d.dtype, block_size, x2d.shape[-1])
    if _lib.native_op():                         # the same call as one C++ op (csrc/bcfft_torch.cpp)
        return _lib.NATIVE_FORWARD(x2d, spec, bias, block_size, out_features, _lib.ALGOS[algo], split_k)
    n, k = x2d.shape
    if block_size > 0 and out_features % block_size == 0 and k % block_size == 0:
        _check_spectra(spec, out_features // block_size, k // block_size, block_size, "bcfft.forward")
    _check_operand(spec, x2d.device, "bcfft.forward", "spectra")
    if bias is not None:
        _check_operand(bias, x2d.device, "bcfft.forward", "bias")
    x2d = x2d.contiguous()
    if x2d.data_ptr() % 16:
        x2d = x2d.clone()
    out_dtype = x2d.dtype if bias is None else torch.promote_types(x2d.dtype, bias.dtype)
    y = torch.empty((n, out_features), dtype=out_dtype, device=x2d.device)
    if n == 0:
        return y
    bias_ptr, bias_code = 0, _lib.BCFFT_NONE
    if bias is not None:
        bias = bias.detach().contiguous()
        if bias.data_ptr() % 16:                 # the epilogue reads bias with 16-B loads
            bias = bias.clone()
        bias_ptr, bias_code = bias.data_ptr(), _lib.dtype_code(bias.dtype)
    lib = _lib.load()
    code = _lib.ALGOS[algo]
    # split-K workspace (short grids of the MFMA and streamed-weight kernels); caller-owned, from
    # torch's allocator
    ws_bytes = lib.bcfft_forward_workspace_bytes_io(n, k, out_features, block_size, code,
                                                    _lib.dtype_code(x2d.dtype), _lib.dtype_code(out_dtype))
    if not split_k:
        ws_bytes = 0
    ws = torch.empty(max(ws_bytes, 0), dtype=torch.uint8, device=x2d.device) if ws_bytes > 0 else None
    _lib.check(lib.bcfft_forward_ws(x2d.data_ptr(), _lib.dtype_code(x2d.dtype), n, k, out_features,
                                    block_size, spec.data_ptr(), bias_ptr, bias_code, y.data_ptr(),
                                    _lib.dtype_code(out_dtype), code, 0 if ws is None else ws.data_ptr(),
                                    max(ws_bytes, 0), _lib.stream_handle(x2d.device)),
               "bcfft_forward")
    return y


def _aligned(t: torch.Tensor) -> torch.Tensor:
    t = t.contiguous()
    return t.clone() if t.data_ptr() % 16 else t


def project_circulant(weight: torch.Tensor, block_size: int) -> torch.Tensor:
    """Loss-aware circulant projection of a dense device weight (out_f, in_f) -> c (nO, nI, b)
    fp32 in one launch (bcfft_project_circulant): from_linear's per-block loop,
    patch_llama_fft.py:207-219 over :82-128, with arithmetic in the weight's dtype."""
    _lib.require_device(weight, "bcfft.project_circulant")
    if weight.dim() != 2:
        raise ValueError("weight must be (out_features, in_features)")
    m, k = weight.shape
    b = block_size
    w = _aligned(weight.detach())
    c = torch.empty((m // b, k // b, b), dtype=torch.float32, device=w.device)
    lib = _lib.load()
    _lib.check(lib.bcfft_project_circulant(w.data_ptr(), _lib.dtype_code(w.dtype), m, k, b, c.data_ptr(),
                                           _lib.stream_handle(w.device)), "bcfft_project_circulant")
    return c


def grad_c(x2d: torch.Tensor, dy: torch.Tensor, block_size: int, c_dtype: torch.dtype = torch.float32) -> torch.Tensor:
    """dL/dc of y = BC(x2d) for upstream gradient dy (N, out_f): (nO, nI, b) of c_dtype
    (bcfft_grad_c; the autograd of patch_llama_fft.py:246-271 with respect to c)."""
    _lib.require_device(x2d, "bcfft.grad_c")
    n, k = x2d.shape
    m = dy.shape[1]
    b = block_size
    x2d, dy = _aligned(x2d), _aligned(dy)
    lib = _lib.load()
    nbytes = lib.bcfft_grad_c_workspace_bytes(n, k, m, b)
    if nbytes < 0:
        raise ValueError(f"invalid grad_c geometry (N={n}, K={k}, M={m}, b={b})")
    ws = torch.empty(max(nbytes // 4, 4), dtype=torch.float32, device=x2d.device)
    dc = torch.empty((m // b, k // b, b), dtype=c_dtype, device=x2d.device)
    _lib.check(lib.bcfft_grad_c(x2d.data_ptr(), _lib.dtype_code(x2d.dtype), dy.data_ptr(), _lib.dtype_code(dy.dtype),
                                n, k, m, b, ws.data_ptr(), dc.data_ptr(), _lib.dtype_code(c_dtype),
                                _lib.stream_handle(x2d.device)), "bcfft_grad_c")
    return dc


def circulant_matvec(c: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """y = C(c) x for one circulant of any length (fft_utils.py:3-34)."""
    _lib.require_device(x, "bcfft.circulant_matvec")
    dt = x.dtype
    c = c.to(dt).contiguous()
    x = x.contiguous()
    y = torch.empty_like(x)
    lib = _lib.load()
    _lib.check(lib.bcfft_circulant_matvec(c.data_ptr(), x.data_ptr(), _lib.dtype_code(dt),
                                          x.numel(), y.data_ptr(), _lib.stream_handle(x.device)),
               "bcfft_circulant_matvec")
    return y
