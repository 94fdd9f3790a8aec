"""torch.library registration of the BC forward and spectra (`torch.ops.bcfft.*`).

The HIP kernels behind bcfft.ops are opaque to PyTorch's tracers; registering them as custom
ops with fake (meta) kernels lets FakeTensor / torch.export / torch.compile trace a model that
calls them, with output shapes and dtypes computed on the host from the C ABI's own sizing
(bcfft_spectra_bytes). The real kernels are bcfft.ops' (C ABI, include/bcfft.h): no CPU path,
a host tensor fails loudly as in bcfft.ops.

    torch.ops.bcfft.forward(x2d, spec, bias, block_size, out_features, algo) -> y
    torch.ops.bcfft.spectra(c, transpose_conj) -> spec
    torch.ops.bcfft.forward_glu(x2d, spec_gu, block_size, gate_features, algo) -> h
    torch.ops.bcfft.forward_mlp(x2d, spec_gu, spec_down, block_size, inter_features, mode) -> y
"""
from __future__ import annotations

import torch

from . import _lib, ops


@torch.library.custom_op("bcfft::forward", mutates_args=())
def forward(x2d: torch.Tensor, spec: torch.Tensor, bias: torch.Tensor | None, block_size: int,
            out_features: int, algo: str = "auto") -> torch.Tensor:
    """y = BC(x2d) (+ bias): bcfft.ops.forward (patch_llama_fft.py:246-271's forward)."""
    return ops.forward(x2d, spec, bias, block_size, out_features, algo=algo)


@forward.register_fake
def _forward_fake(x2d, spec, bias, block_size, out_features, algo="auto"):
    if x2d.dim() != 2:
        raise ValueError("bcfft::forward: x2d must be (N, in_features)")
    if block_size <= 0 or x2d.shape[1] % block_size or out_features % block_size:
        raise ValueError(f"bcfft::forward: features ({x2d.shape[1]}, {out_features}) not multiples of {block_size}")
    out_dtype = x2d.dtype if bias is None else torch.promote_types(x2d.dtype, bias.dtype)
    return x2d.new_empty((x2d.shape[0], out_features), dtype=out_dtype)


@torch.library.custom_op("bcfft::spectra", mutates_args=())
def spectra(c: torch.Tensor, transpose_conj: bool = False) -> torch.Tensor:
    """Packed weight spectra of c (nO, nI, b): bcfft.ops.spectra (rfft of c, :256-257)."""
    return ops.spectra(c, transpose_conj)


@spectra.register_fake
def _spectra_fake(c, transpose_conj=False):
    if c.dim() != 3:
        raise ValueError("bcfft::spectra: c must be (out_blocks, in_blocks, block_size)")
    n_out, n_in, b = c.shape
    if transpose_conj:
        n_out, n_in = n_in, n_out
    return c.new_empty((ops.spectra_numel(n_out, n_in, b),), dtype=torch.float32)


@torch.library.custom_op("bcfft::forward_glu", mutates_args=())
def forward_glu(x2d: torch.Tensor, spec_gu: torch.Tensor, block_size: int, gate_features: int,
                algo: str = "auto") -> torch.Tensor:
    """h = silu(BC_gate(x2d)) * BC_up(x2d): bcfft.ops.forward_glu (the patched LLaMA MLP's inner
    product, patch_llama_fft.py:343-394)."""
    return ops.forward_glu(x2d, spec_gu, block_size, gate_features, algo=algo)


@forward_glu.register_fake
def _forward_glu_fake(x2d, spec_gu, block_size, gate_features, algo="auto"):
    if x2d.dim() != 2 or block_size <= 0 or x2d.shape[1] % block_size or gate_features % block_size:
        raise ValueError("bcfft::forward_glu: x2d must be (N, in_features), features multiples of block_size")
    return x2d.new_empty((x2d.shape[0], gate_features))


@torch.library.custom_op("bcfft::forward_mlp", mutates_args=())
def forward_mlp(x2d: torch.Tensor, spec_gu: torch.Tensor, spec_down: torch.Tensor, block_size: int,
                inter_features: int, mode: str = "auto") -> torch.Tensor:
    """y = BC_down(silu(BC_gate(x2d)) * BC_up(x2d)): bcfft.ops.forward_mlp (SURVEY.md §8 f4;
    microbench_dense_vs_bc.py:183-188)."""
    return ops.forward_mlp(x2d, spec_gu, spec_down, block_size, inter_features, mode=mode)


@forward_mlp.register_fake
def _forward_mlp_fake(x2d, spec_gu, spec_down, block_size, inter_features, mode="auto"):
    if x2d.dim() != 2 or block_size <= 0 or x2d.shape[1] % block_size or inter_features % block_size:
        raise ValueError("bcfft::forward_mlp: x2d must be (N, hidden), features multiples of block_size")
    return x2d.new_empty(x2d.shape)


def registered() -> bool:
    """True once the ops are visible under torch.ops.bcfft (importing this module registers them)."""
    return all(hasattr(torch.ops.bcfft, n) for n in ("forward", "spectra", "forward_glu", "forward_mlp"))


__all__ = ["forward", "spectra", "forward_glu", "forward_mlp", "registered", "_lib"]
