"""Drop-in replacement for the reference's ``patch_llama_fft`` module on MI355X.

Same public surface as Pinguhat/llama-fft ``src/patch_llama_fft.py`` (cited per symbol;
paths relative to the reference's ``src/``): ``MODEL_PATH``, ``BLOCK_SIZE``,
``NUM_LAYERS_TO_PATCH``, ``BlockCirculantLinear`` (ctor, attributes, ``from_linear``,
``forward``), the circulant projection helpers, ``save_bc_params``/``load_bc_params``,
``patch_mlp_with_block_circulant`` and ``main``. Put ``llama-fft_amd/`` on ``sys.path`` where
the reference put ``src/`` and ``import patch_llama_fft`` resolves here.

What differs, by design:
  * ``BlockCirculantLinear.forward`` runs ONE fused HIP kernel (libbcfft.so,
    ``bcfft_forward``) on gfx950 instead of torch's rfft/einsum/irfft/cast/add chain. The
    weight spectra are computed by ``bcfft_spectra`` and cached per module, keyed by the
    parameter's version counter, so an in-place update of ``c`` can never be served stale
    (the reference's cached forward can: bench_all_in_one.py:204-216).
  * There is no CPU path: a non-ROCm tensor raises ``RuntimeError``.
  * Backward: dL/dx runs the same fused kernel on the adjoint spectra; dL/dc runs
    ``bcfft_grad_c`` (bc_grad_c_kernel + bc_grad_c_finish: per-bin cross-correlation, fp64
    split reduction; see DESIGN.md, scope row f3).
"""
from __future__ import annotations

import functools
import os
from typing import Dict

import torch
import torch.nn as nn
from torch.autograd.function import once_differentiable

from bcfft import ops as _ops
from bcfft import _lib
from fft_utils import circulant_matvec_fft

# Same module constants as the reference (patch_llama_fft.py:10-15)
MODEL_PATH = os.environ.get("LLAMA_FFT_MODEL_PATH", r"C:\Users\Lukas\Documents\0-UNI\Seminar\Llama2")
BLOCK_SIZE = 256
NUM_LAYERS_TO_PATCH = 1


# ----------------------------------------------------------------------------- projection helpers
def _detect_best_convention_for_layer(W: torch.Tensor, block_size: int, *, num_probes: int = 3) -> str:
    """patch_llama_fft.py:17-44 — pick "diag" or "diag_inv" by probe error on the top-left block."""
    B = block_size
    block = W[:B, :B].detach().to(dtype=torch.float32)
    dev = block.device
    torch.manual_seed(0)
    xs = [torch.randn(B, device=dev, dtype=torch.float32) for _ in range(num_probes)]

    def score(convention: str) -> float:
        c = dense_block_to_circulant_column(block, convention=convention).to(torch.float32)
        err = 0.0
        for x in xs:
            err += (block @ x - circulant_matvec_fft(c, x)).pow(2).mean().item()
        return err / float(num_probes)

    return "diag" if score("diag") <= score("diag_inv") else "diag_inv"


def dense_block_to_circulant_column(W_block: torch.Tensor, *, convention: str = "diag") -> torch.Tensor:
    """patch_llama_fft.py:47-79 — c[k] = mean_i W[i,(i+k)%B] ("diag") or W[(i+k)%B,i]."""
    assert W_block.dim() == 2
    B0, B1 = W_block.shape
    assert B0 == B1
    if convention not in ("diag", "diag_inv"):
        raise ValueError(f"Unknown convention: {convention}")
    B = B0
    idx = torch.arange(B, device=W_block.device)
    k = idx[:, None]
    if convention == "diag":
        vals = W_block[idx[None, :], (idx[None, :] + k) % B]
    else:
        vals = W_block[(idx[None, :] + k) % B, idx[None, :]]
    return vals.mean(dim=1).to(W_block.dtype)


def _project_loss_aware_batched(blocks: torch.Tensor, eps: float = 1e-12) -> torch.Tensor:
    """Batched dense_block_to_circulant_column_loss_aware over (..., B, B), in blocks.dtype."""
    B = blocks.shape[-1]
    idx = torch.arange(B, device=blocks.device)
    cols = (idx[None, :] - idx[:, None]) % B                     # [t, r] -> column (r - t) % B
    diag = blocks[..., idx[None, :], cols]                       # (..., t, r)   :116-117
    c = diag.mean(dim=-1)                                        # :118
    diag_sums = diag.sum(dim=-1)                                 # :119
    numerator = (c * diag_sums).sum(dim=-1)                      # :124
    denom = (B * (c * c).sum(dim=-1)).clamp_min(eps)             # :125
    alpha = numerator / denom                                    # :126
    return (alpha[..., None] * c).to(blocks.dtype)               # :128


def dense_block_to_circulant_column_loss_aware(W_block: torch.Tensor, eps: float = 1e-12) -> torch.Tensor:
    """patch_llama_fft.py:82-128 — Frobenius projection onto circulants (first-column
    convention C[i,j] = c[(i-j)%B]) with energy-preserving alpha; arithmetic in W's dtype."""
    assert W_block.dim() == 2
    B0, B1 = W_block.shape
    assert B0 == B1
    return _project_loss_aware_batched(W_block, eps)


def circulant_from_first_col(c: torch.Tensor) -> torch.Tensor:
    """patch_llama_fft.py:132-139 — explicit B x B circulant, C[:, j] = roll(c, j)."""
    B = c.numel()
    idx = torch.arange(B, device=c.device)
    return c[(idx[:, None] - idx[None, :]) % B]


# ----------------------------------------------------------------------------- autograd
class _BCFunction(torch.autograd.Function):
    """Fused forward on the HIP engine; backward: dx through the fused kernel on adjoint
    spectra, dc by the per-bin cross-correlation kernel (bcfft_grad_c), dbias by reduction."""

    @staticmethod
    def forward(ctx, x2d, c, bias, module):
        spec = module._spectra(c)
        y = _ops.forward(x2d, spec, bias, module.block_size, module.out_features)
        ctx.module = module
        ctx.save_for_backward(x2d, c, bias)
        return y

    @staticmethod
    @once_differentiable
    def backward(ctx, dy):
        # once_differentiable: the backward runs its kernels under no_grad on both host paths (the
        # C++ operator and the ctypes call), so backward(create_graph=True) gives first-order
        # gradients either way, and a second differentiation raises the same error on both
        x2d, c, bias = ctx.saved_tensors
        m = ctx.module
        dx = dc = dbias = None
        dy = dy.contiguous()
        # The reference adds the bias AFTER y.to(x.dtype) (:266-271): with a 16-bit x and a wider
        # bias, autograd hands the add's x-side input its gradient rounded to x.dtype, and the
        # .to() backward widens it again. dx and dc see that rounded dy; dbias sees dy itself.
        dy_x = dy.to(x2d.dtype) if (bias is not None and dy.dtype != x2d.dtype) else dy
        if ctx.needs_input_grad[0]:
            spec_t = m._spectra(c, adjoint=True)
            dx = _ops.forward(dy_x, spec_t, None, m.block_size, m.in_features).to(x2d.dtype)
        if ctx.needs_input_grad[1]:
            dc = _ops.grad_c(x2d, dy_x, m.block_size, c.dtype)
        if bias is not None and ctx.needs_input_grad[2]:
            dbias = dy.sum(dim=0).to(bias.dtype)
        return dx, dc, dbias, None


def _version_of(x: torch.Tensor):
    """x's in-place version counter; None for inference tensors (created under
    torch.inference_mode, as the reference's harnesses and model.generate run), which have none.
    Caches keyed on it then match by storage identity alone: fused q/k/v outputs are dropped as
    soon as every projection has taken its view, and the spectra of a c created in inference
    mode are not refreshed by in-place edits of that c (edit it outside inference mode)."""
    return None if x.is_inference() else x._version


# ----------------------------------------------------------------------------- the module
class BlockCirculantLinear(nn.Module):
    """Block-circulant linear layer (patch_llama_fft.py:142-275), FFT-multiplied on MI355X.

    c[j, i, :] is the first column of the circulant block C_{j,i} mapping input block i to
    output block j: y_j = sum_i C_{j,i} x_i, C[r, s] = c[(r - s) % block_size].
    """

    def __init__(self, in_features: int, out_features: int, block_size: int = 256, bias: bool = True):
        super().__init__()
        assert in_features % block_size == 0, "in_features must be divisible by block_size"    # :159
        assert out_features % block_size == 0, "out_features must be divisible by block_size"  # :160
        self.in_features = in_features
        self.out_features = out_features
        self.block_size = block_size
        self.in_blocks = in_features // block_size
        self.out_blocks = out_features // block_size
        self.c = nn.Parameter(torch.randn(self.out_blocks, self.in_blocks, self.block_size) * 0.01)  # :171-173
        if bias:
            self.bias = nn.Parameter(torch.zeros(out_features))                               # :175-176
        else:
            self.bias = None
        self._spec_cache: Dict[tuple, torch.Tensor] = {}

    @classmethod
    def from_linear(cls, linear: nn.Linear, block_size: int = 256) -> "BlockCirculantLinear":
        """patch_llama_fft.py:180-224 — project every b x b block of the dense weight onto a
        circulant (loss-aware, in the weight's dtype), keep c in fp32, copy the bias."""
        in_f, out_f = linear.in_features, linear.out_features
        layer = cls(in_features=in_f, out_features=out_f, block_size=block_size,
                    bias=(linear.bias is not None))
        layer = layer.to(linear.weight.device)                                                # :198
        with torch.no_grad():
            W = linear.weight.data
            B = block_size
            if W.device.type == "cuda":                                                        # one launch
                layer.c.data.copy_(_ops.project_circulant(W, B))                               # :207-219
            else:                                                                              # host weights
                blocks = W.view(layer.out_blocks, B, layer.in_blocks, B).permute(0, 2, 1, 3)   # :208-209
                layer.c.data.copy_(_project_loss_aware_batched(blocks))                        # :214-219
            if layer.bias is not None and linear.bias is not None:
                layer.bias.data.copy_(linear.bias.data)                                        # :221-222
        return layer

    # -- spectra cache (device, storage, version, dtype): recomputed after any update of c
    def _spectra(self, c: torch.Tensor, adjoint: bool = False) -> torch.Tensor:
        key = (adjoint, c.device, c.data_ptr(), _version_of(c), c.dtype, tuple(c.shape))
        spec = self._spec_cache.get(key)
        if spec is None:
            self._spec_cache = {k: v for k, v in self._spec_cache.items() if k[0] != adjoint}
            spec = _ops.spectra(c, transpose_conj=adjoint)
            self._spec_cache[key] = spec
        return spec

    def _apply(self, fn, *args, **kwargs):  # .to()/.cuda()/.half(): drop device-bound spectra
        self._spec_cache = {}
        return super()._apply(fn, *args, **kwargs)

    def _flatten(self, x: torch.Tensor) -> torch.Tensor:
        """x -> (N, in_features) with the reference's errors: ValueError for other ranks
        (:238-239), AssertionError for a 3D input of the wrong width (:230), the reshape's
        RuntimeError (:246) for a 2D one."""
        if x.dim() == 3:                                                                       # :228-233
            bs, sl, in_f = x.shape
            assert in_f == self.in_features
            x_flat = x.reshape(bs * sl, in_f)
        elif x.dim() == 2:                                                                     # :234-238
            x_flat = x
        else:
            raise ValueError("Unsupported input dim")                                          # :239
        x_flat.reshape(x_flat.shape[0], self.in_blocks, self.block_size)
        return x_flat

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x_flat = self._flatten(x)
        is_3d = x.dim() == 3
        if is_3d:
            bs, sl = x.shape[0], x.shape[1]
        _lib.require_device(x_flat, "BlockCirculantLinear.forward")
        if torch.is_grad_enabled() and (x_flat.requires_grad or self.c.requires_grad or
                                        (self.bias is not None and self.bias.requires_grad)):
            y_flat = _BCFunction.apply(x_flat, self.c, self.bias, self)
        else:                    # no graph to record (eval, no_grad, inference_mode): skip autograd
            y_flat = _ops.forward(x_flat, self._spectra(self.c), self.bias, self.block_size, self.out_features)
        if is_3d:
            return y_flat.view(bs, sl, self.out_features)                                      # :273-274
        return y_flat

    def extra_repr(self) -> str:
        return (f"in_features={self.in_features}, out_features={self.out_features}, "
                f"block_size={self.block_size}, bias={self.bias is not None}, engine=bcfft-gfx950")


# ----------------------------------------------------------------------------- param I/O
def _get_submodule_by_name(model: nn.Module, name: str) -> nn.Module:
    """patch_llama_fft.py:278-284: the attribute path `name` ("" = the model itself);
    AttributeError for a missing step."""
    return functools.reduce(getattr, name.split("."), model) if name else model


def _bc_tensors(model: nn.Module):
    """(checkpoint key, tensor) of every BlockCirculantLinear's c and bias, in module order."""
    for prefix, mod in model.named_modules():
        if isinstance(mod, BlockCirculantLinear):
            yield f"{prefix}.c", mod.c
            if mod.bias is not None:
                yield f"{prefix}.bias", mod.bias


def save_bc_params(model: nn.Module, path: str) -> None:
    """patch_llama_fft.py:287-300: torch.save of {"<module>.c": (nO,nI,b), "<module>.bias": (M,)}
    for every BC module, host copies."""
    state = {key: t.detach().cpu() for key, t in _bc_tensors(model)}
    parent = os.path.dirname(path)
    os.makedirs(parent if parent else ".", exist_ok=True)
    torch.save(state, path)
    print(f"Saved BC params: {len(state)} tensors -> {path}")


def _load_target(model: nn.Module, key: str, value: torch.Tensor, strict_shapes: bool):
    """The parameter a checkpoint entry restores, or None when the reference loader skips it
    (patch_llama_fft.py:311-336): not a .c / .bias key, no such module or attribute, not a
    tensor, or (strict_shapes) a shape mismatch."""
    if not key.endswith((".c", ".bias")):
        return None
    owner_name, attr = key.rsplit(".", 1)
    try:
        owner = _get_submodule_by_name(model, owner_name)
    except AttributeError:
        return None
    target = getattr(owner, attr, None)
    if not isinstance(target, torch.Tensor) or (strict_shapes and target.shape != value.shape):
        return None
    return target


def load_bc_params(model: nn.Module, path: str, *, strict_shapes: bool = True) -> None:
    """patch_llama_fft.py:303-340: restore a save_bc_params checkpoint in place (tensors only,
    torch.load(weights_only=True)); entries without a matching parameter are counted as skipped."""
    state: Dict[str, torch.Tensor] = torch.load(path, map_location="cpu", weights_only=True)
    restored = 0
    with torch.no_grad():
        for key, value in state.items():
            target = _load_target(model, key, value, strict_shapes)
            if target is not None:
                target.copy_(value.to(target.device, dtype=target.dtype))
                restored += 1
    print(f"Loaded BC params from {path}: loaded={restored}, skipped={len(state) - restored}")


# ----------------------------------------------------------------------------- model patcher
MLP_PROJECTIONS = ("gate_proj", "up_proj", "down_proj")
ATTN_PROJECTIONS = ("q_proj", "k_proj", "v_proj", "o_proj")


def _layer_indices(n_layers: int, num_layers_to_patch: int, patch_position: str):
    if num_layers_to_patch < 0:
        raise ValueError("num_layers_to_patch must be >= 0")                                   # :361-362
    k = min(num_layers_to_patch, n_layers)
    if patch_position not in ("first", "last"):
        raise ValueError("patch_position must be 'first' or 'last'")                           # :365-366
    return list(range(k)) if patch_position == "first" else list(range(n_layers - k, n_layers))


def _patch(model, layer_indices, block_size, targets):
    for layer_idx in layer_indices:
        layer = model.model.layers[layer_idx]
        for parent_name, names in (("mlp", MLP_PROJECTIONS), ("self_attn", ATTN_PROJECTIONS)):
            parent = getattr(layer, parent_name, None)
            if parent is None:
                continue
            sel = [n for n in names if n in targets]
            if sel:
                print(f"  Patching layer {layer_idx} {parent_name.upper() if parent_name == 'mlp' else parent_name}...")
            for name in sel:
                old_layer = getattr(parent, name, None)
                if not isinstance(old_layer, nn.Linear):
                    print(f"    Skip {name}: not an nn.Linear")
                    continue
                print(f"    Replacing {name}: in_features={old_layer.in_features}, "
                      f"out_features={old_layer.out_features}")
                setattr(parent, name, BlockCirculantLinear.from_linear(old_layer, block_size=block_size))


def patch_mlp_with_block_circulant(model, *, num_layers_to_patch: int = NUM_LAYERS_TO_PATCH,
                                   block_size: int = BLOCK_SIZE, patch_position: str = "first") -> None:
    """patch_llama_fft.py:343-394 — replace gate/up/down_proj of the first/last k decoder
    layers with BlockCirculantLinear.from_linear(...)."""
    n_layers = model.config.num_hidden_layers
    print(f"Model has {n_layers} transformer layers.")
    layer_indices = _layer_indices(n_layers, num_layers_to_patch, patch_position)
    print(f"Patching {len(layer_indices)} layer(s) from {patch_position}: {layer_indices}")
    _patch(model, layer_indices, block_size, MLP_PROJECTIONS)


def patch_linear_with_block_circulant(model, *, num_layers_to_patch: int = NUM_LAYERS_TO_PATCH,
                                      block_size: int = BLOCK_SIZE, patch_position: str = "first",
                                      targets=MLP_PROJECTIONS + ATTN_PROJECTIONS) -> None:
    """Extension for BASELINE config 3 ("all linear layers BC"): also q/k/v/o_proj. Same
    kwargs as patch_mlp_with_block_circulant so signature-introspecting harnesses
    (bench_all_in_one.py:127-139) can call either."""
    n_layers = model.config.num_hidden_layers
    print(f"Model has {n_layers} transformer layers.")
    layer_indices = _layer_indices(n_layers, num_layers_to_patch, patch_position)
    print(f"Patching {len(layer_indices)} layer(s) from {patch_position}: {layer_indices}")
    _patch(model, layer_indices, block_size, tuple(targets))


class BCFusedGateUp(nn.Module):
    """act(gate(x)) * up(x) of a BC-patched LLaMA MLP in ONE launch (bcfft_forward_glu,
    include/bcfft.h): the gate and up projections share x's forward FFT in
    each workgroup and neither gate(x) nor up(x) is written to memory.

    Holds plain references to the two BlockCirculantLinear modules (their parameters and
    state_dict keys stay where they are). Uses the two modules + torch SiLU instead when the
    fused kernel does not apply: a bias, autograd recording, or a non-stationary geometry."""

    def __init__(self, gate: BlockCirculantLinear, up: BlockCirculantLinear):
        super().__init__()
        if (gate.in_features, gate.out_features, gate.block_size) != (up.in_features, up.out_features, up.block_size):
            raise ValueError("gate and up projections must have the same shape and block_size")
        object.__setattr__(self, "_gate", gate)          # not submodules: no duplicate parameters
        object.__setattr__(self, "_up", up)
        self._spec = None
        self._key = None

    def _fused_ok(self, x: torch.Tensor) -> bool:
        g, u = self._gate, self._up
        grad = torch.is_grad_enabled() and (g.c.requires_grad or u.c.requires_grad or x.requires_grad)
        # the fused launch only where bcfft_forward_glu_algo serves the geometry with the engine
        # BCFFT_ALGO names (mfma / valu have no fused form): otherwise two launches, never an error
        return (g.bias is None and u.bias is None and not grad and x.is_cuda
                and _ops.glu_eligible(g.in_features, g.block_size, x.dtype,
                                      _ops.resolve_algo(None, x.dtype, g.block_size, g.in_features), g.out_features))

    def _spectra(self) -> torch.Tensor:
        g, u = self._gate.c, self._up.c
        key = (g.device, g.data_ptr(), _version_of(g), u.data_ptr(), _version_of(u), g.dtype)
        if key != self._key:
            self._spec = _ops.spectra(_ops.glu_weights(g, u))
            self._key = key
        return self._spec

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if not self._fused_ok(x):
            return torch.nn.functional.silu(self._gate(x)) * self._up(x)
        shape = x.shape
        x2d = self._gate._flatten(x)                   # the module's rank / width errors
        h = _ops.forward_glu(x2d, self._spectra(), self._gate.block_size, self._gate.out_features)
        return h.view(*shape[:-1], self._gate.out_features)


def _mlp_fused_ok(mlp, x: torch.Tensor) -> bool:
    """The whole MLP as ONE launch (bcfft_forward_mlp) when down_proj is BC too,
    without bias or autograd, on the fused kernel's geometry (bf16, b = 128, hidden 4096)."""
    gu, d = mlp._bc_gate_up, mlp.down_proj
    if not isinstance(d, BlockCirculantLinear) or d.bias is not None or not gu._fused_ok(x):
        return False
    if torch.is_grad_enabled() and d.c.requires_grad:
        return False
    g = gu._gate
    return (d.block_size == g.block_size and d.in_features == g.out_features and d.out_features == g.in_features
            and _ops.default_algo() in ("auto", "dft")
            and _ops.mlp_fused_eligible(d.out_features, d.in_features, d.block_size, x.dtype))


def _fused_mlp_forward(self, x):
    # the one-launch kernel where bcfft_forward_mlp's AUTO takes it (its tiles fill the CUs);
    # otherwise the gate/up launch and down_proj's own forward (which splits K at short grids)
    if _mlp_fused_ok(self, x) and _ops.mlp_auto_is_fused(x.numel() // x.shape[-1], self.down_proj.out_features,
                                                         self.down_proj.in_features, self.down_proj.block_size,
                                                         x.dtype):
        gu, d = self._bc_gate_up, self.down_proj
        shape = x.shape
        x2d = gu._gate._flatten(x)
        y = _ops.forward_mlp(x2d, gu._spectra(), d._spectra(d.c), d.block_size, d.in_features)
        return y.view(*shape[:-1], d.out_features)
    return self.down_proj(self._bc_gate_up(x))


def fuse_mlp_gate_up(model) -> int:
    """Route each decoder MLP whose gate_proj and up_proj are BlockCirculantLinear (same shape,
    act = SiLU, as patch_mlp_with_block_circulant leaves them) through BCFusedGateUp: its
    forward becomes down_proj(silu(gate(x)) * up(x)) with the fused launch. When down_proj is
    BlockCirculantLinear too and the geometry allows it (bf16, b = 128, hidden 4096), the whole
    MLP runs as ONE launch (bcfft_forward_mlp: h never leaves the CU). Parameters and
    state_dict are unchanged. Returns the number of MLPs rewired."""
    import types
    n = 0
    for layer in model.model.layers:
        mlp = getattr(layer, "mlp", None)
        if mlp is None:
            continue
        g, u = getattr(mlp, "gate_proj", None), getattr(mlp, "up_proj", None)
        if not (isinstance(g, BlockCirculantLinear) and isinstance(u, BlockCirculantLinear)):
            continue
        act = getattr(mlp, "act_fn", None)          # nn.SiLU, or transformers' SiLUActivation
        if not (isinstance(act, nn.SiLU) or type(act).__name__ == "SiLUActivation"):
            continue
        if (g.in_features, g.out_features, g.block_size) != (u.in_features, u.out_features, u.block_size):
            continue
        object.__setattr__(mlp, "_bc_gate_up", BCFusedGateUp(g, u))
        mlp.forward = types.MethodType(_fused_mlp_forward, mlp)
        n += 1
    return n


class BCFusedProjections:
    """Several BlockCirculantLinear projections of the SAME input (LLaMA's q/k/v) as ONE launch
    over their concatenated weights: y = x [C_q; C_k; C_v]^T, split into views.
    One launch runs every output group of the three at once, so at small token counts (decode,
    short prompts) it takes about the time of one projection instead of three.

    The projections keep their modules, parameters and state_dict; fuse_attention_qkv points
    each module's forward here. The first call for an input computes all outputs; the others
    return their views of it for the same input (same tensor, same version). Autograd or mixed
    bias / dtype / block size use the modules' own forward."""

    def __init__(self, mods):
        self.mods = list(mods)
        m0 = self.mods[0]
        if any((m.in_features, m.block_size, m.c.dtype) != (m0.in_features, m0.block_size, m0.c.dtype)
               for m in self.mods):
            raise ValueError("fused projections need one in_features, block_size and weight dtype")
        self.splits = [m.out_features for m in self.mods]
        self._spec = self._key = None
        self._x = self._ver = self._outs = None
        self._left = set()

    def _fused_ok(self, x: torch.Tensor) -> bool:
        grad = torch.is_grad_enabled() and (x.requires_grad or any(
            m.c.requires_grad or (m.bias is not None and m.bias.requires_grad) for m in self.mods))
        biases = [m.bias is None for m in self.mods]
        return x.is_cuda and not grad and (all(biases) or not any(biases))

    def _weights(self):
        # the bias is part of the key: bias-only updates (train_bias, a checkpoint that changes
        # only the bias) must reach the fused launch as they reach the modules' own forward
        key = tuple((m.c.data_ptr(), _version_of(m.c),
                     None if m.bias is None else (m.bias.data_ptr(), _version_of(m.bias)))
                    for m in self.mods) + (self.mods[0].c.device,)
        if key != self._key:
            self._spec = _ops.spectra(torch.cat([m.c.detach() for m in self.mods], dim=0))
            self._bias = (None if self.mods[0].bias is None
                          else torch.cat([m.bias.detach() for m in self.mods]))
            self._key = key
        return self._spec, self._bias

    def output(self, idx: int, x: torch.Tensor) -> torch.Tensor:
        m = self.mods[idx]
        if not self._fused_ok(x):
            return BlockCirculantLinear.forward(m, x)
        ver = _version_of(x)
        if not (self._x is x and self._ver == ver and idx in self._left):
            spec, bias = self._weights()
            shape = x.shape
            x2d = m._flatten(x)                         # the module's rank / width errors
            y = _ops.forward(x2d, spec, bias, m.block_size, sum(self.splits))
            outs, o = [], 0
            for n in self.splits:
                outs.append(y[:, o:o + n].view(*shape[:-1], n))
                o += n
            self._x, self._ver, self._outs, self._left = x, ver, outs, set(range(len(self.mods)))
        out = self._outs[idx]
        self._left.discard(idx)
        if not self._left:                              # every view handed out: drop the input
            self._x = self._outs = None
        return out


def fuse_attention_qkv(model) -> int:
    """Route q_proj / k_proj / v_proj of each decoder layer whose three projections are
    BlockCirculantLinear (patch_linear_with_block_circulant) through one BCFusedProjections
    launch. Parameters and state_dict are unchanged. Returns the number of layers rewired."""
    import types
    n = 0
    for layer in model.model.layers:
        attn = getattr(layer, "self_attn", None)
        mods = [getattr(attn, nm, None) for nm in ("q_proj", "k_proj", "v_proj")] if attn is not None else []
        if len(mods) != 3 or not all(isinstance(m, BlockCirculantLinear) for m in mods):
            continue
        try:
            fused = BCFusedProjections(mods)
        except ValueError:
            continue
        for i, m in enumerate(mods):
            m.forward = types.MethodType(lambda self, x, _f=fused, _i=i: _f.output(_i, x), m)
        object.__setattr__(attn, "_bc_qkv", fused)
        n += 1
    return n


def main():
    """patch_llama_fft.py:396-419 — load LLaMA from MODEL_PATH, patch, run a shape check."""
    from transformers import AutoModelForCausalLM
    print(f"Loading Llama-2-7b from local path: {MODEL_PATH}")
    model = AutoModelForCausalLM.from_pretrained(MODEL_PATH, device_map="cpu", torch_dtype=torch.float16,
                                                 low_cpu_mem_usage=True, local_files_only=True)
    model.eval()
    patch_mlp_with_block_circulant(model)
    model = model.to("cuda")
    print("Running a small forward pass to check shapes...")
    input_ids = torch.randint(0, model.config.vocab_size, (1, 8), device="cuda")
    with torch.no_grad():
        outputs = model(input_ids=input_ids)
    print("Forward pass completed.")
    print("Logits shape:", outputs.logits.shape)


if __name__ == "__main__":
    main()
