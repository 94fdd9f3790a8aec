"""BASELINE config 3 in a driver-run test: patch_llama_fft on the LLaMA-2-7B architecture, ALL
linear layers block-circulant at b = 128 (q/k/v fused into one launch, the whole MLP through
bcfft_forward_mlp), a 20-prompt prefill (src/bench_all_in_one.py:297-389; the patcher
src/patch_llama_fft.py:343-394, extended to q/k/v/o).

The model is random-initialised in bf16 on the GPU (no weights offline; tools/model_bench.py is
the timed harness of the same configuration). Layer 0's and the last layer's projections are
checked against the numpy oracle (oracle/bc_oracle.py) on the model's own live activations:
outputs are bf16, so each kernel error is bounded by the unavoidable bf16 rounding of the exact
result (`floor`): the kernel may add at most 10 % on top of it (measured ~2-4 %). The MLP is
checked against the oracle's rounding chain (gate, up -> bf16; silu -> bf16; product -> bf16;
down), at a prefill size (> 2k tokens) where AUTO runs it as ONE launch."""
import argparse
import contextlib
import io
import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

pytestmark = pytest.mark.gpu


def _silu(a):
    a = a.astype(np.float64)
    e = np.exp(-np.abs(a))
    return a * np.where(a >= 0, 1.0 / (1.0 + e), e / (1.0 + e))


def _rel(a, b):
    return float(np.linalg.norm((a - b).astype(np.float64)) / np.linalg.norm(b.astype(np.float64)))


def _check(name, got, exact, rounded, slack=1.10):
    """got: kernel output (bf16 values as fp32); exact: oracle fp32; rounded: the oracle's bf16
    result. The kernel's error vs the exact result within `slack` x the rounding floor."""
    floor = _rel(rounded, exact)
    err = _rel(got, exact)
    print(f"{name}: err {err:.4e} vs exact, floor {floor:.4e} (x{err / floor:.3f}), "
          f"vs rounded {_rel(got, rounded):.4e}")
    assert np.isfinite(got).all(), name
    assert err <= slack * floor, (name, err, floor)


def test_config3_llama7b_all_linear_b128_prefill():
    transformers = pytest.importorskip("transformers")  # noqa: F841
    import bc_eval as E
    import model_bench as MB
    import patch_llama_fft as P
    from bcfft import ops
    from oracle import bc_oracle as O
    dev = torch.device("cuda", 0)
    model = MB.build_model(argparse.Namespace(layers=32, config_overrides="{}", seed=0), dev)
    cfg = model.config
    assert (cfg.hidden_size, cfg.intermediate_size, cfg.num_hidden_layers) == (4096, 11008, 32)
    prompts = E.synthetic_prompts(20, 204, cfg.vocab_size, seed=0, min_len=180)
    ids, mask, last = (t.to(dev) for t in E.pad_batch(prompts, cfg.pad_token_id))
    n_tok = ids.numel()
    assert n_tok >= 2048
    with torch.inference_mode(), contextlib.redirect_stdout(io.StringIO()):
        P.patch_linear_with_block_circulant(model, num_layers_to_patch=32, block_size=128)
    assert P.fuse_attention_qkv(model) == 32 and P.fuse_mlp_gate_up(model) == 32
    # at this prefill size AUTO runs the whole MLP as one launch (bcfft_dmm.hip)
    assert ops.mlp_auto_is_fused(n_tok, 4096, 11008, 128, torch.bfloat16)

    seen = {}
    hooks = []

    def keep(key):
        def hook(m, inp, out):                      # returns None: the module's output is kept
            seen.setdefault(key, (m, inp[0].detach().clone(), out.detach().clone()))
        return hook

    for li in (0, cfg.num_hidden_layers - 1):
        layer = model.model.layers[li]
        for nm in ("q_proj", "k_proj", "v_proj", "o_proj"):
            hooks.append(getattr(layer.self_attn, nm).register_forward_hook(keep((li, nm))))
        hooks.append(layer.mlp.register_forward_hook(keep((li, "mlp"))))
    try:
        with torch.inference_mode():
            logits = model(input_ids=ids, attention_mask=mask).logits
    finally:
        for h in hooks:
            h.remove()
    assert torch.isfinite(logits.float()).all()
    assert len(seen) == 10, sorted(seen)

    for (li, nm), (m, x, y) in sorted(seen.items()):
        xn = x.float().reshape(-1, x.shape[-1]).cpu().numpy()      # bf16 values, exact in fp32
        g = y.float().reshape(xn.shape[0], -1).cpu().numpy()
        assert xn.shape[0] == n_tok
        if nm != "mlp":
            c = m.c.detach().float().cpu().numpy()
            exact = O.bc_forward(xn, c, None, x_dtype=O.F32)
            _check(f"layer {li} {nm}", g, exact, O.round_to(exact, O.BF16))
            continue
        cg, cu, cd = (p.c.detach().float().cpu().numpy() for p in (m.gate_proj, m.up_proj, m.down_proj))
        gt = O.bc_forward(xn, cg, x_dtype=O.F32)
        ut = O.bc_forward(xn, cu, x_dtype=O.F32)
        exact = O.bc_forward((_silu(gt) * ut).astype(np.float32), cd, x_dtype=O.F32)
        gr, ur = O.round_to(gt, O.BF16), O.round_to(ut, O.BF16)
        h = O.round_to((O.round_to(_silu(gr).astype(np.float32), O.BF16).astype(np.float64) * ur).astype(np.float32),
                       O.BF16)
        chain = O.bc_forward(h, cd, x_dtype=O.BF16)
        _check(f"layer {li} mlp (one launch)", g, exact, chain)
