"""Golden vectors for the weight-prep and backward rows, made by importing
the REAL reference (build container only), like make_golden.py.

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_grad.py
  * bwd_*: torch autograd through the reference's BlockCirculantLinear.forward
    (patch_llama_fft.py:226-275) for a seeded upstream gradient dy: dx, dc, dbias.
  * from_linear_*: more from_linear known answers (patch_llama_fft.py:180-224): bf16 weights,
    and fp16 weights at LLaMA's scale (N(0, 0.02)).
Only the data is committed.
"""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from make_golden import REF_SRC, _save  # noqa: E402


def main():
    sys.path.insert(0, REF_SRC)
    import torch
    import patch_llama_fft as plf

    dt = {"fp32": torch.float32, "fp16": torch.float16, "bf16": torch.bfloat16}
    # (name, K, M, b, x shape prefix, x dtype, module dtype, bias)
    cases = [
        ("bwd_256x512_b64_bias", 256, 512, 64, (6,), "fp32", "fp32", True),
        ("bwd_3d_512x256_b128", 512, 256, 128, (2, 5), "fp32", "fp32", False),
        ("bwd_4096sq_b128", 4096, 4096, 128, (3,), "fp32", "fp32", True),        # north-star shape
        ("bwd_256x256_b32_bf16", 256, 256, 32, (9,), "bf16", "bf16", True),      # module.to(bf16)
        ("bwd_512x1024_b256_f16x", 512, 1024, 256, (4,), "fp16", "fp32", False),
        # 16-bit x, fp32 module with a bias: y = y16 + bias promotes to fp32, and autograd rounds
        # the x-side gradient to bf16 before dx / dc (patch_llama_fft.py:266-271)
        ("bwd_promote_bf16x_f32bias_512x256_b64", 512, 256, 64, (7,), "bf16", "fp32", True),
    ]
    only = os.environ.get("GOLDEN_ONLY")          # regenerate selected fixtures only
    print("backward cases:")
    for i, (name, k, m, b, pre, xdt, mdt, bias) in enumerate(cases):
        if only and name not in only.split(","):
            continue
        torch.manual_seed(4000 + i)
        mod = plf.BlockCirculantLinear(k, m, block_size=b, bias=bias)
        with torch.no_grad():
            mod.c.copy_(torch.randn_like(mod.c) * 0.01)
            if bias:
                mod.bias.copy_(torch.randn(m) * 0.1)
        mod = mod.to(dt[mdt])
        x = torch.randn(*pre, k).to(dt[xdt]).requires_grad_(True)
        y = mod(x)
        dy = torch.randn(y.shape).to(y.dtype)
        params = [x, mod.c] + ([mod.bias] if bias else [])
        grads = torch.autograd.grad(y, params, dy)
        _save(name, x=x, c=mod.c, bias=mod.bias, dy=dy, dx=grads[0], dc=grads[1],
              dbias=grads[2] if bias else None, block_size=b, x_dtype=xdt, mod_dtype=mdt)

    print("from_linear cases:")
    if only:
        return
    for i, (m, k, b, d, scale) in enumerate([(256, 512, 64, "bf16", 1.0),
                                             (512, 1024, 128, "fp16", 0.02)]):
        torch.manual_seed(5000 + i)
        lin = torch.nn.Linear(k, m, bias=False)
        with torch.no_grad():
            if scale == 1.0:
                lin.weight.uniform_(-1, 1)
            else:
                lin.weight.normal_(0.0, scale)
        lin = lin.to(dt[d])
        bc = plf.BlockCirculantLinear.from_linear(lin, block_size=b)
        _save(f"from_linear_{m}x{k}_b{b}_{d}", w=lin.weight, c=bc.c, block_size=b, dtype=d)


if __name__ == "__main__":
    main()
