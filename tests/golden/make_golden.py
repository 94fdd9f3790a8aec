"""Generate golden vectors by importing the REAL reference (build container only).

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py
It imports ``fft_utils`` and ``patch_llama_fft`` from /root/reference/src (read-only), runs
them on seeded inputs on the CPU, and writes inputs + outputs as .npz data files next to
this script. Only the resulting data is committed; no reference source or bytecode is
copied (PYTHONDONTWRITEBYTECODE=1 keeps __pycache__ out of /root/reference).

bf16 tensors are stored as their raw uint16 bit patterns (key suffix ``__bf16``).
"""
from __future__ import annotations

import os
import sys

import numpy as np

REF_SRC = "/root/reference/src"
OUT = os.path.dirname(os.path.abspath(__file__))


def _np(t):
    import torch
    t = t.detach().cpu()
    if t.dtype == torch.bfloat16:
        return t.view(torch.int16).numpy().view(np.uint16), "__bf16"
    if t.dtype == torch.float16:
        return t.numpy(), ""
    return t.numpy(), ""


def _save(name, **arrays):
    out = {}
    for k, v in arrays.items():
        if v is None:
            continue
        if isinstance(v, (int, float, str)):
            out[k] = np.asarray(v)
            continue
        a, suf = _np(v)
        out[k + suf] = a
    np.savez_compressed(os.path.join(OUT, name + ".npz"), **out)
    sz = os.path.getsize(os.path.join(OUT, name + ".npz"))
    print(f"  {name}.npz  {sz/1024:.1f} KiB  keys={sorted(out)}")


def main():
    sys.path.insert(0, REF_SRC)
    import torch
    import fft_utils
    import patch_llama_fft as plf

    dt = {"fp32": torch.float32, "fp16": torch.float16, "bf16": torch.bfloat16}

    # ---- forward cases: (name, K, M, b, x_shape_prefix, x dtype, module dtype, bias, bias_std)
    cases = [
        ("fwd_t5_128x64_b32", 128, 64, 32, (4,), "fp32", "fp32", False),      # validate T5 shape
        ("fwd_256x128_b64_bias", 256, 128, 64, (5,), "fp32", "fp32", True),
        ("fwd_4096sq_b128_fp32", 4096, 4096, 128, (3,), "fp32", "fp32", True),  # north-star shape
        ("fwd_4096sq_b128_bf16", 4096, 4096, 128, (17,), "bf16", "bf16", True),  # module.to(bf16)
        ("fwd_4096sq_b64_fp32", 4096, 4096, 64, (2,), "fp32", "fp32", True),    # BASELINE config 1
        ("fwd_4096sq_b256_fp32", 4096, 4096, 256, (3,), "fp32", "fp32", True),
        ("fwd_up_4096x11008_b128_f16", 4096, 11008, 128, (3,), "fp16", "fp32", False),  # LLaMA patched
        ("fwd_down_11008x4096_b128_bf16", 11008, 4096, 128, (2,), "bf16", "fp32", False),
        ("fwd_promote_bf16x_f32bias_512x256_b64", 512, 256, 64, (6,), "bf16", "fp32", True),
        ("fwd_3d_512x512_b128", 512, 512, 128, (2, 3), "fp32", "fp32", True),
        ("fwd_fp16x_fp16mod_1024x512_b256", 1024, 512, 256, (7,), "fp16", "fp16", True),
    ]
    print("forward cases:")
    for i, (name, k, m, b, pre, xdt, mdt, bias) in enumerate(cases):
        torch.manual_seed(1000 + i)
        mod = plf.BlockCirculantLinear(k, m, block_size=b, bias=bias)
        with torch.no_grad():
            mod.c.copy_(torch.randn_like(mod.c) * 0.01)
            if bias:
                mod.bias.copy_(torch.randn(m) * 0.1)
        mod = mod.to(dt[mdt]).eval()
        x = torch.randn(*pre, k).to(dt[xdt])
        with torch.no_grad():
            y = mod(x)
            cf = torch.fft.rfft(mod.c.to(torch.float32), dim=-1)
        small = mod.c.numel() <= 65536   # keep spectra only where they are cheap to store
        _save(name, x=x, c=mod.c, bias=mod.bias, y=y,
              cf_re=cf.real.contiguous() if small else None,
              cf_im=cf.imag.contiguous() if small else None,
              block_size=b, x_dtype=xdt, mod_dtype=mdt, y_dtype=str(y.dtype).replace("torch.", ""))

    # ---- circulant_matvec_fft (fft_utils.py:3-34), incl. non power of two n
    print("circulant_matvec_fft cases:")
    for i, (n, d) in enumerate([(64, "fp32"), (100, "fp32"), (128, "bf16"), (7, "fp32")]):
        torch.manual_seed(2000 + i)
        c = torch.randn(n).to(dt[d])
        x = torch.randn(n).to(dt[d])
        y = fft_utils.circulant_matvec_fft(c, x)
        _save(f"cmv_n{n}_{d}", c=c, x=x, y=y, dtype=d)

    # ---- from_linear (patch_llama_fft.py:180-224) known answers
    print("from_linear cases:")
    for i, (m, k, b, d, bias) in enumerate([(128, 256, 64, "fp32", True),     # validate T4 shape
                                            (256, 512, 128, "fp16", False),   # LLaMA fp16 source
                                            (256, 256, 32, "fp32", False)]):
        torch.manual_seed(3000 + i)
        lin = torch.nn.Linear(k, m, bias=bias)
        with torch.no_grad():
            lin.weight.uniform_(-1, 1)
            if bias:
                lin.bias.uniform_(-0.1, 0.1)
        lin = lin.to(dt[d])
        bc = plf.BlockCirculantLinear.from_linear(lin, block_size=b)
        _save(f"from_linear_{m}x{k}_b{b}_{d}", w=lin.weight, lin_bias=lin.bias,
              c=bc.c, bias=bc.bias, block_size=b, dtype=d)

    # validate T2 exact case c=[1..8]
    ct = torch.tensor([1., 2., 3., 4., 5., 6., 7., 8.])
    idx = torch.arange(8)
    C = ct[(idx[:, None] - idx[None, :]) % 8]
    _save("project_t2_exact", w=C, c=plf.dense_block_to_circulant_column_loss_aware(C))


if __name__ == "__main__":
    main()
