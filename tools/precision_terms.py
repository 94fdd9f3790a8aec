"""Which single fp16 terms of the DFT engine's arithmetic set its error (CPU only; tests/dm_model.py
mirrors the kernels' roundings). For the precise engine's three residual terms (1: the stage-1 DFT
table, 2: the weight spectra, 3: the stage-3 table; dm_model precise=True, terms=...):
  * the structured from_linear layer of tests/test_gpu_0_north_star.py, its 48 most-cancelling
    tokens (raw per-token error, the north star's 1e-3 read per token);
  * the north star's random operator (seed 0), 64 tokens (Frobenius; the reference's T5 bar 1e-4);
  * the weight residual in other formats than e4m3 (exact, and MX-style e2m1 / e2m3 / e3m2 with a
    power-of-two scale per 16 or 4 input blocks), to see how few bits the residual may take.
usage: python tools/precision_terms.py   (writes nothing; profiles/r06q_precision_terms_narrow_residual.txt
holds a run)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "tests"), ROOT, os.path.join(ROOT, "llama-fft_amd")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import dm_model as DM  # noqa: E402
from oracle import bc_oracle as O  # noqa: E402
from test_gpu_0_north_star import _magnitude_norms, _structured_tokens  # noqa: E402


def structured_layer(m=4096, k=4096, b=128, seed=3):
    """tests/test_gpu_0_north_star.py::_structured_layer on the host (the module's host projection)."""
    from patch_llama_fft import BlockCirculantLinear
    g = torch.Generator().manual_seed(seed)
    w = torch.randn(m, k, generator=g) * 0.02
    rs = torch.logspace(-4, 0, m // b)[torch.randperm(m // b, generator=g)]
    cs = torch.logspace(-2, 0, k // b)[torch.randperm(k // b, generator=g)]
    w *= cs.repeat_interleave(b)[None, :]
    t = torch.arange(max(m, k), dtype=torch.float32)
    w += 0.05 * torch.outer(torch.cos(t[:m] * 0.01), torch.exp(-t[:k] / 700.0))
    w *= rs.repeat_interleave(b)[:, None]
    lin = torch.nn.Linear(k, m, bias=False)
    with torch.no_grad():
        lin.weight.copy_(w)
    return BlockCirculantLinear.from_linear(lin, block_size=b).c.detach().float().numpy()


def raw_residual(c):
    """conj(C) s_o - fp16(conj(C) s_o) before any rounding (dm_model.lo8_image without the e4m3)."""
    b = c.shape[-1]
    h = b // 2
    xf = np.fft.rfft(c.astype(np.float64), axis=-1) / (2.0 * b)
    p = xf[..., :h].astype(np.complex64).astype(np.complex128)
    p[..., 0] = np.float32(xf[..., 0].real) + 1j * np.float32(xf[..., h].real)
    mx = np.maximum(np.abs(p.real), np.abs(p.imag)).reshape(p.shape[0], -1).max(axis=1)
    n2 = np.array([int(np.clip(15 - np.frexp(np.float32(v))[1], -126, 126)) if v > 0 else 0 for v in mx])
    sc = (2.0 ** n2)[:, None, None]
    out = []
    for part in (p.real, p.imag):
        v = (part * sc).astype(np.float32)
        out.append(v.astype(np.float64) - v.astype(np.float16).astype(np.float64))
    return out


def mx_quant(r, i, mant, maxv, grp=16):
    """Element format with `mant` mantissa bits up to maxv, one power-of-two scale per (o, grp input
    blocks, bin) over the re and im parts."""
    no, ni, h = r.shape
    R, I = r.reshape(no, ni // grp, grp, h), i.reshape(no, ni // grp, grp, h)
    amax = np.maximum(np.abs(R).max(axis=2, keepdims=True), np.abs(I).max(axis=2, keepdims=True))
    s = 2.0 ** np.ceil(np.log2(np.maximum(amax, 1e-300) / maxv))

    def q(v):
        a = np.abs(v) / s
        step = 2.0 ** (np.maximum(np.floor(np.log2(np.maximum(a, 1e-300))), 0) - mant)
        return np.sign(v) * np.minimum(np.round(a / step) * step, maxv) * s
    return q(R).reshape(no, ni, h), q(I).reshape(no, ni, h)


# (name, mantissa bits, largest value, input blocks per power-of-two scale)
NARROW = (("e2m1, scale per 16 blocks", 1, 6.0, 16), ("e2m1, scale per 4 blocks", 1, 6.0, 4),
          ("e2m3, scale per 16 blocks", 3, 7.5, 16), ("e3m2, scale per 16 blocks", 2, 28.0, 16))


def report(name, x, c, ref, **kw):
    y = DM.dm_forward(x, c, **kw)
    d = (y - ref).astype(np.float64)
    pt = np.linalg.norm(d, axis=1) / np.linalg.norm(ref.astype(np.float64), axis=1)
    print(f"  {name:34s} worst token {pt.max():.3e}   Frobenius {np.linalg.norm(d) / np.linalg.norm(ref):.3e}",
          flush=True)


def main():
    c = structured_layer()
    x = _structured_tokens(512, 4096, seed=4)
    ref = O.bc_forward(x, c, None)
    amp = _magnitude_norms(x, c) / np.linalg.norm(ref.astype(np.float64), axis=1)
    idx = np.argsort(-amp)[:48]
    print(f"structured layer, 48 most-cancelling tokens (cancellation x{amp[idx].min():.0f} .. x{amp[idx].max():.0f})")
    xs, rs = x[idx], ref[idx]
    report("dftx", xs, c, rs, exact=True)
    for t in [(0, 0, 0), (1, 0, 0), (0, 1, 0), (0, 0, 1), (1, 1, 0), (0, 1, 1), (1, 1, 1)]:
        report(f"precise, residual terms {t}", xs, c, rs, precise=True, terms=t)
    orig = DM.lo8_image
    try:
        DM.lo8_image = lambda cc: tuple(raw_residual(cc))
        report("weight residual exact", xs, c, rs, precise=True)
        for name, mant, maxv, grp in NARROW:
            DM.lo8_image = lambda cc, m=mant, v=maxv, g=grp: mx_quant(*raw_residual(cc), m, v, g)
            report(f"weight residual {name}", xs, c, rs, precise=True)
    finally:
        DM.lo8_image = orig
    rng = np.random.default_rng(0)
    c = (rng.standard_normal((32, 32, 128)) * 0.01).astype(np.float32)
    rng.standard_normal(4096)
    x = rng.standard_normal((8192, 4096)).astype(np.float32)[:64]
    ref = O.bc_forward(x, c, None)
    print("north-star operator (random, seed 0), 64 tokens")
    report("dft", x, c, ref, exact=False)
    report("dftx", x, c, ref, exact=True)
    for t in [(1, 0, 0), (0, 1, 0), (0, 0, 1), (1, 1, 0), (1, 0, 1), (0, 1, 1), (1, 1, 1)]:
        report(f"precise, residual terms {t}", x, c, ref, precise=True, terms=t)
    print("north-star operator (random, seed 0), 64 tokens: narrow weight residuals", flush=True)
    try:
        for name, mant, maxv, grp in NARROW:
            DM.lo8_image = lambda cc, m=mant, v=maxv, g=grp: mx_quant(*raw_residual(cc), m, v, g)
            report(f"weight residual {name}", x, c, ref, precise=True)
    finally:
        DM.lo8_image = orig


if __name__ == "__main__":
    main()
