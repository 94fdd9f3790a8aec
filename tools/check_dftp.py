"""Quick GPU check of the precise engine (BCFFT_ALGO_DFTP) against dftx at the north star:
accuracy vs the oracle (random and structured weights) and event-timed launch time.
usage: python tools/check_dftp.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "llama-fft_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bcfft import ops  # noqa: E402
from oracle import bc_oracle as O  # noqa: E402


def timeit(fn, iters=100):
    for _ in range(20):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def errs(g, ref):
    d = (g - ref).astype(np.float64)
    pt = np.linalg.norm(d, axis=1) / np.maximum(np.linalg.norm(ref.astype(np.float64), axis=1), 1e-30)
    return float(np.linalg.norm(d) / np.linalg.norm(ref)), float(pt.max())


def main():
    dev = torch.device("cuda")
    rng = np.random.default_rng(0)
    c = (rng.standard_normal((32, 32, 128)) * 0.01).astype(np.float32)
    bv = (rng.standard_normal(4096) * 0.1).astype(np.float32)
    x = rng.standard_normal((8192, 4096)).astype(np.float32)
    ref = O.bc_forward(x, c, bv)
    ref_nb = O.bc_forward(x[:1024], c, None)
    cd, xd, bd = torch.from_numpy(c).to(dev), torch.from_numpy(x).to(dev), torch.from_numpy(bv).to(dev)
    spec = ops.spectra(cd)
    for algo in ("dftx", "dftp"):
        y = ops.forward(xd, spec, bd, 128, 4096, algo=algo)
        y2 = ops.forward(xd[:1024], spec, None, 128, 4096, algo=algo)
        torch.cuda.synchronize()
        f, t = errs(y.cpu().numpy(), ref)
        f2, t2 = errs(y2.cpu().numpy(), ref_nb)
        quick = os.environ.get("QUICK") == "1"
        us = 0.0 if quick else timeit(lambda: ops.forward(xd, spec, None, 128, 4096, algo=algo))
        us_b = 0.0 if quick else timeit(lambda: ops.forward(xd, spec, bd, 128, 4096, algo=algo))
        print(f"{algo}: random+bias fro {f:.3e} worst tok {t:.3e} | no bias fro {f2:.3e} | "
              f"{us:.2f} us ({268967936 / max(us, 1e-9) / 1e6 / 8:.3f} of 8 TB/s), with bias {us_b:.2f} us", flush=True)
    # structured weights (tests/test_gpu_0_north_star.py's construction)
    from test_gpu_0_north_star import _structured_tokens
    import torch as T
    from patch_llama_fft import BlockCirculantLinear
    g = T.Generator().manual_seed(3)
    m = k = 4096
    b = 128
    w = T.randn(m, k, generator=g) * 0.02
    rs = T.logspace(-4, 0, m // b)[T.randperm(m // b, generator=g)]
    cs = T.logspace(-2, 0, k // b)[T.randperm(k // b, generator=g)]
    w *= cs.repeat_interleave(b)[None, :]
    t = T.arange(max(m, k), dtype=T.float32)
    w += 0.05 * T.outer(T.cos(t[:m] * 0.01), T.exp(-t[:k] / 700.0))
    w *= rs.repeat_interleave(b)[:, None]
    lin = T.nn.Linear(k, m, bias=False)
    with T.no_grad():
        lin.weight.copy_(w)
    mod = BlockCirculantLinear.from_linear(lin.to(dev), block_size=b).eval()
    cs_np = mod.c.detach().float().cpu().numpy()
    xs = _structured_tokens(512, k, seed=4)
    refs = O.bc_forward(xs, cs_np)
    specs = ops.spectra(mod.c.detach())
    for algo in ("dftx", "dftp", "mfma"):
        y = ops.forward(T.from_numpy(xs).to(dev), specs, None, 128, 4096, algo=algo)
        f, tk = errs(y.cpu().numpy(), refs)
        print(f"structured {algo}: fro {f:.3e} worst tok {tk:.3e}", flush=True)


if __name__ == "__main__":
    main()
