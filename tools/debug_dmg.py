"""Debug aid: the multi-group DFT kernel against the 8-token kernel run per output group (bit
comparison per group, token and 16-block N-tile)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "llama-fft_amd"))
from bcfft import ops  # noqa: E402

dev = torch.device("cuda:0")
k, b = 4096, 128
for m, n in ((11008, 37), (8192, 8), (8192, 1)):
    torch.manual_seed(5)
    c = (torch.randn(m // b, k // b, b, device=dev) * 0.01).to(torch.bfloat16)
    x = torch.randn(n, k, device=dev).to(torch.bfloat16)
    y = ops.forward(x, ops.spectra(c), None, b, m, algo="dft").float()
    torch.cuda.synchronize()
    for gi, g0 in enumerate(range(0, m // b, 32)):
        cg = c[g0:g0 + 32].contiguous()
        r = ops.forward(x, ops.spectra(cg), None, b, cg.shape[0] * b, algo="dft").float()
        yy = y[:, g0 * b:g0 * b + r.shape[1]]
        d = (yy - r).abs()
        per_tok = d.amax(dim=1)
        per_blk = d.view(n, -1, b).amax(dim=(0, 2))
        print(f"M={m} N={n} group {gi}: max|d| {d.max().item():.3e} (|r| max {r.abs().max().item():.3e}); "
              f"bad tokens {int((per_tok > 0).sum())}/{n}; bad blocks {[int(i) for i in torch.nonzero(per_blk > 0).flatten()][:40]}")

# the bias case of tests/test_gpu_dmg.py: where are the elements beyond ~1 ulp?
import numpy as np  # noqa: E402
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_gpu_stationary import _run  # noqa: E402
for m, n, bias in ((11008, 2049, True), (11008, 2049, False), (4096, 2049, True)):
    rng = np.random.default_rng(m + n)
    c = (rng.standard_normal((m // b, k // b, b)) * 0.01).astype(np.float32)
    bv = (rng.standard_normal(m) * 0.1).astype(np.float32) if bias else None
    x = rng.standard_normal((n, k)).astype(np.float32)
    x[0] *= 300.0
    x[n // 2, 1000:1100] *= 1e-3
    y, ref = _run(dev, x, c, bv, "bfloat16", "bfloat16", algo="dft")
    g = y.float().cpu().numpy()
    ulp = 2.0 ** -7
    rms = float(np.sqrt(np.mean(ref.astype(np.float64) ** 2)))
    bad = np.abs(g - ref) > 2 * ulp * np.abs(ref) + 2 * ulp * rms
    idx = np.argwhere(bad)
    print(f"M={m} N={n} bias={bias}: {len(idx)} bad; tokens {sorted(set(idx[:, 0].tolist()))[:10]}; "
          f"cols {idx[:5, 1].tolist()}; got {g[bad][:5]}; ref {ref[bad][:5]}; rms {rms:.3f}")
