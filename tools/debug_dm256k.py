"""Debug: bc_forward_dm256k_kernel against the oracle on small cases (finite fraction, error)."""
import os
import sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama-fft_amd"))
sys.path.insert(0, ROOT)
from bcfft import ops  # noqa: E402
from oracle import bc_oracle as O  # noqa: E402

for (k, m, n) in [(2048, 4096, 8), (4096 + 256, 4096, 8), (8192, 4096, 8), (11008, 4096, 8), (11008, 4096, 37)]:
    b = 256
    rng = np.random.default_rng(1)
    c = O.round_to((rng.standard_normal((m // b, k // b, b)) * 0.01).astype(np.float32), O.BF16)
    x = O.round_to(rng.standard_normal((n, k)).astype(np.float32), O.BF16)
    spec = ops.spectra(torch.from_numpy(c).cuda().to(torch.bfloat16))
    y = ops.forward(torch.from_numpy(x).cuda().to(torch.bfloat16), spec, None, b, m, algo="dft").float().cpu().numpy()
    ref = O.bc_forward(x, c, None, x_dtype=O.BF16)
    fin = np.isfinite(y)
    e = np.abs(np.where(fin, y, 0) - ref)
    print(f"K={k} M={m} N={n}: finite {fin.mean():.3f}; nonfinite tokens {sorted(set(np.where(~fin)[0].tolist()))[:10]}"
          f" blocks {sorted(set((np.where(~fin)[1] // b).tolist()))[:16]}; max err (finite) {e[fin].max() if fin.any() else -1:.3e}"
          f" |ref| {np.abs(ref).max():.3e}", flush=True)
    print("   y[0,:6]", y[0, :6], "ref", ref[0, :6], flush=True)
