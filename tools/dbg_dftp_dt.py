"""Debug: dftx / dftp error vs the oracle per x dtype and bias, for the library in BCFFT_LIB_PATH."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "llama-fft_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bcfft import ops  # noqa: E402
from oracle import bc_oracle as O  # noqa: E402

dev = torch.device("cuda")
rng = np.random.default_rng(3)
c = (rng.standard_normal((32, 32, 128)) * 0.01).astype(np.float32)
spec = ops.spectra(torch.from_numpy(c).to(dev))
for n in (50, 2000):
    x = rng.standard_normal((n, 4096)).astype(np.float32)
    bv = (rng.standard_normal(4096) * 0.1).astype(np.float32)
    for xdt, odt in (("float32", O.F32), ("bfloat16", O.BF16), ("float16", O.F16)):
        xt = torch.from_numpy(x).to(dev).to(getattr(torch, xdt))
        xr = O.round_to(x, odt)
        for bias in (False, True):
            ref = O.bc_forward(xr, c, bv if bias else None, x_dtype=odt, bias_dtype=O.F32 if bias else None)
            out = []
            for algo in ("dftx", "dftp"):
                y = ops.forward(xt, spec, torch.from_numpy(bv).to(dev) if bias else None, 128, 4096, algo=algo)
                g = y.float().cpu().numpy()
                out.append(f"{algo} {np.linalg.norm(g - ref) / np.linalg.norm(ref):.2e} ({y.dtype})")
            print(f"N={n} x {xdt} bias {bias}: " + ", ".join(out), flush=True)
