"""Debug (analysis builds of tools/dbg_dftp16_build.sh, BIAS16=1): the precise engine on fp32 x
with a 16-bit bias (its BM = 2 instantiation) against the oracle, per token, for bias dtypes
bf16 and fp16; the same call with an fp32 bias of equal values beside it."""
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
rng = np.random.default_rng(5)
c = (rng.standard_normal((32, 32, 128)) * 0.01).astype(np.float32)
spec = ops.spectra(torch.from_numpy(c).to(dev))
x = rng.standard_normal((67, 4096)).astype(np.float32)
np.set_printoptions(precision=2, suppress=False, linewidth=150)
for name, bdt, odt in (("bf16", torch.bfloat16, O.BF16), ("fp16", torch.float16, O.F16)):
    b = O.round_to((rng.standard_normal(4096) * 0.1).astype(np.float32), odt)
    ref = O.bc_forward(x, c, b)
    xt = torch.from_numpy(x).to(dev)
    y16 = ops.forward(xt, spec, torch.from_numpy(b).to(dev).to(bdt), 128, 4096, algo="dftp").float().cpu().numpy()
    y32 = ops.forward(xt, spec, torch.from_numpy(b).to(dev), 128, 4096, algo="dftp").float().cpu().numpy()
    e16 = np.linalg.norm(y16 - ref, axis=1) / np.linalg.norm(ref, axis=1)
    e32 = np.linalg.norm(y32 - ref, axis=1) / np.linalg.norm(ref, axis=1)
    print(f"{name} bias: worst token {e16.max():.3e} (fp32 bias, same values: {e32.max():.3e}); "
          f"worst output block {max(np.linalg.norm((y16 - ref)[:, 128 * o:128 * o + 128]) / np.linalg.norm(ref[:, 128 * o:128 * o + 128]) for o in range(32)):.3e}")
    print("  per token:", e16[:12])
