"""Debug: EP=9 16-bit x vs fp32 x with the same values, one nonzero input block per token."""
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
x = np.zeros((40, 4096), np.float32)
for t in range(32):
    x[t, 128 * t:128 * t + 128] = rng.standard_normal(128)
x[32] = rng.standard_normal(4096)                    # dense
x[33, :2048] = rng.standard_normal(2048)             # half 0 only
x[34, 2048:] = rng.standard_normal(2048)             # half 1 only
x[35, 5] = 1.0                                       # one element t=5 of block 0
x[36, 64 + 5] = 1.0                                  # t=69 of block 0
x[37, 2048 + 5] = 1.0                                # block 16
xr = O.round_to(x, O.BF16)
zb = torch.zeros(4096, device=dev)
y32 = ops.forward(torch.from_numpy(xr).to(dev), spec, zb, 128, 4096, algo="dftp").cpu().numpy()
y16 = ops.forward(torch.from_numpy(xr).to(dev).to(torch.bfloat16), spec, zb, 128, 4096, algo="dftp").cpu().numpy()
ref = O.round_to(y32, O.BF16)
err = np.linalg.norm(y16 - ref, axis=1) / np.maximum(np.linalg.norm(ref, axis=1), 1e-30)
np.set_printoptions(precision=4, suppress=True, linewidth=150)
print("per token (block t for t < 32; 32 dense, 33 half0, 34 half1, 35-37 single elements):")
print(err)
