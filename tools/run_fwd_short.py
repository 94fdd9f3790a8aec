"""rocprof driver: back-to-back forwards of BASELINE config 1 (4096 -> 4096, b = 64, fp32) and the
b = 128 decode shape at a few token counts, per engine, so a kernel trace gives the kernel's own
duration beside the launch gaps. usage: python tools/run_fwd_short.py [iters]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama-fft_amd"))
import torch  # noqa: E402
from bcfft import ops  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 200
for b in (64, 128):
    torch.manual_seed(1)
    c = torch.randn(4096 // b, 4096 // b, b, device="cuda") * 0.01
    spec = ops.spectra(c)
    for n in (1, 128):
        x = torch.randn(n, 4096, device="cuda")
        for algo in ("short", "stationary"):
            with torch.inference_mode():
                for _ in range(iters):
                    ops.forward(x, spec, None, b, 4096, algo=algo)
            torch.cuda.synchronize()
print("done")
