"""Ablation timing of bcfft_grad_c (analysis builds, BCFFT_GRAD_ABL): which phase sets its time.
usage: BCFFT_LIB_PATH=<lib> python tools/time_grad_abl.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama-fft_amd"))
import torch  # noqa: E402

from bcfft import ops  # noqa: E402

x = torch.randn(8192, 4096, device="cuda")
dy = torch.randn(8192, 4096, device="cuda")
for _ in range(3):
    ops.grad_c(x, dy, 128)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(20):
    ops.grad_c(x, dy, 128)
e.record()
torch.cuda.synchronize()
print(os.environ.get("BCFFT_LIB_PATH", "product"), f"{s.elapsed_time(e) / 20 * 1e3:.1f} us")
