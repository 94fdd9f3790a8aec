"""Phase timeline of the short-N kernel (analysis build only: lib/libbcfft_stamps.so from
`make -C llama-fft_amd stamps`). Slots per wave (bcfft_sn.hip): 0 start | 1 x DMA issued | 2 table
written, fragments issued | 3 x and table landed | 4 prologue barrier | 5 stage 1 | 6 barrier | 7
stage 2 | 8 barrier | 9 stage 3. Prints median segment cycles over all waves, and the in-kernel
clock (s_memtime ticks over the event-timed wall). usage: python tools/timeline_sn.py"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["BCFFT_LIB_PATH"] = os.path.join(ROOT, "llama-fft_amd", "lib", "libbcfft_stamps.so")
sys.path.insert(0, os.path.join(ROOT, "llama-fft_amd"))
import torch  # noqa: E402
from bcfft import _lib, ops  # noqa: E402

SEG = ["dma issue", "tab+frag", "x wait", "bar0", "stage1", "bar1", "stage2", "bar2", "stage3"]


def run(b, n, m=4096, k=4096, io="fp32"):
    dt = {"fp32": torch.float32, "bf16": torch.bfloat16}[io]
    lib = _lib.load()
    lib.bcfft_set_stamps_sn.restype = ctypes.c_int
    lib.bcfft_set_stamps_sn.argtypes = [ctypes.c_void_p]
    torch.manual_seed(0)
    c = (torch.randn(m // b, k // b, b) * 0.01).cuda()
    spec = ops.spectra(c)
    x = torch.randn(n, k, device="cuda").to(dt)
    fwd = lambda: ops.forward(x, spec, None, b, m, algo="short")  # noqa: E731
    for _ in range(300):
        fwd()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(100):
        fwd()
    e.record()
    torch.cuda.synchronize()
    wall = s.elapsed_time(e) / 100 * 1e3
    wgs = -(-n // 4) * -(-(m // b) // 16)
    buf = torch.zeros(wgs * 8 * 64, dtype=torch.int64, device="cuda")
    _lib.check(lib.bcfft_set_stamps_sn(buf.data_ptr()), "stamps")
    fwd()
    torch.cuda.synchronize()
    _lib.check(lib.bcfft_set_stamps_sn(None), "stamps")
    st = buf.view(-1, 64).cpu().numpy().astype(np.int64)[:, :10]
    st = st[st[:, 0] != 0]
    seg = np.diff(st, axis=1)
    tot = np.median(st[:, 9] - st[:, 0])
    print(f"b={b} N={n} {io}: {wgs} workgroups, event wall {wall:.2f} us per launch, in-kernel median "
          f"{tot:.0f} cycles, start spread {(st[:, 0].max() - st[:, 0].min()):.0f}")
    print("  " + " ".join(f"{h:>9s}" for h in SEG))
    print("  " + " ".join(f"{v:9.0f}" for v in np.median(seg, axis=0)))
    print("  " + " ".join(f"{v:9.0f}" for v in np.max(seg, axis=0)) + "   (max)")


if __name__ == "__main__":
    for b, n in ((64, 1), (64, 128), (128, 1), (128, 128), (128, 512)):
        run(b, n)
