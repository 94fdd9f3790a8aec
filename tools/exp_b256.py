"""b = 256 on the split-bf16 MFMA kernel (build with BCFFT_MFMA_MAXB=256) vs the fp32-VALU kernel:
agreement with the VALU output (exact fp32 CMAC) and with the oracle at small sizes, then kernel
time at the block-size sweep shapes (N = 8192). Analysis tool; select the library with
BCFFT_LIB_PATH."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama-fft_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
from bcfft import ops  # noqa: E402
from oracle import bc_oracle as O  # noqa: E402


def parity():
    for k, m, n, io, bias in ((1024, 512, 37, torch.float32, True), (4096, 4096, 64, torch.float32, False),
                              (4096, 11008, 19, torch.bfloat16, True), (11008, 4096, 8, torch.float32, True)):
        torch.manual_seed(0)
        c = torch.randn(m // 256, k // 256, 256) * 0.01
        bvec = torch.randn(m) * 0.1 if bias else None
        x = torch.randn(n, k).to(io)
        spec = ops.spectra(c.cuda())
        bd = bvec.cuda() if bias else None
        ym = ops.forward(x.cuda(), spec, bd, 256, m, algo="mfma").float().cpu()
        yv = ops.forward(x.cuda(), spec, bd, 256, m, algo="valu").float().cpu()
        ref = O.bc_forward(x.float().numpy(), c.numpy(), None if bvec is None else bvec.numpy())
        e_or = float(np.linalg.norm(ym.numpy() - ref) / np.linalg.norm(ref))
        e_mv = float((ym - yv).norm() / yv.norm())
        print(f"parity b256 {k}->{m} N={n} {io}: mfma vs oracle {e_or:.2e}, mfma vs valu {e_mv:.2e}", flush=True)
        assert e_or < (1e-3 if io == torch.float32 else 5e-3), e_or


def timing(k, m, io, algo, n=8192, iters=30):
    torch.manual_seed(1)
    c = (torch.randn(m // 256, k // 256, 256) * 0.01).cuda()
    spec = ops.spectra(c)
    x = torch.randn(n, k, device="cuda").to(io)
    for _ in range(5):
        ops.forward(x, spec, None, 256, m, algo=algo)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        ops.forward(x, spec, None, 256, m, algo=algo)
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / iters * 1e3
    es = x.element_size()
    nbytes = n * k * es + n * m * es + (m // 256) * (k // 256) * 129 * 8
    print(f"{algo:6s} {k}x{m} b256 {io} N={n}: {us:8.1f} us {nbytes / us / 1e3:7.1f} GB/s "
          f"{nbytes / us / 1e3 / 8000:.3f}", flush=True)


if __name__ == "__main__":
    parity()
    for k, m in ((4096, 4096), (4096, 11008), (11008, 4096)):
        for algo in ("mfma", "valu"):
            timing(k, m, torch.bfloat16, algo)
    timing(4096, 4096, torch.float32, "mfma")
    timing(4096, 4096, torch.float32, "valu")
