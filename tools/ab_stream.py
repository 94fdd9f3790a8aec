"""A/B timing of one library build over the kernels that stream weights from L2 beside the x / y
stream (HIP events, median of 5 repeats of 30 launches): the fp32 headline (dftx, dftp), the bf16
north star, config 2, the K > 4096 shapes at b = 64 / 128, and the one-launch MLP.
usage: BCFFT_LIB_PATH=... python tools/ab_stream.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama-fft_amd"))
import torch  # noqa: E402
from bcfft import ops  # noqa: E402

DT = {"fp32": torch.float32, "bf16": torch.bfloat16}


def med(fn, iters=30):
    for _ in range(60):
        fn()
    reps = []
    for _ in range(5):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        reps.append(s.elapsed_time(e) / iters * 1e3)
    return sorted(reps)[2]


def main():
    torch.manual_seed(1)
    shapes = ((4096, 4096, 128, "fp32", "dftx"), (4096, 4096, 128, "fp32", "dftp"),
              (4096, 4096, 128, "bf16", "auto"), (4096, 11008, 128, "bf16", "auto"),
              (11008, 4096, 128, "bf16", "auto"), (11008, 4096, 64, "bf16", "auto"),
              (4096, 11008, 64, "bf16", "auto"))
    if os.environ.get("AB_SET") == "more":          # the kernels the first A/B did not cover
        shapes = ((4096, 4096, 256, "bf16", "auto"), (4096, 11008, 256, "bf16", "auto"),
                  (11008, 4096, 256, "bf16", "auto"), (4096, 4096, 64, "bf16", "auto"),
                  (4096, 4096, 128, "fp32", "stationary"), (4096, 4096, 64, "fp32", "auto"))
    for (k, m, b, io, algo) in shapes:
        c = (torch.randn(m // b, k // b, b) * 0.01).cuda()
        spec = ops.spectra(c)
        x = torch.randn(8192, k, device="cuda").to(DT[io])
        us = med(lambda: ops.forward(x, spec, None, b, m, algo=algo))
        print(f"{k}x{m} b{b} {io} {algo}: {us:8.1f} us", flush=True)
    if os.environ.get("AB_SET") == "more":
        for b in (64, 256):                         # fused gate/up at the other block sizes
            cg, cu = ((torch.randn(11008 // b, 4096 // b, b) * 0.01).cuda() for _ in range(2))
            sgu = ops.spectra(ops.glu_weights(cg, cu))
            x = torch.randn(8192, 4096, device="cuda").to(torch.bfloat16)
            print(f"glu b{b}: {med(lambda: ops.forward_glu(x, sgu, b, 11008), 10):8.1f} us", flush=True)
        return
    k, m, b = 4096, 11008, 128
    cg, cu = ((torch.randn(m // b, k // b, b) * 0.01).cuda() for _ in range(2))
    cd = (torch.randn(k // b, m // b, b) * 0.01).cuda()
    x = torch.randn(8192, k, device="cuda").to(torch.bfloat16)
    sgu, sd = ops.spectra(ops.glu_weights(cg, cu)), ops.spectra(cd)
    print(f"MLP fused: {med(lambda: ops.forward_mlp(x, sgu, sd, b, m, mode='fused'), 10):8.1f} us", flush=True)


if __name__ == "__main__":
    main()
