"""Per-algorithm kernel timing of the BC forward at the bench shapes (HIP events on the launch
stream, mean over iterations). Analysis tool; bench.py is the contract."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama-fft_amd"))
import torch  # noqa: E402
from bcfft import ops  # noqa: E402

DT = {"fp32": torch.float32, "bf16": torch.bfloat16}


def t_one(k, m, b, io, algo, n=8192, iters=50):
    torch.manual_seed(1)
    c = (torch.randn(m // b, k // b, b) * 0.01).cuda()
    spec = ops.spectra(c)
    x = torch.randn(n, k, device="cuda").to(DT[io])
    for _ in range(150):                            # ~10 ms: clocks settle before timing
        ops.forward(x, spec, None, b, m, algo=algo)
    reps = []
    for _ in range(5):                              # median of 5 repeats
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(iters):
            ops.forward(x, spec, None, b, m, algo=algo)
        e.record()
        torch.cuda.synchronize()
        reps.append(s.elapsed_time(e) / iters * 1e3)
    us = sorted(reps)[2]
    es = 4 if io == "fp32" else 2
    nbytes = n * k * es + n * m * es + (m // b) * (k // b) * (b // 2 + 1) * 8
    print(f"{algo:10s} {k}x{m} b{b} {io} N={n}: {us:8.1f} us  {nbytes / us / 1e3:7.1f} GB/s  "
          f"{nbytes / us / 1e3 / 8000:.3f} of 8 TB/s", flush=True)


def t_glu(k=4096, m=11008, b=128, n=8192, iters=50):
    """fused gate/up + SwiGLU (bcfft_forward_glu) at config 2, bf16"""
    torch.manual_seed(1)
    cg = (torch.randn(m // b, k // b, b) * 0.01).cuda().to(torch.bfloat16)
    cu = (torch.randn(m // b, k // b, b) * 0.01).cuda().to(torch.bfloat16)
    spec = ops.spectra(ops.glu_weights(cg, cu))
    x = torch.randn(n, k, device="cuda").to(torch.bfloat16)
    for _ in range(150):
        ops.forward_glu(x, spec, b, m)
    reps = []
    for _ in range(5):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(iters):
            ops.forward_glu(x, spec, b, m)
        e.record()
        torch.cuda.synchronize()
        reps.append(s.elapsed_time(e) / iters * 1e3)
    print(f"glu        {k}x{m} b{b} bf16 N={n}: {sorted(reps)[2]:8.1f} us", flush=True)


if __name__ == "__main__":
    shapes = [(4096, 4096, 128, "fp32", 8192), (4096, 4096, 128, "bf16", 8192), (4096, 11008, 128, "bf16", 8192),
              (4096, 4096, 64, "fp32", 8192)]
    algos = [a for a in sys.argv[1:] if not a.startswith("--")] or ["stationary", "mfma", "valu"]
    if "--down" in sys.argv:                        # K > 4096: the streamed-weight kernel vs split-K MFMA
        shapes = [(11008, 4096, 128, "bf16", n) for n in (16, 64, 256, 1024, 1700, 8192)]
    if "--xcd" in sys.argv:                         # shapes with several output groups (+ fused gate/up)
        shapes = [(4096, 11008, 128, "bf16", 8192), (4096, 11008, 64, "bf16", 8192), (4096, 4096, 64, "bf16", 8192)]
        t_glu()
    if "--cfg2" in sys.argv:                        # config 2 and its fused gate/up (bcfft_dmg.hip)
        shapes = [(4096, 11008, 128, "bf16", 8192)]
        t_glu()
    if "--downmid" in sys.argv:                     # the 8/16-token tile switch point
        shapes = [(11008, 4096, 128, "bf16", n) for n in (3000, 4096, 5000, 6144)]
    if "--b64down" in sys.argv:
        shapes = [(11008, 4096, 64, "bf16", n) for n in (1700, 8192)]
    if "--downsmall" in sys.argv:                   # decode sizes: AUTO's floor for the streamed kernel
        shapes = [(11008, 4096, 128, "bf16", n) for n in (1, 2, 4, 8, 16, 32)]
    if "--fp32n" in sys.argv:                       # the fp32 headline and its 1024-token shard
        shapes = [(4096, 4096, 128, "fp32", 8192), (4096, 4096, 128, "fp32", 1024)]
    if "--pipe" in sys.argv:                        # the bf16 K = 4096 DFT kernels (dm8, dmg, dm256, dm64)
        shapes = [(4096, 4096, 128, "bf16", 8192), (4096, 11008, 128, "bf16", 8192), (4096, 4096, 256, "bf16", 8192),
                  (4096, 11008, 256, "bf16", 8192), (4096, 4096, 64, "bf16", 8192), (4096, 4096, 128, "bf16", 1024)]
    if "--b64" in sys.argv:                         # the b = 64 sweep rows (bcfft_dm64.hip, bcfft_dm64k.hip)
        shapes = [(4096, 4096, 64, "bf16", 8192), (4096, 11008, 64, "bf16", 8192), (11008, 4096, 64, "bf16", 8192),
                  (11008, 4096, 64, "bf16", 1024), (11008, 4096, 64, "bf16", 64)]
    if "--b64up" in sys.argv:                       # b = 64, K = 4096: 2 and 6 output groups, fused gate/up
        shapes = [(4096, 4096, 64, "bf16", 8192), (4096, 11008, 64, "bf16", 8192), (4096, 11008, 64, "bf16", 1700)]
        t_glu(b=64)
    if "--b256" in sys.argv:                        # the b = 256 sweep rows (bcfft_dm256.hip)
        t_glu(b=256)
        shapes = [(4096, 4096, 256, "bf16", 8192), (4096, 11008, 256, "bf16", 8192), (11008, 4096, 256, "bf16", 8192),
                  (4096, 11008, 256, "bf16", 1700), (11008, 4096, 256, "bf16", 1024), (11008, 4096, 256, "bf16", 64)]
    if "--down2" in sys.argv:
        shapes = [(11008, 4096, 128, "bf16", n) for n in (1700, 8192)]
    if "--short" in sys.argv:                       # the short-N kernel against the persistent engines
        shapes = ([(4096, 4096, 64, "fp32", n) for n in (1, 16, 64, 128, 256, 512, 1024)]
                  + [(4096, 4096, 128, io, n) for io in ("fp32", "bf16") for n in (1, 16, 64, 128, 256, 512, 1024)]
                  + [(4096, 11008, 128, "bf16", n) for n in (20, 128, 256, 512)])
    if "--bf16all" in sys.argv:                     # every bf16 DFT kernel at the sweep's N = 8192 shapes
        shapes = [(k, m, b, "bf16", 8192) for b in (128, 64, 256)
                  for k, m in ((4096, 4096), (4096, 11008), (11008, 4096))]
    if "--smalln" in sys.argv:                      # AUTO's small-N crossover
        shapes = [(4096, 4096, b, io, n) for b in (64, 128) for io in ("fp32",) for n in (16, 64, 128, 256, 512, 1024, 2048)]
    for k, m, b, io, n in shapes:
        for algo in algos:
            try:
                t_one(k, m, b, io, algo, n=n)
            except RuntimeError as ex:
                print(algo, (k, m, b, io, n), "n/a:", str(ex)[:80])
