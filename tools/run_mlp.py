"""Run the LLaMA-7B BC-MLP (4096 -> 11008 -> 4096, b = 128, bf16) `iters` times in one mode (fused /
split) for rocprofv3 PMC passes (tools/pmc_mlp.sh). usage: run_mlp.py N MODE ITERS"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama-fft_amd"))
import torch  # noqa: E402
from bcfft import ops  # noqa: E402


def main():
    n, mode, iters = int(sys.argv[1]), sys.argv[2], int(sys.argv[3])
    b, h, f = 128, 4096, 11008
    torch.manual_seed(0)
    c = lambda o, i: (torch.randn(o // b, i // b, b) * 0.01).cuda()  # noqa: E731
    sgu = ops.spectra(ops.glu_weights(c(f, h), c(f, h)))
    sd = ops.spectra(c(h, f))
    x = torch.randn(n, h, device="cuda").to(torch.bfloat16)
    for _ in range(iters):
        ops.forward_mlp(x, sgu, sd, b, f, mode=mode)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
