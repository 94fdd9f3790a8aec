"""Dump the 8-token kernels' outputs at N = 4104 (bf16 bias forward and fused gate/up, b = 128
and 64) for a bitwise comparison of two library builds (e.g. the mixed stage order against
-DBCFFT_DM8_MIX=0 -DBCFFT_DM64_MIX=0). usage: python tools/dump_mixed.py OUT.pt"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama-fft_amd"))
import torch  # noqa: E402
from bcfft import ops  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    out = {}
    for b in (128, 64):
        g = torch.Generator(device="cpu").manual_seed(b)
        k, m, n = 4096, 4096, 4104
        c = (torch.randn(m // b, k // b, b, generator=g) * 0.01).to(dev).to(torch.bfloat16)
        bias = (torch.randn(m, generator=g) * 0.1).to(dev).to(torch.bfloat16)
        x = torch.randn(n, k, generator=g).to(dev).to(torch.bfloat16)
        out[f"y{b}"] = ops.forward(x, ops.spectra(c), bias, b, m, algo="dft").cpu()
        mg = 2048 if b == 128 else 1024
        cg = (torch.randn(mg // b, k // b, b, generator=g) * 0.01).to(dev)
        cu = (torch.randn(mg // b, k // b, b, generator=g) * 0.01).to(dev)
        out[f"h{b}"] = ops.forward_glu(x, ops.spectra(ops.glu_weights(cg, cu)), b, mg, algo="dft").cpu()
        out[f"h{b}_again"] = ops.forward_glu(x, ops.spectra(ops.glu_weights(cg, cu)), b, mg, algo="dft").cpu()
    torch.save(out, sys.argv[1])
    for k_, v in out.items():
        print(k_, tuple(v.shape), float(v.float().abs().mean()))


if __name__ == "__main__":
    main()
