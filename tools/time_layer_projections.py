"""Kernel time of each BC launch of one patched LLaMA-7B decoder layer (b = 128, bf16) at decode
and prefill token counts: fused q/k/v (4096 -> 12288), o (4096 -> 4096), fused gate/up + SwiGLU
(4096 -> 2 x 11008) and down (11008 -> 4096, split-K where the grid is short). HIP events on the
launch stream, mean over iterations. One JSON line per N."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama-fft_amd"))
import torch  # noqa: E402
from bcfft import ops  # noqa: E402


def timed(fn, iters=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    b, h, f = 128, 4096, 11008
    torch.manual_seed(0)
    c = lambda o, i: (torch.randn(o // b, i // b, b) * 0.01).cuda()  # noqa: E731
    s_qkv = ops.spectra(c(3 * h, h))
    s_o = ops.spectra(c(h, h))
    s_gu = ops.spectra(ops.glu_weights(c(f, h), c(f, h)))
    s_d = ops.spectra(c(h, f))
    for n in (20, 256, 1700, 8192):
        x = torch.randn(n, h, device="cuda").to(torch.bfloat16)
        xm = torch.randn(n, f, device="cuda").to(torch.bfloat16)
        t = {"qkv": timed(lambda: ops.forward(x, s_qkv, None, b, 3 * h)),
             "o": timed(lambda: ops.forward(x, s_o, None, b, h)),
             "gate_up_swiglu": timed(lambda: ops.forward_glu(x, s_gu, b, f)),
             "down": timed(lambda: ops.forward(xm, s_d, None, b, h)),
             # the whole MLP as the patched module runs it (one launch where AUTO takes it)
             "mlp_auto": timed(lambda: ops.forward_mlp(x, s_gu, s_d, b, f) if ops.mlp_auto_is_fused(
                 n, h, f, b, torch.bfloat16) else ops.forward(ops.forward_glu(x, s_gu, b, f), s_d, None, b, h))}
        print(json.dumps({"N": n, "us": {k: round(v, 1) for k, v in t.items()},
                          "layer_us": round(t["qkv"] + t["o"] + t["mlp_auto"], 1)}), flush=True)


if __name__ == "__main__":
    main()
