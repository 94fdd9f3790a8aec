"""Times the §8 f1/f3 kernels against the torch expressions they replace, on the device:
  * bcfft_grad_c (dc) at 4096 -> 4096, b = 128 / 64, N = 8192, fp32 and bf16 inputs, vs
    torch.fft rfft / einsum / irfft (the module's previous backward for dc);
  * bcfft_project_circulant (from_linear) on a LLaMA-7B gate weight (11008 x 4096 fp16, b = 128)
    vs the batched torch projection (patch_llama_fft._project_loss_aware_batched).
Prints one JSON line per measurement (median of 5 event-timed repeats of `iters` launches)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama-fft_amd"))
import torch  # noqa: E402

import patch_llama_fft as P  # noqa: E402
from bcfft import ops  # noqa: E402


def timed(fn, iters=10, reps=5):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    out = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        out.append(s.elapsed_time(e) / iters)
    return sorted(out)[len(out) // 2]


def torch_grad_c(x, dy, b):
    n = x.shape[0]
    xf = torch.fft.rfft(x.float().reshape(n, -1, b), dim=-1)
    df = torch.fft.rfft(dy.float().reshape(n, -1, b), dim=-1)
    return torch.fft.irfft(torch.einsum("nof,nif->oif", df, xf.conj()), n=b, dim=-1)


def main():
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    n, k, m = 8192, 4096, 4096
    for b in (128, 64):
        for dt in (torch.float32, torch.bfloat16):
            x = torch.randn(n, k, device=dev).to(dt)
            dy = torch.randn(n, m, device=dev).to(dt)
            t_k = timed(lambda: ops.grad_c(x, dy, b))
            t_t = timed(lambda: torch_grad_c(x, dy, b), iters=3)
            es = x.element_size()
            flops = 8 * (m // b) * (k // b) * (b // 2) * n + (k // b + m // b) * 2.5 * b * (b.bit_length() - 1) * n
            print(json.dumps({"op": "grad_c", "shape": f"{k}->{m} b={b} N={n}", "dtype": str(dt)[6:],
                              "ms": round(t_k, 4), "torch_fft_ms": round(t_t, 4), "speedup": round(t_t / t_k, 2),
                              "input_GB_s": round((n * k + n * m) * es / t_k / 1e6, 1),
                              "TFLOP_s": round(flops / t_k / 1e9, 1)}), flush=True)
    w = (torch.randn(11008, 4096, device=dev) * 0.02).half()
    b = 128
    t_k = timed(lambda: ops.project_circulant(w, b))
    blocks = w.view(11008 // b, b, 4096 // b, b).permute(0, 2, 1, 3)
    t_t = timed(lambda: P._project_loss_aware_batched(blocks), iters=3)
    same = torch.equal(ops.project_circulant(w, b), P._project_loss_aware_batched(blocks).float())
    print(json.dumps({"op": "project_circulant", "shape": "11008x4096 fp16 b=128", "ms": round(t_k, 4),
                      "torch_batched_ms": round(t_t, 4), "speedup": round(t_t / t_k, 2),
                      "GB_s": round(w.numel() * 2 / t_k / 1e6, 1), "equal_to_torch_batched": same}), flush=True)


if __name__ == "__main__":
    main()
