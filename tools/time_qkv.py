"""q/k/v of a LLaMA-7B layer (3 x 4096->4096, b = 128, fp32 and bf16) as three launches vs one
fused launch over the concatenated weights (patch_llama_fft.fuse_attention_qkv), at decode,
short-prompt and prefill token counts. Prints one JSON line per (N, dtype)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama-fft_amd"))
import torch  # noqa: E402

from bcfft import ops  # noqa: E402


def timed(fn, iters=50, reps=5):
    for _ in range(5):
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
        out.append(s.elapsed_time(e) / iters * 1e3)
    return sorted(out)[len(out) // 2]


def main():
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    b, k = 128, 4096
    cs = [torch.randn(32, 32, b, device=dev) * 0.01 for _ in range(3)]
    specs = [ops.spectra(c) for c in cs]
    spec_f = ops.spectra(torch.cat(cs, 0))
    for dt in (torch.float32, torch.bfloat16):
        for n in (1, 16, 128, 1024, 8192):
            x = torch.randn(n, k, device=dev).to(dt)
            t_sep = timed(lambda: [ops.forward(x, s, None, b, 4096) for s in specs])
            t_fused = timed(lambda: ops.forward(x, spec_f, None, b, 3 * 4096))
            print(json.dumps({"op": "qkv 3x4096->4096 b=128", "N": n, "dtype": str(dt)[6:],
                              "separate_us": round(t_sep, 1), "fused_us": round(t_fused, 1),
                              "speedup": round(t_sep / t_fused, 2)}), flush=True)


if __name__ == "__main__":
    main()
