"""Phase ablation of the fused forward (performance analysis only; outputs are wrong when a
flag is set). Times the kernel with HIP events for each BCFFT_DEBUG_FLAGS combination."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama-fft_amd"))
import torch  # noqa: E402
from patch_llama_fft import BlockCirculantLinear  # noqa: E402


def timeit(layer, x, iters=30):
    with torch.inference_mode():
        for _ in range(5):
            layer(x)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(iters):
            layer(x)
        e.record()
        torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3   # us


def main():
    dev = torch.device("cuda:0")
    shapes = [(4096, 4096, 128, torch.float32), (4096, 4096, 128, torch.bfloat16)]
    flags = {"full": 0, "no_mfma": 1, "no_bload": 2, "no_mfma_no_bload": 3, "no_fwdfft": 4,
             "no_invfft": 8, "no_xpref": 16, "no_fft_both": 12, "only_loads_x_b": 12 | 1,
             "nothing": 31}
    out = {}
    for algo in ("mfma", "valu"):
        os.environ["BCFFT_ALGO"] = algo
        for k, m, b, dt in shapes:
            torch.manual_seed(0)
            layer = BlockCirculantLinear(k, m, block_size=b, bias=False).to(dev).to(dt).eval()
            x = torch.randn(8192, k, device=dev).to(dt)
            for name, f in (flags.items() if algo == "mfma" else [("full", 0)]):
                os.environ["BCFFT_DEBUG_FLAGS"] = str(f)
                us = timeit(layer, x)
                out[f"{algo} {k}x{m} b{b} {str(dt)[6:]} {name}"] = round(us, 1)
                print(f"{algo:5s} {k}x{m} b{b} {str(dt)[6:]:9s} {name:18s} {us:8.1f} us", flush=True)
            os.environ["BCFFT_DEBUG_FLAGS"] = "0"
    print(json.dumps(out))


if __name__ == "__main__":
    main()
