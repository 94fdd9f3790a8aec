"""Phase ablation of the fused MFMA forward (performance analysis only: outputs are WRONG when a
switch is set). Loads the analysis build lib/libbcfft_ablate.so (`make -C llama-fft_amd ablate`),
whose kernels read a device flag word (bcfft_set_ablation), and times each combination with
HIP events. The product library has no such switches.
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["BCFFT_LIB_PATH"] = os.path.join(ROOT, "llama-fft_amd", "lib", "libbcfft_ablate.so")
sys.path.insert(0, os.path.join(ROOT, "llama-fft_amd"))
import torch  # noqa: E402
from bcfft import _lib  # noqa: E402
from patch_llama_fft import BlockCirculantLinear  # noqa: E402

FLAGS = {"full": 0, "no_mfma": 1, "no_bload": 2, "no_fwdfft": 4, "no_invfft": 8, "no_xdma": 16,
         "no_fft_both": 12, "no_mfma_no_bload": 3, "only_mem": 15, "nothing": 31}


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
    lib = _lib.load()
    lib.bcfft_set_ablation.restype = ctypes.c_int
    lib.bcfft_set_ablation.argtypes = [ctypes.c_int]
    dev = torch.device("cuda:0")
    shapes = [(4096, 4096, 128, torch.float32), (4096, 4096, 128, torch.bfloat16)]
    out = {}
    for algo in ("mfma", "valu"):
        os.environ["BCFFT_ALGO"] = algo
        for k, m, b, dt in shapes:
            torch.manual_seed(0)
            layer = BlockCirculantLinear(k, m, block_size=b, bias=False).to(dev).to(dt).eval()
            x = torch.randn(8192, k, device=dev).to(dt)
            for name, f in (FLAGS.items() if algo == "mfma" else [("full", 0)]):
                _lib.check(lib.bcfft_set_ablation(f), "bcfft_set_ablation")
                us = timeit(layer, x)
                key = f"{algo} {k}x{m} b{b} {str(dt)[6:]} {name}"
                out[key] = round(us, 1)
                print(f"{key:45s} {us:8.1f} us", flush=True)
            _lib.check(lib.bcfft_set_ablation(0), "bcfft_set_ablation")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
