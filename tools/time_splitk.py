"""Short-grid launches at decode / prefill token counts, bf16: the down projection (11008 -> 4096)
at b = 128 (MFMA kernel) and b = 256 (VALU kernel), and 4096 -> 4096 at b = 256 (VALU kernel).
Split-K (ops.forward supplies the workspace) vs the unsplit launch (bcfft_forward_algo, no
workspace). HIP events on the launch stream, mean over iterations. One JSON line per (shape, N)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama-fft_amd"))
import torch  # noqa: E402
from bcfft import _lib, ops  # noqa: E402


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
    lib = _lib.load()
    for k, m, b, ns in ((11008, 4096, 128, (20, 256, 1024, 1700, 2040, 2048, 4096)),
                        (11008, 4096, 256, (20, 256, 1024, 2048)),
                        (4096, 4096, 256, (20, 256, 1024, 2048))):
        torch.manual_seed(0)
        spec = ops.spectra((torch.randn(m // b, k // b, b) * 0.01).cuda())
        for n in ns:
            x = torch.randn(n, k, device="cuda").to(torch.bfloat16)
            y = torch.empty(n, m, device="cuda", dtype=torch.bfloat16)
            s = _lib.stream_handle(x.device)

            def unsplit():
                lib.bcfft_forward_algo(x.data_ptr(), _lib.BCFFT_BF16, n, k, m, b, spec.data_ptr(), 0,
                                       _lib.BCFFT_NONE, y.data_ptr(), _lib.BCFFT_BF16, _lib.ALGOS["auto"], s)

            t_split = timed(lambda: ops.forward(x, spec, None, b, m))
            t_unsplit = timed(unsplit)
            ws = int(lib.bcfft_forward_workspace_bytes(n, k, m, b, 0))
            print(json.dumps({"shape": f"{k}->{m} b{b} bf16", "N": n, "slices": ws // (n * m * 4),
                              "split_us": round(t_split, 1), "unsplit_us": round(t_unsplit, 1)}), flush=True)


if __name__ == "__main__":
    main()
