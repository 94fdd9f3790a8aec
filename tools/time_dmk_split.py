"""The down projection 11008 -> 4096 (b = 128, bf16) at decode / short-prefill token counts: the
streamed-weight kernel unsplit vs its K-chunk split (kz slices + the finishing pass), through the
C ABI with preallocated buffers; HIP events around back-to-back calls. One JSON line per N."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama-fft_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402
from bcfft import _lib, ops  # noqa: E402
from time_dmg_switch import timed  # noqa: E402


def main():
    b, k, m = 128, 11008, 4096
    torch.manual_seed(0)
    spec = ops.spectra((torch.randn(m // b, k // b, b) * 0.01).cuda())
    lib = _lib.load()
    st = _lib.stream_handle(torch.device("cuda:0"))
    BF16, NONE, AUTO = _lib.BCFFT_BF16, _lib.BCFFT_NONE, _lib.ALGO_AUTO
    for n in [int(a) for a in sys.argv[1:]] or [1, 20, 64, 128, 256, 512, 768, 1024]:
        x = torch.randn(n, k, device="cuda").to(torch.bfloat16)
        y = torch.empty(n, m, device="cuda", dtype=torch.bfloat16)
        wsb = lib.bcfft_forward_workspace_bytes_io(n, k, m, b, AUTO, BF16, BF16)
        ws = torch.empty(max(wsb, 16), dtype=torch.uint8, device="cuda")
        t = {"unsplit": timed(lambda: lib.bcfft_forward_ws(x.data_ptr(), BF16, n, k, m, b, spec.data_ptr(), None, NONE,
                                                           y.data_ptr(), BF16, AUTO, None, 0, st)),
             "split": timed(lambda: lib.bcfft_forward_ws(x.data_ptr(), BF16, n, k, m, b, spec.data_ptr(), None, NONE,
                                                         y.data_ptr(), BF16, AUTO, ws.data_ptr(), wsb, st)),
             "kz": wsb // (n * m * 4) if wsb > 0 else 1}
        print(json.dumps({"N": n, "us": t}), flush=True)


if __name__ == "__main__":
    main()
