"""Kernel time of the LLaMA-7B BC-MLP (b = 128, bf16, 4096 -> 11008 -> 4096) per token count:
the one-launch fused kernel (bcfft_forward_mlp FUSED, bcfft_dmm.hip) against the split form
(gate/up + SwiGLU launch, h in HBM, down launch), both through the C ABI with preallocated
buffers. HIP events on the launch stream around `iters` back-to-back calls. One JSON line per N."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama-fft_amd"))
import torch  # noqa: E402
from bcfft import _lib, ops  # noqa: E402


def timed(fn, iters):
    for _ in range(5):
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
    ns = [int(a) for a in sys.argv[1:]] or [20, 256, 1700, 4096, 8192]
    torch.manual_seed(0)
    c = lambda o, i: (torch.randn(o // b, i // b, b) * 0.01).cuda()  # noqa: E731
    s_gu = ops.spectra(ops.glu_weights(c(f, h), c(f, h)))
    s_d = ops.spectra(c(h, f))
    lib = _lib.load()
    stream = _lib.stream_handle(torch.device("cuda:0"))
    BF16 = _lib.BCFFT_BF16
    for n in ns:
        x = torch.randn(n, h, device="cuda").to(torch.bfloat16)
        y = torch.empty(n, h, device="cuda", dtype=torch.bfloat16)
        wsb = max(lib.bcfft_forward_mlp_workspace_bytes(n, h, f, b, BF16, _lib.MLP_MODES[m])
                  for m in ("split", "fused_splitk"))
        ws = torch.empty(wsb, dtype=torch.uint8, device="cuda")
        out = {}
        for mode in ("fused", "split", "fused_splitk"):
            code = _lib.MLP_MODES[mode]

            def call():
                _lib.check(lib.bcfft_forward_mlp(x.data_ptr(), BF16, n, h, f, b, s_gu.data_ptr(), s_d.data_ptr(),
                                                 y.data_ptr(), code, ws.data_ptr(), wsb, stream), "mlp")
            out[mode] = round(timed(call, 20 if n >= 4096 else 50), 1)
        # algorithmic HBM bytes of the fused unit: x and y (bf16) + both weight images once
        alg = 2 * n * h * 2
        print(json.dumps({"N": n, "us": out, "fused_vs_split": round(out["split"] / out["fused"], 3),
                          "fused_GBps_xy": round(alg / out["fused"] / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
