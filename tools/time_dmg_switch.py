"""Token counts where the multi-group kernels (bcfft_dmg.hip: one workgroup per 8-token tile for
ALL output groups) stop beating the per-group kernel (bcfft_dm8.hip: one workgroup per (tile,
group)): bf16 4096 -> 11008 and 4096 -> 12288 (fused q/k/v) forwards, the fused gate/up + SwiGLU,
and the whole MLP (fused one-launch and split). Run once with the product library and once with
an experiment build (BCFFT_LIB_PATH=... of `make exp NAME=nodmg DEFS=-DBCFFT_NO_DMG`).
HIP events around back-to-back launches; one JSON line per N."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama-fft_amd"))
import torch  # noqa: E402
from bcfft import _lib, ops  # noqa: E402


def timed(fn, iters=40):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return round(s.elapsed_time(e) / iters * 1e3, 1)


def main():
    b, h, f = 128, 4096, 11008
    tag = sys.argv[1]
    ns = [int(a) for a in sys.argv[2:]]
    torch.manual_seed(0)
    c = lambda o, i: (torch.randn(o // b, i // b, b) * 0.01).cuda()  # noqa: E731
    s_up = ops.spectra(c(f, h))
    s_qkv = ops.spectra(c(3 * h, h))
    s_gu = ops.spectra(ops.glu_weights(c(f, h), c(f, h)))
    s_d = ops.spectra(c(h, f))
    lib = _lib.load()
    st = _lib.stream_handle(torch.device("cuda:0"))
    BF16, NONE, AUTO = _lib.BCFFT_BF16, _lib.BCFFT_NONE, _lib.ALGO_AUTO
    for n in ns:
        x = torch.randn(n, h, device="cuda").to(torch.bfloat16)
        y_up = torch.empty(n, f, device="cuda", dtype=torch.bfloat16)
        y_qkv = torch.empty(n, 3 * h, device="cuda", dtype=torch.bfloat16)
        y = torch.empty(n, h, device="cuda", dtype=torch.bfloat16)
        wsb = lib.bcfft_forward_mlp_workspace_bytes(n, h, f, b, BF16, 2)
        ws = torch.empty(wsb, dtype=torch.uint8, device="cuda")
        t = {
            "up": timed(lambda: lib.bcfft_forward_ws(x.data_ptr(), BF16, n, h, f, b, s_up.data_ptr(), None, NONE,
                                                     y_up.data_ptr(), BF16, AUTO, None, 0, st)),
            "qkv": timed(lambda: lib.bcfft_forward_ws(x.data_ptr(), BF16, n, h, 3 * h, b, s_qkv.data_ptr(), None, NONE,
                                                      y_qkv.data_ptr(), BF16, AUTO, None, 0, st)),
            "glu": timed(lambda: lib.bcfft_forward_glu(x.data_ptr(), BF16, n, h, f, b, s_gu.data_ptr(),
                                                       y_up.data_ptr(), st)),
            "mlp_fused": timed(lambda: lib.bcfft_forward_mlp(x.data_ptr(), BF16, n, h, f, b, s_gu.data_ptr(),
                                                             s_d.data_ptr(), y.data_ptr(), 1, None, 0, st)),
            "mlp_split": timed(lambda: lib.bcfft_forward_mlp(x.data_ptr(), BF16, n, h, f, b, s_gu.data_ptr(),
                                                             s_d.data_ptr(), y.data_ptr(), 2, ws.data_ptr(), wsb, st)),
        }
        print(json.dumps({"lib": tag, "N": n, "us": t}), flush=True)


if __name__ == "__main__":
    main()
