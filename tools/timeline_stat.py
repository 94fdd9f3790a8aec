"""Phase timeline and ablations of the stationary-weight kernel (analysis build only).

Loads lib/libbcfft_ablate.so (`make -C llama-fft_amd ablate`), or with TIMELINE_BUILD=stamps
lib/libbcfft_stamps.so (`make stamps`: stamps only, the product's control flow, no switches). Every wave stamps s_memtime at
the STAMP points of bc_forward_stat_kernel (bcfft_stat.hip):
  0 start | per M-tile it (base 1 + 7 min(it, 7)): +0 loop top, +1 inverse done, +2 stores and
  next DMA issued, +3 forward done, +4 after barrier Ba, +5 MFMAs + Y written, +6 after Bb | 63 end
and the phase switches (outputs are WRONG when set) time what each phase costs.
usage: python tools/timeline_stat.py [K M B IO N]   (GLU=1: the fused gate/up + SwiGLU launch,
       M = gate features, same weights for gate and up)
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STAMPS_ONLY = os.environ.get("TIMELINE_BUILD", "ablate") == "stamps"   # product control flow
os.environ["BCFFT_LIB_PATH"] = os.path.join(ROOT, "llama-fft_amd", "lib",
                                            "libbcfft_stamps.so" if STAMPS_ONLY else "libbcfft_ablate.so")
sys.path.insert(0, os.path.join(ROOT, "llama-fft_amd"))
import torch  # noqa: E402
from bcfft import _lib, ops  # noqa: E402

SEG = ["inverse", "stores+dma", "forward", "Ba wait", "cmac", "Bb wait"]
FLAGS = {"full": 0, "no_mfma": 1, "no_store": 2, "no_fwdfft": 4, "no_invfft": 8, "no_xdma": 16,
         "no_mem": 18, "no_fft": 12, "no_fft_no_mem": 30, "no_mem_no_aread": 18 | 32,
         "no_mem_no_atrans": 18 | 64, "no_mem_no_a_no_mfma": 18 | 32 | 64 | 1}


def run(k, m, b, io, n):
    dt = {"fp32": torch.float32, "bf16": torch.bfloat16}[io]
    lib = _lib.load()
    for f in ("bcfft_set_stamps_stat", "bcfft_set_ablation_stat"):
        getattr(lib, f).restype = ctypes.c_int
    lib.bcfft_set_stamps_stat.argtypes = [ctypes.c_void_p]
    lib.bcfft_set_ablation_stat.argtypes = [ctypes.c_int]
    torch.manual_seed(0)
    c = (torch.randn(m // b, k // b, b) * 0.01).cuda()
    glu = os.environ.get("GLU", "0") == "1"
    spec = ops.spectra(ops.glu_weights(c, c) if glu else c)
    x = torch.randn(n, k, device="cuda").to(dt)

    def fwd():
        if glu:
            return ops.forward_glu(x, spec, b, m)
        return ops.forward(x, spec, None, b, m, algo="stationary")

    def timeit(iters=30):
        for _ in range(3):
            fwd()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(iters):
            fwd()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / iters * 1e3

    groups = -(-(m // b) // (16 if glu else 32))
    buf = torch.zeros(256 * groups * 8 * 64, dtype=torch.int64, device="cuda")

    def stamps():
        buf.zero_()
        _lib.check(lib.bcfft_set_stamps_stat(buf.data_ptr()), "stamps")
        fwd()
        torch.cuda.synchronize()
        _lib.check(lib.bcfft_set_stamps_stat(None), "stamps")
        st = buf.view(-1, 64).cpu().numpy().astype(np.int64)
        st = st[st[:, 0] != 0]
        tiles = max(1, min(8, -(-(-(-n // 4)) // max(1, len(st) // 8))))   # M-tiles per workgroup
        seg = np.zeros((len(st), tiles, 6))
        for it in range(tiles):
            base = 1 + 7 * it
            for j in range(6):
                seg[:, it, j] = st[:, base + j + 1] - st[:, base + j]
        return st, seg

    print(f"{'flags':14s} {'us':>7s} " + " ".join(f"{h:>11s}" for h in SEG) + "   sum/tile")
    for name, fl in ({"full": 0} if STAMPS_ONLY else FLAGS).items():
        _lib.check(lib.bcfft_set_ablation_stat(fl), "ablation")
        us = timeit()
        _, seg = stamps()
        med = [np.median(seg[:, :, j]) for j in range(6)]
        print(f"{name:14s} {us:7.1f} " + " ".join(f"{v:11.0f}" for v in med) +
              f"   {np.median(seg.sum(axis=2)):8.0f}", flush=True)
    _lib.check(lib.bcfft_set_ablation_stat(0), "ablation")
    wall = timeit()
    st, seg = stamps()
    pro = np.median(st[:, 1] - st[:, 0])
    tot = np.median(st[:, 63] - st[:, 0])
    end = np.median(st[:, 63] - st[:, 1 + 7 * seg.shape[1]]) if seg.shape[1] < 8 else float("nan")
    wv = np.nonzero(buf.view(-1, 64).cpu().numpy()[:, 0])[0] % 8
    for w in range(8):
        sel = wv == w
        if sel.any():
            mid = seg[sel][:, 1:-1] if seg.shape[1] > 2 else seg[sel]
            print(f"wave {w}        " + " ".join(f"{np.median(mid[:, :, j]):11.0f}" for j in range(6)))
    print(f"waves {len(st)}, wall {wall:.1f} us, kernel cycles median {tot:.0f} "
          f"-> {tot / wall / 1e3:.2f} GHz implied; prologue {pro:.0f} cycles; first-tile sum "
          f"{np.median(seg[:, 0].sum(axis=1)):.0f}, last-tile sum {np.median(seg[:, -1].sum(axis=1)):.0f}, "
          f"after the last tile (drain) {end:.0f}")


if __name__ == "__main__":
    a = sys.argv[1:]
    k, m, b = (int(a[0]), int(a[1]), int(a[2])) if len(a) >= 3 else (4096, 4096, 128)
    io = a[3] if len(a) >= 4 else "fp32"
    n = int(a[4]) if len(a) >= 5 else 8192
    run(k, m, b, io, n)
