"""Per-phase timeline of the fused MFMA forward (analysis build only).

Loads lib/libbcfft_ablate.so, hands it a stamp buffer (bcfft_set_stamps) and runs one forward;
every wave records s_memtime at the STAMP points of bc_forward_mfma_kernel:
  0 start | per chunk c (base 1+6c): +0 loop top, +1 after wait+barrier (half 0 landed),
  +2 after half-0 FFTs, +3 after wait+barrier (half 1 landed), +4 after half-1 FFTs,
  +5 after barrier (X image complete) -> MFMA phase runs until the next loop top
  49 loop end | 50/52 epilogue N-tile 0/1 after acc->LDS barriers | 51/53 after inverse+stores
Prints the mean/median duration of each segment over all waves, and the clock rate implied by
the launch's wall time. usage: python tools/timeline.py [K M B IO N]
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["BCFFT_LIB_PATH"] = os.path.join(ROOT, "llama-fft_amd", "lib", "libbcfft_ablate.so")
sys.path.insert(0, os.path.join(ROOT, "llama-fft_amd"))
import torch  # noqa: E402
from bcfft import _lib  # noqa: E402
from patch_llama_fft import BlockCirculantLinear  # noqa: E402


def main():
    a = sys.argv[1:]
    k, m, b = (int(a[0]), int(a[1]), int(a[2])) if len(a) >= 3 else (4096, 4096, 128)
    io = a[3] if len(a) >= 4 else "fp32"
    n = int(a[4]) if len(a) >= 5 else 8192
    dt = {"fp32": torch.float32, "bf16": torch.bfloat16, "fp16": torch.float16}[io]
    os.environ["BCFFT_ALGO"] = "mfma"
    lib = _lib.load()
    lib.bcfft_set_stamps.restype = ctypes.c_int
    lib.bcfft_set_stamps.argtypes = [ctypes.c_void_p]
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    layer = BlockCirculantLinear(k, m, block_size=b, bias=False).to(dev).to(dt).eval()
    x = torch.randn(n, k, device=dev).to(dt)
    tt, nw = 8, 4
    opw = 4096 // b
    n_blocks = ((n + tt - 1) // tt) * ((m // b + opw - 1) // opw)
    buf = torch.zeros(n_blocks * nw * 64, dtype=torch.int64, device=dev)
    with torch.inference_mode():
        for _ in range(3):
            layer(x)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(10):
            layer(x)
        e.record()
        torch.cuda.synchronize()
        wall_us = s.elapsed_time(e) / 10 * 1e3
        _lib.check(lib.bcfft_set_stamps(buf.data_ptr()), "set_stamps")
        layer(x)
        torch.cuda.synchronize()
        _lib.check(lib.bcfft_set_stamps(None), "set_stamps")
    st = buf.view(n_blocks * nw, 64).cpu().numpy().astype(np.int64)
    n_chunks = (k // b + 7) // 8
    t_start = st[:, 0]
    t_end = st[:, 53] if (4096 // b) // 16 > 1 else st[:, 51]
    span = t_end.max() - t_start.min()
    print(f"wall (no stamps) {wall_us:.1f} us; stamped span {span} ticks -> {span / wall_us:.0f} ticks/us")
    life = t_end - t_start
    print(f"wave lifetime: mean {life.mean():.0f} median {np.median(life):.0f} ticks")
    segs = [("dma prologue", 0, 1)]
    for c in range(n_chunks):
        bb = 1 + 6 * c
        nxt = 1 + 6 * (c + 1) if c + 1 < n_chunks else 49
        segs += [(f"c{c} wait+bar h0", bb, bb + 1), (f"c{c} fft h0", bb + 1, bb + 2),
                 (f"c{c} wait+bar h1", bb + 2, bb + 3), (f"c{c} dma+bload+fft h1", bb + 3, bb + 4),
                 (f"c{c} bar X", bb + 4, bb + 5), (f"c{c} mfma+dma h1", bb + 5, nxt)]
    segs += [("epi nt0 acc->lds", 49, 50), ("epi nt0 inv+store", 50, 51)]
    if (4096 // b) // 16 > 1:
        segs += [("epi nt1 acc->lds", 51, 52), ("epi nt1 inv+store", 52, 53)]
    tot = 0.0
    for name, i, j in segs:
        d = st[:, j] - st[:, i]
        tot += d.mean()
        print(f"{name:24s} mean {d.mean():8.0f}  median {np.median(d):8.0f}  p90 {np.percentile(d, 90):8.0f}")
    print(f"sum of means {tot:.0f}")
    # concurrency: how many waves alive over time (sampled)
    ts = np.linspace(t_start.min(), t_end.max(), 20)
    alive = [int(((t_start <= t) & (t_end > t)).sum()) for t in ts]
    print("waves alive over the launch:", alive)


if __name__ == "__main__":
    main()
