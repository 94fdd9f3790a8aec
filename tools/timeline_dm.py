"""Phase timeline of the DFT-on-MFMA kernel (analysis build only: lib/libbcfft_stamps.so from
`make -C llama-fft_amd stamps`, the product's control flow with s_memtime stamps). Slots per wave
(bcfft_dm.hip): 0 start | per M-tile it (base 1 + 6 min(it, 8)): +0 loop top, +1 stage 1 (F waves
0-3) / stage 3 + DMA issue (I waves 4-7) done, +2 after barrier Ba, +3 x DMA issued (F waves), +4 stage 2 done,
+5 after Bb | 55-62 sub-phases of iteration 4 | 63 end. Prints per-wave-class medians of the segments in cycles.
usage: python tools/timeline_dm.py [M IO N]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["BCFFT_LIB_PATH"] = os.path.join(ROOT, "llama-fft_amd", "lib",
                                           os.environ.get("TIMELINE_LIB", "libbcfft_stamps.so"))
sys.path.insert(0, os.path.join(ROOT, "llama-fft_amd"))
import torch  # noqa: E402
from bcfft import _lib, ops  # noqa: E402

SEG = ["P1 work", "Ba wait", "dma issue", "stage2", "Bb wait"]


def run(m, io, n, k=4096, b=128):
    dt = {"fp32": torch.float32, "bf16": torch.bfloat16}[io]
    lib = _lib.load()
    lib.bcfft_set_stamps_dm.restype = ctypes.c_int
    lib.bcfft_set_stamps_dm.argtypes = [ctypes.c_void_p]
    torch.manual_seed(0)
    c = (torch.randn(m // b, k // b, b) * 0.01).cuda()
    spec = ops.spectra(c)
    x = torch.randn(n, k, device="cuda").to(dt)
    fwd = lambda: ops.forward(x, spec, None, b, m, algo=os.environ.get("TIMELINE_ALGO", "dft"))  # noqa: E731
    for _ in range(200):                         # settle the clock
        fwd()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(50):
        fwd()
    e.record()
    torch.cuda.synchronize()
    wall = s.elapsed_time(e) / 50 * 1e3
    groups = -(-(m // b) // 32)
    buf = torch.zeros(256 * groups * 8 * 64, dtype=torch.int64, device="cuda")
    _lib.check(lib.bcfft_set_stamps_dm(buf.data_ptr()), "stamps")
    fwd()
    torch.cuda.synchronize()
    _lib.check(lib.bcfft_set_stamps_dm(None), "stamps")
    raw = buf.view(-1, 64).cpu().numpy().astype(np.int64)
    rows = np.nonzero(raw[:, 0])[0]
    st = raw[rows]
    wv = rows % 8
    tiles = min(8, -(-n // 4) // max(1, len(st) // 8))
    seg = np.zeros((len(st), tiles, 5))
    for it in range(tiles):
        base = 1 + 6 * it
        for j in range(5):
            seg[:, it, j] = st[:, base + j + 1] - st[:, base + j]
    print(f"M={m} {io} N={n}: wall {wall:.1f} us, waves {len(st)}, tiles/WG {tiles}")
    print(f"{'':10s}" + " ".join(f"{h:>10s}" for h in SEG) + "   sum/tile")
    for name, sel in (("F 0-3", wv < 4), ("I 4-7", wv >= 4)):
        med = [np.median(seg[sel][:, 1:-1, j]) for j in range(5)] if tiles > 2 else [np.median(seg[sel][:, :, j]) for j in range(5)]
        print(f"{name:10s}" + " ".join(f"{v:10.0f}" for v in med) + f"   {sum(med):8.0f}")
    for w in range(8):
        sel = wv == w
        med = [np.median(seg[sel][:, 1:-1, j]) for j in range(5)] if tiles > 2 else [0] * 5
        print(f"wave {w}    " + " ".join(f"{v:10.0f}" for v in med))
    for it in range(tiles):                      # per iteration (iteration 4 carries the sub-phase stamps)
        row = []
        for name, sel in (("F", wv < 4), ("I", wv >= 4)):
            row.append(name + " " + " ".join(f"{np.median(seg[sel][:, it, j]):6.0f}" for j in range(5)))
        print(f"  it {it}: " + "   ".join(row))
    if tiles > 4:                                # sub-phases of iteration 4 (from its loop top)
        top = st[:, 1 + 6 * 4]
        fsub = ["dma wait", "h0 rd+max", "h0 mfma", "h0 X wr", "h1 rd+max", "h1 mfma", "h1 X wr", "-"]
        isub = ["Y+G read", "-", "compute", "stores", "-", "-", "-", "-"]
        for name, sel, lab in (("F", wv < 4, fsub), ("I", wv >= 4, isub)):
            prev = top[sel]
            out = []
            for j in range(8):
                cur = st[sel, 55 + j]
                ok = cur != 0
                d = np.where(ok, cur - prev, 0)
                out.append(f"{lab[j]} {np.median(d[ok]) if ok.any() else 0:.0f}")
                prev = np.where(ok, cur, prev)
            print(f"sub {name}: " + ", ".join(out))
    pro = np.median(st[:, 1] - st[:, 0])
    tot = np.median(st[:, 63] - st[:, 0])
    print(f"kernel cycles median {tot:.0f} -> {tot / wall / 1e3:.2f} GHz implied; prologue {pro:.0f} cycles; "
          f"first tile {np.median(seg[:, 0].sum(axis=1)):.0f}, per-tile sums: "
          + " ".join(f"{np.median(seg[:, i].sum(axis=1)):.0f}" for i in range(tiles)))


if __name__ == "__main__":
    a = sys.argv[1:]
    run(int(a[0]) if a else 4096, a[1] if len(a) > 1 else "fp32", int(a[2]) if len(a) > 2 else 8192)
