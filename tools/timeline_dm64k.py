"""Per-phase timeline of the b = 64 streamed-weight DFT kernel (bcfft_dm64k.hip) from a stamps
build (`make -C llama-fft_amd stamps` -> lib/libbcfft_stamps.so, or `make exp NAME=x
DEFS="-DBCFFT_STAMPS ..."`). Analysis tool.

Slots 8 c + p for the chunks c of each workgroup's second tile: p = 0 step top, 1 stage 3 (first
chunk only), 2 x DMA issued, 3 x landed, 4 stage 1, 5 Ba, 6 stage 2, 7 Bb. Prints per phase the
median over workgroups of the slowest and the fastest wave, in s_memtime ticks.
usage (GPU box): BCFFT_LIB_PATH=llama-fft_amd/lib/<stamps lib> python tools/timeline_dm64k.py [N]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("BCFFT_LIB_PATH", os.path.join(ROOT, "llama-fft_amd", "lib", "libbcfft_stamps.so"))
sys.path.insert(0, os.path.join(ROOT, "llama-fft_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from bcfft import _lib, ops  # noqa: E402

PH = ["stage3", "dma issue", "x wait", "stage1", "Ba", "stage2", "Bb"]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    k, m, b = 11008, 4096, 64
    lib = _lib.load()
    lib.bcfft_set_stamps_dm64k.argtypes = [ctypes.c_void_p]
    torch.manual_seed(0)
    c = (torch.randn(m // b, k // b, b) * 0.01).cuda().to(torch.bfloat16)
    spec = ops.spectra(c)
    x = torch.randn(n, k, device="cuda").to(torch.bfloat16)
    fwd = lambda: ops.forward(x, spec, None, b, m, algo="dft")  # noqa: E731
    for _ in range(100):
        fwd()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(50):
        fwd()
    e.record()
    torch.cuda.synchronize()
    wall = s.elapsed_time(e) / 50 * 1e3
    wgs = 4 * torch.cuda.get_device_properties(0).multi_processor_count
    buf = torch.zeros(wgs * 8 * 64, dtype=torch.int64, device="cuda")
    _lib.check(lib.bcfft_set_stamps_dm64k(buf.data_ptr()), "stamps")
    fwd()
    torch.cuda.synchronize()
    _lib.check(lib.bcfft_set_stamps_dm64k(None), "stamps")
    st = buf.view(wgs, 8, 64).cpu().numpy().astype(np.int64)
    st = st[(st[:, :, 0] != 0).all(1)]
    nch = (k // b + 31) // 32
    print(f"N={n}: event wall {wall:.1f} us per launch; {st.shape[0]} workgroups stamped (second tile, "
          f"{nch} chunks)")
    steps = []
    for cc in range(nch):
        t = st[:, :, 8 * cc: 8 * cc + 8]
        d = np.diff(t, axis=2)                     # (wg, wave, 7)
        nxt = st[:, :, 8 * (cc + 1)] if cc + 1 < nch else None
        row = {PH[i]: (np.median(d[:, :, i].max(1)), np.median(d[:, :, i].min(1))) for i in range(7)}
        if nxt is not None:
            row["tail"] = (np.median((nxt - t[:, :, 7]).max(1)), np.median((nxt - t[:, :, 7]).min(1)))
            steps.append(np.median((nxt - t[:, :, 0]).max(1)))
        print(f"-- chunk {cc}: " + "  ".join(f"{k_} {v[0]:.0f}/{v[1]:.0f}" for k_, v in row.items()))
    if steps:
        print(f"step (top to next top, slowest wave) median {np.median(steps):.0f} ticks")
    # per wave (chunk 1): median over workgroups of its stage-1 length, its stage-1 end after the
    # step top of the workgroup's earliest wave, and how often it is the workgroup's slowest
    t = st[:, :, 8: 16]
    top = t[:, :, 0].min(1, keepdims=True)
    s1 = t[:, :, 4] - t[:, :, 3]
    end = t[:, :, 4] - top
    slow = np.bincount(s1.argmax(1), minlength=8) / s1.shape[0]
    for w in range(8):
        print(f"   wave {w}: stage1 {np.median(s1[:, w]):.0f}  stage1 end {np.median(end[:, w]):.0f}  "
              f"stage2 {np.median(t[:, w, 6] - t[:, w, 5]):.0f}  slowest in {100 * slow[w]:.0f} % of workgroups")


if __name__ == "__main__":
    main()
