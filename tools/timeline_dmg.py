"""Per-phase timeline of the multi-group 8-token kernel (bcfft_dmg.hip) from a stamps build
(tools/exp_one.sh st_dmg bcfft_dmg "-DBCFFT_STAMPS" -> lib/libbcfft_exp_st_dmg.so). Analysis tool.

Slots of each workgroup's second tile: 0 top, 1 x DMA issued, 2 stage 1, 3 Ba, 4 A fragments, 5 Bx,
then per output group g: stage 2, Bb, stage 3 (+ stores), Bc. Prints per phase the median over
workgroups of the slowest and the fastest wave, and per wave its median phase lengths, in
s_memtime ticks (100 MHz).
usage (GPU box): BCFFT_LIB_PATH=llama-fft_amd/lib/<stamps lib> python tools/timeline_dmg.py [N] [M]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama-fft_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from bcfft import _lib, ops  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    m = int(sys.argv[2]) if len(sys.argv) > 2 else 11008
    k, b = 4096, 128
    lib = _lib.load()
    lib.bcfft_set_stamps_dmg.argtypes = [ctypes.c_void_p]
    torch.manual_seed(0)
    c = (torch.randn(m // b, k // b, b) * 0.01).cuda().to(torch.bfloat16)
    spec = ops.spectra(c)
    x = torch.randn(n, k, device="cuda").to(torch.bfloat16)
    fwd = lambda: ops.forward(x, spec, None, b, m, algo="dft")  # noqa: E731
    for _ in range(50):
        fwd()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(20):
        fwd()
    e.record()
    torch.cuda.synchronize()
    wall = s.elapsed_time(e) / 20 * 1e3
    wgs = 2 * torch.cuda.get_device_properties(0).multi_processor_count
    buf = torch.zeros(wgs * 8 * 64, dtype=torch.int64, device="cuda")
    _lib.check(lib.bcfft_set_stamps_dmg(buf.data_ptr()), "stamps")
    fwd()
    torch.cuda.synchronize()
    _lib.check(lib.bcfft_set_stamps_dmg(None), "stamps")
    st = buf.view(wgs, 8, 64).cpu().numpy().astype(np.int64)
    ng = min(4, (m // b + 31) // 32)
    last = 9 + 4 * (ng - 1)
    st = st[(st[:, :, : last + 1] != 0).all((1, 2))]
    names = ["dma issue", "stage1", "Ba", "A frags", "Bx"]
    for g in range(ng):
        names += [f"g{g} stage2", f"g{g} Bb", f"g{g} stage3", f"g{g} Bc"]
    d = np.diff(st[:, :, : last + 1], axis=2)        # (wg, wave, phases)
    print(f"N={n} M={m}: event wall {wall:.1f} us per launch; {st.shape[0]} workgroups stamped (second tile)")
    print("  " + "  ".join(f"{nm} {np.median(d[:, :, i].max(1)):.0f}/{np.median(d[:, :, i].min(1)):.0f}"
                           for i, nm in enumerate(names)))
    print(f"  tile (slot 0 -> last Bc, slowest wave) median {np.median((st[:, :, last] - st[:, :, 0]).max(1)):.0f} ticks")
    for w in range(8):
        print(f"   wave {w}: " + "  ".join(f"{nm} {np.median(d[:, w, i]):.0f}" for i, nm in enumerate(names)))


if __name__ == "__main__":
    main()
