"""Per-phase timeline of the 8-token DFT kernel (bcfft_dm8.hip) from its stamps build
(make -C llama-fft_amd exp NAME=st DEFS=-DBCFFT_STAMPS -> lib/libbcfft_exp_st.so). Analysis tool.

usage (on the GPU box): BCFFT_LIB_PATH=llama-fft_amd/lib/libbcfft_exp_st.so python tools/timeline_dm8.py [N]
Prints, per phase of iterations 0-8, the median over workgroups of the slowest and the fastest
wave's duration in s_memtime ticks (100 MHz)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama-fft_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from bcfft import _lib, ops  # noqa: E402

NAMES = {1: "wait own x", 2: "stage 1", 3: "stage 3 + DMA issue", 4: "Ba wait", 5: "stage 2 + Bb"}


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    k, m, b = 4096, 4096, 128
    lib = _lib.load()
    lib.bcfft_set_stamps_dm8.argtypes = [ctypes.c_void_p]
    torch.manual_seed(0)
    c = (torch.randn(m // b, k // b, b) * 0.01).cuda().to(torch.bfloat16)
    spec = ops.spectra(c)
    x = torch.randn(n, k, device="cuda").to(torch.bfloat16)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    for _ in range(50):
        ops.forward(x, spec, None, b, m, algo="dft")
    buf = torch.zeros(cus * 8 * 64, dtype=torch.int64, device="cuda")
    lib.bcfft_set_stamps_dm8(buf.data_ptr())
    ops.forward(x, spec, None, b, m, algo="dft")
    torch.cuda.synchronize()
    lib.bcfft_set_stamps_dm8(None)
    st = buf.view(cus, 8, 64).cpu().numpy().astype(np.int64)
    st = st[st[:, 0, 0] != 0]
    t0 = st[:, :, 0].min(1)
    print(f"N={n}: {st.shape[0]} workgroups stamped; start->end median {np.median(st[:, :, 63].max(1) - t0):.0f} "
          f"ticks; start spread {np.ptp(t0)}")
    if (st[:, :, 62] != 0).all():                   # slot 62: kernel entry, before the prologue
        pro = st[:, :, 0].min(1) - st[:, :, 62].min(1)
        print(f"prologue (entry -> loop start, x + table + weights): median {np.median(pro):.0f} ticks, "
              f"max {pro.max()}; entry spread over workgroups {np.ptp(st[:, :, 62].min(1))}")
    for it in range(9):
        base = 1 + 6 * it
        if not (st[:, :, base] != 0).all():
            break
        print(f"-- iteration {it}: top at {np.median(st[:, :, base].min(1) - t0):.0f}")
        prev = base
        for i in range(1, 6):
            cur = base + i
            if not (st[:, :, cur] != 0).all():
                continue
            d = st[:, :, cur] - st[:, :, prev]
            print(f"  {NAMES[i]:22s} slowest {np.median(d.max(1)):7.0f}  fastest {np.median(d.min(1)):7.0f}")
            prev = cur
    # per wave, iteration 3 (steady state): median phase lengths over workgroups
    base = 1 + 6 * 3
    if (st[:, :, base: base + 6] != 0).all():
        d = np.diff(st[:, :, base: base + 6], axis=2)
        for w in range(8):
            print(f"   wave {w}: " + "  ".join(f"{NAMES[i + 1]} {np.median(d[:, w, i]):.0f}" for i in range(5)))


if __name__ == "__main__":
    main()
