"""Per-phase timeline of the streamed-weight DFT kernel (bcfft_dmk.hip) from its stamps build
(tools/ab_dmk.sh build st -DBCFFT_STAMPS -> lib/libbcfft_exp_st.so). Analysis tool.

usage (on the GPU box): BCFFT_LIB_PATH=llama-fft_amd/lib/libbcfft_exp_st.so python tools/timeline_dmk.py N
Prints, per phase of tiles 0 and 1, the median over workgroups of the slowest wave's duration
and of the fastest wave's, in s_memtime ticks."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama-fft_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from bcfft import _lib, ops  # noqa: E402

NAMES = {0: "step0 top", 1: "B(0)+stage1", 3: "stage3 (prev half)", 4: "Ba wait",
         5: "DMA+stage2 (first)", 6: "Bb wait"}
for c in range(1, 6):
    NAMES[7 + 3 * (c - 1)] = f"c{c}: wait+DMA+stage1"
    NAMES[8 + 3 * (c - 1)] = f"c{c}: Ba wait"
    NAMES[9 + 3 * (c - 1)] = f"c{c}: stage2+Bb"
NAMES.update({22: "ywrite0+Bc", 23: "stage3 half0", 24: "Bd wait", 25: "ywrite+Be"})


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    k, m, b = 11008, 4096, 128
    lib = _lib.load()
    lib.bcfft_set_stamps_dmk.argtypes = [ctypes.c_void_p]
    torch.manual_seed(0)
    c = (torch.randn(m // b, k // b, b) * 0.01).cuda().to(torch.bfloat16)
    spec = ops.spectra(c)
    x = torch.randn(n, k, device="cuda").to(torch.bfloat16)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    for _ in range(20):
        ops.forward(x, spec, None, b, m, algo="dft")
    buf = torch.zeros(cus * 8 * 64, dtype=torch.int64, device="cuda")
    lib.bcfft_set_stamps_dmk(buf.data_ptr())
    ops.forward(x, spec, None, b, m, algo="dft")
    torch.cuda.synchronize()
    lib.bcfft_set_stamps_dmk(None)
    st = buf.view(cus, 8, 64).cpu().numpy().astype(np.int64)
    used = st[:, 0, 0] != 0
    st = st[used]
    print(f"N={n}: {st.shape[0]} workgroups stamped; total (start->end) median "
          f"{np.median(st[:, :, 63].max(1) - st[:, :, 0].min(1)):.0f} ticks")
    for t in range(2):
        base = 1 + 30 * t
        ids = [i for i in range(26) if (st[:, :, base + i] != 0).all()]
        if not ids:
            continue
        prev = base + ids[0]
        print(f"-- tile {t}: top at {np.median(st[:, :, prev].min(1) - st[:, :, 0].min(1)):.0f}")
        for i in ids[1:]:
            cur = base + i
            d = st[:, :, cur] - st[:, :, prev]
            print(f"  {NAMES.get(i, i):24s} slowest {np.median(d.max(1)):7.0f}  fastest {np.median(d.min(1)):7.0f}")
            prev = cur
    # per wave, tile 1, chunk step 2 (steady state): median over workgroups
    base = 1 + 30
    cols = [(10, 9), (11, 10), (12, 11)]          # (end slot, start slot) of c2's three phases
    if all((st[:, :, base + a] != 0).all() and (st[:, :, base + b] != 0).all() for a, b in cols):
        for w in range(8):
            parts = [f"{NAMES[a]} {np.median(st[:, w, base + a] - st[:, w, base + b]):.0f}" for a, b in cols]
            print(f"   wave {w}: " + "  ".join(parts))


if __name__ == "__main__":
    main()
