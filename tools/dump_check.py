"""Determinism of LDS contents at a given chunk (padding masked out): flag 256 dumps staging
(after the x load), flag 128 dumps the split-X image (after the FFT phase)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama-fft_amd"))
import torch  # noqa: E402
from patch_llama_fft import BlockCirculantLinear  # noqa: E402

b = int(os.environ.get("DBG_B", "64"))
extra = int(os.environ.get("DBG_EXTRA", "0"))
n = 8192
H = b // 2
L = 4 if H <= 32 else 8
P = H // L
SROW = max(b + 2 * L, 2 * P * (L + 1))
SROW = (SROW + 3) // 4 * 4
XS = 2 * 8 * 8 + 4
torch.manual_seed(0)
layer = BlockCirculantLinear(4096, 4096, block_size=b, bias=False).cuda().eval()
x = torch.randn(n, 4096, device="cuda")
os.environ["BCFFT_ALGO"] = "mfma"
for what, flag, width, valid, count in (("staging", 256 | extra, SROW, b, 64),
                                        ("x-image", 128 | extra, XS, 128, H)):
    for ch in range(4):
        os.environ["BCFFT_DEBUG_FLAGS"] = str(flag | (ch << 16))
        with torch.inference_mode():
            ys = [layer(x).view(torch.int32).view(n // 8, 8 * 4096)[:, : count * width].clone()
                  for _ in range(3)]
        ys = [y.view(n // 8, count, width)[:, :, :valid] for y in ys]
        d = ys[0] != ys[1]
        ntile = int(d.any(dim=2).any(dim=1).sum())
        info = ""
        if ntile:
            tl, r, c = d.nonzero()[0].tolist()
            cells = d.nonzero()
            info = f"first tile {tl} row/bin {r} col {c}; #cells {cells.shape[0]}; "
            if what == "x-image":
                cc = cells[:, 2]
                prec, t, blk = cc // 64, (cc % 64) // 8, cc % 8
                info += f"t-hist {torch.bincount(t, minlength=8).tolist()} blk-hist {torch.bincount(blk, minlength=8).tolist()}"
            else:
                rr = cells[:, 1]
                info += f"row(t*8+blk) t-hist {torch.bincount(rr // 8, minlength=8).tolist()}"
        print(f"{what:8s} chunk {ch}: tiles differing {ntile}  {info}", flush=True)
