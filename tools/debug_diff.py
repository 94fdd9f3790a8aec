"""Locate mismatches between the MFMA and VALU forward (debug aid)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama-fft_amd"))
import torch  # noqa: E402
from patch_llama_fft import BlockCirculantLinear  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
if len(sys.argv) > 2:
    os.environ["BCFFT_DEBUG_FLAGS"] = sys.argv[2]
bsz = int(os.environ.get("DBG_B", "128"))
torch.manual_seed(0)
layer = BlockCirculantLinear(4096, 4096, block_size=bsz, bias=False).cuda().eval()
x = torch.randn(n, 4096, device="cuda")
with torch.inference_mode():
    os.environ["BCFFT_ALGO"] = "valu"
    f = os.environ.pop("BCFFT_DEBUG_FLAGS", None)
    yv = layer(x)
    if f:
        os.environ["BCFFT_DEBUG_FLAGS"] = f
    os.environ["BCFFT_ALGO"] = "mfma"
    ym = layer(x)
    ym2 = layer(x)
d = (ym - yv).abs()
rel = d.norm() / yv.norm()
print(f"N={n} rel err {rel:.3e}  max abs {d.max():.3e}  run-to-run diff {(ym - ym2).abs().max():.3e}")
bad = d > 1e-3 * yv.abs().max()
print("bad elements:", int(bad.sum()), "of", bad.numel())
tok_bad = bad.any(dim=1).nonzero().flatten()
print("bad tokens:", tok_bad.numel(), tok_bad[:40].tolist())
if tok_bad.numel():
    wg = (tok_bad // 8).unique()
    print("bad tiles (token//8):", wg.numel(), wg[:40].tolist())
    print("token%8 histogram:", torch.bincount(tok_bad % 8, minlength=8).tolist())
    blk_bad = bad.view(n, 4096 // bsz, bsz).any(dim=2).any(dim=0).nonzero().flatten()
    print("bad output blocks:", blk_bad.tolist())
    t0 = int(tok_bad[0])
    print("first bad token row, bad cols:", bad[t0].nonzero().flatten()[:20].tolist())
