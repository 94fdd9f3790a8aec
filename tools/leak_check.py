"""For corrupted (token, block) rows of the MFMA forward, look for the token whose CORRECT
row matches best: a match from another tile means data leaked across workgroups."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama-fft_amd"))
import torch  # noqa: E402
from patch_llama_fft import BlockCirculantLinear  # noqa: E402

b = int(os.environ.get("DBG_B", "64"))
n = 8192
torch.manual_seed(0)
layer = BlockCirculantLinear(4096, 4096, block_size=b, bias=False).cuda().eval()
x = torch.randn(n, 4096, device="cuda")
with torch.inference_mode():
    os.environ["BCFFT_ALGO"] = "valu"
    yv = layer(x)
    os.environ["BCFFT_ALGO"] = "mfma"
    ym = layer(x)
nb = 4096 // b
dv = yv.view(n, nb, b)
dm = ym.view(n, nb, b)
err = (dm - dv).norm(dim=2) / dv.norm(dim=2)
bad = (err > 1e-3).nonzero()
print("bad (token, block) rows:", bad.shape[0])
for t, o in bad[:12].tolist():
    w = dm[t, o]                                   # wrong row
    cand = dv[:, o, :]                             # correct rows of every token, same block
    cos = (cand @ w) / (cand.norm(dim=1) * w.norm() + 1e-30)
    best = int(cos.argmax())
    # also: is the wrong row a mix? fit w = a*correct(t) + residual
    a = float((dv[t, o] @ w) / (dv[t, o] @ dv[t, o]))
    resid = float((w - a * dv[t, o]).norm() / w.norm())
    print(f"tok {t:5d} (tile {t//8:4d}, t%8={t%8}) blk {o:2d}: rel err {float(err[t, o]):.3f} "
          f"best-match tok {best:5d} (tile {best//8:4d}) cos {float(cos[best]):.3f} | "
          f"self-proj a={a:.3f} resid={resid:.3f}")
