"""Which phase carries the nondeterminism? For each ablation flag, run the MFMA forward
several times and report max |y_a - y_b| between runs (0 => deterministic)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama-fft_amd"))
import torch  # noqa: E402
from patch_llama_fft import BlockCirculantLinear  # noqa: E402

bsz = int(os.environ.get("DBG_B", "64"))
torch.manual_seed(0)
layer = BlockCirculantLinear(4096, 4096, block_size=bsz, bias=False).cuda().eval()
x = torch.randn(8192, 4096, device="cuda")
os.environ["BCFFT_ALGO"] = "mfma"
for f in [0, 1, 2, 4, 8, 16, 32, 4 | 8, 1 | 2, 16 | 32]:
    os.environ["BCFFT_DEBUG_FLAGS"] = str(f)
    with torch.inference_mode():
        ys = [layer(x).clone() for _ in range(4)]
    d = max(float((ys[0] - y).abs().max()) for y in ys[1:])
    print(f"b={bsz} flags={f:3d}  run-to-run max diff {d:.3e}", flush=True)
