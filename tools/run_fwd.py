"""Run the BC forward a few times (for rocprofv3 counter passes / traces).
usage: run_fwd.py K M B IO N ITERS   (env BCFFT_ALGO honoured)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama-fft_amd"))
import torch  # noqa: E402
from patch_llama_fft import BlockCirculantLinear  # noqa: E402

k, m, b, io, n, iters = (int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4],
                         int(sys.argv[5]), int(sys.argv[6]))
dt = {"fp32": torch.float32, "bf16": torch.bfloat16, "fp16": torch.float16}[io]
torch.manual_seed(1)
layer = BlockCirculantLinear(k, m, block_size=b, bias=False).cuda().to(dt).eval()
x = torch.randn(n, k, device="cuda").to(dt)
with torch.inference_mode():
    for _ in range(iters):
        y = layer(x)
torch.cuda.synchronize()
print("done", tuple(y.shape), flush=True)
