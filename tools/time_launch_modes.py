"""Per-forward time of the fp32 north-star layer (4096 -> 4096, b = 128) at a rank's shard sizes
of the strong-scaling partition (8192 / g tokens): eager back-to-back launches vs HIP-graph
replays of 1 and 10 forwards per graph (bcfft.graph.GraphedCall). HIP events around the loop;
shows how much of a short launch is the inter-kernel gap. One JSON line per N."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama-fft_amd"))
import torch  # noqa: E402
from bcfft.graph import GraphedCall  # noqa: E402
from patch_llama_fft import BlockCirculantLinear  # noqa: E402


def timed(fn, iters, per):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return round(s.elapsed_time(e) / iters / per * 1e3, 2)


def main():
    torch.manual_seed(1)
    layer = BlockCirculantLinear(4096, 4096, block_size=128, bias=False).cuda().eval()
    for n in [int(a) for a in sys.argv[1:]] or [1024, 2048, 4096, 8192]:
        x = torch.randn(n, 4096, device="cuda")
        with torch.inference_mode():
            layer(x)
            out = {"eager": timed(lambda: layer(x), 200, 1)}
            for rep in (1, 10):
                g = GraphedCall(lambda t: layer(t), [x], repeat=rep)
                out[f"graph{rep}"] = timed(g.replay, 100, rep)
                del g
        print(json.dumps({"N": n, "us_per_forward": out}), flush=True)


if __name__ == "__main__":
    main()
