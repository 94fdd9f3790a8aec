"""BASELINE config 1 (4096 -> 4096, b = 64, N = 128, fp32 I/O) per engine: eager (HIP events around
back-to-back module calls) and HIP-graph replay of 10 forwards (bcfft.graph). One JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama-fft_amd"))
import torch  # noqa: E402
from bcfft import ops  # noqa: E402
from bcfft.graph import GraphedCall  # noqa: E402


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
    k = m = 4096
    b = 64
    torch.manual_seed(1)
    c = torch.randn(m // b, k // b, b, device="cuda") * 0.01
    spec = ops.spectra(c)
    out = {}
    for n in (128, 256, 1024):
        x = torch.randn(n, k, device="cuda")
        for algo in ("auto", "short", "stationary", "mfma", "valu"):
            f = lambda t, a=algo: ops.forward(t, spec, None, b, m, algo=a)  # noqa: E731
            with torch.inference_mode():
                e = timed(lambda: f(x), 100, 1)
                g = GraphedCall(f, [x], repeat=10)
                gr = timed(g.replay, 50, 10)
                del g
            out[f"N{n}_{algo}"] = {"eager_us": e, "graph_us": gr}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
