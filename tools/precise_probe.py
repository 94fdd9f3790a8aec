"""The fp32 engines' accuracy AND time in one run, for A/B builds of the precise engine
(BCFFT_LIB_PATH selects the library): per algorithm, the kernel time at the north star (8192 tokens)
and its 1024-token shard, the raw worst token on structured from_linear weights (the test of
tests/test_gpu_0_north_star.py::test_structured_weights_per_block_and_token) and the Frobenius
error on the north-star operator (first 1024 tokens) against the oracle.
usage: python tools/precise_probe.py [algo ...]   (default: dftx dftp)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "llama-fft_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bcfft import ops  # noqa: E402
from oracle import bc_oracle as O  # noqa: E402
from test_gpu_0_north_star import _per_token, _structured_layer, _structured_tokens  # noqa: E402


def kernel_us(x, spec, algo, iters=50):
    for _ in range(100):
        ops.forward(x, spec, None, 128, 4096, algo=algo)
    reps = []
    for _ in range(5):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(iters):
            ops.forward(x, spec, None, 128, 4096, algo=algo)
        e.record()
        torch.cuda.synchronize()
        reps.append(s.elapsed_time(e) / iters * 1e3)
    return sorted(reps)[2]


def main():
    algos = [a for a in sys.argv[1:]] or ["dftx", "dftp"]
    dev = torch.device("cuda")
    lib = os.path.basename(os.environ.get("BCFFT_LIB_PATH", "libbcfft.so"))
    rng = np.random.default_rng(0)
    c = (rng.standard_normal((32, 32, 128)) * 0.01).astype(np.float32)
    x = rng.standard_normal((8192, 4096)).astype(np.float32)
    ref = O.bc_forward(x[:1024], c, None)
    spec = ops.spectra(torch.from_numpy(c).to(dev))
    xd = torch.from_numpy(x).to(dev)
    mod = _structured_layer(dev, 4096, 4096, 128, seed=3)
    cs = mod.c.detach().float().cpu().numpy()
    xs = _structured_tokens(512, 4096, seed=4)
    refs = O.bc_forward(xs, cs, None)
    sspec = mod._spectra(mod.c)
    for algo in algos:
        t8 = kernel_us(xd, spec, algo)
        t1 = kernel_us(xd[:1024], spec, algo)
        g = ops.forward(xd[:1024], spec, None, 128, 4096, algo=algo).cpu().numpy()
        fro = float(np.linalg.norm(g - ref) / np.linalg.norm(ref))
        gs = ops.forward(torch.from_numpy(xs).to(dev), sspec, None, 128, 4096, algo=algo).cpu().numpy()
        pt = _per_token(gs, refs)
        print(f"{lib:26s} {algo:6s} N=8192 {t8:7.2f} us ({268967936 / t8 / 8e6:.4f} of 8 TB/s)  N=1024 {t1:6.2f} us  "
              f"north-star Frobenius {fro:.3e}  structured worst token {pt.max():.3e} (token {int(pt.argmax())})",
              flush=True)


if __name__ == "__main__":
    main()
