"""Debug aid: which tokens and which K-chunks the streamed-weight kernel
(bcfft_dmk.hip) gets wrong in an analysis build, by chunk-tagged inputs.

Every token t of a 4090-token, 11008 -> 4096, b = 128 bf16 batch holds data in ONE 16-block
K-chunk, chunk t % 6, so each output row is that one chunk's contribution (or zero, or another
chunk's, when the kernel mixes them up). `run` writes the output of the library named by
BCFFT_LIB_PATH to gpurun_out/ep/dmk_<lib>.npy; `compare A B` prints, per chunk and per tile
position, how many tokens differ between two libraries' outputs and how (zero rows, rows equal to
the other library's row of another token).
usage: python tools/dbg_dmk_late.py run | python tools/dbg_dmk_late.py compare a.npy b.npy"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N, K, M, B = 4090, 11008, 4096, 128


def run():
    sys.path.insert(0, os.path.join(ROOT, "llama-fft_amd"))
    import torch
    from bcfft import ops
    rng = np.random.default_rng(11)
    c = (rng.standard_normal((M // B, K // B, B)) * 0.01).astype(np.float32)
    x = np.zeros((N, K), np.float32)
    for t in range(N):
        ch = t % 6
        lo, hi = ch * 2048, min(K, ch * 2048 + 2048)
        x[t, lo:hi] = rng.standard_normal(hi - lo)
    dev = torch.device("cuda")
    spec = ops.spectra(torch.from_numpy(c).to(dev).to(torch.bfloat16))
    xt = torch.from_numpy(x).to(dev).to(torch.bfloat16)
    y = ops.forward(xt, spec, None, B, M, algo="dft").float().cpu().numpy()
    lib = os.path.basename(os.environ.get("BCFFT_LIB_PATH", "libbcfft.so")).replace(".so", "")
    out = os.path.join(ROOT, "gpurun_out", "ep", f"dmk_{lib}.npy")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    # compact (gpurun_out travels back under 64 MiB): per token its row norm and 31 sample columns
    cols = np.arange(0, M, M // 31)[:31]
    np.save(out, np.concatenate([np.linalg.norm(y, axis=1)[:, None], y[:, cols]], axis=1).astype(np.float32))
    print("saved", out, "norm", float(np.linalg.norm(y)))


def compare(a, b):
    ya, yb = np.load(a), np.load(b)              # (N, 32): row norm, 31 sample columns
    d = np.linalg.norm(ya - yb, axis=1) / np.maximum(np.linalg.norm(yb, axis=1), 1e-30)
    bad = np.nonzero(d > 1e-6)[0]
    print(f"{len(bad)} of {N} tokens differ (> 1e-6 relative); worst {d.max():.3e}")
    if len(bad) == 0:
        return
    zero = [t for t in bad if not np.any(ya[t])]
    print(f"  zero rows in {os.path.basename(a)}: {len(zero)}")
    for name, key in (("chunk (t % 6)", lambda t: t % 6), ("slot in tile (t % 16)", lambda t: t % 16),
                      ("wave (t % 16 // 2)", lambda t: (t % 16) // 2), ("tile (t // 16)", lambda t: t // 16)):
        cnt = {}
        for t in bad:
            cnt[key(t)] = cnt.get(key(t), 0) + 1
        print(f"  by {name}: " + " ".join(f"{k}:{v}" for k, v in sorted(cnt.items())[:40]))
    print("  first bad tokens:", " ".join(f"{t}({d[t]:.2f})" for t in bad[:24]))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        compare(sys.argv[2], sys.argv[3])
