"""A/B of a dm64k experiment build (BCFFT_LIB_PATH) against the product library: the b = 64 down
projection 11008 -> 4096 (bf16) at N = 8192 and 1024, outputs saved for a bitwise comparison
(usage: ab_dm64k.py TAG OUTDIR; ab_dm64k.py --compare OUTDIR TAG1 TAG2)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama-fft_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402


def main():
    if sys.argv[1] == "--compare":
        d, a, b = sys.argv[2:5]
        A, B = torch.load(os.path.join(d, a + ".pt")), torch.load(os.path.join(d, b + ".pt"))
        print(json.dumps({k: bool(torch.equal(A[k], B[k])) for k in A}))
        return
    from bcfft import ops
    from time_dmg_switch import timed
    tag, out = sys.argv[1], sys.argv[2]
    b, k, m = 64, 11008, 4096
    torch.manual_seed(0)
    s = ops.spectra((torch.randn(m // b, k // b, b) * 0.01).cuda())
    res, outs = {}, {}
    for n in (8192, 1024):
        x = torch.randn(n, k, device="cuda").to(torch.bfloat16)
        x[3, 100:200] *= 1e3
        res[f"N{n}"] = timed(lambda: ops.forward(x, s, None, b, m), 30)
        outs[f"y{n}"] = ops.forward(x, s, None, b, m).cpu()
    os.makedirs(out, exist_ok=True)
    torch.save(outs, os.path.join(out, tag + ".pt"))
    print(json.dumps({"lib": tag, "us": res}), flush=True)


if __name__ == "__main__":
    main()
