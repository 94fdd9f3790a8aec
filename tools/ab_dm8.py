"""A/B of a dm8 experiment build (BCFFT_LIB_PATH) against the product library: times of the bf16
north star (4096^2, b = 128, N = 8192 and 2048) and of the per-group fused gate/up at N = 256,
and the outputs saved for a bitwise comparison (usage: ab_dm8.py TAG OUTDIR; then
ab_dm8.py --compare OUTDIR TAG1 TAG2)."""
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
    b, h, f = 128, 4096, 11008
    torch.manual_seed(0)
    c = (torch.randn(h // b, h // b, b) * 0.01).cuda()
    s = ops.spectra(c)
    sgu = ops.spectra(ops.glu_weights((torch.randn(f // b, h // b, b) * 0.01).cuda(),
                                      (torch.randn(f // b, h // b, b) * 0.01).cuda()))
    res, outs = {}, {}
    for n in (8192, 2048):
        x = torch.randn(n, h, device="cuda").to(torch.bfloat16)
        res[f"bf16_4096sq_N{n}"] = timed(lambda: ops.forward(x, s, None, b, h), 50)
        outs[f"y{n}"] = ops.forward(x, s, None, b, h).cpu()
    x = torch.randn(256, h, device="cuda").to(torch.bfloat16)
    res["glu_N256"] = timed(lambda: ops.forward_glu(x, sgu, b, f), 50)
    outs["h256"] = ops.forward_glu(x, sgu, b, f).cpu()
    # the multi-group kernels at N = 8192: config 2 (4096 -> 11008) and the fused gate/up
    sup = ops.spectra((torch.randn(f // b, h // b, b) * 0.01).cuda())
    x = torch.randn(8192, h, device="cuda").to(torch.bfloat16)
    res["up_N8192"] = timed(lambda: ops.forward(x, sup, None, b, f), 30)
    outs["up8192"] = ops.forward(x, sup, None, b, f).cpu()
    res["glu_N8192"] = timed(lambda: ops.forward_glu(x, sgu, b, f), 30)
    outs["h8192"] = ops.forward_glu(x, sgu, b, f).cpu()
    os.makedirs(out, exist_ok=True)
    torch.save(outs, os.path.join(out, tag + ".pt"))
    print(json.dumps({"lib": tag, "us": res}), flush=True)


if __name__ == "__main__":
    main()
