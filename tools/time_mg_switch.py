"""b = 64 and b = 256 counterpart of tools/time_dmg_switch.py: the multi-group kernels
(bcfft_dm64g.hip, bc_forward_dm256g_kernel) against the per-group ones at small and mid token
counts, bf16 4096 -> 11008 (and the b = 64 fused gate/up). Run with the product library and with
`make exp NAME=nomg DEFS="-DBCFFT_NO_DM64G -DBCFFT_NO_DM256G -DBCFFT_NO_DMG"`. One JSON line per N."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama-fft_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402
from bcfft import _lib, ops  # noqa: E402
from time_dmg_switch import timed  # noqa: E402


def main():
    h, f = 4096, 11008
    tag = sys.argv[1]
    ns = [int(a) for a in sys.argv[2:]]
    torch.manual_seed(0)
    lib = _lib.load()
    st = _lib.stream_handle(torch.device("cuda:0"))
    BF16, NONE, AUTO = _lib.BCFFT_BF16, _lib.BCFFT_NONE, _lib.ALGO_AUTO
    specs = {}
    for b in (64, 256):
        c = lambda o, i: (torch.randn(o // b, i // b, b) * 0.01).cuda()  # noqa: E731
        specs[b] = (ops.spectra(c(f, h)), ops.spectra(ops.glu_weights(c(f, h), c(f, h))) if b == 64 else None)
    for n in ns:
        x = torch.randn(n, h, device="cuda").to(torch.bfloat16)
        y = torch.empty(n, f, device="cuda", dtype=torch.bfloat16)
        t = {}
        for b, (s_up, s_gu) in specs.items():
            t[f"up_b{b}"] = timed(lambda: lib.bcfft_forward_ws(x.data_ptr(), BF16, n, h, f, b, s_up.data_ptr(), None,
                                                               NONE, y.data_ptr(), BF16, AUTO, None, 0, st))
            if s_gu is not None:
                t[f"glu_b{b}"] = timed(lambda: lib.bcfft_forward_glu(x.data_ptr(), BF16, n, h, f, b, s_gu.data_ptr(),
                                                                     y.data_ptr(), st))
        print(json.dumps({"lib": tag, "N": n, "us": t}), flush=True)


if __name__ == "__main__":
    main()
