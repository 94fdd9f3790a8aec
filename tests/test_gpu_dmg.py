"""GPU parity of the multi-group DFT kernel (bcfft_dmg.hip: bf16 I/O, b = 128, K = 4096, two or
more output groups; BASELINE config 2's 4096 -> 11008 and the fused gate/up + SwiGLU).

Its three stages are the 8-token kernel's (bcfft_dm8.hip) with stage 1 run once per tile and the
weight fragments streamed per group, in the same arithmetic order. So beside the oracle it is
checked BIT FOR BIT against the 8-token kernel run on each output group separately (one group:
bcfft_dm8.hip), and the fused gate/up against its own two-projection composition."""
import numpy as np
import pytest
import torch

from golden_io import rel_err
from oracle import bc_oracle as O
from test_gpu_stationary import _check, _run, _check_auto

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    import bcfft
    bcfft.load()
    return torch.device("cuda:0")


CASES = [
    # (M, N, bias): K = 4096, b = 128, bf16 I/O
    (11008, 37, False),       # 3 groups, the last partial (22 blocks); ragged last tile
    (8192, 1, False),         # 2 groups, one token
    (11008, 2049, True),      # several tiles per workgroup, bf16 bias
    (12288, 300, False),      # 3 full groups
    (4096 * 5, 64, False),    # 5 groups
]


@pytest.mark.parametrize("m,n,bias", CASES)
def test_dmg_vs_oracle(dev, m, n, bias):
    k, b = 4096, 128
    rng = np.random.default_rng(m + n)
    c = (rng.standard_normal((m // b, k // b, b)) * 0.01).astype(np.float32)
    bv = (rng.standard_normal(m) * 0.1).astype(np.float32) if bias else None
    x = rng.standard_normal((n, k)).astype(np.float32)
    y, ref = _run(dev, x, c, bv, "bfloat16", "bfloat16", algo="dft")
    _check(y, ref, "bfloat16")                      # ~1 bf16 ulp elementwise
    ya, _ = _run(dev, x, c, bv, "bfloat16", "bfloat16", algo="auto")
    _check_auto(y, ya, ref, n, k, m, b, "bfloat16")   # AUTO resolves to it (short N: the sn kernel)
    # per-token power-of-two scales: a 300x token and a token with a 1e-3-quiet stretch, each
    # within the bf16 floor relative to its own norm
    x[0] *= 300.0
    x[n // 2, 1000:1100] *= 1e-3
    y, ref = _run(dev, x, c, bv, "bfloat16", "bfloat16", algo="dft")
    g = y.float().cpu().numpy()
    for t in sorted({0, n // 2, n - 1}):
        assert rel_err(g[t], ref[t]) < 4e-3, (t, rel_err(g[t], ref[t]))


def test_dmg_bit_equal_to_per_group_dm8(dev):
    """4096 -> 11008 in one multi-group launch == the 8-token kernel on each group's 32 (22) output
    blocks alone, bit for bit (same stages, roundings and per-bin summation order)."""
    from bcfft import ops
    k, m, b, n = 4096, 11008, 128, 1000
    torch.manual_seed(5)
    c = (torch.randn(m // b, k // b, b, device=dev) * 0.01).to(torch.bfloat16)
    x = torch.randn(n, k, device=dev).to(torch.bfloat16)
    y = ops.forward(x, ops.spectra(c), None, b, m, algo="dft")
    parts = []
    for g0 in range(0, m // b, 32):
        cg = c[g0:g0 + 32].contiguous()
        parts.append(ops.forward(x, ops.spectra(cg), None, b, cg.shape[0] * b, algo="dft"))
    assert torch.equal(y, torch.cat(parts, dim=1))


def test_dmg_full_size_config2(dev):
    """BASELINE config 2 at its full size (4096 -> 11008, b = 128, bf16, N = 8192): every token
    against the oracle (~1 bf16 ulp), run-to-run bit equality."""
    from bcfft import ops
    k, m, b, n = 4096, 11008, 128, 8192
    rng = np.random.default_rng(2)
    c = O.round_to((rng.standard_normal((m // b, k // b, b)) * 0.01).astype(np.float32), O.BF16)
    x = O.round_to(rng.standard_normal((n, k)).astype(np.float32), O.BF16)
    spec = ops.spectra(torch.from_numpy(c).to(dev).to(torch.bfloat16))
    xt = torch.from_numpy(x).to(dev).to(torch.bfloat16)
    y = ops.forward(xt, spec, None, b, m, algo="auto")
    assert torch.equal(y, ops.forward(xt, spec, None, b, m, algo="auto"))
    g = y.float().cpu().numpy()
    ref = O.bc_forward(x, c, None, x_dtype=O.BF16)
    ulp = 2.0 ** -7
    rms = float(np.sqrt(np.mean(ref.astype(np.float64) ** 2)))
    bad = np.abs(g - ref) > 2 * ulp * np.abs(ref) + 2 * ulp * rms
    assert not bad.any(), f"{int(bad.sum())} elements beyond ~1 ulp"
    assert rel_err(g, ref) < 4e-3


@pytest.mark.parametrize("n", [1, 37, 1700])
def test_dmg_glu_matches_composition(dev, n):
    """The fused gate/up + SwiGLU (6 groups of 16 gate + 16 up blocks) against silu(gate) * up of
    the same engine's two separate launches (each a multi-group launch itself)."""
    from bcfft import ops
    torch.manual_seed(3)
    k, m, b = 4096, 11008, 128
    cg = torch.randn(m // b, k // b, b, device=dev) * 0.01
    cu = torch.randn(m // b, k // b, b, device=dev) * 0.01
    x = torch.randn(n, k, device=dev).to(torch.bfloat16)
    h = ops.forward_glu(x, ops.spectra(ops.glu_weights(cg, cu)), b, m, algo="dft")
    gt = ops.forward(x, ops.spectra(cg), None, b, m, algo="dft")
    ut = ops.forward(x, ops.spectra(cu), None, b, m, algo="dft")
    ref = (torch.nn.functional.silu(gt.float()).to(torch.bfloat16).float() * ut.float()).to(torch.bfloat16)
    d = (h.float() - ref.float()).abs()
    assert (d <= 2 * 2.0 ** -7 * ref.float().abs() + 1e-6).float().mean().item() > 0.999
    assert ((h.float() - ref.float()).norm() / ref.float().norm()).item() < 4e-3
