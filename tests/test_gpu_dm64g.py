"""GPU parity of the b = 64 multi-group DFT kernel (bcfft_dm64g.hip: bf16 I/O, b = 64, K = 4096,
three or more output groups; the block-size sweep's b = 64 gate / up 4096 -> 11008 and the fused
gate/up + SwiGLU). Its stages are bcfft_dm64.hip's in the same arithmetic order, so beside the
oracle it is checked bit for bit against the per-group kernel run on each output group alone."""
import numpy as np
import pytest
import torch

from golden_io import rel_err
from test_gpu_stationary import _check, _run, _check_auto

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    import bcfft
    bcfft.load()
    return torch.device("cuda:0")


CASES = [
    # (M, N, bias): K = 4096, b = 64, bf16 I/O
    (11008, 37, False),       # 172 output blocks: 6 groups, the last partial (12); ragged tile
    (6144, 1, True),          # 3 groups, one token, bf16 bias
    (11008, 2049, True),      # several tiles per workgroup
    (6144, 300, False),       # 3 full groups
]


@pytest.mark.parametrize("m,n,bias", CASES)
def test_dm64g_vs_oracle(dev, m, n, bias):
    k, b = 4096, 64
    rng = np.random.default_rng(m + 5 * n)
    c = (rng.standard_normal((m // b, k // b, b)) * 0.01).astype(np.float32)
    bv = (rng.standard_normal(m) * 0.1).astype(np.float32) if bias else None
    x = rng.standard_normal((n, k)).astype(np.float32)
    y, ref = _run(dev, x, c, bv, "bfloat16", "bfloat16", algo="dft")
    _check(y, ref, "bfloat16")
    ya, _ = _run(dev, x, c, bv, "bfloat16", "bfloat16", algo="auto")
    _check_auto(y, ya, ref, n, k, m, b, "bfloat16")   # AUTO resolves to it (short N: the sn kernel)
    x[0] *= 300.0                                   # per-(token, quarter) scales
    x[n // 2, 1000:1100] *= 1e-3
    y, ref = _run(dev, x, c, bv, "bfloat16", "bfloat16", algo="dft")
    g = y.float().cpu().numpy()
    for t in sorted({0, n // 2, n - 1}):
        assert rel_err(g[t], ref[t]) < 4e-3, (t, rel_err(g[t], ref[t]))


def test_dm64g_bit_equal_to_per_group_dm64(dev):
    """4096 -> 11008 at b = 64 in one multi-group launch == the per-group kernel on each group's
    32 (12) output blocks alone, bit for bit. (N = 1100: 138 tiles, past the multi-group
    kernel's 4/8-of-the-CUs threshold.)"""
    from bcfft import ops
    k, m, b, n = 4096, 11008, 64, 1100
    torch.manual_seed(6)
    c = (torch.randn(m // b, k // b, b, device=dev) * 0.01).to(torch.bfloat16)
    x = torch.randn(n, k, device=dev).to(torch.bfloat16)
    y = ops.forward(x, ops.spectra(c), None, b, m, algo="dft")
    parts = []
    for g0 in range(0, m // b, 32):
        cg = c[g0:g0 + 32].contiguous()
        parts.append(ops.forward(x, ops.spectra(cg), None, b, cg.shape[0] * b, algo="dft"))
    assert torch.equal(y, torch.cat(parts, dim=1))


def test_dm64g_full_size(dev):
    """The sweep's b = 64 up projection at full size (4096 -> 11008, N = 8192): every token within
    ~1 bf16 ulp of the oracle, run-to-run bit equality."""
    from bcfft import ops
    from oracle import bc_oracle as O
    k, m, b, n = 4096, 11008, 64, 8192
    rng = np.random.default_rng(4)
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
def test_dm64g_glu_matches_composition(dev, n):
    """The fused gate/up + SwiGLU at b = 64 (11 groups of 16 gate + 16 up blocks) against
    silu(gate) * up of the same engine's two separate launches."""
    from bcfft import ops
    torch.manual_seed(3)
    k, m, b = 4096, 11008, 64
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
