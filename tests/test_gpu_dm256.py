"""GPU parity of the b = 256 DFT-on-MFMA kernel (bcfft_dm256.hip: K = 4096, bf16 I/O; the
reference's default block size, patch_llama_fft.py:13). The 256-point transforms are built from
the 128-point table on three virtual rows (tests/dm256_model.py restates the algebra); the
checks are the oracle (~1 bf16 ulp, per-token scales) and AUTO's resolution to it."""
import numpy as np
import pytest
import torch

from golden_io import rel_err
from test_gpu_stationary import _check, _run

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    import bcfft
    bcfft.load()
    return torch.device("cuda:0")


CASES = [
    # (M, N, bias): K = 4096, b = 256, bf16 I/O
    (4096, 37, False),        # one group of 16 output blocks; ragged last tile of 8
    (4096, 1, True),          # one token, bf16 bias
    (11008, 19, False),       # 43 output blocks: 3 groups, the last partial (11)
    (2048, 300, True),        # 8 output blocks: a partial group; several tiles per workgroup
    (4096, 2049, False),      # several tiles per workgroup on every CU
]
# K != 4096 at b = 256: the streamed-weight chunk kernel (bc_forward_dm256k_kernel)
CASES_K = [
    # (K, M, N, bias)
    (11008, 4096, 37, False),   # the down projection: 43 input blocks = 2 full chunks + 11
    (11008, 4096, 1, True),     # one token, bf16 bias
    (11008, 4096, 2049, False), # several tiles per workgroup
    (8192, 2048, 300, True),    # 2 full chunks; 8 output blocks (a partial N-tile)
    (2048, 4096, 19, False),    # K < 4096: one partial chunk (8 blocks)
    (5120, 11008, 64, False),   # 20 input blocks, 3 N-tile groups
]


@pytest.mark.parametrize("m,n,bias", CASES)
def test_dm256_vs_oracle(dev, m, n, bias):
    k, b = 4096, 256
    rng = np.random.default_rng(m + 3 * n)
    c = (rng.standard_normal((m // b, k // b, b)) * 0.01).astype(np.float32)
    bv = (rng.standard_normal(m) * 0.1).astype(np.float32) if bias else None
    x = rng.standard_normal((n, k)).astype(np.float32)
    y, ref = _run(dev, x, c, bv, "bfloat16", "bfloat16", algo="dft")
    _check(y, ref, "bfloat16")
    ya, _ = _run(dev, x, c, bv, "bfloat16", "bfloat16", algo="auto")
    assert torch.equal(y, ya)                       # AUTO resolves to it
    x[0] *= 300.0                                   # per-token power-of-two scale
    x[n - 1, 1000:1100] *= 1e-3
    x[n // 2, 4000] = 50.0                          # one loud channel in the last block
    y, ref = _run(dev, x, c, bv, "bfloat16", "bfloat16", algo="dft")
    g = y.float().cpu().numpy()
    for t in sorted({0, n // 2, n - 1}):
        assert rel_err(g[t], ref[t]) < 4e-3, (t, rel_err(g[t], ref[t]))


@pytest.mark.parametrize("k,m,n,bias", CASES_K)
def test_dm256k_vs_oracle(dev, k, m, n, bias):
    b = 256
    rng = np.random.default_rng(k + m + n)
    c = (rng.standard_normal((m // b, k // b, b)) * 0.01).astype(np.float32)
    bv = (rng.standard_normal(m) * 0.1).astype(np.float32) if bias else None
    x = rng.standard_normal((n, k)).astype(np.float32)
    y, ref = _run(dev, x, c, bv, "bfloat16", "bfloat16", algo="dft")
    _check(y, ref, "bfloat16")
    ya, _ = _run(dev, x, c, bv, "bfloat16", "bfloat16", algo="auto")
    assert torch.equal(y, ya)
    # per-(token, chunk) scales: a 300x token; a token whose first chunk is 1e-3-quiet and
    # whose last is loud (the reference exponent drops: accumulator rows rescale); a token with
    # one all-zero chunk
    x[0] *= 300.0
    x[n - 1, :4096] *= 1e-3
    x[n - 1, -100:] *= 40.0
    if n > 2 and k > 4096:
        x[n // 2, 4096:8192] = 0.0
    y, ref = _run(dev, x, c, bv, "bfloat16", "bfloat16", algo="dft")
    g = y.float().cpu().numpy()
    for t in sorted({0, n // 2, n - 1}):
        assert rel_err(g[t], ref[t]) < 4e-3, (t, rel_err(g[t], ref[t]))


def test_dm256k_full_size_down(dev):
    """The block-size sweep's down projection at b = 256 (11008 -> 4096, N = 8192): every token
    within ~1 bf16 ulp of the oracle, run-to-run bit equality."""
    from bcfft import ops
    from oracle import bc_oracle as O
    k, m, b, n = 11008, 4096, 256, 8192
    rng = np.random.default_rng(8)
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


def test_dm256_full_size_sweep_shape(dev):
    """The block-size sweep's q/k/v/o shape at b = 256 (4096 -> 4096, N = 8192): every token
    within ~1 bf16 ulp of the oracle, run-to-run bit equality."""
    from bcfft import ops
    from oracle import bc_oracle as O
    k, m, b, n = 4096, 4096, 256, 8192
    rng = np.random.default_rng(7)
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


def test_dm256g_bit_equal_to_per_group(dev):
    """4096 -> 11008 at b = 256 (43 output blocks: 3 groups, the multi-group kernel) == the
    one-group kernel on each group's 16 (11) output blocks alone, bit for bit."""
    from bcfft import ops
    k, m, b, n = 4096, 11008, 256, 1000
    torch.manual_seed(8)
    c = (torch.randn(m // b, k // b, b, device=dev) * 0.01).to(torch.bfloat16)
    x = torch.randn(n, k, device=dev).to(torch.bfloat16)
    y = ops.forward(x, ops.spectra(c), None, b, m, algo="dft")
    parts = []
    for g0 in range(0, m // b, 16):
        cg = c[g0:g0 + 16].contiguous()
        parts.append(ops.forward(x, ops.spectra(cg), None, b, cg.shape[0] * b, algo="dft"))
    assert torch.equal(y, torch.cat(parts, dim=1))


@pytest.mark.parametrize("n", [1, 37, 1700])
def test_dm256_glu_matches_composition(dev, n):
    """The fused gate/up + SwiGLU at b = 256 (bf16; virtual groups of 8 gate + 8 up blocks of the
    multi-group kernel, paired by a DPP row rotation) against silu(gate) * up of the same
    engine's two separate launches, and through the module path (BCFusedGateUp)."""
    from bcfft import ops
    torch.manual_seed(4)
    k, m, b = 4096, 11008, 256
    cg = torch.randn(m // b, k // b, b, device=dev) * 0.01
    cu = torch.randn(m // b, k // b, b, device=dev) * 0.01
    x = torch.randn(n, k, device=dev).to(torch.bfloat16)
    assert ops.glu_eligible(k, b, torch.bfloat16) and not ops.glu_eligible(k, b, torch.float32)
    h = ops.forward_glu(x, ops.spectra(ops.glu_weights(cg, cu)), b, m, algo="auto")
    gt = ops.forward(x, ops.spectra(cg), None, b, m, algo="dft")
    ut = ops.forward(x, ops.spectra(cu), None, b, m, algo="dft")
    ref = (torch.nn.functional.silu(gt.float()).to(torch.bfloat16).float() * ut.float()).to(torch.bfloat16)
    d = (h.float() - ref.float()).abs()
    assert (d <= 2 * 2.0 ** -7 * ref.float().abs() + 1e-6).float().mean().item() > 0.999
    assert ((h.float() - ref.float()).norm() / ref.float().norm()).item() < 4e-3


def test_dm256_glu_module_path(dev):
    """BCFusedGateUp at b = 256 bf16 takes the fused launch and matches the two modules."""
    from patch_llama_fft import BCFusedGateUp, BlockCirculantLinear
    torch.manual_seed(5)
    g = BlockCirculantLinear(4096, 11008, block_size=256, bias=False).to(dev).to(torch.bfloat16).eval()
    u = BlockCirculantLinear(4096, 11008, block_size=256, bias=False).to(dev).to(torch.bfloat16).eval()
    f = BCFusedGateUp(g, u)
    x = torch.randn(2, 50, 4096, device=dev).to(torch.bfloat16)
    with torch.inference_mode():
        assert f._fused_ok(x)
        h = f(x)
        ref = torch.nn.functional.silu(g(x)) * u(x)
    assert h.shape == ref.shape
    assert ((h.float() - ref.float()).norm() / ref.float().norm()).item() < 4e-3
