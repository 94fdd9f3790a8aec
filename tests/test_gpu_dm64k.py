"""GPU parity of the b = 64 streamed-weight DFT kernel (bcfft_dm64k.hip: K > 4096, bf16 I/O; the
block-size sweep's down projection 11008 -> 4096 at b = 64). Checked against the oracle (~1 bf16
ulp elementwise) with per-(token, quarter) scale edge cases, and AUTO's resolution to it."""
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
    # (K, M, N, bias): b = 64
    (11008, 4096, 37, False),   # 172 input blocks: 5 full 32-block chunks + 12; 2 output groups
    (11008, 4096, 1, True),     # one token, bf16 bias
    (11008, 4096, 2049, False), # several 16-token tiles per workgroup
    (4160, 2048, 300, True),    # 65 blocks: 2 chunks + 1 block (an odd K-step count)
    (16320, 1024, 19, False),   # 255 blocks: the largest K
    (8192, 11008, 64, False),   # 172 output blocks: 6 groups, the last partial
    (4160, 2048, 8200, True),   # bias, two or three tiles per workgroup (HB path, empty-range B loads)
]


@pytest.mark.parametrize("k,m,n,bias", CASES)
def test_dm64k_vs_oracle(dev, k, m, n, bias):
    b = 64
    rng = np.random.default_rng(k + 7 * m + n)
    c = (rng.standard_normal((m // b, k // b, b)) * 0.01).astype(np.float32)
    bv = (rng.standard_normal(m) * 0.1).astype(np.float32) if bias else None
    x = rng.standard_normal((n, k)).astype(np.float32)
    y, ref = _run(dev, x, c, bv, "bfloat16", "bfloat16", algo="dft")
    _check(y, ref, "bfloat16")
    ya, _ = _run(dev, x, c, bv, "bfloat16", "bfloat16", algo="auto")
    if n >= 128:                                    # AUTO resolves to it from 128 tokens
        assert torch.equal(y, ya)
    else:                                           # below: the split-K MFMA kernel
        _check(ya, ref, "bfloat16")
    # a 300x token; a token whose first chunk is 1e-3-quiet and whose last blocks are loud (the
    # reference exponent drops mid-tile); a token with an all-zero 32-block chunk
    x[0] *= 300.0
    x[n - 1, :2048] *= 1e-3
    x[n - 1, -100:] *= 40.0
    if n > 2:
        x[n // 2, 2048:4096] = 0.0
    y, ref = _run(dev, x, c, bv, "bfloat16", "bfloat16", algo="dft")
    g = y.float().cpu().numpy()
    for t in sorted({0, n // 2, n - 1}):
        assert rel_err(g[t], ref[t]) < 4e-3, (t, rel_err(g[t], ref[t]))


def test_dm64k_full_size_down(dev):
    """The sweep's down projection at b = 64 (11008 -> 4096, N = 8192): every token within ~1 bf16
    ulp of the oracle, run-to-run bit equality."""
    from bcfft import ops
    from oracle import bc_oracle as O
    k, m, b, n = 11008, 4096, 64, 8192
    rng = np.random.default_rng(9)
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
