"""GPU parity of the short-N DFT kernel (algo="short", bcfft_sn.hip) against the CPU oracle
(BlockCirculantLinear.forward, patch_llama_fft.py:226-275) and the dftx mirror (tests/dm_model.py,
exact=True: the same table, splits and scales; only the work split differs).

The kernel serves the STAT geometries (b = 128 with K = 4096; b = 64 with K = 2048 or 4096), every
x dtype and bias, one workgroup per 2- or 4-token tile (2 while those workgroups fit one round)
and 16 output blocks; AUTO takes it up to
the short-N rule's token count (sn_pays: workgroups <= CUs; BASELINE config 1: 4096 -> 4096, b = 64, N = 128, fp32). Tolerances as
dftx: < 6e-4 relative Frobenius and < 1e-3 per token (north star) for fp32 outputs, ~1 ulp of the
output rounding for 16-bit ones."""
import numpy as np
import pytest
import torch

from golden_io import rel_err
from oracle import bc_oracle as O
from test_gpu_stationary import _check, _run

pytestmark = pytest.mark.gpu
SN_TOL = 6e-4


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    import bcfft
    bcfft.load()
    return torch.device("cuda:0")


CASES = [
    # (K, M, b, N, x dtype, module dtype, bias)
    (4096, 4096, 64, 128, "float32", "float32", False),     # BASELINE config 1
    (4096, 4096, 64, 1, "float32", "float32", True),        # one token: 3 zero-filled rows
    (4096, 4096, 64, 5, "float32", "float32", True),        # ragged second tile
    (4096, 4096, 64, 37, "bfloat16", "bfloat16", False),
    (4096, 1088, 64, 9, "float32", "float32", True),        # 17 output blocks: a 1-block N-tile
    (2048, 1024, 64, 7, "float32", "float32", True),        # K-steps 2
    (2048, 3072, 64, 23, "float16", "float32", False),      # fp16 x, fp32 module -> fp32 out
    (4096, 4096, 128, 1, "float32", "float32", True),
    (4096, 4096, 128, 20, "bfloat16", "bfloat16", True),    # a decode step of a 20-prompt batch
    (4096, 11008, 128, 13, "bfloat16", "bfloat16", False),  # 86 output blocks: 6 N-tiles, last partial
    (4096, 4096, 128, 64, "float16", "float16", True),
    (4096, 4096, 128, 50, "bfloat16", "float32", True),     # promotion -> fp32 output
    (4096, 4096, 128, 255, "float32", "float32", False),    # 128 2-token tiles, the last one of 1 token
    # 4-token tiles (the 2-token grid would exceed one round of 256 workgroups)
    (4096, 4096, 128, 400, "float32", "float32", True),
    (4096, 4096, 64, 203, "bfloat16", "bfloat16", False),   # the last tile of 3 tokens
    (2048, 3072, 64, 300, "float32", "float32", True),
]


@pytest.mark.parametrize("k,m,b,n,xdt,mdt,bias", CASES)
def test_short_vs_oracle(dev, k, m, b, n, xdt, mdt, bias):
    rng = np.random.default_rng(k + m + b + n)
    c = (rng.standard_normal((m // b, k // b, b)) * 0.01).astype(np.float32)
    bv = (rng.standard_normal(m) * 0.1).astype(np.float32) if bias else None
    x = rng.standard_normal((n, k)).astype(np.float32)
    y, ref = _run(dev, x, c, bv, xdt, mdt, algo="short")
    _check(y, ref, xdt)
    if xdt == "float32":                              # 16-bit x: the output is rounded to x's dtype (:266)
        g = y.cpu().numpy().astype(np.float64)
        pt = np.linalg.norm(g - ref, axis=1) / np.maximum(np.linalg.norm(ref, axis=1), 1e-30)
        assert pt.max() < 1e-3, (int(pt.argmax()), pt.max())


def test_short_matches_dftx_mirror(dev):
    """b = 128: the numpy mirror of the dftx arithmetic (dm_model, exact=True) agrees with the
    short-N kernel far below the quantisation error (fp32 summation order only)."""
    from dm_model import dm_forward
    rng = np.random.default_rng(11)
    c = (rng.standard_normal((32, 32, 128)) * 0.01).astype(np.float32)
    x = rng.standard_normal((8, 4096)).astype(np.float32)
    x[1] *= 300.0
    x[5, 2048:] *= 1e-3                               # the two K halves at different scales
    y, ref = _run(dev, x, c, None, "float32", "float32", algo="short")
    g = y.cpu().numpy()
    mdl = dm_forward(x, c, exact=True)
    assert rel_err(g, mdl) < 2e-5, rel_err(g, mdl)
    assert rel_err(g, ref) < SN_TOL


def test_short_per_token_scale(dev):
    """Tokens 10^9 apart, a zero token, one massive channel, a token far below fp16's range, K
    chunks at very different scales: per-(token, chunk) scales keep each at full accuracy."""
    rng = np.random.default_rng(2)
    for b in (64, 128):
        c = (rng.standard_normal((4096 // b, 4096 // b, b)) * 0.01).astype(np.float32)
        x = rng.standard_normal((9, 4096)).astype(np.float32)
        x[0] *= 1e4
        x[1] *= 1e-5
        x[2] = 0.0
        x[3, 77] = 3000.0
        x[4, 2100:2300] *= 1e3
        x[5] *= 1e-30
        y, ref = _run(dev, x, c, None, "float32", "float32", algo="short")
        g = y.cpu().numpy()
        assert np.all(g[2] == 0.0)
        for t in (0, 1, 3, 4, 5, 6, 7, 8):
            assert rel_err(g[t], ref[t]) < SN_TOL, (b, t, rel_err(g[t], ref[t]))


@pytest.mark.parametrize("b,n", [(64, 128), (128, 16), (128, 256)])
def test_auto_takes_short_at_small_n(dev, b, n):
    """AUTO resolves to the short-N kernel while its grid fits one round of the device's CUs (the
    sn_pays rule: workgroups <= CU count; bit-equal to algo=short) and to the persistent engines
    above it. The test's token counts fit on 128 or more CUs."""
    if torch.cuda.get_device_properties(0).multi_processor_count < 128:
        pytest.skip("the short-N threshold scales with the CU count; these N assume >= 128 CUs")
    from bcfft import _lib, ops
    lib = _lib.load()
    code = _lib.dtype_code(torch.float32)
    assert lib.bcfft_forward_resolve(n, 4096, 4096, b, 0, code, code) == _lib.ALGOS["short"]
    assert lib.bcfft_forward_kernel_name(n, 4096, 4096, b, 0, code, code).decode() == "bc_forward_sn_kernel"
    assert lib.bcfft_forward_resolve(8192, 4096, 4096, b, 0, code, code) != _lib.ALGOS["short"]
    rng = np.random.default_rng(5)
    c = torch.from_numpy((rng.standard_normal((4096 // b, 4096 // b, b)) * 0.01).astype(np.float32)).to(dev)
    x = torch.from_numpy(rng.standard_normal((n, 4096)).astype(np.float32)).to(dev)
    spec = ops.spectra(c)
    ya = ops.forward(x, spec, None, b, 4096, algo="auto")
    ys = ops.forward(x, spec, None, b, 4096, algo="short")
    assert torch.equal(ya, ys)


@pytest.mark.parametrize("b,k,n_small,n_big", [(64, 4096, 128, 130), (128, 4096, 256, 258), (64, 2048, 170, 172)])
def test_tile_size_does_not_change_results(dev, b, k, n_small, n_big):
    """The 2-token tiles (n_small fits one round of their workgroups) and the 4-token tiles
    (n_big does not) give bit-identical rows: a token's stage 1, its MFMA rows in stage 2 and its
    stage 3 do not depend on which tokens share its workgroup."""
    from bcfft import ops
    m = 3072 if k == 2048 else 4096
    rng = np.random.default_rng(b + n_big)
    c = torch.from_numpy((rng.standard_normal((m // b, k // b, b)) * 0.01).astype(np.float32)).to(dev)
    x = torch.from_numpy(rng.standard_normal((n_big, k)).astype(np.float32)).to(dev)
    spec = ops.spectra(c)
    y_big = ops.forward(x, spec, None, b, m, algo="short")
    y_small = ops.forward(x[:n_small].contiguous(), spec, None, b, m, algo="short")
    assert torch.equal(y_small, y_big[:n_small])
