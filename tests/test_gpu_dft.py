"""GPU parity of the DFT-on-MFMA kernel (algo="dft", bcfft_dm.hip) against the CPU oracle and
against its numpy mirror (tests/dm_model.py).

Numerics (dm_model.py): the table and C are one fp16 term each, X two; a/d and the per-bin
products Y one RNE fp16 term each ("dft", ~4e-4 relative Frobenius on random data) or two
("dftx", and every fp16-output launch: ~2.8e-4, linear in x to ~1e-6); fp32 accumulation. The tests assert
< 6e-4 (north star: 1e-3), per token where scales differ; 16-bit outputs within ~1 output ulp
plus the norm bound."""
import numpy as np
import pytest
import torch

from golden_io import rel_err
from oracle import bc_oracle as O
from test_gpu_stationary import TDT, ODT, _check, _run, _check_auto

pytestmark = pytest.mark.gpu
DFT_TOL = 6e-4


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    import bcfft
    bcfft.load()
    return torch.device("cuda:0")


CASES = [
    # (M, N, x dtype, module dtype, bias)
    (4096, 1, "float32", "float32", True),        # one token: partial M-tile, 3 zero-filled slots
    (4096, 4, "float32", "float32", False),
    (4096, 37, "float32", "float32", True),
    (4096, 301, "bfloat16", "bfloat16", False),   # ragged, many tiles per workgroup
    (4096, 64, "float16", "float16", True),
    (4096, 50, "bfloat16", "float32", True),      # promotion -> fp32 output
    (11008, 31, "bfloat16", "bfloat16", False),   # 3 output groups, the last one partial
    (11008, 9, "float32", "float32", True),
    (1024, 23, "float32", "float32", False),      # a single partial group (32 of 8 blocks)
    (4096, 2000, "float32", "float32", False),    # > 1 tile per workgroup on every CU
    (4096, 19, "bfloat16", "bfloat16", True),     # 8-token kernel: bf16 bias, ragged last tile
    (4096, 1, "bfloat16", "bfloat16", False),     # 8-token kernel: one token, 7 empty slots
    (1024, 9, "bfloat16", "bfloat16", True),      # 8-token kernel: one partial group
]


@pytest.mark.parametrize("algo", ["dft", "dftx"])
@pytest.mark.parametrize("m,n,xdt,mdt,bias", CASES)
def test_dft_vs_oracle(dev, m, n, xdt, mdt, bias, algo):
    k, b = 4096, 128
    rng = np.random.default_rng(m + n + len(xdt))
    c = (rng.standard_normal((m // b, k // b, b)) * 0.01).astype(np.float32)
    bv = (rng.standard_normal(m) * 0.1).astype(np.float32) if bias else None
    x = rng.standard_normal((n, k)).astype(np.float32)
    if n > 600:                                    # oracle on a slice, all tokens computed
        y, _ = _run(dev, x, c, bv, xdt, mdt, algo=algo)
        sl = slice(n - 300, n)
        ref = O.bc_forward(x[sl], c, bv)
        e = rel_err(y[sl].float().cpu().numpy(), ref)
        assert e < DFT_TOL, e
        return
    y, ref = _run(dev, x, c, bv, xdt, mdt, algo=algo)
    _check(y, ref, xdt)              # fp32: < 6e-4 (= DFT_TOL); 16-bit x: ~1 ulp of the rounding


@pytest.mark.parametrize("algo", ["dft", "dftx"])
def test_dft_matches_numpy_model(dev, algo):
    """The kernel and its numpy mirror agree far below the quantisation error: same table,
    splits, scales and packed-bin order (only the fp32 summation order differs)."""
    from dm_model import dm_forward
    rng = np.random.default_rng(11)
    c = (rng.standard_normal((32, 32, 128)) * 0.01).astype(np.float32)
    x = rng.standard_normal((8, 4096)).astype(np.float32)
    x[1] *= 300.0
    y, ref = _run(dev, x, c, None, "float32", "float32", algo=algo)
    g = y.cpu().numpy()
    mdl = dm_forward(x, c, exact=algo == "dftx")
    # one-term Y: an fp32 summation-order difference can flip an fp16 rounding of a product
    assert rel_err(g, mdl) < (2e-5 if algo == "dftx" else 1e-4), rel_err(g, mdl)
    assert rel_err(g, ref) < DFT_TOL


@pytest.mark.parametrize("algo", ["dft", "dftx"])
def test_dft_per_token_scale(dev, algo):
    """Tokens 10^9 apart in magnitude, zero tokens, one massive channel, a token far below fp16's
    range: the per-(token, half) power-of-two scales keep every token at full relative accuracy."""
    rng = np.random.default_rng(2)
    c = (rng.standard_normal((32, 32, 128)) * 0.01).astype(np.float32)
    x = rng.standard_normal((9, 4096)).astype(np.float32)
    x[0] *= 1e4
    x[1] *= 1e-5
    x[2] = 0.0
    x[3, 77] = 3000.0
    x[4, 2100:2300] *= 1e3                # the two K halves at very different scales
    x[5] *= 1e-30
    y, ref = _run(dev, x, c, None, "float32", "float32", algo=algo)
    g = y.cpu().numpy()
    assert np.all(g[2] == 0.0)
    for t in (0, 1, 3, 4, 5, 6, 7, 8):
        e = rel_err(g[t], ref[t])
        assert e < DFT_TOL, (t, e)


@pytest.mark.parametrize("algo,lin_tol", [("dft", 1e-3), ("dftx", 1e-5)])
def test_dft_full_size_and_linearity(dev, algo, lin_tol):
    """North-star size (4096^2, b=128, N=8192, fp32): oracle parity on a 256-token slice plus
    linearity over all 8192 tokens, and run-to-run bit equality."""
    from bcfft import ops
    rng = np.random.default_rng(0)
    c = (rng.standard_normal((32, 32, 128)) * 0.01).astype(np.float32)
    x = rng.standard_normal((8192, 4096)).astype(np.float32)
    spec = ops.spectra(torch.from_numpy(c).to(dev))
    xt = torch.from_numpy(x).to(dev)
    y = ops.forward(xt, spec, None, 128, 4096, algo=algo)
    sl = slice(4000, 4256)
    e = rel_err(y[sl].cpu().numpy(), O.bc_forward(x[sl], c))
    assert e < DFT_TOL, e
    assert torch.equal(y, ops.forward(xt, spec, None, 128, 4096, algo=algo))
    x2 = torch.randn(8192, 4096, device=dev)
    lhs = ops.forward(2.0 * xt + x2, spec, None, 128, 4096, algo=algo)
    rhs = 2.0 * y + ops.forward(x2, spec, None, 128, 4096, algo=algo)
    assert ((lhs - rhs).norm() / rhs.norm()).item() < lin_tol


def test_dft_rejects_ineligible_geometry(dev):
    from bcfft import ops
    c = torch.zeros(4, 8, 64, device=dev)
    spec = ops.spectra(c)
    with pytest.raises(RuntimeError, match="block_size"):
        ops.forward(torch.zeros(3, 512, device=dev), spec, None, 64, 256, algo="dft")


def test_dft8_bf16_matches_numpy_model(dev):
    """bf16 I/O runs the 8-token kernel (bcfft_dm8.hip: X one fp16 term): its bf16 output equals
    the numpy mirror's (single_x) rounded to bf16 except for rounding flips at the bf16 ties."""
    from dm_model import dm_forward
    rng = np.random.default_rng(12)
    c = (rng.standard_normal((32, 32, 128)) * 0.01).astype(np.float32)
    x = rng.standard_normal((21, 4096)).astype(np.float32)   # 3 M-tiles of 8, the last partial
    x[3] *= 500.0
    x[9] *= 1e-4
    xr = O.round_to(x, O.BF16)
    y, ref = _run(dev, x, c, None, "bfloat16", "bfloat16", algo="dft")
    g = y.float().cpu().numpy()
    mdl = O.round_to(dm_forward(xr, O.round_to(c, O.BF16), exact=False, single_x=True), O.BF16)
    assert np.mean(g == mdl) > 0.97, np.mean(g == mdl)
    assert rel_err(g, mdl) < 1e-3
    for t in range(x.shape[0]):
        assert rel_err(g[t], ref[t]) < 4e-3, t


CASES64 = [
    # (M, N, bias): b = 64 with K = 4096, bf16 I/O -> bc_forward_dm64_kernel (bcfft_dm64.hip)
    (4096, 37, False),        # ragged last tile of 8
    (11008, 19, True),        # 6 output groups, the last partial; bf16 bias
    (2048, 1, False),         # one token, one group
    (4096, 600, True),        # several tiles per workgroup
]


@pytest.mark.parametrize("m,n,bias", CASES64)
def test_dft64_bf16_vs_oracle(dev, m, n, bias):
    k, b = 4096, 64
    rng = np.random.default_rng(m + n)
    c = (rng.standard_normal((m // b, k // b, b)) * 0.01).astype(np.float32)
    bv = (rng.standard_normal(m) * 0.1).astype(np.float32) if bias else None
    x = rng.standard_normal((n, k)).astype(np.float32)
    y, ref = _run(dev, x, c, bv, "bfloat16", "bfloat16", algo="dft")
    _check(y, ref, "bfloat16")
    ya, _ = _run(dev, x, c, bv, "bfloat16", "bfloat16", algo="auto")
    _check_auto(y, ya, ref, n, k, m, b, "bfloat16")   # AUTO resolves to it (short N: the sn kernel)
    x[0] *= 300.0                                # per-(token, quarter) scales: a loud token
    x[n - 1, 1000:1100] *= 1e-3
    y, ref = _run(dev, x, c, bv, "bfloat16", "bfloat16", algo="dft")
    g = y.float().cpu().numpy()
    for t in (0, n - 1):
        assert rel_err(g[t], ref[t]) < 4e-3, (t, rel_err(g[t], ref[t]))


@pytest.mark.parametrize("b", [128, 64])
def test_mixed_order_multi_tile_bias_and_glu(dev, b):
    """N = 4104: every workgroup of the 8-token kernels (bcfft_dm8.hip at b = 128,
    bcfft_dm64.hip at b = 64) runs two or more tiles, the last ragged, so the mixed stage order
    (waves 0-3 run stage 3 and the next x DMA before stage 1, their x waits counting those stores
    and that DMA) is exercised with a bf16 bias (the HB instantiation) and in the fused gate/up
    (GLU: 4 stores per stage 3 instead of 8), against the oracle."""
    from bcfft import ops
    from test_gpu_glu import oracle_glu
    k, m, n = 4096, 4096, 4104
    rng = np.random.default_rng(b + 41)
    c = (rng.standard_normal((m // b, k // b, b)) * 0.01).astype(np.float32)
    bv = (rng.standard_normal(m) * 0.1).astype(np.float32)
    x = rng.standard_normal((n, k)).astype(np.float32)
    y, ref = _run(dev, x, c, bv, "bfloat16", "bfloat16", algo="dft")
    _check(y, ref, "bfloat16")
    mg = 2048 if b == 128 else 1024                  # one output group of the GLU form
    cg = (rng.standard_normal((mg // b, k // b, b)) * 0.01).astype(np.float32)
    cu = (rng.standard_normal((mg // b, k // b, b)) * 0.01).astype(np.float32)
    spec = ops.spectra(ops.glu_weights(torch.from_numpy(cg).to(dev), torch.from_numpy(cu).to(dev)))
    h = ops.forward_glu(torch.from_numpy(x).to(dev).to(torch.bfloat16), spec, b, mg, algo="dft")
    torch.cuda.synchronize()
    # 8.4 M products of two bf16-rounded projections: a handful sit 2 ulps off where the
    # oracle's and the kernel's gate / up round to neighbouring values, so the bound is on the
    # fraction (the mixed order itself is bit-identical to the plain one: tools/dump_mixed.py)
    g = h.float().cpu().numpy()
    ref = oracle_glu(x, cg, cu, "bfloat16")
    ulp = 2.0 ** -7
    rms = float(np.sqrt(np.mean(ref.astype(np.float64) ** 2)))
    bad = np.abs(g - ref) > 2 * ulp * np.abs(ref) + 2 * ulp * rms
    assert bad.mean() < 1e-5, (int(bad.sum()), bad.size)
    assert rel_err(g, ref) < 4e-3
