"""GPU parity of the streamed-weight DFT kernel (bcfft_dmk.hip: b = 128, K > 4096, bf16 I/O;
the LLaMA down projection 11008 -> 4096) against the CPU oracle.

Numerics are the 8-token bf16 kernel's (tests/dm_model.py, single_x): per-(token, chunk)
power-of-two scales, a/d, X and Y one RNE fp16 term each, C and the table one term each, fp32
accumulation; chunks are aligned to each token's loudest chunk so far, and accumulator rows are
scaled down when a later chunk is louder. Outputs are bf16: within ~1 output ulp plus the norm
bound (_check), as every bf16 case of the other DFT kernels."""
import numpy as np
import pytest
import torch

from golden_io import rel_err
from oracle import bc_oracle as O
from test_gpu_stationary import _check, _run

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    import bcfft
    bcfft.load()
    return torch.device("cuda:0")


def _extremes(rng, k):
    x = rng.standard_normal((11, k)).astype(np.float32)
    x[0, 9000:9500] *= 3e3            # chunk 4 of token 0 far louder than chunks 0-3
    x[1, :2048] *= 3e3                # chunk 0 far louder than the rest
    x[2] = 0.0
    x[3] *= 1e-20
    x[4, 10000] = 5000.0              # one massive channel in the last (partial) chunk
    x[5, 2048:4096] *= 1e-6           # one very quiet chunk in the middle
    x[6, 4096:] *= 1e5                # every chunk after the second louder
    return x


CASES = [
    # (K, M, N, bias)
    (11008, 4096, 37, False),      # down projection: 86 input blocks = 6 chunks, the last of 6
    (11008, 4096, 1, False),       # one token: 7 empty slots in the tile
    (11008, 4096, 300, True),      # many tiles per workgroup; bf16 bias
    (5120, 1024, 17, True),        # 40 input blocks (last chunk of 8), one partial output group
    (6144, 5120, 50, False),       # 48 input blocks (3 full chunks), 2 groups, the last partial
    (16256, 512, 9, False),        # 127 input blocks: the largest K the kernel takes
]


@pytest.mark.parametrize("k,m,n,bias", CASES)
def test_dmk_bf16_vs_oracle(dev, k, m, n, bias):
    b = 128
    rng = np.random.default_rng(k + m + n)
    c = (rng.standard_normal((m // b, k // b, b)) * 0.01).astype(np.float32)
    bv = (rng.standard_normal(m) * 0.1).astype(np.float32) if bias else None
    x = rng.standard_normal((n, k)).astype(np.float32)
    y, ref = _run(dev, x, c, bv, "bfloat16", "bfloat16", algo="dft")
    _check(y, ref, "bfloat16")
    ya, _ = _run(dev, x, c, bv, "bfloat16", "bfloat16", algo="auto")   # AUTO resolves to it
    assert torch.equal(y, ya)


@pytest.mark.parametrize("n", [11, 4090])
def test_dmk_per_token_chunk_scales(dev, n):
    """Chunks of one token at very different magnitudes, in both orders (a later louder chunk
    scales the accumulated rows down), zero and tiny tokens, a single massive channel. n = 11
    runs 8-token tiles; n = 4090 runs one 16-token tile per CU (the launcher's makespan rule;
    the last tile ragged)."""
    from bcfft import ops
    k, m, b = 11008, 4096, 128
    rng = np.random.default_rng(5)
    c = (rng.standard_normal((m // b, k // b, b)) * 0.01).astype(np.float32)
    if n > 11:                                    # oracle on the special rows and the ragged tail
        x = rng.standard_normal((n, k)).astype(np.float32)
        x[:11] = _extremes(rng, k)
        spec = ops.spectra(torch.from_numpy(c).to(dev).to(torch.bfloat16))
        xt = torch.from_numpy(x).to(dev).to(torch.bfloat16)
        y = ops.forward(xt, spec, None, b, m, algo="dft").float().cpu().numpy()
        rows = list(range(11)) + list(range(n - 20, n))
        xr = xt[rows].float().cpu().numpy()
        ref = O.bc_forward(xr, O.round_to(c, O.BF16), x_dtype=O.BF16)
        assert np.all(y[2] == 0.0)
        for i, t in enumerate(rows):
            if t != 2:
                assert rel_err(y[t], ref[i]) < 4e-3, (t, rel_err(y[t], ref[i]))
        return
    x = _extremes(rng, k)
    y, ref = _run(dev, x, c, None, "bfloat16", "bfloat16", algo="dft")
    g = y.float().cpu().numpy()
    assert np.all(g[2] == 0.0)
    for t in range(x.shape[0]):
        if t == 2:
            continue
        e = rel_err(g[t], ref[t])
        assert e < 4e-3, (t, e)


def test_dmk_full_size_and_linearity(dev):
    """11008 -> 4096, N = 8192 (the sweep's down projection): every token against the oracle
    (~1 bf16 ulp per element, 4e-3 per token), run-to-run bit equality, and linearity over all
    tokens within the bf16 rounding."""
    from bcfft import ops
    k, m, b, n = 11008, 4096, 128, 8192
    rng = np.random.default_rng(0)
    c = (rng.standard_normal((m // b, k // b, b)) * 0.01).astype(np.float32)
    spec = ops.spectra(torch.from_numpy(c).to(dev).to(torch.bfloat16))
    xt = torch.randn(n, k, device=dev).to(torch.bfloat16)
    y = ops.forward(xt, spec, None, b, m, algo="dft")
    ref = O.bc_forward(xt.float().cpu().numpy(), O.round_to(c, O.BF16), x_dtype=O.BF16)
    g = y.float().cpu().numpy()
    assert rel_err(g, ref) < 4e-3
    ulp = 2.0 ** -7
    rms = float(np.sqrt(np.mean(ref.astype(np.float64) ** 2)))
    bad = np.abs(g - ref) > 2 * ulp * np.abs(ref) + 2 * ulp * rms
    assert not bad.any(), f"{int(bad.sum())} elements beyond ~1 ulp"
    tok = np.sqrt(((g.astype(np.float64) - ref) ** 2).sum(1) / (ref.astype(np.float64) ** 2).sum(1))
    print(f"dmk full size: worst token {tok.max():.3e}, Frobenius {rel_err(g, ref):.3e}")
    assert tok.max() < 4e-3, (int(tok.argmax()), tok.max())
    assert torch.equal(y, ops.forward(xt, spec, None, b, m, algo="dft"))
    x2 = torch.randn(n, k, device=dev).to(torch.bfloat16)
    lhs = ops.forward((xt.float() + x2.float()).to(torch.bfloat16), spec, None, b, m, algo="dft").float()
    rhs = y.float() + ops.forward(x2, spec, None, b, m, algo="dft").float()
    assert ((lhs - rhs).norm() / rhs.norm()).item() < 1e-2


def test_dmk_bf16_matches_numpy_model(dev):
    """The kernel's bf16 output equals its numpy mirror (tests/dm_model.py, head=4: chunked
    scales, headroom, running reference) rounded to bf16, except for rounding flips at bf16
    ties; both 8-token tiles (N = 21) and the chunk-scale extremes are covered."""
    from dm_model import dm_forward
    k, m, b = 5120, 1024, 128                      # nI = 40: chunks of 16, 16 and 8 blocks
    rng = np.random.default_rng(13)
    c = (rng.standard_normal((m // b, k // b, b)) * 0.01).astype(np.float32)
    x = rng.standard_normal((21, k)).astype(np.float32)
    x[1, 4200:4300] *= 3e3
    x[2, :2048] *= 3e3
    x[3, 2048:4096] *= 10.0
    x[9] *= 1e-4
    xr = O.round_to(x, O.BF16)
    _, ref = _run(dev, x, c, None, "bfloat16", "bfloat16", algo="dft")
    from bcfft import ops
    spec = ops.spectra(torch.from_numpy(c).to(dev).to(torch.bfloat16))
    y = ops.forward(torch.from_numpy(x).to(dev).to(torch.bfloat16), spec, None, b, m, algo="dft",
                    split_k=False)                  # the unsplit kernel the model mirrors
    g = y.float().cpu().numpy()
    mdl = O.round_to(dm_forward(xr, O.round_to(c, O.BF16), head=4), O.BF16)
    assert np.mean(g == mdl) > 0.97, np.mean(g == mdl)
    assert rel_err(g, mdl) < 1e-3
    for t in range(x.shape[0]):
        assert rel_err(g[t], ref[t]) < 4e-3, t


@pytest.mark.parametrize("k,m,n,bias", [(11008, 4096, 1, False), (11008, 4096, 20, True), (11008, 4096, 37, False),
                                        (11008, 4096, 128, True), (16256, 512, 9, False), (5120, 1024, 17, True)])
def test_dmk_split_k_short_grids(dev, k, m, n, bias):
    """Decode / short-prefill sizes: the K-chunks split over kz workgroup slices whose fp32 partial
    outputs a finishing pass sums in a fixed order, then rounds (+ bias) once. Against the oracle
    (bf16 bounds) and the unsplit launch (same numerics up to the partials' fp16 Y roundings)."""
    from bcfft import _lib, ops
    b = 128
    lib = _lib.load()
    wsb = lib.bcfft_forward_workspace_bytes_io(n, k, m, b, _lib.ALGOS["auto"], _lib.BCFFT_BF16, _lib.BCFFT_BF16)
    assert wsb > 0 and wsb % (n * m * 4) == 0 and wsb // (n * m * 4) >= 2
    rng = np.random.default_rng(k + 3 * n)
    c = (rng.standard_normal((m // b, k // b, b)) * 0.01).astype(np.float32)
    bv = (rng.standard_normal(m) * 0.1).astype(np.float32) if bias else None
    x = rng.standard_normal((n, k)).astype(np.float32)
    if n >= 11:
        x[:11] = _extremes(rng, k)[:, :k] if k >= 11008 else x[:11]
    y, ref = _run(dev, x, c, bv, "bfloat16", "bfloat16", algo="dft")
    g = y.float().cpu().numpy()
    for t in range(n):
        if np.any(ref[t] != 0):
            assert rel_err(g[t], ref[t]) < 4e-3, (t, rel_err(g[t], ref[t]))
    spec = ops.spectra(torch.from_numpy(c).to(dev).to(torch.bfloat16))
    bt = torch.from_numpy(bv).to(dev).to(torch.bfloat16) if bias else None
    xt = torch.from_numpy(x).to(dev).to(torch.bfloat16)
    yu = ops.forward(xt, spec, bt, b, m, algo="dft", split_k=False)
    d = (y.float() - yu.float()).abs()
    rms = yu.float().pow(2).mean().sqrt().item()
    assert (d <= 2.0 ** -7 * (yu.float().abs() + rms)).float().mean().item() > 0.999
    assert ((y.float() - yu.float()).norm() / yu.float().norm()).item() < 3e-3
    assert torch.equal(y, ops.forward(xt, spec, bt, b, m, algo="dft"))     # deterministic
