"""The north star's parity, first in a `-x` run: the benchmarked engines over ALL 8192 tokens
of the bench workload, structured (from_linear-projected) weights with per-output-block and
per-token errors, and the reference's golden vectors under every DFT engine explicitly.

North star: <= 1e-3 relative error vs the reference CPU fft_utils path, fp32, fixed seeds
(BlockCirculantLinear.forward, patch_llama_fft.py:226-275; the reference's own known-answer
test is validate_implementation.py:145-187, T5). The bounds asserted here are tighter than the
contract where the engine is (measured: dftx / dft ~2.8e-4 / ~4e-4, mfma ~5e-6, valu ~2e-7), so
a regression shows long before the contract is at risk."""
import numpy as np
import pytest
import torch

from golden_io import load, names, rel_err
from oracle import bc_oracle as O

pytestmark = pytest.mark.gpu

N_STAR, K_STAR, B_STAR = 8192, 4096, 128
TOL = {"auto": 6e-4, "precise": 6e-5, "dftx": 6e-4, "dft": 6e-4, "dftp": 6e-5, "stationary": 6e-4, "mfma": 5e-5, "valu": 2e-6}
TOKEN_TOL = 1e-3                 # north star, per token
TDT = {"float32": torch.float32, "float16": torch.float16, "bfloat16": torch.bfloat16}
_cache = {}


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    import bcfft
    bcfft.load()                 # fail loudly if the native library is missing
    return torch.device("cuda:0")


def _star_inputs():
    """The bench workload's operator at its full size (seeded), and the oracle's output over all
    8192 tokens (computed once for the module: ~3 s of numpy)."""
    if "star" not in _cache:
        rng = np.random.default_rng(0)
        c = (rng.standard_normal((32, 32, B_STAR)) * 0.01).astype(np.float32)
        bv = (rng.standard_normal(K_STAR) * 0.1).astype(np.float32)
        x = rng.standard_normal((N_STAR, K_STAR)).astype(np.float32)
        _cache["star"] = (c, bv, x, O.bc_forward(x, c, bv))
    return _cache["star"]


def _per_token(g, ref):
    num = np.linalg.norm((g - ref).astype(np.float64), axis=1)
    den = np.linalg.norm(ref.astype(np.float64), axis=1)
    return num / np.maximum(den, 1e-30)


@pytest.mark.parametrize("algo", ["auto", "precise", "dftx", "dftp", "dft", "stationary", "mfma", "valu"])
def test_north_star_all_tokens_vs_oracle(dev, monkeypatch, algo):
    """4096 -> 4096, b = 128, N = batch*seq = 8192, fp32 I/O (+ bias): every token of the bench
    workload against the oracle, Frobenius and per token. AUTO is the engine bench.py times."""
    from patch_llama_fft import BlockCirculantLinear
    monkeypatch.setenv("BCFFT_ALGO", "auto" if algo == "precise" else algo)
    monkeypatch.setenv("BCFFT_PRECISE", "1" if algo == "precise" else "0")
    c, bv, x, ref = _star_inputs()
    mod = BlockCirculantLinear(K_STAR, K_STAR, block_size=B_STAR, bias=True)
    with torch.no_grad():
        mod.c.copy_(torch.from_numpy(c))
        mod.bias.copy_(torch.from_numpy(bv))
    mod = mod.to(dev).eval()
    with torch.no_grad():
        y = mod(torch.from_numpy(x).to(dev))
    g = y.cpu().numpy()
    assert np.isfinite(g).all()
    e = rel_err(g, ref)
    pt = _per_token(g, ref)
    print(f"{algo}: rel err {e:.3e}, worst token {pt.max():.3e}")
    assert e < TOL[algo], e
    assert pt.max() < TOKEN_TOL, (int(pt.argmax()), pt.max())


def test_north_star_bf16_all_tokens_vs_oracle(dev):
    """The bf16-I/O form of the north star (AUTO: the 8-token DFT kernel) over all 8192 tokens:
    every element within ~1 bf16 ulp of the oracle's rounded output, norm-wise < 4e-3."""
    from bcfft import ops
    rng = np.random.default_rng(1)
    c = O.round_to((rng.standard_normal((32, 32, B_STAR)) * 0.01).astype(np.float32), O.BF16)
    x = O.round_to(rng.standard_normal((N_STAR, K_STAR)).astype(np.float32), O.BF16)
    spec = ops.spectra(torch.from_numpy(c).to(dev).to(torch.bfloat16))
    y = ops.forward(torch.from_numpy(x).to(dev).to(torch.bfloat16), spec, None, B_STAR, K_STAR, algo="auto")
    g = y.float().cpu().numpy()
    ref = O.bc_forward(x, c, None, x_dtype=O.BF16)
    ulp = 2.0 ** -7
    rms = float(np.sqrt(np.mean(ref.astype(np.float64) ** 2)))
    bad = np.abs(g - ref) > 2 * ulp * np.abs(ref) + 2 * ulp * rms
    assert not bad.any(), f"{int(bad.sum())} elements beyond ~1 ulp"
    assert rel_err(g, ref) < 4e-3
    assert _per_token(g, ref).max() < 4e-3


def _structured_layer(dev, m, k, b, seed):
    """A LLaMA-like dense weight with very different block norms, projected by from_linear (the
    GPU loss-aware projection): N(0, 0.02) entries with input-block columns scaled over 1e-2..1,
    plus a smooth rank-1 part (blocks with decaying circulant spectra, dominated by the DC bin);
    output-block rows of the sum scaled over 1e-4..1."""
    from patch_llama_fft import BlockCirculantLinear
    g = torch.Generator().manual_seed(seed)
    w = torch.randn(m, k, generator=g) * 0.02
    rs = torch.logspace(-4, 0, m // b)[torch.randperm(m // b, generator=g)]
    cs = torch.logspace(-2, 0, k // b)[torch.randperm(k // b, generator=g)]
    w *= cs.repeat_interleave(b)[None, :]
    t = torch.arange(max(m, k), dtype=torch.float32)
    w += 0.05 * torch.outer(torch.cos(t[:m] * 0.01), torch.exp(-t[:k] / 700.0))
    w *= rs.repeat_interleave(b)[:, None]
    lin = torch.nn.Linear(k, m, bias=False)
    with torch.no_grad():
        lin.weight.copy_(w)
    return BlockCirculantLinear.from_linear(lin.to(dev), block_size=b).eval()


def _structured_tokens(n, k, seed):
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((n, k)).astype(np.float32)
    x *= np.logspace(-2, 2, n).astype(np.float32)[rng.permutation(n)][:, None]   # token norms 1e-2..1e2
    x[:, rng.choice(k, 6, replace=False)] *= 40.0                                 # outlier channels
    return x


def _magnitude_norms(x, c):
    """Per token, the norm of the layer evaluated on magnitudes: sum_i |C_oi[f]| |X_i[f]| per
    output block and bin, through irfft's Parseval weights. It is the scale of the standard
    floating-point error bound of the per-bin sums (|fl(sum a b) - sum a b| <= g sum |a||b|):
    a token whose output is a near-cancellation of large terms is measured against it."""
    n, k = x.shape
    no, ni, b = c.shape
    xf = np.abs(np.fft.rfft(x.reshape(n, ni, b).astype(np.float64), axis=-1))
    cf = np.abs(np.fft.rfft(c.astype(np.float64), axis=-1))
    mag = np.einsum("oif,nif->nof", cf, xf)
    w = np.full(b // 2 + 1, 2.0)
    w[0] = w[-1] = 1.0
    return np.sqrt(np.einsum("nof,f->n", mag ** 2, w) / b)


@pytest.mark.parametrize("algo,xdt", [("auto", "float32"), ("precise", "float32"), ("dftx", "float32"), ("dftp", "float32"),
                                      ("dft", "float32"),
                                      ("stationary", "float32"), ("mfma", "float32"), ("auto", "bfloat16")])
def test_structured_weights_per_block_and_token(dev, monkeypatch, algo, xdt):
    """from_linear weights (output blocks ~1e4 apart in norm) through the forward, errors reported
    per output block and per token:
      * every output block within the north star's 1e-3 (16-bit I/O: the bf16 floor, 4e-3), so no
        quiet block hides behind loud ones in a Frobenius norm;
      * every token within the same bound measured against its magnitude evaluation
        (_magnitude_norms). The raw per-token relative error is printed: for tokens whose output
        nearly cancels (the rank-1 part's projection of x close to zero) it is the weight
        spectra's fp16 rounding (~2^-12) times that cancellation, ~1e-2 on the DFT engines here
        and ~1e-4 on the split-bf16 'mfma' engine."""
    monkeypatch.setenv("BCFFT_ALGO", "auto" if algo == "precise" else algo)
    monkeypatch.setenv("BCFFT_PRECISE", "1" if algo == "precise" else "0")   # precise: AUTO -> dftp
    m, k, b, n = 4096, 4096, 128, 512
    mod = _structured_layer(dev, m, k, b, seed=3)
    if xdt != "float32":
        mod = mod.to(TDT[xdt])
    c = mod.c.detach().float().cpu().numpy()
    x = _structured_tokens(n, k, seed=4)
    xr = O.round_to(x, O.BF16) if xdt == "bfloat16" else x
    with torch.no_grad():
        y = mod(torch.from_numpy(xr).to(dev).to(TDT[xdt]))
    g = y.float().cpu().numpy()
    ref = O.bc_forward(xr, c, None, x_dtype=O.BF16 if xdt == "bfloat16" else O.F32)
    tol = 1e-3 if xdt == "float32" else 4e-3
    d = (g - ref).astype(np.float64).reshape(n, m // b, b)
    r = ref.astype(np.float64).reshape(n, m // b, b)
    per_block = np.sqrt((d ** 2).sum(axis=(0, 2)) / (r ** 2).sum(axis=(0, 2)))
    pt = _per_token(g, ref)
    mag = _magnitude_norms(xr, c)
    pt_cond = np.linalg.norm(d.reshape(n, m), axis=1) / mag
    norms = np.sqrt((r ** 2).sum(axis=(0, 2)))
    amp = mag / np.maximum(np.linalg.norm(ref.astype(np.float64), axis=1), 1e-30)
    print(f"{algo}/{xdt}: block norms span {norms.max() / norms.min():.1e}; worst block "
          f"{per_block.max():.3e} (block {per_block.argmax()}); worst token {pt.max():.3e} raw "
          f"(cancellation x{amp[pt.argmax()]:.0f}), {pt_cond.max():.3e} vs its magnitude evaluation; "
          f"Frobenius {rel_err(g, ref):.3e}")
    assert norms.max() / norms.min() > 1000.0         # the test really has quiet and loud blocks
    assert rel_err(g, ref) < (TOL[algo] if xdt == "float32" else 4e-3)
    assert per_block.max() < tol, (int(per_block.argmax()), per_block.max())
    assert pt_cond.max() < tol, (int(pt_cond.argmax()), pt_cond.max())
    assert pt.max() < 50 * tol                        # gross-error guard on the raw figure
    if algo in ("dftp", "precise"):
        # the precise engine: RAW per token within the north star, with margin (measured 1.8e-4:
        # the weight residual against e4m3 (RNE) of X; 8.8e-4 with round 4's bf8 operand)
        assert pt.max() < TOKEN_TOL / 2, (int(pt.argmax()), pt.max())
    elif algo in ("auto", "dftx") and xdt == "float32":
        # NOT per-token faithful on cancelling tokens (measured 5.9e-3 raw at x26-54 cancellation):
        # the weight spectra's single fp16 term. Pinned here so a change
        # either way shows; BCFFT_PRECISE=1 (dftp) is the engine that meets 1e-3 per token raw.
        assert 1e-3 < pt.max() < 1e-2, pt.max()


DFT_GOLDEN = [nm for nm in names("fwd_") if nm.startswith(("fwd_4096sq_b128", "fwd_up_4096x11008_b128"))]


@pytest.mark.parametrize("algo", ["dft", "dftx", "dftp"])
@pytest.mark.parametrize("name", DFT_GOLDEN)
def test_golden_under_dft_engines(dev, monkeypatch, name, algo):
    """The reference's golden vectors of the DFT geometries (b = 128, K = 4096) through the module
    with each DFT engine forced; bf16 x under 'dft' is the 8-token kernel (bcfft_dm8.hip)."""
    from patch_llama_fft import BlockCirculantLinear
    monkeypatch.setenv("BCFFT_ALGO", algo)
    gv = load(name)
    c = gv["c"]
    n_out, n_in, b = c.shape
    mdt = {"fp32": torch.float32, "fp16": torch.float16, "bf16": torch.bfloat16}[gv["mod_dtype"]]
    mod = BlockCirculantLinear(n_in * b, n_out * b, block_size=b, bias="bias" in gv)
    with torch.no_grad():
        mod.c.copy_(torch.from_numpy(c))
        if "bias" in gv:
            mod.bias.copy_(torch.from_numpy(gv["bias"]))
    mod = mod.to(mdt).to(dev).eval()
    x = torch.from_numpy(gv["x"]).to(dev).to(TDT[gv["x__dt"]])
    with torch.no_grad():
        y = mod(x)
    assert str(y.dtype).replace("torch.", "") == gv["y__dt"]
    g, ref = y.float().cpu().numpy(), gv["y"]
    if gv["y__dt"] == "float32":
        assert rel_err(g, ref) < TOL[algo]
    else:
        ulp = 2.0 ** -7 if gv["y__dt"] == "bfloat16" else 2.0 ** -10
        rms = float(np.sqrt(np.mean(ref.astype(np.float64) ** 2)))
        assert np.all(np.abs(g - ref) <= 2 * ulp * np.abs(ref) + 2 * ulp * rms)
        assert rel_err(g, ref) < 4e-3
