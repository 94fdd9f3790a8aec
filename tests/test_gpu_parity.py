"""GPU parity: the HIP engine (libbcfft.so through the drop-in module) vs the oracle and the
reference's golden vectors. Tolerance (north_star): <= 1e-3 relative (Frobenius) error for
fp32 outputs. Low-precision outputs are additionally rounded to bf16/fp16 by both sides, so
they are checked to be within one output ulp elementwise plus a norm-wise bound."""
import numpy as np
import pytest
import torch

from golden_io import load, names, rel_err
from oracle import bc_oracle as O

pytestmark = pytest.mark.gpu

TOL_F32 = 1e-3          # north_star: <= 1e-3 rel fp32
TDT = {"float32": torch.float32, "float16": torch.float16, "bfloat16": torch.bfloat16}
ODT = {"float32": O.F32, "float16": O.F16, "bfloat16": O.BF16}


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    import bcfft
    bcfft.load()   # fail loudly if the native library is missing
    return torch.device("cuda:0")


def _to_dev(a, dtname, dev):
    return torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev).to(TDT[dtname])


def _check(got: torch.Tensor, ref: np.ndarray, out_dt: str, tol=TOL_F32):
    g = got.detach().float().cpu().numpy()
    assert g.shape == ref.shape
    assert np.isfinite(g).all()
    e = rel_err(g, ref)
    if out_dt == "float32":
        assert e < tol, f"rel err {e:.3e}"
    else:
        # both sides round to the output dtype; allow rounding-boundary flips of <= ~1 ulp
        ulp = 2.0 ** -7 if out_dt == "bfloat16" else 2.0 ** -10
        rms = float(np.sqrt(np.mean(ref.astype(np.float64) ** 2)))
        assert np.all(np.abs(g - ref) <= 2 * ulp * np.abs(ref) + ulp * rms), "more than ~1 ulp off"
        assert e < 4e-3, f"rel err {e:.3e}"
    return e


def _module(c, bias, mod_dt, dev):
    from patch_llama_fft import BlockCirculantLinear
    n_out, n_in, b = c.shape
    m = BlockCirculantLinear(n_in * b, n_out * b, block_size=b, bias=bias is not None)
    with torch.no_grad():
        m.c.copy_(torch.from_numpy(c))
        if bias is not None:
            m.bias.copy_(torch.from_numpy(bias))
    return m.to(TDT[mod_dt]).to(dev).eval()


# ---------------------------------------------------------------- golden vectors (reference)
@pytest.mark.parametrize("name", names("fwd_"))
def test_forward_vs_reference_golden(dev, name):
    g = load(name)
    mdt = {"fp32": "float32", "fp16": "float16", "bf16": "bfloat16"}[g["mod_dtype"]]
    m = _module(g["c"], g.get("bias"), mdt, dev)
    x = _to_dev(g["x"], g["x__dt"], dev)
    with torch.no_grad():
        y = m(x)
    assert str(y.dtype).replace("torch.", "") == g["y__dt"]
    _check(y, g["y"], g["y__dt"])


@pytest.mark.parametrize("name", names("cmv_"))
def test_circulant_matvec_vs_reference_golden(dev, name):
    from fft_utils import circulant_matvec_fft
    g = load(name)
    c = _to_dev(g["c"], g["c__dt"], dev)
    x = _to_dev(g["x"], g["x__dt"], dev)
    y = circulant_matvec_fft(c, x)
    _check(y, g["y"], g["y__dt"])


def test_spectra_vs_reference_golden(dev):
    """bcfft_spectra's packed, scaled bins == rfft(c)/(2b) of the golden spectra."""
    from bcfft import ops
    for name in names("fwd_"):
        g = load(name)
        if "cf_re" not in g:
            continue
        c = torch.from_numpy(g["c"]).to(dev)
        b = c.shape[-1]
        h = b // 2
        n = c.shape[0] * c.shape[1]
        s = ops.spectra(c).cpu().numpy()[: n * h * 2].reshape(c.shape[0], c.shape[1], h, 2)
        ref = (g["cf_re"] + 1j * g["cf_im"]) / (2 * b)
        got = s[..., 0] + 1j * s[..., 1]
        assert rel_err(got[..., 1:], ref[..., 1:h]) < 1e-6
        assert rel_err(got[..., 0].real, ref[..., 0].real) < 1e-6
        assert rel_err(got[..., 0].imag, ref[..., h].real) < 1e-6


# ---------------------------------------------------------------- seeded cases vs the oracle
CASES = [
    # (K, M, b, N, x dtype, module dtype, bias)
    (128, 64, 32, 4, "float32", "float32", False),
    (384, 256, 128, 17, "float32", "float32", True),     # nI=3 < IC: partial chunk; ragged N
    (4096, 4096, 128, 1, "float32", "float32", True),
    (4096, 4096, 128, 33, "bfloat16", "float32", False),
    (4096, 4096, 64, 15, "float32", "float32", True),
    (4096, 4096, 256, 16, "float32", "float32", True),
    (4096, 11008, 128, 31, "bfloat16", "bfloat16", False),  # nO=86: partial output group
    (11008, 4096, 128, 9, "float16", "float32", False),     # nI=86: partial last chunk
    (512, 1536, 64, 40, "float16", "float16", True),
    (1024, 768, 256, 23, "bfloat16", "float32", True),       # promotion -> fp32 output
    (256, 256, 32, 64, "float32", "float32", True),
]


@pytest.mark.parametrize("algo", ["auto", "valu"])
@pytest.mark.parametrize("k,m,b,n,xdt,mdt,bias", CASES)
def test_forward_vs_oracle(dev, monkeypatch, algo, k, m, b, n, xdt, mdt, bias):
    monkeypatch.setenv("BCFFT_ALGO", algo)
    rng = np.random.default_rng(k * 7 + m * 3 + b + n)
    c = (rng.standard_normal((m // b, k // b, b)) * 0.01).astype(np.float32)
    bv = (rng.standard_normal(m) * 0.1).astype(np.float32) if bias else None
    x = rng.standard_normal((n, k)).astype(np.float32)
    mod = _module(c, bv, mdt, dev)
    xt = _to_dev(x, xdt, dev)
    with torch.no_grad():
        y = mod(xt)
    c_eff = O.round_to(c, ODT[mdt])
    b_eff = O.round_to(bv, ODT[mdt]) if bias else None
    ref = O.bc_forward(O.round_to(x, ODT[xdt]), c_eff, b_eff, x_dtype=ODT[xdt],
                       bias_dtype=ODT[mdt] if bias else None)
    _check(y, ref, str(y.dtype).replace("torch.", ""))


def test_three_d_input_and_shapes(dev):
    rng = np.random.default_rng(5)
    c = (rng.standard_normal((4, 4, 128)) * 0.01).astype(np.float32)
    mod = _module(c, None, "float32", dev)
    x = rng.standard_normal((2, 5, 512)).astype(np.float32)
    y = mod(torch.from_numpy(x).to(dev))
    assert y.shape == (2, 5, 512)
    _check(y, O.bc_forward(x, c), "float32")


def test_empty_batch(dev):
    mod = _module(np.zeros((2, 2, 64), np.float32), np.zeros(128, np.float32), "float32", dev)
    y = mod(torch.zeros(0, 128, device=dev))
    assert y.shape == (0, 128)


def test_reference_error_behaviour(dev):
    mod = _module(np.zeros((2, 2, 64), np.float32), None, "float32", dev)
    with pytest.raises(ValueError, match="Unsupported input dim"):
        mod(torch.zeros(1, 1, 1, 128, device=dev))
    with pytest.raises(AssertionError):
        mod(torch.zeros(1, 2, 64, device=dev))
    with pytest.raises(RuntimeError):
        mod(torch.zeros(3, 100, device=dev))
    with pytest.raises(RuntimeError, match="ROCm device"):
        mod(torch.zeros(3, 128))


# ---------------------------------------------------------------- full size (north star)
# (every engine over all 8192 tokens of the bench workload: tests/test_gpu_0_north_star.py)
@pytest.mark.parametrize("algo,tol", [
    ("auto", 1e-5),        # fp32 outputs resolve to dftx (products split hi + lo): linear to ~1e-6
    ("dft", 1e-3),         # the per-bin products rounded once to fp16 (~3e-4 noise per call)
    ("dftx", 1e-5),
    ("stationary", 1e-5),
])
def test_linearity_full_size(dev, monkeypatch, algo, tol):
    """BC(a x1 + x2) = a BC(x1) + BC(x2) at the bench shape (size-independent property)."""
    monkeypatch.setenv("BCFFT_ALGO", algo)
    torch.manual_seed(0)
    from patch_llama_fft import BlockCirculantLinear
    mod = BlockCirculantLinear(4096, 11008, block_size=128, bias=False).to(dev).eval()
    x1 = torch.randn(8192, 4096, device=dev)
    x2 = torch.randn(8192, 4096, device=dev)
    with torch.no_grad():
        lhs = mod(2.5 * x1 + x2)
        rhs = 2.5 * mod(x1) + mod(x2)
    assert (lhs - rhs).norm() / rhs.norm() < tol


def test_spectra_cache_invalidation(dev):
    """An in-place update of c must be seen by the next forward (no stale spectra)."""
    rng = np.random.default_rng(9)
    c = (rng.standard_normal((2, 2, 64)) * 0.01).astype(np.float32)
    mod = _module(c, None, "float32", dev)
    x = torch.randn(3, 128, device=dev)
    with torch.no_grad():
        y1 = mod(x)
        mod.c.mul_(2.0)
        y2 = mod(x)
    assert torch.allclose(y2, 2 * y1, rtol=1e-5, atol=1e-6)


# ---------------------------------------------------------------- backward (calibration path)
def test_backward_vs_dense(dev):
    rng = np.random.default_rng(3)
    k, m, b, n = 512, 256, 64, 7
    c = (rng.standard_normal((m // b, k // b, b)) * 0.1).astype(np.float32)
    bv = (rng.standard_normal(m) * 0.1).astype(np.float32)
    x = rng.standard_normal((n, k)).astype(np.float32)
    gy = rng.standard_normal((n, m)).astype(np.float32)
    mod = _module(c, bv, "float32", dev).train()
    xt = torch.from_numpy(x).to(dev).requires_grad_(True)
    y = mod(xt)
    y.backward(torch.from_numpy(gy).to(dev))
    w = O.bc_dense_weight(c.astype(np.float64))
    assert rel_err(xt.grad.cpu().numpy(), gy @ w) < 1e-5
    # dL/dc[o,i,t] = sum_n sum_r gy[n, o*b + r] x[n, i*b + (r - t) % b]
    gyb = gy.reshape(n, m // b, b).astype(np.float64)
    xb = x.reshape(n, k // b, b).astype(np.float64)
    r = np.arange(b)
    xs = xb[:, :, (r[:, None] - r[None, :]) % b]            # [n, i, r, t]
    dc = np.einsum("nor,nirt->oit", gyb, xs)
    assert rel_err(mod.c.grad.cpu().numpy(), dc) < 1e-5
    assert rel_err(mod.bias.grad.cpu().numpy(), gy.sum(0)) < 1e-6


# ------------------------------------------------- split-K MFMA launches (short grids, K >= 32 blocks)
SPLIT_CASES = [
    # (K, M, b, N, x dtype, bias dtype or None, algo)
    (11008, 4096, 128, 1700, "bfloat16", None, "auto"),       # LLaMA down projection, prefill batch
    (11008, 4096, 128, 3, "float32", "float32", "auto"),      # 11 slices of 1 chunk (decode-size N)
    (11008, 4096, 128, 40, "bfloat16", "bfloat16", "auto"),   # 6 slices of 2 chunks
    (4224, 640, 128, 37, "bfloat16", "float32", "auto"),      # 5 chunks: slices of 2 + 2 + 1, fp32 promotion
    (1024, 512, 32, 61, "float16", "float16", "auto"),        # b = 32: exactly 4 chunks
    (4096, 4096, 256, 20, "bfloat16", None, "auto"),          # VALU kernel, b = 256: 4 chunks, 4 slices
    (11008, 4096, 256, 37, "float32", "float32", "auto"),     # VALU b = 256: 11 chunks, 11 slices
    (4096, 4096, 256, 1500, "float32", None, "auto"),         # VALU b = 256: 94 rows, 2 slices of 2
    (11008, 4096, 128, 50, "float32", "bfloat16", "valu"),    # VALU b = 128: 22 chunks, 22 slices
]


def _split_inputs(k, m, b, n, xdt, bdt, dev):
    rng = np.random.default_rng(k + m + n)
    c = (rng.standard_normal((m // b, k // b, b)) * 0.01).astype(np.float32)
    bv = (rng.standard_normal(m) * 0.1).astype(np.float32) if bdt else None
    x = rng.standard_normal((n, k)).astype(np.float32)
    return c, bv, x


@pytest.mark.parametrize("k,m,b,n,xdt,bdt,algo", SPLIT_CASES)
def test_split_k_vs_oracle_and_unsplit(dev, k, m, b, n, xdt, bdt, algo):
    """The split path (workspace from ops.forward) vs the oracle, bit-reproducible run to run, and
    within fp32 summation-order noise of the unsplit launch (bcfft_forward_algo, no workspace)."""
    from bcfft import _lib, ops
    c, bv, x = _split_inputs(k, m, b, n, xdt, bdt, dev)
    lib = _lib.load()
    wsb = lib.bcfft_forward_workspace_bytes(n, k, m, b, _lib.ALGOS[algo])
    assert wsb > 0 and wsb % (n * m * 4) == 0 and wsb // (n * m * 4) >= 2
    spec = ops.spectra(torch.from_numpy(c).to(dev))
    xt = _to_dev(x, xdt, dev)
    bt = None if bdt is None else torch.from_numpy(bv).to(dev).to(getattr(torch, bdt))
    y1 = ops.forward(xt, spec, bt, b, m, algo=algo)
    y2 = ops.forward(xt, spec, bt, b, m, algo=algo)
    assert torch.equal(y1, y2)
    y0 = torch.empty_like(y1)
    _lib.check(lib.bcfft_forward_algo(xt.data_ptr(), _lib.dtype_code(xt.dtype), n, k, m, b, spec.data_ptr(),
                                      0 if bt is None else bt.data_ptr(),
                                      _lib.BCFFT_NONE if bt is None else _lib.dtype_code(bt.dtype),
                                      y0.data_ptr(), _lib.dtype_code(y0.dtype), _lib.ALGOS[algo],
                                      _lib.stream_handle(xt.device)), "unsplit")
    rel = ((y1.float() - y0.float()).norm() / y0.float().norm()).item()
    # 16-bit x: the epilogue rounds to x's dtype before the bias, so order noise can flip roundings
    assert rel < (1e-5 if xt.dtype == torch.float32 else 2e-3), rel
    b_eff = None if bdt is None else O.round_to(bv, ODT[bdt])
    ref = O.bc_forward(O.round_to(x, ODT[xdt]), c, b_eff, x_dtype=ODT[xdt], bias_dtype=ODT[bdt] if bdt else None)
    _check(y1, ref, str(y1.dtype).replace("torch.", ""))
