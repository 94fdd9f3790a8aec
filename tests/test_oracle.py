"""Pin the CPU oracle (oracle/bc_oracle.py) against the reference's golden vectors and
against the reference's own known-answer tests (validate_implementation.py T1-T5)."""
import numpy as np
import pytest

from golden_io import load, names, rel_err
from oracle import bc_oracle as O

DT = {"float32": O.F32, "float16": O.F16, "bfloat16": O.BF16}


@pytest.mark.parametrize("name", names("fwd_"))
def test_forward_matches_reference_golden(name):
    g = load(name)
    xdt = DT[g["x__dt"]]
    bdt = DT[g["bias__dt"]] if "bias" in g else None
    y = O.bc_forward(g["x"], g["c"], g.get("bias"), x_dtype=xdt, bias_dtype=bdt)
    assert y.shape == g["y"].shape
    # the oracle uses pocketfft (numpy) in fp32/complex64 like torch CPU; differences are
    # rounding-order only, well inside the 1e-3 product tolerance
    assert rel_err(y, g["y"]) < 2e-5 if g["y__dt"] == "float32" else rel_err(y, g["y"]) < 1e-2
    if "cf_re" in g:
        cf = O.spectra(g["c"])
        assert rel_err(cf.real, g["cf_re"]) < 1e-6 and rel_err(cf.imag, g["cf_im"]) < 1e-6


@pytest.mark.parametrize("name", names("fwd_"))
def test_forward_equals_explicit_dense(name):
    """Closed form: y = x W^T with W the explicit block-circulant matrix (validate T5)."""
    g = load(name)
    x = g["x"].reshape(-1, g["x"].shape[-1]).astype(np.float64)
    w = O.bc_dense_weight(g["c"].astype(np.float64))
    y = x @ w.T
    if "bias" in g:
        y = y + g["bias"]
    tol = 1e-5 if g["x__dt"] == "float32" else 1e-2   # y rounded to x.dtype first (:266)
    assert rel_err(g["y"].reshape(y.shape), y) < tol


@pytest.mark.parametrize("name", names("cmv_"))
def test_circulant_matvec_golden(name):
    g = load(name)
    d = DT[g["x__dt"]]
    y = O.circulant_matvec_fft(g["c"], g["x"], d)
    assert rel_err(y, g["y"]) < (1e-5 if d == O.F32 else 1e-2)


def test_t1_fft_convention():
    """validate_implementation.py:20-44 — FFT matvec == C[i,j] = c[(i-j) % B], B=64."""
    rng = np.random.default_rng(42)
    c = rng.standard_normal(64).astype(np.float32)
    x = rng.standard_normal(64).astype(np.float32)
    idx = np.arange(64)
    cm = c[(idx[:, None] - idx[None, :]) % 64]
    assert rel_err(O.circulant_matvec_fft(c, x), cm @ x) < 1e-5


@pytest.mark.parametrize("name", names("from_linear_"))
def test_from_linear_golden(name):
    g = load(name)
    d = DT[g["w__dt"]]
    c = O.from_linear_c(g["w"], int(g["block_size"]), d)
    tol = 1e-5 if d == O.F32 else 2e-3
    assert rel_err(c, g["c"]) < tol
    assert np.max(np.abs(c - g["c"])) < (1e-5 if d == O.F32 else 1e-3)


@pytest.mark.parametrize("name", names("from_linear_"))
def test_from_linear_16bit_bit_exact(name):
    """16-bit weights: the oracle reproduces the reference's CPU loop bit for bit."""
    g = load(name)
    if g["w__dt"] == "float32":
        pytest.skip("fp32 reductions differ in summation order (checked to 1e-5 above)")
    c = O.from_linear_c(g["w"], int(g["block_size"]), DT[g["w__dt"]])
    assert np.array_equal(c, g["c"])


@pytest.mark.parametrize("name", names("bwd_"))
def test_backward_golden(name):
    """bc_grad_c / bc_grad_x against torch autograd through the reference forward
    (tests/golden/make_golden_grad.py)."""
    g = load(name)
    b = int(g["block_size"])
    x = g["x"].reshape(-1, g["x"].shape[-1])
    dy = g["dy"].reshape(x.shape[0], -1)
    # bias added after y.to(x.dtype) (patch_llama_fft.py:266-271): the x side gets dy rounded
    # to x's dtype when the output was promoted past it
    dy_x = dy
    if "bias" in g and g["x__dt"] != "float32" and g.get("dy__dt", "float32") == "float32":
        dy_x = O.round_to(dy, DT[g["x__dt"]])
    dc = O.round_to(O.bc_grad_c(x, dy_x, b), DT[g["dc__dt"]])
    dx = O.bc_grad_x(dy_x, g["c"], DT[g["x__dt"]])
    if g["dc__dt"] == "float32":
        assert rel_err(dc, g["dc"]) < 1e-6
    else:
        assert np.array_equal(dc, g["dc"])
    tol = 1e-6 if g["x__dt"] == "float32" else 2e-3
    assert rel_err(dx, g["dx"].reshape(dx.shape)) < tol
    if "dbias" in g:
        assert rel_err(O.round_to(dy.sum(0), DT[g["dbias__dt"]]), g["dbias"]) < 1e-6


def test_project_t2_exact():
    """validate_implementation.py:47-78 — projection of a true circulant recovers c up to alpha."""
    g = load("project_t2_exact")
    c = O.project_loss_aware(g["w"])
    assert np.allclose(c, g["c"], rtol=1e-6, atol=1e-6)
    ratio = c / np.arange(1, 9)
    assert ratio.std() < 1e-5
