"""GPU parity of the weight-prep kernel (bcfft_project_circulant) and the dc
backward kernel (bcfft_grad_c, §8 f3), both called through the C ABI (bcfft.ops).

* Projection: bit-exact with the oracle (and so with the reference's golden vectors) for 16-bit
  weights; fp32 within 1e-6 (summation order).
* dc: the oracle (fp64) within 1e-5 relative Frobenius for fp32 (fp32 FFTs and accumulation
  over N tokens); the reference's autograd golden vectors through the module's backward; at
  the north-star size (N = 8192) against torch's fp32 FFT expression of the same gradient on
  the device, and through linearity in dy.
"""
import numpy as np
import pytest
import torch

from golden_io import load, names, rel_err
from oracle import bc_oracle as O

pytestmark = pytest.mark.gpu

TDT = {"float32": torch.float32, "float16": torch.float16, "bfloat16": torch.bfloat16}
ODT = {"float32": O.F32, "float16": O.F16, "bfloat16": O.BF16}


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    import bcfft
    bcfft.load()
    return torch.device("cuda:0")


# ----------------------------------------------------------------------------- f1 projection
@pytest.mark.parametrize("name", names("from_linear_"))
def test_project_vs_reference_golden(dev, name):
    from bcfft import ops
    g = load(name)
    w = torch.from_numpy(g["w"]).to(dev).to(TDT[g["w__dt"]])
    c = ops.project_circulant(w, int(g["block_size"])).cpu().numpy()
    if g["w__dt"] == "float32":
        assert rel_err(c, g["c"]) < 1e-6
    else:
        assert np.array_equal(c, g["c"])


@pytest.mark.parametrize("m,k,b,dt", [(1024, 2048, 128, "float16"), (512, 768, 256, "bfloat16"),
                                      (384, 256, 64, "float16"), (96, 64, 32, "bfloat16"),
                                      (512, 1024, 64, "float32")])
def test_project_vs_oracle(dev, m, k, b, dt):
    from bcfft import ops
    rng = np.random.default_rng(m + k + b)
    w = O.round_to((rng.standard_normal((m, k)) * 0.02).astype(np.float32), ODT[dt])
    c = ops.project_circulant(torch.from_numpy(w).to(dev).to(TDT[dt]), b).cpu().numpy()
    ref = O.from_linear_c(w, b, ODT[dt])
    if dt == "float32":
        assert rel_err(c, ref) < 1e-6
    else:
        assert np.array_equal(c, ref)


def test_project_zero_block_and_errors(dev):
    """An all-zero fp32 block: alpha = 0 / eps = 0 (the reference's clamp_min, :125)."""
    from bcfft import ops
    w = torch.zeros(128, 256, device=dev)
    w[:, 128:] = torch.randn(128, 128, device=dev)
    c = ops.project_circulant(w, 128)
    assert torch.all(c[0, 0] == 0) and torch.isfinite(c).all()
    with pytest.raises(RuntimeError, match="block_size"):
        ops.project_circulant(torch.zeros(96, 96, device=dev), 48)


def test_from_linear_on_device_uses_kernel(dev):
    import patch_llama_fft as P
    torch.manual_seed(5)
    lin = torch.nn.Linear(1024, 512, bias=True).half().to(dev)
    bc = P.BlockCirculantLinear.from_linear(lin, block_size=128)
    assert bc.c.device.type == "cuda" and bc.c.dtype == torch.float32
    ref = O.from_linear_c(lin.weight.detach().float().cpu().numpy(), 128, O.F16)
    assert np.array_equal(bc.c.detach().cpu().numpy(), ref)
    assert torch.equal(bc.bias, lin.bias)


# ----------------------------------------------------------------------------- f3 dc
@pytest.mark.parametrize("n,k,m,b,xdt", [
    (37, 512, 768, 128, "float32"),      # ragged tokens; 6 x 4 blocks (partial tiles)
    (1, 4096, 4096, 128, "float32"),     # one token
    (300, 1024, 512, 64, "bfloat16"),
    (64, 256, 1024, 32, "float16"),
    (45, 1024, 2048, 256, "float32"),
    (513, 384, 640, 128, "bfloat16"),    # 3 x 5 blocks
])
def test_grad_c_vs_oracle(dev, n, k, m, b, xdt):
    from bcfft import ops
    rng = np.random.default_rng(n + k + m + b)
    x = O.round_to(rng.standard_normal((n, k)).astype(np.float32), ODT[xdt])
    dy = O.round_to(rng.standard_normal((n, m)).astype(np.float32), ODT[xdt])
    dc = ops.grad_c(torch.from_numpy(x).to(dev).to(TDT[xdt]), torch.from_numpy(dy).to(dev).to(TDT[xdt]), b)
    torch.cuda.synchronize()
    assert dc.shape == (m // b, k // b, b) and dc.dtype == torch.float32
    assert rel_err(dc.cpu().numpy(), O.bc_grad_c(x, dy, b)) < 1e-5


def test_grad_c_zero_tokens_and_dtype(dev):
    from bcfft import ops
    x = torch.zeros(0, 512, device=dev)
    dy = torch.zeros(0, 256, device=dev)
    dc = ops.grad_c(x, dy, 128)
    assert dc.shape == (2, 4, 128) and torch.all(dc == 0)
    x = torch.randn(20, 512, device=dev)
    dy = torch.randn(20, 256, device=dev)
    d16 = ops.grad_c(x, dy, 128, torch.bfloat16)
    d32 = ops.grad_c(x, dy, 128)
    assert d16.dtype == torch.bfloat16 and torch.equal(d16, d32.to(torch.bfloat16))


def test_grad_c_deterministic(dev):
    from bcfft import ops
    x = torch.randn(4096, 4096, device=dev)
    dy = torch.randn(4096, 4096, device=dev)
    assert torch.equal(ops.grad_c(x, dy, 128), ops.grad_c(x, dy, 128))


def _torch_grad_c(x, dy, b):
    n = x.shape[0]
    xf = torch.fft.rfft(x.float().reshape(n, -1, b), dim=-1)
    df = torch.fft.rfft(dy.float().reshape(n, -1, b), dim=-1)
    return torch.fft.irfft(torch.einsum("nof,nif->oif", df, xf.conj()), n=b, dim=-1)


@pytest.mark.parametrize("b", [64, 128])
def test_grad_c_full_size(dev, b):
    """North-star size: N = 8192, 4096 -> 4096, against torch's fp32 FFT expression, plus
    linearity in dy (dc(dy1 + dy2) = dc(dy1) + dc(dy2))."""
    from bcfft import ops
    torch.manual_seed(b)
    x = torch.randn(8192, 4096, device=dev)
    d1 = torch.randn(8192, 4096, device=dev)
    d2 = torch.randn(8192, 4096, device=dev)
    g1 = ops.grad_c(x, d1, b)
    ref = _torch_grad_c(x, d1, b)
    assert ((g1 - ref).norm() / ref.norm()).item() < 1e-5
    g12 = ops.grad_c(x, d1 + d2, b)
    g2 = ops.grad_c(x, d2, b)
    assert ((g12 - g1 - g2).norm() / g12.norm()).item() < 1e-5


@pytest.mark.parametrize("name", names("bwd_"))
def test_module_backward_vs_reference_golden(dev, name):
    """dx, dc, dbias of the module (HIP forward on adjoint spectra, bcfft_grad_c, reduction)
    against torch autograd through the reference's forward."""
    import patch_llama_fft as P
    g = load(name)
    b = int(g["block_size"])
    xs = g["x"]
    k = xs.shape[-1]
    n_out, n_in, _ = g["c"].shape
    mdt, xdt = TDT[g["c__dt"]], TDT[g["x__dt"]]
    mod = P.BlockCirculantLinear(k, n_out * b, block_size=b, bias="bias" in g).to(mdt).to(dev)
    with torch.no_grad():
        mod.c.copy_(torch.from_numpy(g["c"]))
        if "bias" in g:
            mod.bias.copy_(torch.from_numpy(g["bias"]))
    x = torch.from_numpy(xs).to(dev).to(xdt).requires_grad_(True)
    y = mod(x)
    dy = torch.from_numpy(g["dy"]).to(dev).to(y.dtype)
    params = [x, mod.c] + ([mod.bias] if "bias" in g else [])
    grads = torch.autograd.grad(y, params, dy)
    dx, dc = grads[0].float().cpu().numpy(), grads[1].float().cpu().numpy()
    assert grads[1].dtype == mdt and grads[0].dtype == xdt
    # dx runs through the forward engine (stationary fp16 weights where eligible, ~3e-4)
    assert rel_err(dx, g["dx"]) < (1e-3 if g["x__dt"] == "float32" else 4e-3)
    assert rel_err(dc, g["dc"]) < (1e-5 if g["c__dt"] == "float32" else 4e-3)
    if "dbias" in g:
        assert rel_err(grads[2].float().cpu().numpy(), g["dbias"]) < 1e-5
