"""The C++ operator path (torch.ops.bcfft_native) against the ctypes path on the GPU: the same
kernels, so bit-identical outputs, and the host cost per call of each (printed)."""
import time

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    import bcfft
    bcfft.load()
    return torch.device("cuda:0")


def _ctypes_path(monkeypatch):
    from bcfft import _lib
    monkeypatch.setattr(_lib, "_native", False)


def test_native_forward_bit_identical(dev, monkeypatch):
    from bcfft import _lib, ops
    assert _lib.native_op(), "libbcfft_torch.so not loaded"
    g = torch.Generator(device="cpu").manual_seed(0)
    for (k, m, b, n, dt, bias) in ((4096, 4096, 128, 37, torch.float32, True), (4096, 11008, 128, 300, torch.bfloat16, False),
                                   (2048, 5632, 64, 9, torch.float16, True), (4096, 4096, 128, 0, torch.float32, False)):
        c = (torch.randn(m // b, k // b, b, generator=g) * 0.01).to(dev)
        x = torch.randn(n, k, generator=g).to(dev).to(dt)
        bv = (torch.randn(m, generator=g) * 0.1).to(dev).to(dt) if bias else None
        spec = ops.spectra(c)
        y = ops.forward(x, spec, bv, b, m)
        with monkeypatch.context() as mp:
            _ctypes_path(mp)
            yc = ops.forward(x, spec, bv, b, m)
        assert y.dtype == yc.dtype and torch.equal(y, yc), (k, m, b, n)
    with pytest.raises(ValueError, match="spectra"):            # as the Python path
        ops.forward(torch.zeros(3, 4096, device=dev), spec, None, 64, 4096)


def test_native_glu_bit_identical(dev, monkeypatch):
    from bcfft import ops
    g = torch.Generator(device="cpu").manual_seed(1)
    cg, cu = ((torch.randn(86, 32, 128, generator=g) * 0.01).to(dev) for _ in range(2))
    x = torch.randn(45, 4096, generator=g).to(dev).to(torch.bfloat16)
    spec = ops.spectra(ops.glu_weights(cg, cu))
    h = ops.forward_glu(x, spec, 128, 11008)
    with monkeypatch.context() as mp:
        _ctypes_path(mp)
        hc = ops.forward_glu(x, spec, 128, 11008)
    assert torch.equal(h, hc)


def test_native_host_cost(dev, monkeypatch):
    """Host issue cost per call, native vs ctypes (N=4, GPU time negligible): printed, and the
    native op not slower."""
    from bcfft import ops
    from patch_llama_fft import BlockCirculantLinear
    layer = BlockCirculantLinear(4096, 4096, block_size=128, bias=False).to(dev).eval()
    x = torch.randn(4, 4096, device=dev)
    spec = layer._spectra(layer.c)

    def per_call(fn, iters=3000):
        for _ in range(100):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        return (t1 - t0) / iters * 1e6

    with torch.inference_mode():
        nat = per_call(lambda: ops.forward(x, spec, None, 128, 4096))
        mod = per_call(lambda: layer(x))
        with monkeypatch.context() as mp:
            _ctypes_path(mp)
            cty = per_call(lambda: ops.forward(x, spec, None, 128, 4096))
            modc = per_call(lambda: layer(x))
    print(f"host us/call: ops.forward native {nat:.1f} vs ctypes {cty:.1f}; module native {mod:.1f} vs ctypes {modc:.1f}")
    assert nat < cty * 1.1


@pytest.mark.parametrize("native", [True, False])
def test_operands_on_other_device_or_strided(dev, monkeypatch, native):
    """A spectra buffer or bias on the host (or a strided spectra view) is refused before any
    launch, with the same ValueError on the C++ and the ctypes path: the kernels read them by raw
    device pointer."""
    from bcfft import ops
    g = torch.Generator(device="cpu").manual_seed(2)
    c = (torch.randn(32, 32, 128, generator=g) * 0.01).to(dev)
    spec = ops.spectra(c)
    x = torch.randn(5, 4096, generator=g).to(dev)
    with monkeypatch.context() as mp:
        if not native:
            _ctypes_path(mp)
        with pytest.raises(ValueError, match="spectra is on cpu"):
            ops.forward(x, spec.cpu(), None, 128, 4096)
        with pytest.raises(ValueError, match="bias is on cpu"):
            ops.forward(x, spec, torch.zeros(4096), 128, 4096)
        wide = torch.zeros(2 * spec.numel(), device=dev)
        wide[::2] = spec
        with pytest.raises(ValueError, match="contiguous"):
            ops.forward(x, wide[::2], None, 128, 4096)
        sgu = ops.spectra(ops.glu_weights(c, c))
        with pytest.raises(ValueError, match="spectra is on cpu"):
            ops.forward_glu(x, sgu.cpu(), 128, 4096)
        assert torch.equal(ops.forward(x, spec, None, 128, 4096), ops.forward(x, spec, None, 128, 4096))


@pytest.mark.parametrize("native", [True, False])
def test_backward_create_graph_same_on_both_paths(dev, monkeypatch, native):
    """backward(create_graph=True) through BlockCirculantLinear: first-order gradients equal to the
    plain backward on the C++ operator path and the ctypes path alike (the custom Function's
    backward is once_differentiable: its kernels run under no_grad), and differentiating them again
    raises the same RuntimeError on both."""
    from patch_llama_fft import BlockCirculantLinear
    torch.manual_seed(3)
    layer = BlockCirculantLinear(256, 128, block_size=64, bias=True).to(dev)
    x = torch.randn(6, 256, device=dev, requires_grad=True)
    with monkeypatch.context() as mp:
        if not native:
            _ctypes_path(mp)
        gx, gc = torch.autograd.grad(layer(x).square().sum(), (x, layer.c))
        gx2, gc2 = torch.autograd.grad(layer(x).square().sum(), (x, layer.c), create_graph=True)
        assert torch.equal(gx, gx2.detach()) and torch.equal(gc, gc2.detach())
        with pytest.raises(RuntimeError, match="once_differentiable|differentiate"):
            torch.autograd.grad(gx2.sum(), x)
