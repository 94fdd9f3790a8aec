"""torch.library registration (bcfft.torch_ops) on the CPU: the fake kernels give the real ops'
output shapes / dtypes under FakeTensorMode (no device, no launch), and the real kernels refuse
host tensors loudly."""
import pytest
import torch
from torch._subclasses.fake_tensor import FakeTensorMode


def test_ops_registered():
    from bcfft import torch_ops
    assert torch_ops.registered()


@pytest.mark.parametrize("k,m,b,xdt,bdt", [(4096, 4096, 128, torch.float32, None),
                                            (4096, 11008, 128, torch.bfloat16, torch.bfloat16),
                                            (11008, 4096, 64, torch.bfloat16, torch.float32),
                                            (4096, 4096, 256, torch.float16, None)])
def test_forward_fake_shapes(k, m, b, xdt, bdt):
    import bcfft.torch_ops  # noqa: F401
    from bcfft import ops
    with FakeTensorMode():
        x = torch.empty(37, k, dtype=xdt)
        c = torch.empty(m // b, k // b, b, dtype=torch.float32)
        spec = torch.ops.bcfft.spectra(c, False)
        assert spec.shape == (ops.spectra_numel(m // b, k // b, b),) and spec.dtype == torch.float32
        bias = torch.empty(m, dtype=bdt) if bdt is not None else None
        y = torch.ops.bcfft.forward(x, spec, bias, b, m, "auto")
        assert y.shape == (37, m)
        assert y.dtype == (xdt if bdt is None else torch.promote_types(xdt, bdt))
        adj = torch.ops.bcfft.spectra(c, True)
        assert adj.shape == (ops.spectra_numel(k // b, m // b, b),)


def test_forward_fake_rejects_bad_geometry():
    import bcfft.torch_ops  # noqa: F401
    with FakeTensorMode():
        x = torch.empty(4, 1000)
        with pytest.raises(ValueError):
            torch.ops.bcfft.forward(x, torch.empty(10), None, 128, 4096, "auto")


def test_real_op_refuses_host_tensors():
    import bcfft.torch_ops  # noqa: F401
    with pytest.raises(RuntimeError, match="ROCm device"):
        torch.ops.bcfft.forward(torch.zeros(2, 128), torch.zeros(10), None, 64, 128, "auto")


def test_glu_and_mlp_fake_shapes():
    import bcfft.torch_ops  # noqa: F401
    from bcfft import ops
    b, h, f = 128, 4096, 11008
    with FakeTensorMode():
        x = torch.empty(21, h, dtype=torch.bfloat16)
        sgu = torch.empty(ops.spectra_numel(32 * 6, h // b, b), dtype=torch.float32)
        sd = torch.empty(ops.spectra_numel(h // b, f // b, b), dtype=torch.float32)
        hh = torch.ops.bcfft.forward_glu(x, sgu, b, f, "auto")
        assert hh.shape == (21, f) and hh.dtype == torch.bfloat16
        y = torch.ops.bcfft.forward_mlp(x, sgu, sd, b, f, "auto")
        assert y.shape == (21, h) and y.dtype == torch.bfloat16
        with pytest.raises(ValueError):
            torch.ops.bcfft.forward_mlp(torch.empty(3, 1000), sgu, sd, b, f, "auto")


def test_real_mlp_op_refuses_host_tensors():
    import bcfft.torch_ops  # noqa: F401
    with pytest.raises(RuntimeError, match="ROCm device"):
        torch.ops.bcfft.forward_mlp(torch.zeros(2, 4096), torch.zeros(10), torch.zeros(10), 128, 11008, "auto")
