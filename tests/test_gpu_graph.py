"""HIP-graph replay of the BC forward (bcfft.graph.GraphedCall): bit-identical to the eager
launches, new inputs copied into the static buffers, several forwards per graph."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    import bcfft
    bcfft.load()
    return torch.device("cuda:0")


@pytest.mark.parametrize("k,m,b,io,n", [(4096, 4096, 64, torch.float32, 128),    # BASELINE config 1
                                         (4096, 4096, 128, torch.bfloat16, 64),
                                         (11008, 4096, 128, torch.bfloat16, 16)])
def test_graph_replay_matches_eager(dev, k, m, b, io, n):
    from bcfft import ops
    from bcfft.graph import GraphedCall
    torch.manual_seed(0)
    c = torch.randn(m // b, k // b, b, device=dev) * 0.01
    spec = ops.spectra(c)
    x = torch.randn(n, k, device=dev).to(io)
    fwd = lambda t: ops.forward(t, spec, None, b, m)  # noqa: E731
    y_eager = fwd(x)
    g = GraphedCall(fwd, [x], repeat=3)
    y_graph = g(x).clone()
    torch.cuda.synchronize()
    assert torch.equal(y_graph, y_eager)
    x2 = torch.randn(n, k, device=dev).to(io)       # a new input is copied in
    y2 = g(x2).clone()
    assert torch.equal(y2, fwd(x2))
    with pytest.raises(ValueError):
        g(torch.randn(n + 1, k, device=dev).to(io))


def test_torch_library_ops_match_bcfft_ops(dev):
    """torch.ops.bcfft.* run the same kernels as bcfft.ops (bit-identical), and torch.library's
    opcheck accepts the registrations (schema, fake kernel vs the real one)."""
    import bcfft.torch_ops  # noqa: F401
    from bcfft import ops
    torch.manual_seed(1)
    c = torch.randn(32, 32, 128, device=dev) * 0.01
    x = torch.randn(64, 4096, device=dev).to(torch.bfloat16)
    spec = torch.ops.bcfft.spectra(c, False)
    assert torch.equal(spec, ops.spectra(c))
    y = torch.ops.bcfft.forward(x, spec, None, 128, 4096, "auto")
    assert torch.equal(y, ops.forward(x, spec, None, 128, 4096, algo="auto"))
    torch.library.opcheck(torch.ops.bcfft.forward.default, (x, spec, None, 128, 4096, "auto"),
                          test_utils=("test_schema", "test_faketensor"))
