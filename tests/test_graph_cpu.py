"""bcfft.graph on the CPU: it refuses loudly without a ROCm device (no silent eager fallback)."""
import pytest
import torch


def test_graph_requires_device():
    from bcfft.graph import GraphedCall
    if torch.cuda.is_available():
        pytest.skip("a device is present")
    with pytest.raises(RuntimeError, match="ROCm device"):
        GraphedCall(lambda t: t, [torch.zeros(2)])
