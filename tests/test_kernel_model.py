"""The numpy mirror of the kernel dataflow (tests/kernel_model.py) equals the oracle."""
import numpy as np
import pytest

from golden_io import rel_err
import kernel_model as KM
from oracle import bc_oracle as O


@pytest.mark.parametrize("b", [32, 64, 128, 256])
@pytest.mark.parametrize("k,m", [(256, 512), (512, 256)])
def test_model_matches_oracle(b, k, m):
    rng = np.random.default_rng(b + k)
    c = (rng.standard_normal((m // b, k // b, b)) * 0.01).astype(np.float32)
    x = rng.standard_normal((5, k)).astype(np.float32)
    bias = (rng.standard_normal(m) * 0.1).astype(np.float32)
    ref = O.bc_forward(x, c, bias)
    got = KM.bc_forward_model(x, c, bias)
    assert rel_err(got, ref) < 1e-5


@pytest.mark.parametrize("b", [32, 64, 128, 256])
def test_four_step_is_dft(b):
    rng = np.random.default_rng(b)
    h, lanes, _ = KM.fft_lane_split(b)
    z = rng.standard_normal((3, h)) + 1j * rng.standard_normal((3, h))
    assert rel_err(KM.four_step(z, lanes, -1), np.fft.fft(z, axis=-1)) < 1e-12
    assert rel_err(KM.four_step(z, lanes, +1), np.fft.ifft(z, axis=-1) * h) < 1e-12
