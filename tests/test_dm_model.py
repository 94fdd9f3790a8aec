"""CPU checks of the DFT-on-MFMA kernel's decomposition (tests/dm_model.py) against the oracle:
the table, the even/odd split, the packed-bin order, the scale bookkeeping and the fp16
roundings reproduce the reference forward (patch_llama_fft.py:226-275) within the kernel's
parity tolerance, before any GPU run."""
import numpy as np
import pytest

from dm_model import dm_forward, dm_table
from oracle import bc_oracle as orc


def test_table_matches_dft():
    F = dm_table() * 2.0 ** 7
    t = np.arange(64)
    assert np.allclose(F[:, 0], 1) and np.allclose(F[:, 1], (-1.0) ** t)
    assert np.allclose(F[:, 2 * 5], np.cos(2 * np.pi * 5 * t / 64), atol=1e-3)
    assert np.allclose(F[:, 64 + 2 * 5 + 1], -np.sin(2 * np.pi * 11 * t / 128), atol=1e-3)


@pytest.mark.parametrize("scale,exact", [(1.0, True), (1e-5, True), (3e4, True), (1.0, False), (1e-5, False), (3e4, False)])
def test_dm_model_vs_oracle(scale, exact):
    rng = np.random.default_rng(7)
    x = (rng.standard_normal((6, 4096)) * scale).astype(np.float32)
    x[1] *= 1e3                                    # token scales differ
    x[2, 100] = 500 * scale                        # one big channel in half 0
    c = (rng.standard_normal((32, 32, 128)) * 0.01).astype(np.float32)
    ref = orc.bc_forward(x, c)
    got = dm_forward(x, c, exact)
    rel = np.linalg.norm(got - ref) / np.linalg.norm(ref)
    assert rel < (3.2e-4 if exact else 4.8e-4), rel
    for t in range(x.shape[0]):                   # per token as well
        r = np.linalg.norm(got[t] - ref[t]) / np.linalg.norm(ref[t])
        assert r < 6e-4, (t, r)


def test_dm8_model_single_x_vs_oracle():
    """The bf16-I/O kernel's arithmetic (X one fp16 term as well) before the bf16 output rounding:
    well under bf16's own 2^-9."""
    rng = np.random.default_rng(8)
    x = rng.standard_normal((4, 4096)).astype(np.float32)
    c = (rng.standard_normal((32, 32, 128)) * 0.01).astype(np.float32)
    ref = orc.bc_forward(x, c)
    got = dm_forward(x, c, exact=False, single_x=True)
    rel = np.linalg.norm(got - ref) / np.linalg.norm(ref)
    assert rel < 6e-4, rel


def test_dmk_mirror_vs_oracle():
    """The streamed-weight kernel's numerics (bcfft_dmk.hip): 16-block chunks with their own
    scales, a partial last chunk, 2^4 alignment headroom and the running reference, checked on
    the CPU against the oracle. Tokens with one chunk 3e3 louder after (and before) the others
    exercise the reference drop; the output of a bf16 kernel is then within its rounding."""
    from golden_io import rel_err
    rng = np.random.default_rng(21)
    c = (rng.standard_normal((4, 40, 128)) * 0.01).astype(np.float32)   # nI = 40: chunks 16+16+8
    x = rng.standard_normal((5, 40 * 128)).astype(np.float32)
    x[1, 4200:4300] *= 3e3             # last chunk far louder: the reference drops
    x[2, :2048] *= 3e3                 # first chunk far louder
    x[3, 2048:4096] *= 10.0            # within the 2^4 headroom: no drop
    x[4] *= 1e-6
    ref = orc.bc_forward(x, c)
    mdl = dm_forward(x, c, head=4)
    for t in range(x.shape[0]):
        assert rel_err(mdl[t], ref[t]) < 6e-4, (t, rel_err(mdl[t], ref[t]))   # measured 4.3-5.0e-4
