"""CPU checks of the DFT-on-MFMA kernel's decomposition (tests/dm_model.py) against the oracle:
the table, the even/odd split, the packed-bin order, the scale bookkeeping and the fp16
roundings reproduce the reference forward (patch_llama_fft.py:226-275) within the kernel's
parity tolerance, before any GPU run."""
import numpy as np
import pytest

import dm_model as DM
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


def test_precise_tables_are_the_residual_split():
    """kDmFp (F 2^8 in fp16) is the dftx table times 2^15 bit for bit, and kDmFl8 is the e4m3 rounding
    of its residual: together within e4m3's 2^-4 relative step of the residual (and of 2^-10 absolute
    for the subnormal codes) of the exact DFT."""
    from dm_model import dm_table_precise
    fp, fl = dm_table_precise()
    assert np.array_equal(fp, dm_table() * 2.0 ** 15)
    t = np.arange(64)[:, None]
    j = np.arange(32)[None, :]
    F = np.zeros((64, 128))
    F[:, 0], F[:, 1] = 1.0, (-1.0) ** np.arange(64)
    F[:, 2:64:2] = np.cos(2 * np.pi * (2 * j[:, 1:]) * t / 128)
    F[:, 3:64:2] = -np.sin(2 * np.pi * (2 * j[:, 1:]) * t / 128)
    F[:, 64::2] = np.cos(2 * np.pi * (2 * j + 1) * t / 128)
    F[:, 65::2] = -np.sin(2 * np.pi * (2 * j + 1) * t / 128)
    res = F * 2.0 ** 8 - fp
    assert np.abs(res).max() <= 2.0 ** -4
    assert np.all(np.abs(fl - res) <= 2.0 ** -4 * np.abs(res) + 2.0 ** -10)


@pytest.mark.parametrize("scale", [1.0, 1e-5, 3e4])
def test_precise_model_vs_oracle(scale):
    """The precise engine's arithmetic (BCFFT_ALGO_DFTP): an order of magnitude under dftx's, per
    token as well; each residual term removes its share (dftx ~2.8e-4 -> ~2.8e-5)."""
    rng = np.random.default_rng(9)
    x = (rng.standard_normal((6, 4096)) * scale).astype(np.float32)
    x[1] *= 1e3
    x[2, 100] = 500 * scale
    c = (rng.standard_normal((32, 32, 128)) * 0.01).astype(np.float32)
    ref = orc.bc_forward(x, c)
    got = dm_forward(x, c, precise=True)
    rel = np.linalg.norm(got - ref) / np.linalg.norm(ref)
    assert rel < 5e-5, rel
    for t in range(x.shape[0]):
        r = np.linalg.norm(got[t] - ref[t]) / np.linalg.norm(ref[t])
        assert r < 8e-5, (t, r)
    partial = dm_forward(x, c, precise=True, terms=(1, 0, 1))   # no weight residual: dftx-like
    assert np.linalg.norm(partial - ref) / np.linalg.norm(ref) > 3 * rel


def _table_words(name, count):
    text = open(DM._TABLE).read()
    body = text[text.index(f"{name}[{count}]"):]
    body = body[:body.index("};")]
    return np.array([int(w, 16) for w in __import__("re").findall(r"0x([0-9a-f]{8})u", body)], dtype=np.uint32)


def _bf16(bits):
    return (bits.astype(np.uint32) << 16).view(np.float32).astype(np.float64)


def test_dm64k_bf16_fragments_are_the_dft():
    """kDmB64 (bcfft_dm64k.hip's stage-1 A fragments, [pr][mt][term][lane][8] bf16): hi + lo of the
    b = 64 even / odd DFT columns times 2^-7 to ~2^-17, hi the RNE bf16 of each entry, and the
    fragment layout A[m = lane & 15][k = 8 (lane >> 4) + e] = column 32 pr + 16 mt + m, row t = k."""
    w = _table_words("kDmB64", 2048).reshape(2, 2, 2, 64, 4)
    el = np.empty((2, 2, 2, 64, 8))
    el[..., 0::2] = _bf16(w & 0xFFFF)
    el[..., 1::2] = _bf16(w >> 16)
    t = np.arange(32)
    F = np.zeros((32, 64))
    F[:, 0], F[:, 1] = 1.0, (-1.0) ** t
    for j in range(1, 16):
        F[:, 2 * j], F[:, 2 * j + 1] = np.cos(2 * np.pi * j * t / 32), -np.sin(2 * np.pi * j * t / 32)
    for j in range(16):
        th = 2 * np.pi * (2 * j + 1) * t / 64
        F[:, 32 + 2 * j], F[:, 32 + 2 * j + 1] = np.cos(th), -np.sin(th)
    ref = F * 2.0 ** -7
    for pr in range(2):
        for mt in range(2):
            for ln in range(64):
                col, ts = 32 * pr + 16 * mt + (ln & 15), 8 * (ln >> 4) + np.arange(8)
                hi, lo = el[pr, mt, 0, ln], el[pr, mt, 1, ln]
                np.testing.assert_allclose(hi + lo, ref[ts, col], rtol=0, atol=2.0 ** -24)
                # hi is bf16(v): |v - hi| within half a bf16 ulp of v (8 significant bits)
                assert np.all(np.abs(ref[ts, col] - hi) <= 2.0 ** -8 * np.abs(ref[ts, col]) + 1e-30)


def test_dm64k_direct_stage1_model():
    """The direct stage 1 of bcfft_dm64k.hip in numpy: X = (F_hi + F_lo) x over all 64 points
    (x_{t+32} negated for the odd bins), then X 2^sx rounded once to fp16, equals the exact
    64-point rfft of the bf16 x to the fp16 rounding of X (the even / odd fp16 form it replaces
    also rounds a, d and the table: its error is larger)."""
    rng = np.random.default_rng(3)
    w = _table_words("kDmB64", 2048).reshape(2, 2, 2, 64, 4)
    el = np.empty((2, 2, 2, 64, 8))
    el[..., 0::2] = _bf16(w & 0xFFFF)
    el[..., 1::2] = _bf16(w >> 16)
    A = np.zeros((64, 32))                            # [column][t]: hi + lo
    for pr in range(2):
        for mt in range(2):
            for ln in range(64):
                A[32 * pr + 16 * mt + (ln & 15), 8 * (ln >> 4) + np.arange(8)] = el[pr, mt, 0, ln] + el[pr, mt, 1, ln]
    x = rng.standard_normal((16, 64)).astype(np.float32)
    xb = _bf16(x.view(np.uint32) >> 16)               # bf16 truncation: any bf16 input
    Xs = np.zeros((16, 64))
    Xs[:, :32] = (xb[:, :32] + xb[:, 32:]) @ A[:32].T     # even columns: x_{t+32} as is
    Xs[:, 32:] = (xb[:, :32] - xb[:, 32:]) @ A[32:].T     # odd columns: x_{t+32} negated
    Xs *= 2.0 ** 7
    full = np.fft.rfft(xb, axis=1)                   # bins 0..32
    ref = np.zeros((16, 64))
    ref[:, 0], ref[:, 1] = full[:, 0].real, full[:, 32].real
    for j in range(1, 16):
        ref[:, 2 * j], ref[:, 2 * j + 1] = full[:, 2 * j].real, full[:, 2 * j].imag
    for j in range(16):
        ref[:, 32 + 2 * j], ref[:, 32 + 2 * j + 1] = full[:, 2 * j + 1].real, full[:, 2 * j + 1].imag
    err = np.abs(Xs - ref).max() / np.abs(ref).max()
    assert err < 2.0 ** -15, err
