"""Numpy mirror of the b = 256 DFT-on-MFMA kernel's transform algebra (bcfft_dm256.hip) — test
infrastructure. A 256-point real block is transformed with the 128-point fp16 table of the b = 128
kernels (csrc/bcfft_dm_table.h, 2^-7 scaled) applied to three 128-point "virtual rows":

  forward   a_t = x_t + x_{t+128}, d_t = x_t - x_{t+128}, psi_t = 2 pi t / 256 (t < 128);
            p_t = d_t cos psi_t, q_t = -d_t sin psi_t;
            X_{2j} = A_j (A = the packed 128-point spectrum of a: bin 0 = (X_0, X_128)),
            X_{2j+1} = P_j + i Q_j (P_0, Q_0 from the re slot of packed bin 0), j < 64.
  inverse   per output block, three 128-point inverses of the stage-3 kernel INV (the b = 128
            stage 3 fed with b = 256 spectra, so INV(p) = irfft_128(p) / 2):
            E = the even bins (packed bin 0 (Y_0, Y_128) / 2, as the b = 128 MAC makes it),
            W = the odd bins Z_j = Y_{2j+1} with packed bin 0 (Re Z_0, 0),
            W' = -i Z with packed bin 0 (Im Z_0, 0);
            y_t = INV(E)_t + cos psi_t INV(W)_t - sin psi_t INV(W')_t,
            y_{t+128} = INV(E)_t - cos psi_t INV(W)_t + sin psi_t INV(W')_t.
"""
import numpy as np

from dm_model import dm_table


def _tables():
    f = dm_table()
    return f[:, :64], f[:, 64:]


def fwd128(v):
    """v (..., 128) -> the packed 64-bin spectrum (..., 64, 2) times 2^-7, as stage 1 makes it."""
    fe, fo = _tables()
    lo, hi = v[..., :64], v[..., 64:]
    ev = (lo + hi) @ fe
    od = (lo - hi) @ fo
    pk = np.zeros(v.shape[:-1] + (64, 2))
    pk[..., 0::2, 0], pk[..., 0::2, 1] = ev[..., 0::2], ev[..., 1::2]
    pk[..., 1::2, 0], pk[..., 1::2, 1] = od[..., 0::2], od[..., 1::2]
    return pk


def inv128(pk):
    """packed (..., 64, 2) -> 128 outputs, as stage 3 makes them (E = Fe Y_even, O = Fo Y_odd)."""
    fe, fo = _tables()
    ye = np.stack([pk[..., 0::2, 0], pk[..., 0::2, 1]], -1).reshape(pk.shape[:-2] + (64,))
    yo = np.stack([pk[..., 1::2, 0], pk[..., 1::2, 1]], -1).reshape(pk.shape[:-2] + (64,))
    e, o = ye @ fe.T, yo @ fo.T
    return np.concatenate([e + o, e - o], -1)


def psi():
    t = np.arange(128)
    return np.cos(2 * np.pi * t / 256), np.sin(2 * np.pi * t / 256)


def fwd256(x):
    """x (..., 256) -> the packed 128-bin b = 256 spectrum (..., 128, 2) times 2^-7."""
    cs, sn = psi()
    a = x[..., :128] + x[..., 128:]
    d = x[..., :128] - x[..., 128:]
    pa, pp, pq = fwd128(a), fwd128(d * cs), fwd128(-d * sn)
    out = np.zeros(x.shape[:-1] + (128, 2))
    out[..., 0::2, :] = pa
    out[..., 1::2, 0] = pp[..., :, 0] - pq[..., :, 1]
    out[..., 1::2, 1] = pp[..., :, 1] + pq[..., :, 0]
    out[..., 1, 0], out[..., 1, 1] = pp[..., 0, 0], pq[..., 0, 0]      # X_1 = P_0 + i Q_0
    return out


def inv256(y):
    """y (..., 128, 2): the b = 256 stage-2 output (packed bin 0 = (Y_0, Y_128) already halved, as
    the MAC makes it) -> 256 outputs, 2 INV(...) = irfft_256 convention of the kernels."""
    cs, sn = psi()
    e = y[..., 0::2, :]
    w = y[..., 1::2, :].copy()
    wp = np.stack([w[..., 1], -w[..., 0]], -1)
    w[..., 0, 1] = 0.0
    wp[..., 0, 0], wp[..., 0, 1] = y[..., 1, 1], 0.0
    ie, iw, iwp = inv128(e), inv128(w), inv128(wp)
    o = cs * iw[..., :128] - sn * iwp[..., :128]
    return np.concatenate([ie[..., :128] + o, ie[..., :128] - o], -1)
