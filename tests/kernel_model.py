"""Numpy mirror of the HIP kernel's dataflow (test infrastructure).

It restates, step by step and in the same index conventions, what
llama-fft_amd/csrc/bcfft_kernels.hip computes, so the decomposition can be checked on the CPU
against the oracle before (and independently of) the GPU:

  * spectra: packed bins P[0] = (X[0], X[H]) (both real), P[k] = X[k] for 0<k<H, scaled by
    1/(2b)  (1/b = irfft normalisation, 1/2 = the real-FFT untangling factor).
  * forward real FFT of b points = H=b/2 point complex FFT of z[n] = x[2n] + i x[2n+1],
    four-step H = L x P: lane n1 < L holds z[n1 + L*n2] (n2 < P), P-point DFT, twiddle
    W_H^(n1*k2), transpose, L-point DFT -> Z[P*k1 + k2]; untangle (without the 1/2).
  * CMAC with the branch-free bin-0 rule: yr += cr*xr - ci'*xi ; yi += cr'*xi + ci*xr.
  * inverse: E = Y[k] + conj(Y[H-k]), O = (Y[k] - conj(Y[H-k])) W_b^-k, Zi = E + iO,
    same four-step with conjugate twiddles, y[2n] = Re z[n], y[2n+1] = Im z[n].
"""
import numpy as np


def fft_lane_split(b):
    h = b // 2
    lanes = 4 if h <= 32 else 8
    return h, lanes, h // lanes


def spectra_packed(c):
    b = c.shape[-1]
    h = b // 2
    x = np.fft.rfft(c.astype(np.float64), axis=-1) / (2.0 * b)
    p = x[..., :h].copy()
    p[..., 0] = x[..., 0].real + 1j * x[..., h].real
    return p.astype(np.complex64)


def four_step(z, lanes, sign):
    """z: (..., H) complex. Returns the unnormalised DFT with exp(sign*2*pi*i*nk/H)."""
    h = z.shape[-1]
    p = h // lanes
    w = lambda n, m: np.exp(sign * 2j * np.pi * np.outer(np.arange(n), np.arange(n)) / m)  # noqa
    # lane n1 holds z[n1 + L*n2]
    v = z.reshape(*z.shape[:-1], p, lanes)              # [..., n2, n1]
    a = np.einsum("...ql,qk->...lk", v, w(p, p))        # P-point DFT over n2 -> [..., n1, k2]
    tw = np.exp(sign * 2j * np.pi * np.outer(np.arange(lanes), np.arange(p)) / h)
    a = a * tw                                           # W_H^(n1*k2)
    zz = np.einsum("...lk,lm->...mk", a, w(lanes, lanes))  # L-point DFT over n1 -> [..., k1, k2]
    return zz.reshape(*z.shape[:-1], h)                 # index P*k1 + k2


def forward_real(x):
    """x (..., b) real -> packed X' = 2*X (bins 0..H-1; bin 0 = (X0, XH))."""
    b = x.shape[-1]
    h, lanes, _ = fft_lane_split(b)
    z = x[..., 0::2] + 1j * x[..., 1::2]
    zk = four_step(z, lanes, -1)
    zm = np.conj(np.roll(zk[..., ::-1], 1, axis=-1))     # conj(Z[(H-k) % H])
    k = np.arange(h)
    wb = np.exp(-2j * np.pi * k / b)
    out = (zk + zm) - 1j * wb * (zk - zm)                # 2 X[k]
    z0 = zk[..., 0]
    out[..., 0] = 2 * (z0.real + z0.imag) + 1j * 2 * (z0.real - z0.imag)
    return out


def inverse_real(yp, b):
    h, lanes, _ = fft_lane_split(b)
    k = np.arange(h)
    ym = np.conj(np.roll(yp[..., ::-1], 1, axis=-1))     # conj(Y[(H-k) % H])
    e = yp + ym
    o = (yp - ym) * np.exp(2j * np.pi * k / b)
    zi = e + 1j * o
    y0, yh = yp[..., 0].real, yp[..., 0].imag
    zi[..., 0] = (y0 + yh) + 1j * (y0 - yh)
    z = four_step(zi, lanes, +1)
    out = np.empty(z.shape[:-1] + (b,))
    out[..., 0::2] = z.real
    out[..., 1::2] = z.imag
    return out


def cmac(cp, xp):
    """cp (nO, nI, H) packed spectra, xp (N, nI, H) packed X' -> Y (N, nO, H) with the
    branch-free bin-0 rule."""
    cr, ci = cp.real, cp.imag
    crp = cr.copy()
    cip = ci.copy()
    crp[..., 0] = ci[..., 0]     # cr' = CH on bin 0
    cip[..., 0] = 0.0            # ci' = 0
    cin = ci.copy()
    cin[..., 0] = 0.0            # ci  = 0
    xr, xi = xp.real, xp.imag
    yr = np.einsum("oif,nif->nof", cr, xr) - np.einsum("oif,nif->nof", cip, xi)
    yi = np.einsum("oif,nif->nof", crp, xi) + np.einsum("oif,nif->nof", cin, xr)
    return yr + 1j * yi


def bc_forward_model(x, c, bias=None):
    n_out, n_in, b = c.shape
    n = x.shape[0]
    xp = forward_real(x.reshape(n, n_in, b).astype(np.float64))
    y = inverse_real(cmac(spectra_packed(c).astype(np.complex128), xp), b)
    y = y.reshape(n, n_out * b)
    if bias is not None:
        y = y + bias
    return y
