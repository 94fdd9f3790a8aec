"""Numpy mirror of bc_forward_dm_kernel's dataflow (llama-fft_amd/csrc/bcfft_dm.hip) — test
infrastructure.

It restates, in the kernel's index conventions and roundings, the three matrix-core stages, so
the decomposition, the DFT table (csrc/bcfft_dm_table.h, parsed here) and the scale bookkeeping
are checked on the CPU against the oracle before the GPU runs them:

  stage 1  per (token, half h of 16 input blocks): s = 2^sx with 2^sx * 2 max|x| < 2^15;
           a_t = (x_t + x_{t+64}) s, d_t = (x_t - x_{t+64}) s (t < 64), each split into fp16
           hi (round toward zero) + lo (exact) or rounded once to fp16 (RNE); X = [a Fe | d Fo]
           with the fp16 table F = DFT * 2^-7 (fp32 accumulation), i.e. X * 2^(sx - 7); split
           into fp16 hi + lo.
  stage 2  per packed bin: the halves brought to the token's smaller exponent (exact), times the
           STAT image conj(C)/(2b) s_C (fp16), bin 0 with an extra 1/2; Y * 2^-21 split into fp16
           hi + lo (exact) or rounded once to fp16.
  stage 3  E = Fe Y16_even, O = Fo Y16_odd (fp32 accumulation); y_t = (E + O) sc,
           y_{t+64} = (E - O) sc with sc = 2^(30 - nmin) / s_C.

precise=True mirrors the precise engine (BCFFT_ALGO_DFTP, the kernel's EP = 7 variant): the table
is F 2^8 in fp16 (kDmFp) and a, d are scaled 2^15 lower; each fp16 single term gets its rounding
residual back in e4m3 (kDmFl8 for the table, the lo8 image e4m3(conj(C) s_o - fp16(.)) for the
weights), multiplied by bf8 (the fp16 value's high byte) of the other operand's fp16 terms in
the table terms, and by e4m3 (RNE) of the aligned X terms in the weight term (x8="e4m3", the
kernel's BCFFT_DFTP_X8 = 1; x8="bf8" mirrors round 4's form).
"""
import os
import re

import numpy as np

_TABLE = os.path.join(os.path.dirname(__file__), "..", "llama-fft_amd", "csrc", "bcfft_dm_table.h")


def dm_table():
    """F[t][col] * 2^-7 (64 x 128) exactly as the kernel's fp16 table holds it."""
    text = open(_TABLE).read()
    body = text[text.index("kDmF[4096]"):]
    body = body[:body.index("};")]
    words = [int(w, 16) for w in re.findall(r"0x([0-9a-f]{8})u", body)]
    w = np.array(words, dtype=np.uint32).reshape(64, 64)
    bits = np.empty((64, 128), dtype=np.uint16)
    bits[:, 0::2] = (w & 0xFFFF).astype(np.uint16)
    bits[:, 1::2] = (w >> 16).astype(np.uint16)
    return bits.view(np.float16).astype(np.float64)


def _rtz16(v):
    """fp32 -> fp16 round toward zero (v_cvt_pkrtz_f16_f32), as float64."""
    v = np.asarray(v, dtype=np.float32).astype(np.float64)
    r = v.astype(np.float16).astype(np.float64)            # nearest
    over = np.abs(r) > np.abs(v)
    nxt = np.nextafter(r.astype(np.float16), np.float16(0)).astype(np.float64)
    return np.where(over, nxt, r)


def dm_table_precise():
    """(F 2^8 as the kernel's fp16 kDmFp, its e4m3 residual kDmFl8 decoded), both 64 x 128."""
    text = open(_TABLE).read()

    def words(name, n):
        body = text[text.index(name):]
        body = body[:body.index("};")]
        w = np.array([int(v, 16) for v in re.findall(r"0x([0-9a-f]{8})u", body)], dtype=np.uint32)
        assert w.size == n, (name, w.size)
        return w
    w = words("kDmFp[4096]", 4096).reshape(64, 64)
    bits = np.empty((64, 128), dtype=np.uint16)
    bits[:, 0::2] = (w & 0xFFFF).astype(np.uint16)
    bits[:, 1::2] = (w >> 16).astype(np.uint16)
    fp = bits.view(np.float16).astype(np.float64)
    w8 = words("kDmFl8[2048]", 2048).reshape(32, 64)         # pair-row p, column pair
    pairs = np.empty((32, 128), dtype=np.uint32)
    pairs[:, 0::2] = w8 & 0xFFFF
    pairs[:, 1::2] = w8 >> 16
    codes = np.empty((64, 128), dtype=np.uint32)
    codes[0::2] = pairs & 0xFF
    codes[1::2] = pairs >> 8
    return fp, e4m3_decode(codes)


def e4m3_decode(codes):
    """OCP e4m3fn codes -> float64 (no NaN codes occur here)."""
    c = np.asarray(codes, dtype=np.int64)
    e, m = (c >> 3) & 15, c & 7
    v = np.where(e == 0, m / 8.0 * 2.0 ** -6, (1 + m / 8.0) * 2.0 ** (e - 7.0))
    return np.where(c & 0x80, -v, v)


def e4m3(v):
    """fp32 -> OCP e4m3fn value, round to nearest even (v_cvt_pk_fp8_f32; |v| < 448 here)."""
    v = np.asarray(v, np.float32).astype(np.float64)
    a = np.abs(v)
    e = np.maximum(np.floor(np.log2(np.maximum(a, 2.0 ** -40))), -6)
    q = 2.0 ** (e - 3)
    return np.sign(v) * np.round(a / q) * q


def bf8(v):
    """bf8 (e5m2) of fp16 values: the high byte, i.e. the mantissa truncated to 2 bits."""
    h = np.asarray(v, np.float64).astype(np.float16).view(np.uint16) & np.uint16(0xFF00)
    return h.view(np.float16).astype(np.float64)


def _split16(v):
    hi = _rtz16(v)
    lo = _rtz16(np.asarray(v, np.float32).astype(np.float64) - hi)
    return hi, lo


def _scale_exp(mx):
    """stat_scale_exp: 15 - frexp exponent, clamped to [-126, 126]; an all-zero piece 126."""
    if mx == 0:
        return 126
    e = np.frexp(np.float32(mx))[1]
    return int(np.clip(15 - e, -126, 126))


def stat_image(c):
    """conj(C)/(2b) s_o as fp16 values (the STAT image's arithmetic: one power-of-two scale per
    output block o, bc_stat_scale_kernel), packed bins, and 1/s_o per output block (shape (nO, 1))."""
    b = c.shape[-1]
    h = b // 2
    xf = np.fft.rfft(c.astype(np.float64), axis=-1) / (2.0 * b)
    p = xf[..., :h].astype(np.complex64).astype(np.complex128)
    p[..., 0] = np.float32(xf[..., 0].real) + 1j * np.float32(xf[..., h].real)
    mx = np.maximum(np.abs(p.real), np.abs(p.imag)).reshape(p.shape[0], -1).max(axis=1)
    n2 = np.array([int(np.clip(15 - np.frexp(np.float32(m))[1], -126, 126)) if m > 0 else 0 for m in mx])
    sc = (2.0 ** n2)[:, None, None]
    re = (p.real * sc).astype(np.float32).astype(np.float16).astype(np.float64)
    im = (p.imag * sc).astype(np.float32).astype(np.float16).astype(np.float64)
    return re, im, 1.0 / sc[:, :, 0]                         # im of bins > 0 are Im(C) (not conj)


def _rne16(v):
    return np.asarray(v, np.float32).astype(np.float16).astype(np.float64)


def lo8_image(c):
    """The precise engine's weight residuals e4m3(v s_o - fp16(v s_o)) (bc_lo8_image_kernel), in
    stat_image's layout: (re, im), the same packed bins."""
    b = c.shape[-1]
    h = b // 2
    xf = np.fft.rfft(c.astype(np.float64), axis=-1) / (2.0 * b)
    p = xf[..., :h].astype(np.complex64).astype(np.complex128)
    p[..., 0] = np.float32(xf[..., 0].real) + 1j * np.float32(xf[..., h].real)
    mx = np.maximum(np.abs(p.real), np.abs(p.imag)).reshape(p.shape[0], -1).max(axis=1)
    n2 = np.array([int(np.clip(15 - np.frexp(np.float32(m))[1], -126, 126)) if m > 0 else 0 for m in mx])
    sc = (2.0 ** n2)[:, None, None]
    out = []
    for part in (p.real, p.imag):
        v = (part * sc).astype(np.float32)
        out.append(e4m3(v.astype(np.float64) - v.astype(np.float16).astype(np.float64)))
    return out[0], out[1]


def e4m3_s6(v):
    """The precise engine's stage-2 residual operand (BCFFT_DFTP_X8 = 1): e4m3 (RNE) of the fp16 A
    values times 2^-6, returned at the values' own scale (the kernel joins that accumulator to the
    main one times 2^6)."""
    return e4m3(np.asarray(v, np.float64) / 64.0) * 64.0


def dm_forward(x, c, exact=True, single_x=False, head=None, precise=False, terms=(1, 1, 1), x8="e4m3"):
    """x (N, K) float32, c (nO, nI, 128): the kernel's fp32 output (no bias). exact: the
    BCFFT_ALGO_DFTX variant (a, d and Y as hi + lo); else "dft" (one RNE term each). single_x:
    the bf16-I/O kernel of bcfft_dm8.hip, whose X is one RNE fp16 term too.

    head: the streamed-weight kernel of bcfft_dmk.hip (K > 4096, any nI; single_x implied).
    Each 16-block chunk (the last zero-padded) gets the scale exponent sx - head, and the chunks
    are aligned to the token's running reference: R = the first chunk's exponent, lowered to
    e + head by a chunk of exponent e < R - head (whose accumulated products then scale down by
    the same power of two). Powers of two are exact, so the result is each chunk aligned to the
    final R."""
    n, k = x.shape
    no, ni, b = c.shape
    if precise:
        exact = True
    if head is not None:
        single_x = True
        exact = False
        pad = (-ni) % 16
        if pad:
            c = np.concatenate([c, np.zeros((no, pad, b), c.dtype)], axis=1)
            x = np.concatenate([x, np.zeros((n, pad * b), x.dtype)], axis=1)
            ni += pad
            k += pad * b
    assert b == 128 and ni * b == k and ni % 16 == 0
    h = 64
    if precise:
        F, FL = dm_table_precise()                                # F 2^8: the data scale 2^-15 lower
        FLe, FLo = FL[:, :64], FL[:, 64:]
        lre, lim = lo8_image(c)
        t1, t2, t3 = (bool(t) for t in terms)
    else:
        F = dm_table()
    Fe, Fo = F[:, :64], F[:, 64:]
    cre, cim, inv_sc = stat_image(c)
    y = np.zeros((n, no * b))
    halves = ni // 16
    for tok in range(n):
        xr = x[tok].astype(np.float32).reshape(ni, b).astype(np.float64)
        X = np.zeros((ni, h), dtype=np.complex128)
        if precise:
            XB = np.zeros((ni, h), dtype=np.complex128)               # bf8 of X's fp16 terms, summed
        nsc = []
        for hh in range(halves):
            blk = xr[16 * hh:16 * hh + 16]
            sx = _scale_exp(2.0 * np.abs(blk).max()) - (head or 0)
            s = 2.0 ** (max(sx - 15, -126) if precise else sx)
            lo, hi = blk[:, :64], blk[:, 64:]
            a = ((lo + hi).astype(np.float32) * np.float32(s)).astype(np.float64)
            d = ((lo - hi).astype(np.float32) * np.float32(s)).astype(np.float64)
            if exact:
                ah, al = _split16(a)
                dh, dl = _split16(d)
                ev = ah @ Fe + al @ Fe                                   # (16, 64): even packed bins
                od = dh @ Fo + dl @ Fo
                if precise and t1:
                    ev = ev + bf8(ah) @ FLe
                    od = od + bf8(dh) @ FLo
                ev, od = ev.astype(np.float32), od.astype(np.float32)
            else:
                ev = (_rne16(a) @ Fe).astype(np.float32)
                od = (_rne16(d) @ Fo).astype(np.float32)
            # packed bins: even f = 2j at ev[:, 2j], ev[:, 2j+1]; odd f = 2j+1 at od[:, 2j], od[:, 2j+1]
            pk = np.zeros((16, 64, 2))
            pk[:, 0::2, 0], pk[:, 0::2, 1] = ev[:, 0::2], ev[:, 1::2]
            pk[:, 1::2, 0], pk[:, 1::2, 1] = od[:, 0::2], od[:, 1::2]
            if single_x:
                shi, slo = _rne16(pk), np.zeros_like(pk)
            else:
                shi, slo = _split16(pk)
            X[16 * hh:16 * hh + 16] = (shi[..., 0] + slo[..., 0]) + 1j * (shi[..., 1] + slo[..., 1])
            if precise:                        # bf8 / e4m3 commute with the exact 2^-d alignment below
                q = e4m3_s6 if x8 == "e4m3" else bf8
                XB[16 * hh:16 * hh + 16] = (q(shi[..., 0]) + q(slo[..., 0])) + 1j * (q(shi[..., 1]) + q(slo[..., 1]))
            nsc.append(sx - 7)
        nmin = min(nsc)
        if head is not None:                                      # the running reference
            nmin = nsc[0]
            for e in nsc[1:]:
                nmin = min(nmin, e + head)
        for hh in range(halves):                                  # exact power-of-two alignment
            X[16 * hh:16 * hh + 16] *= 2.0 ** (nmin - nsc[hh])
            if precise:
                XB[16 * hh:16 * hh + 16] *= 2.0 ** (nmin - nsc[hh])
        # stage 2: complex MAC per bin, bin 0 as two real products with the extra 1/2
        yr = np.einsum("oif,if->of", cre[..., 1:], X.real[:, 1:]) - np.einsum("oif,if->of", cim[..., 1:], X.imag[:, 1:])
        yi = np.einsum("oif,if->of", cre[..., 1:], X.imag[:, 1:]) + np.einsum("oif,if->of", cim[..., 1:], X.real[:, 1:])
        y0 = 0.5 * np.einsum("oi,i->o", cre[..., 0], X.real[:, 0])
        y64 = 0.5 * np.einsum("oi,i->o", cim[..., 0], X.imag[:, 0])
        if precise and t2:
            yr = yr + np.einsum("oif,if->of", lre[..., 1:], XB.real[:, 1:]) - np.einsum("oif,if->of", lim[..., 1:], XB.imag[:, 1:])
            yi = yi + np.einsum("oif,if->of", lre[..., 1:], XB.imag[:, 1:]) + np.einsum("oif,if->of", lim[..., 1:], XB.real[:, 1:])
            y0 = y0 + 0.5 * np.einsum("oi,i->o", lre[..., 0], XB.real[:, 0])
            y64 = y64 + 0.5 * np.einsum("oi,i->o", lim[..., 0], XB.imag[:, 0])
        Y = np.zeros((no, 64, 2))
        Y[:, 1:, 0], Y[:, 1:, 1] = yr, yi
        Y[:, 0, 0], Y[:, 0, 1] = y0, y64
        ys = (Y.astype(np.float32) * np.float32(2.0 ** -21)).astype(np.float32)
        if exact:
            yh, yl = _split16(ys)
            Y16 = yh + yl
        else:
            Y16 = _rne16(ys)
        # stage 3: columns in table order
        ye = np.stack([Y16[:, 0::2, 0], Y16[:, 0::2, 1]], -1).reshape(no, 64)
        yo = np.stack([Y16[:, 1::2, 0], Y16[:, 1::2, 1]], -1).reshape(no, 64)
        E = ye @ Fe.T
        O = yo @ Fo.T
        if precise and t3:
            yhb = bf8(yh)
            E = E + np.stack([yhb[:, 0::2, 0], yhb[:, 0::2, 1]], -1).reshape(no, 64) @ FLe.T
            O = O + np.stack([yhb[:, 1::2, 0], yhb[:, 1::2, 1]], -1).reshape(no, 64) @ FLo.T
        E = E.astype(np.float32).astype(np.float64)   # (no, 64 t)
        O = O.astype(np.float32).astype(np.float64)
        sc = 2.0 ** ((15 if precise else 30) - nmin) * inv_sc
        yt = np.concatenate([(E + O) * sc, (E - O) * sc], -1)
        y[tok] = yt.reshape(-1)
    return y.astype(np.float32)

