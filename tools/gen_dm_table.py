"""Writes llama-fft_amd/csrc/bcfft_dm_table.h: the DFT matrix image of bc_forward_dm_kernel
(bcfft_dm.hip), F[t][col] for t < 64 and 128 columns, times 2^-7, as fp16 (fp64 trig, one
round-to-nearest-even). Columns 0-63 = Fe (even packed bins from a_t = x_t + x_{t+64}), 64-127 =
Fo (odd packed bins from d_t = x_t - x_{t+64}); packed bin f occupies columns (2 (f >> 1), +1)
of its half: (re, im) of X_f, and for f = 0 (X_0, X_64).
  Fe[t][2j]   = cos(2 pi j t / 64),  Fe[t][2j+1] = -sin(2 pi j t / 64)   (j >= 1)
  Fe[t][0]    = 1,                   Fe[t][1]    = (-1)^t                 (X_0, X_64)
  Fo[t][2j]   = cos(2 pi (2j+1) t / 128), Fo[t][2j+1] = -sin(2 pi (2j+1) t / 128)
Also kDmF64, the b = 64 table of bc_forward_dm64_kernel (bcfft_dm64.hip), built the same way,
and kDmB64, the same b = 64 table as bf16 hi + lo MFMA A fragments (bc_forward_dm64k_kernel's
stage 1 on raw bf16 x).
The precise engine (BCFFT_ALGO_DFTP, bcfft_dm.hip's EP variant) takes the same table times 2^8 as
fp16 (kDmFp: entries 12.6 .. 256, the same 11 significant bits) plus its rounding residual
F 2^8 - kDmFp as OCP e4m3 (kDmFl8, |value| <= 2^-3), pair-packed for the kernel's fp8 MFMA
operands: word (p, c) holds the 16-bit pair (row 2p, row 2p + 1) of column c, 32 pair-rows x 128
columns, row-major, unswizzled.
usage: python tools/gen_dm_table.py"""
import os
import numpy as np

t = np.arange(64)[:, None]
F = np.zeros((64, 128))
for j in range(32):
    if j == 0:
        F[:, 0] = 1.0
        F[:, 1] = (-1.0) ** t[:, 0]
    else:
        F[:, 2 * j] = np.cos(2 * np.pi * j * t[:, 0] / 64)
        F[:, 2 * j + 1] = -np.sin(2 * np.pi * j * t[:, 0] / 64)
    th = 2 * np.pi * (2 * j + 1) * t[:, 0] / 128
    F[:, 64 + 2 * j] = np.cos(th)
    F[:, 64 + 2 * j + 1] = -np.sin(th)
bits = (F * 2.0 ** -7).astype(np.float16).view(np.uint16).astype(np.uint32)
words = (bits[:, 0::2] | (bits[:, 1::2] << 16)).reshape(-1)          # (64 rows x 64 words)

# b = 64 (bc_forward_dm64_kernel, bcfft_dm64.hip): t < 32, 64 columns, the same construction
# with x_{t+32}: Fe[t][2j] = cos(2 pi j t / 32) (j >= 1), Fe[t][0..1] = (1, (-1)^t),
# Fo[t][2j] = cos(2 pi (2j+1) t / 64), the -sin columns beside them
t64 = np.arange(32)
F64 = np.zeros((32, 64))
for j in range(16):
    if j == 0:
        F64[:, 0] = 1.0
        F64[:, 1] = (-1.0) ** t64
    else:
        F64[:, 2 * j] = np.cos(2 * np.pi * j * t64 / 32)
        F64[:, 2 * j + 1] = -np.sin(2 * np.pi * j * t64 / 32)
    th = 2 * np.pi * (2 * j + 1) * t64 / 64
    F64[:, 32 + 2 * j] = np.cos(th)
    F64[:, 32 + 2 * j + 1] = -np.sin(th)
bits64 = (F64 * 2.0 ** -7).astype(np.float16).view(np.uint16).astype(np.uint32)
words64 = (bits64[:, 0::2] | (bits64[:, 1::2] << 16)).reshape(-1)     # (32 rows x 32 words)


def bf16_rne(v):
    """v rounded to bf16 (8 significant bits, round half to even) in fp64; normal range only."""
    m, e = np.frexp(np.asarray(v, np.float64))
    return np.ldexp(np.round(m * 256.0), e - 8)


def bf16_bits(v):
    """bf16 bits of values exactly representable in bf16."""
    return (np.asarray(v, np.float32).view(np.uint32) >> 16).astype(np.uint32)


# b = 64, the bf16 direct stage 1 of bc_forward_dm64k_kernel (bcfft_dm64k.hip): the MFMA A
# fragments of F64 2^-7 as bf16 hi + lo (hi = bf16(v), lo = bf16(v - hi): ~16 significant bits).
# Fragment (pr, mt, term), lane l, element e = A[m = l & 15][k = 8 (l >> 4) + e] = column
# 32 pr + 16 mt + m, row t = k; layout [pr][mt][term][lane][8 bf16] (16 B per lane)
v64 = F64 * 2.0 ** -7
hi64 = bf16_rne(v64)
lo64 = bf16_rne(v64 - hi64)
assert np.abs(v64 - hi64 - lo64).max() <= 2.0 ** -23
fragb = np.zeros((2, 2, 2, 64, 8), np.uint32)
for pr in range(2):
    for mt in range(2):
        for ln in range(64):
            col = 32 * pr + 16 * mt + (ln & 15)
            ts = 8 * (ln >> 4) + np.arange(8)
            fragb[pr, mt, 0, ln] = bf16_bits(hi64[ts, col])
            fragb[pr, mt, 1, ln] = bf16_bits(lo64[ts, col])
wordsb64 = (fragb[..., 0::2] | (fragb[..., 1::2] << 16)).reshape(-1)  # 2048 words


def e4m3(v):
    """OCP e4m3fn encoding (bias 7, max 448, no infinities), round to nearest even."""
    v = np.asarray(v, np.float64)
    a = np.abs(v)
    e = np.floor(np.log2(np.maximum(a, 2.0 ** -30)))
    e = np.maximum(e, -6)                                             # subnormals: step 2^-9
    q = 2.0 ** (e - 3)
    m = np.round(a / q)                                               # numpy rounds half to even
    val = m * q
    assert (val <= 448).all()
    code = np.zeros(v.shape, np.uint32)
    sub = val < 2.0 ** -6
    code[sub] = (val[sub] / 2.0 ** -9).astype(np.uint32)
    ee = np.floor(np.log2(np.maximum(val, 2.0 ** -30)))
    mant = np.round(val / 2.0 ** ee * 8) - 8
    code[~sub] = (((ee[~sub] + 7).astype(np.uint32)) << 3) | mant[~sub].astype(np.uint32)
    code[val == 0] = 0
    code |= np.where(v < 0, 0x80, 0).astype(np.uint32)
    return code, np.where(v < 0, -val, val)


fp = (F * 2.0 ** 8).astype(np.float16)
bitsp = fp.view(np.uint16).astype(np.uint32)
wordsp = (bitsp[:, 0::2] | (bitsp[:, 1::2] << 16)).reshape(-1)       # (64 rows x 64 words)
res = F * 2.0 ** 8 - fp.astype(np.float64)
l8, l8v = e4m3(res)
assert (np.abs(l8v - res) <= 2.0 ** -4 * np.abs(res) + 2.0 ** -10).all() and np.abs(res).max() <= 2.0 ** -3
pairs = l8[0::2, :] | (l8[1::2, :] << 8)                              # (32 pair-rows, 128 cols) 16-bit
wordsl8 = (pairs[:, 0::2] | (pairs[:, 1::2] << 16)).reshape(-1)      # (32 x 64 words)
out = os.path.join(os.path.dirname(__file__), "..", "llama-fft_amd", "csrc", "bcfft_dm_table.h")
with open(out, "w") as f:
    f.write("// generated by tools/gen_dm_table.py -- do not edit\n")
    f.write("// F[t][col] * 2^-7 as fp16 pairs, row-major, unswizzled: kDmF (b = 128) 64 rows x 256 B,\n")
    f.write("// kDmF64 (b = 64) 32 rows x 128 B\n")
    f.write("#pragma once\n#include <stdint.h>\nnamespace bcfft {\n")
    f.write("__device__ const uint32_t kDmF[4096] __attribute__((aligned(16))) = {\n")
    for r in range(0, 4096, 8):
        f.write("  " + ", ".join("0x%08xu" % w for w in words[r:r + 8]) + ",\n")
    f.write("};\n")
    f.write("__device__ const uint32_t kDmF64[1024] __attribute__((aligned(16))) = {\n")
    for r in range(0, 1024, 8):
        f.write("  " + ", ".join("0x%08xu" % w for w in words64[r:r + 8]) + ",\n")
    f.write("};\n")
    f.write("// F64 * 2^-7 as bf16 hi + lo MFMA A fragments [pr][mt][term][lane][8] (bcfft_dm64k.hip)\n")
    f.write("__device__ const uint32_t kDmB64[2048] __attribute__((aligned(16))) = {\n")
    for r in range(0, 2048, 8):
        f.write("  " + ", ".join("0x%08xu" % w for w in wordsb64[r:r + 8]) + ",\n")
    f.write("};\n")
    f.write("// F[t][col] * 2^8 as fp16 pairs (the precise engine), layout of kDmF\n")
    f.write("__device__ const uint32_t kDmFp[4096] __attribute__((aligned(16))) = {\n")
    for r in range(0, 4096, 8):
        f.write("  " + ", ".join("0x%08xu" % w for w in wordsp[r:r + 8]) + ",\n")
    f.write("};\n")
    f.write("// e4m3(F 2^8 - kDmFp), byte pairs (row 2p, row 2p + 1) per column: 32 pair-rows x 256 B\n")
    f.write("__device__ const uint32_t kDmFl8[2048] __attribute__((aligned(16))) = {\n")
    for r in range(0, 2048, 8):
        f.write("  " + ", ".join("0x%08xu" % w for w in wordsl8[r:r + 8]) + ",\n")
    f.write("};\n}  // namespace bcfft\n")
print("wrote", out)
