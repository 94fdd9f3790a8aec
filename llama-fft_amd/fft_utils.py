"""Drop-in for the reference's ``fft_utils`` (src/fft_utils.py:3-34) on MI355X."""
import torch

from bcfft import ops as _ops


def circulant_matvec_fft(c: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """y = C x for the circulant C with first column c (C[i, j] = c[(i - j) % n]).

    Same contract as fft_utils.py:3-34: 1-D c and x of equal length, any float dtype,
    result in x's dtype. Runs the ``bcfft_circulant_matvec`` HIP kernel (any n)."""
    assert c.dim() == 1                                            # :14
    assert x.dim() == 1                                            # :15
    n = c.shape[0]
    assert x.shape[0] == n                                         # :17
    c = c.to(x.device)
    if c.dtype != x.dtype:   # reference: both go to fp32 (:22-23), result cast to x.dtype (:34)
        return _ops.circulant_matvec(c.float(), x.float()).to(x.dtype)
    return _ops.circulant_matvec(c, x)
