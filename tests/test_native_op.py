"""The C++ torch operators (torch.ops.bcfft_native, llama-fft_amd/csrc/bcfft_torch.cpp) without a
GPU: the library loads beside libbcfft.so, Meta kernels give the output shapes and dtypes
(promote(x, bias) as patch_llama_fft.py:266-271), and host tensors fail loudly like the Python
path — there is no CPU engine."""
import os

import pytest
import torch

import bcfft
from bcfft import _lib


def _loaded():
    if not os.path.exists(_lib.TORCH_OP_PATH):
        pytest.fail(f"{_lib.TORCH_OP_PATH} not built (make -C llama-fft_amd)")
    assert _lib.native_op()
    return torch.ops.bcfft_native


def test_native_op_meta_shapes():
    ops = _loaded()
    x = torch.empty(5, 4096, device="meta")
    spec = torch.empty(16, device="meta")
    y = ops.forward(x.to(torch.bfloat16), spec, None, 128, 11008, 0)
    assert y.shape == (5, 11008) and y.dtype == torch.bfloat16
    assert ops.forward(x.to(torch.bfloat16), spec, torch.empty(4096, device="meta"), 128, 4096, 0).dtype == torch.float32
    assert ops.forward_glu(x, spec, 128, 11008, 0).shape == (5, 11008)
    with pytest.raises(ValueError, match="multiples"):
        ops.forward(torch.empty(3, 100, device="meta"), spec, None, 128, 4096, 0)


def test_native_op_host_tensors_fail_loudly():
    ops = _loaded()
    with pytest.raises(RuntimeError, match="no CPU path"):
        ops.forward(torch.zeros(3, 4096), torch.zeros(8), None, 128, 4096, 0)
    with pytest.raises(RuntimeError, match="no CPU path"):
        ops.forward_glu(torch.zeros(3, 4096), torch.zeros(8), 128, 4096, 0)
    with pytest.raises(RuntimeError, match="no CPU path"):      # bcfft.ops with the native op loaded
        bcfft.ops.forward(torch.zeros(3, 4096), torch.zeros(8), None, 128, 4096)


def test_broken_native_library_falls_back_to_ctypes(tmp_path, monkeypatch):
    """A libbcfft_torch.so that exists but does not load (stale build against another torch, a
    truncated file) must not take the forward path down: one warning, then the ctypes binding of
    the same libbcfft.so. Host tensors still fail loudly there."""
    bogus = tmp_path / "libbcfft_torch.so"
    bogus.write_bytes(b"not an ELF object")
    monkeypatch.setattr(_lib, "TORCH_OP_PATH", str(bogus))
    monkeypatch.setattr(_lib, "_native", None)
    with pytest.warns(RuntimeWarning, match="did not load"):
        assert _lib.native_op() is False
    assert _lib.native_op() is False                         # decided once, no second warning
    with pytest.raises(RuntimeError, match="no CPU path"):  # bcfft.ops on the ctypes path
        bcfft.ops.forward(torch.zeros(3, 4096), torch.zeros(8), None, 128, 4096)
