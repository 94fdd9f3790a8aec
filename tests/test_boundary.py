"""The C-ABI boundary on the CPU: the library loads, exports every symbol include/bcfft.h
declares, and validates arguments before launching anything (no GPU needed for that)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "bcfft.h")


def header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(bcfft_[a-z_]+)\s*\(", text)))


def test_header_declares_expected_entry_points():
    fns = header_functions()
    for f in ("bcfft_forward", "bcfft_spectra", "bcfft_spectra_bytes", "bcfft_circulant_matvec",
              "bcfft_abi_version", "bcfft_status_string", "bcfft_last_hip_error"):
        assert f in fns


def test_library_exports_every_header_symbol(built_lib):
    lib = ctypes.CDLL(built_lib)
    for f in header_functions():
        assert hasattr(lib, f), f"{f} declared in bcfft.h but not exported"


def test_binding_signatures_cover_header(built_lib):
    from bcfft import _lib
    assert set(_lib._SIGNATURES) == set(header_functions())
    lib = _lib.load()
    assert lib.bcfft_abi_version() == _lib.ABI_VERSION


def test_status_strings_and_sizes(built_lib):
    from bcfft import _lib
    lib = _lib.load()
    assert lib.bcfft_status_string(0) == b"ok"
    assert b"block_size" in lib.bcfft_status_string(2)
    # (nO*nI*b/2 + b) complex64
    assert lib.bcfft_spectra_bytes(32, 32, 128) == (32 * 32 * 64 + 128) * 8
    assert lib.bcfft_spectra_bytes(86, 32, 128) == (86 * 32 * 64 + 128) * 8
    assert lib.bcfft_spectra_bytes(2, 2, 100) == -1
    assert lib.bcfft_spectra_bytes(0, 2, 64) == -1


def test_argument_validation_without_launch(built_lib):
    """Every rejected call returns before any HIP launch, so this runs without a GPU."""
    from bcfft import _lib
    lib = _lib.load()
    F32, BF16, NONE = _lib.BCFFT_F32, _lib.BCFFT_BF16, _lib.BCFFT_NONE
    fake = 4096  # never dereferenced: validation fails first
    fwd = lib.bcfft_forward
    assert fwd(fake, F32, 8, 4096, 4096, 100, fake, None, NONE, fake, F32, None) == 2   # block
    assert fwd(fake, F32, 8, 4000, 4096, 128, fake, None, NONE, fake, F32, None) == 1   # shape
    assert fwd(fake, F32, 8, 4096, 4096, 128, fake, None, NONE, fake, BF16, None) == 3  # y dtype
    assert fwd(fake, BF16, 8, 4096, 4096, 128, fake, fake, F32, fake, BF16, None) == 3  # promote
    assert fwd(fake, 7, 8, 4096, 4096, 128, fake, None, NONE, fake, F32, None) == 3     # dtype
    assert fwd(fake, F32, 8, 4096, 4096, 128, fake, fake, NONE, fake, F32, None) == 6   # bias arg
    assert fwd(None, F32, 8, 4096, 4096, 128, fake, None, NONE, fake, F32, None) == 6   # NULL x
    assert fwd(fake + 4, F32, 8, 4096, 4096, 128, fake, None, NONE, fake, F32, None) == 4  # align
    assert fwd(None, F32, 0, 4096, 4096, 128, None, None, NONE, None, F32, None) == 0   # N=0 no-op
    spec = lib.bcfft_spectra
    assert spec(fake, F32, 2, 2, 48, 0, fake, None) == 2
    assert spec(None, F32, 2, 2, 64, 0, fake, None) == 6
    assert spec(fake, F32, 0, 2, 64, 0, fake, None) == 1
    assert spec(fake, F32, 2, 2, 64, 0, fake + 8, None) == 4
    assert lib.bcfft_circulant_matvec(fake, fake, F32, 0, fake, None) == 1


def test_python_layer_fails_loudly_on_cpu_tensors(built_lib):
    import torch
    from bcfft import ops
    with pytest.raises(RuntimeError, match="ROCm device"):
        ops.forward(torch.zeros(2, 128), torch.zeros(10), None, 64, 128)
    with pytest.raises(RuntimeError, match="ROCm device"):
        ops.spectra(torch.zeros(2, 2, 64))
