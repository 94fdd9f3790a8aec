"""ctypes binding of libbcfft.so (the C ABI declared in include/bcfft.h).

The library is built in-tree (``make -C llama-fft_amd`` or ``__graft_entry__.build()``) into
``llama-fft_amd/lib/libbcfft.so``. There is no fallback: if the library is missing or a
call fails, a ``RuntimeError`` is raised.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("BCFFT_LIB_PATH") or os.path.join(os.path.dirname(_HERE), "lib", "libbcfft.so")
ABI_VERSION = 1

BCFFT_NONE, BCFFT_F32, BCFFT_F16, BCFFT_BF16 = -1, 0, 1, 2
ALGO_AUTO, ALGO_MFMA, ALGO_VALU, ALGO_STAT, ALGO_DFT, ALGO_DFTX, ALGO_DFTP, ALGO_SHORT = 0, 1, 2, 3, 4, 5, 6, 7
ALGOS = {"auto": ALGO_AUTO, "mfma": ALGO_MFMA, "valu": ALGO_VALU, "stationary": ALGO_STAT, "dft": ALGO_DFT,
         "dftx": ALGO_DFTX, "dftp": ALGO_DFTP, "short": ALGO_SHORT}
DTYPE_CODE = {torch.float32: BCFFT_F32, torch.float16: BCFFT_F16, torch.bfloat16: BCFFT_BF16}
SUPPORTED_BLOCKS = (32, 64, 128, 256)
MLP_MODES = {"auto": 0, "fused": 1, "split": 2, "fused_splitk": 3}

# every symbol include/bcfft.h declares, with its ctypes signature
_SIGNATURES = {
    "bcfft_abi_version": (ctypes.c_int, []),
    "bcfft_status_string": (ctypes.c_char_p, [ctypes.c_int]),
    "bcfft_last_hip_error": (ctypes.c_char_p, []),
    "bcfft_last_error_detail": (ctypes.c_char_p, []),
    "bcfft_spectra_bytes": (ctypes.c_int64, [ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "bcfft_spectra": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]),
    "bcfft_forward": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
    "bcfft_forward_algo": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_int,
                                          ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_void_p]),
    "bcfft_forward_resolve": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                             ctypes.c_int, ctypes.c_int]),
    "bcfft_forward_kernel_name": (ctypes.c_char_p, [ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                    ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "bcfft_forward_workspace_bytes": (ctypes.c_int64, [ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                       ctypes.c_int]),
    "bcfft_forward_workspace_bytes_io": (ctypes.c_int64, [ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                          ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "bcfft_forward_ws": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_int,
                                        ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]),
    "bcfft_forward_glu": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_int,
                                         ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_void_p]),
    "bcfft_forward_glu_algo": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_int,
                                              ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_int, ctypes.c_void_p]),
    "bcfft_forward_mlp_mode": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                              ctypes.c_int]),
    "bcfft_forward_mlp_workspace_bytes": (ctypes.c_int64, [ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                          ctypes.c_int, ctypes.c_int]),
    "bcfft_forward_mlp": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]),
    "bcfft_project_circulant": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                               ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]),
    "bcfft_grad_c_workspace_bytes": (ctypes.c_int64, [ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "bcfft_grad_c": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int64,
                                    ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_int, ctypes.c_void_p]),
    "bcfft_circulant_matvec": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                              ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]),
}

_lib = None
_native = None
# the operators' handles (OpOverload), looked up once: torch.ops attribute access costs ~1 us a call
NATIVE_FORWARD = None
NATIVE_FORWARD_GLU = None
_lock = threading.RLock()
# torch.ops.bcfft_native (csrc/bcfft_torch.cpp): the C++ operators over this ABI, built next to it
TORCH_OP_PATH = os.path.join(os.path.dirname(LIB_PATH), "libbcfft_torch.so")


def load() -> ctypes.CDLL:
    """Load (once) and return the library; raise RuntimeError if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"libbcfft.so not found at {LIB_PATH}: build it with `make -C llama-fft_amd` "
                "(or __graft_entry__.build()). The MI355X engine has no CPU/torch fallback.")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.bcfft_abi_version() != ABI_VERSION:
            raise RuntimeError(f"libbcfft ABI {lib.bcfft_abi_version()} != expected {ABI_VERSION}")
        _lib = lib
    return _lib


def native_op() -> bool:
    """True once torch.ops.bcfft_native is loaded: the hot forward / forward_glu calls then go
    through one C++ dispatcher op (argument checks, allocation, stream lookup and the launch in
    C++) instead of ctypes. False when that library is not built, when BCFFT_NATIVE_OP=0, when
    BCFFT_LIB_PATH names another engine library (the operators link the in-tree libbcfft.so), or
    when the library is present but does not load (e.g. built against another torch: undefined
    c10 symbols), which warns once. Either way the kernels are libbcfft.so's (the ctypes path
    calls the same ABI): there is no CPU path."""
    global _native, NATIVE_FORWARD, NATIVE_FORWARD_GLU
    if _native is None:
        with _lock:
            if _native is None:
                ok = (os.environ.get("BCFFT_NATIVE_OP", "1") != "0" and os.path.exists(TORCH_OP_PATH)
                      and os.path.basename(LIB_PATH) == "libbcfft.so")
                if ok:
                    load()                                    # the ABI version check first (raises)
                    try:
                        torch.ops.load_library(TORCH_OP_PATH)
                    except (OSError, RuntimeError) as e:      # stale / foreign build: the ctypes path
                        import warnings
                        warnings.warn(f"{TORCH_OP_PATH} did not load ({e}); bcfft calls libbcfft.so through "
                                      "ctypes instead. Rebuild with `make -C llama-fft_amd`.", RuntimeWarning)
                        ok = False
                if ok:
                    NATIVE_FORWARD = torch.ops.bcfft_native.forward.default
                    NATIVE_FORWARD_GLU = torch.ops.bcfft_native.forward_glu.default
                _native = ok
    return _native


def check(status: int, what: str) -> None:
    if status != 0:
        lib = load()
        msg = lib.bcfft_status_string(status).decode()
        hip = lib.bcfft_last_hip_error().decode() if status == 5 else ""
        detail = lib.bcfft_last_error_detail().decode() if status == 2 else ""
        raise RuntimeError(f"{what} failed: {msg}" + (f" ({hip})" if hip else "") + (f" [{detail}]" if detail else ""))


def dtype_code(dt: torch.dtype) -> int:
    try:
        return DTYPE_CODE[dt]
    except KeyError:
        raise TypeError(f"unsupported dtype {dt}; BC engine supports float32/float16/bfloat16")


def stream_handle(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def require_device(t: torch.Tensor, what: str) -> None:
    if not t.is_cuda:
        raise RuntimeError(
            f"{what}: the MI355X BC engine runs on ROCm device tensors only (got {t.device}); "
            "move the module and inputs to the GPU. There is no CPU path in the product.")
