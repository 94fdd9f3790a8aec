"""bcfft — MI355X-native block-circulant linear engine (Python side of libbcfft.so).

`bcfft.torch_ops` (the torch.library registration of the ops under torch.ops.bcfft) is imported
on first access, so the ctypes ops stay importable on a torch without torch.library.custom_op."""
from . import _lib, graph, ops  # noqa: F401
from ._lib import LIB_PATH, SUPPORTED_BLOCKS, load  # noqa: F401

__all__ = ["ops", "graph", "torch_ops", "load", "LIB_PATH", "SUPPORTED_BLOCKS"]


def __getattr__(name):
    if name == "torch_ops":
        import importlib
        return importlib.import_module(".torch_ops", __name__)
    raise AttributeError(f"module 'bcfft' has no attribute {name!r}")
