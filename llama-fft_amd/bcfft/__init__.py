"""bcfft — MI355X-native block-circulant linear engine (Python side of libbcfft.so)."""
from . import _lib, graph, ops, torch_ops  # noqa: F401
from ._lib import LIB_PATH, SUPPORTED_BLOCKS, load  # noqa: F401

__all__ = ["ops", "graph", "torch_ops", "load", "LIB_PATH", "SUPPORTED_BLOCKS"]
