"""pghip — MI355X-native PaliGemma image->text path (HIP kernels behind the reference's module API).

Layout: csrc/*.hip (kernels + C-ABI, include/pghip.h) -> libpghip.so -> _lib (ctypes) -> ops (tensor
wrappers) -> weights (packing) / engine (vision, prefill, graph-captured decode) -> the drop-in modules
modeling_siglip.py / modeling_gemma.py / modeling_paligemma.py / inference.py next to this package.
"""
from . import _lib  # noqa: F401

__all__ = ["_lib"]
