"""Numeric ops: gfx950 HIP kernel wrappers (``kernels``) and fp32 golden models (``reference``)."""
from . import kernels, reference
from ._ext import available as native_available
from ._ext import load as load_native

__all__ = ["kernels", "reference", "native_available", "load_native"]
