"""fq_amd -- MI355X-native DataBlock expression + aggregation hot path of
fuse-query (dantengsky/fuse-query), behind the reference's Function /
IProcessor surfaces.

Layers:
  abi     ctypes mirror of include/fq_gpu.h (layouts, constants)
  _lib    loads lib/libfq_amd.so (gfx950 kernels + C ABI + C++ engine)
  expr    fused-expression descriptors (numerical_coercion-typed chains)
  ops     tensor-level wrappers of the kernels (fill, aggregate, arith,
          compare, filter compaction, state merge)
"""
from . import abi  # noqa: F401
from ._lib import FQError, LIB_PATH, last_error, lib  # noqa: F401

__all__ = ["abi", "FQError", "LIB_PATH", "last_error", "lib"]
