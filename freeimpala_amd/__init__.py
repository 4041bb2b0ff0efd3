"""freeimpala_amd -- MI355X-native batched IMPALA learner step for freeimpala.

The product is libfi_learner.so (HIP for gfx950) behind the C ABI in include/fi_learner.h;
this package holds its sources (csrc/), the in-tree build (lib/) and the ctypes binding.
"""
from ._abi import LIB_PATH, FiError, lib  # noqa: F401

__all__ = ["LIB_PATH", "FiError", "lib"]
