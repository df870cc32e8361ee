"""lifeapi_amd -- MI355X-native batched ``LifeState::Step()``.

The product is the C-ABI shared library ``lifeapi_amd/liblifeapi_hip.so``
(hand-written HIP for gfx950, entry points declared in
``include/lifeapi_hip.h``) and the C++ facade in ``include/lifeapi/``.  This
Python module is a thin ctypes binding used by the tests and ``bench.py``:
PyTorch provides device memory and streams (plumbing), every compute call goes
through the C ABI.  There is no CPU fallback: if the HIP library is missing or
fails to load, importing :mod:`lifeapi_amd.hip` raises.
"""
from .layout import N, UNIVERSE_BYTES, UNIVERSE_WORDS  # noqa: F401

__all__ = ["N", "UNIVERSE_BYTES", "UNIVERSE_WORDS"]
