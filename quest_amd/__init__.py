"""quest_amd: an MI355X-native full-state quantum circuit simulator with the
QuEST v2 API.

Layers (see docs/ARCHITECTURE.md):

* native library (``quest_amd/lib/libQuEST_*.so``): the C API of
  ``include/QuEST.h`` implemented by a C++ front-end, a distributed router
  (RCCL over xGMI, one process per GPU) and hand-written HIP kernels for
  gfx950 - or, in the host build, plain C++ loops;
* :mod:`quest_amd.ops` - ctypes binding of the whole C API (``capi``) and a
  Pythonic :class:`Register` / :class:`Env`;
* :mod:`quest_amd.models` - circuit families (random benchmark circuits, QFT,
  Bernstein-Vazirani, GHZ, the fork's 30-qubit benchmark);
* :mod:`quest_amd.parallel` - multi-process launch / bootstrap helpers
  (torchrun-compatible);
* :mod:`quest_amd.utils` - NumPy reference simulator (test oracle), the
  golden ``.test`` runner, timers.
"""
from ._lib import load, resolve  # noqa: F401
from .ops import capi  # noqa: F401
from .ops.capi import QuESTError  # noqa: F401
from .ops.register import Env, Register  # noqa: F401

__version__ = "0.1.0"
