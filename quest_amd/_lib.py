"""Locate and load the native QuEST-for-MI355X library.

Four builds live in ``quest_amd/lib`` (see the Makefile): HIP for gfx950 and
the host plumbing build, each in fp64 and fp32 (compile-time precision, as in
the reference's ``QuEST_precision.h``).  Selection:

* ``QUEST_BACKEND`` = ``hip`` | ``cpu`` | ``auto`` (default ``auto``: HIP when
  a GPU is visible, else CPU);
* ``QUEST_PREC`` = ``2`` (fp64, default) | ``1`` (fp32).

On the HIP path PyTorch is imported *before* the library so that both share
one HIP runtime (and the RCCL that the library dlopens is torch's).  A
missing HIP library on a GPU machine is an error, never a silent fallback.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(_HERE, "lib")

_loaded = {}


def gpu_visible() -> bool:
    """True when an AMD GPU device node exists and torch sees a device."""
    if not os.path.exists("/dev/kfd"):
        return False
    try:
        import torch  # noqa: F401

        return torch.cuda.device_count() > 0
    except Exception:  # pragma: no cover - torch missing
        return False


def resolve(backend: str | None = None, prec: int | None = None) -> tuple[str, int, str]:
    backend = (backend or os.environ.get("QUEST_BACKEND", "auto")).lower()
    prec = int(prec or os.environ.get("QUEST_PREC", "2"))
    if prec not in (1, 2, 4):
        raise ValueError("QUEST_PREC must be 1 (fp32), 2 (fp64) or 4 (long double, host build only)")
    if backend == "auto":
        backend = "cpu" if prec == 4 else ("hip" if gpu_visible() else "cpu")
    if backend not in ("hip", "cpu"):
        raise ValueError(f"unknown QUEST_BACKEND {backend!r}")
    if prec == 4 and backend != "cpu":
        raise ValueError("QUEST_PREC=4 (long double) exists for the host build only, as in the reference")
    name = f"libQuEST_{backend}_f{ {1: 32, 2: 64, 4: 128}[prec] }.so"
    override = os.environ.get("QUEST_LIB")  # e.g. a CMake build's library
    if override:
        return backend, prec, override
    return backend, prec, os.path.join(LIB_DIR, name)


def load(backend: str | None = None, prec: int | None = None) -> ctypes.CDLL:
    backend, prec, path = resolve(backend, prec)
    key = (backend, prec)
    if key in _loaded:
        return _loaded[key]
    if not os.path.exists(path):
        raise RuntimeError(
            f"native library {path} is missing: run `make {'hip' if backend == 'hip' else 'cpu'}` "
            "(or __graft_entry__.build()) first"
        )
    if backend == "hip":
        import torch  # noqa: F401  (share torch's HIP runtime / RCCL)
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
    lib._quest_backend = backend
    lib._quest_prec = prec
    lib._quest_path = path
    _loaded[key] = lib
    return lib
