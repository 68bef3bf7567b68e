"""Loader for the in-tree native extension ``hipdsml._C``.

Rule: on a machine with a GPU the HIP path is mandatory — if ``_C.so`` is
missing or fails to import while ``torch.cuda.is_available()``, every GPU entry
point raises instead of silently falling back to PyTorch.  On a CPU-only host
the torch reference backend is used for host tensors only.
"""
from __future__ import annotations

import importlib
import os
from types import ModuleType
from typing import Optional

_native: Optional[ModuleType] = None
_error: Optional[BaseException] = None


def load_native(build_if_missing: bool = False) -> Optional[ModuleType]:
    global _native, _error
    if _native is not None:
        return _native
    import torch  # noqa: F401  (libtorch / libamdhip64 / librccl must be loaded first)

    try:
        _native = importlib.import_module("hipdsml._C")
        _error = None
    except ImportError as e:  # pragma: no cover - depends on build state
        _error = e
        if build_if_missing or os.environ.get("HIPDSML_AUTOBUILD") == "1":
            from .. import _build

            _build.build()
            _native = importlib.import_module("hipdsml._C")
            _error = None
    return _native


def native_available() -> bool:
    return load_native() is not None


def require_native() -> ModuleType:
    m = load_native()
    if m is None:
        raise RuntimeError(
            "hipdsml native extension (_C.so) is not built or failed to import: "
            f"{_error!r}. Run `python -m hipdsml._build` (hipcc --offload-arch=gfx950)."
        )
    return m
