"""Native (HIP/CDNA4) operator entry points with strict loading rules."""
from .native import load_native, native_available, require_native  # noqa: F401
from . import functional  # noqa: F401
