"""Reference path src/utils/__init__.py -> polarcode_and_ldpc_amd.utils (import shim)."""
import sys as _sys
from pathlib import Path as _Path

_ROOT = str(_Path(__file__).resolve().parents[4])
if _ROOT not in _sys.path:
    _sys.path.insert(0, _ROOT)

from polarcode_and_ldpc_amd.utils import *  # noqa: F401,F403
from polarcode_and_ldpc_amd.utils import __all__  # noqa: F401
