"""`src` package of the reference layout (tests import `src.polar.decoder`)."""
import sys as _sys
from pathlib import Path as _Path

_ROOT = str(_Path(__file__).resolve().parents[3])
if _ROOT not in _sys.path:
    _sys.path.insert(0, _ROOT)
