"""Reference path src/polar/decoder.py -> polarcode_and_ldpc_amd.polar.decoder (import shim)."""
import sys as _sys
from pathlib import Path as _Path

_ROOT = str(_Path(__file__).resolve().parents[4])
if _ROOT not in _sys.path:
    _sys.path.insert(0, _ROOT)

from polarcode_and_ldpc_amd.polar.decoder import SCDecoder, SCLDecoder, CASCLDecoder  # noqa: F401

__all__ = ['SCDecoder', 'SCLDecoder', 'CASCLDecoder']
