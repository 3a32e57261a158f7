"""Reference path src/channel/bsc.py -> polarcode_and_ldpc_amd.channel.bsc (import shim)."""
import sys as _sys
from pathlib import Path as _Path

_ROOT = str(_Path(__file__).resolve().parents[4])
if _ROOT not in _sys.path:
    _sys.path.insert(0, _ROOT)

from polarcode_and_ldpc_amd.channel.bsc import BSCChannel  # noqa: F401

__all__ = ['BSCChannel']
