"""Reference path src/polar/utils.py -> polarcode_and_ldpc_amd.polar.utils (import shim)."""
import sys as _sys
from pathlib import Path as _Path

_ROOT = str(_Path(__file__).resolve().parents[4])
if _ROOT not in _sys.path:
    _sys.path.insert(0, _ROOT)

from polarcode_and_ldpc_amd.polar.utils import (bit_reverse, bit_reverse_array, generate_frozen_bits, crc_encode, crc_check, polar_transform_recursive, polar_transform_iterative, polar_transform)  # noqa: F401

__all__ = ['bit_reverse', 'bit_reverse_array', 'generate_frozen_bits', 'crc_encode', 'crc_check', 'polar_transform_recursive', 'polar_transform_iterative', 'polar_transform']
