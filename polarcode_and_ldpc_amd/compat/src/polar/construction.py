"""Reference path src/polar/construction.py -> polarcode_and_ldpc_amd.polar.construction (import shim)."""
import sys as _sys
from pathlib import Path as _Path

_ROOT = str(_Path(__file__).resolve().parents[4])
if _ROOT not in _sys.path:
    _sys.path.insert(0, _ROOT)

from polarcode_and_ldpc_amd.polar.construction import (bhattacharyya_bounds, gaussian_approximation, construct_polar_code, calculate_channel_capacities, construct_frozen_set)  # noqa: F401

__all__ = ['bhattacharyya_bounds', 'gaussian_approximation', 'construct_polar_code', 'calculate_channel_capacities', 'construct_frozen_set']
