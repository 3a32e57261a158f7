"""Reference path src/ldpc/utils.py -> polarcode_and_ldpc_amd.ldpc.utils (import shim)."""
import sys as _sys
from pathlib import Path as _Path

_ROOT = str(_Path(__file__).resolve().parents[4])
if _ROOT not in _sys.path:
    _sys.path.insert(0, _ROOT)

from polarcode_and_ldpc_amd.ldpc.utils import create_tanner_graph, check_syndrome, calculate_syndrome, count_errors, hamming_distance  # noqa: F401

__all__ = ['create_tanner_graph', 'check_syndrome', 'calculate_syndrome', 'count_errors', 'hamming_distance']
