"""Reference path src/ldpc/matrix.py -> polarcode_and_ldpc_amd.ldpc.matrix (import shim)."""
import sys as _sys
from pathlib import Path as _Path

_ROOT = str(_Path(__file__).resolve().parents[4])
if _ROOT not in _sys.path:
    _sys.path.insert(0, _ROOT)

from polarcode_and_ldpc_amd.ldpc.matrix import mackay_construction, generate_ldpc_matrix, peg_construction, create_systematic_generator, check_matrix_rank, calculate_girth  # noqa: F401

__all__ = ['mackay_construction', 'generate_ldpc_matrix', 'peg_construction', 'create_systematic_generator', 'check_matrix_rank', 'calculate_girth']
