"""Reference path src/utils/metrics.py -> polarcode_and_ldpc_amd.utils.metrics (import shim)."""
import sys as _sys
from pathlib import Path as _Path

_ROOT = str(_Path(__file__).resolve().parents[4])
if _ROOT not in _sys.path:
    _sys.path.insert(0, _ROOT)

from polarcode_and_ldpc_amd.utils.metrics import calculate_ber, calculate_fer, calculate_throughput, measure_encoding_throughput, measure_decoding_throughput, calculate_ber_with_confidence, calculate_snr_from_ebn0, calculate_ebn0_from_snr  # noqa: F401

__all__ = ['calculate_ber', 'calculate_fer', 'calculate_throughput', 'measure_encoding_throughput', 'measure_decoding_throughput', 'calculate_ber_with_confidence', 'calculate_snr_from_ebn0', 'calculate_ebn0_from_snr']
