"""Metrics and result helpers with the reference's API (src/utils/)."""
from .metrics import (calculate_ber, calculate_ber_with_confidence, calculate_ebn0_from_snr, calculate_fer,
                      calculate_snr_from_ebn0, calculate_throughput, measure_decoding_throughput,
                      measure_encoding_throughput)
from .visualization import plot_ber_curves, plot_comparison, save_results

__all__ = ["calculate_ber", "calculate_fer", "calculate_throughput", "calculate_ber_with_confidence",
           "calculate_snr_from_ebn0", "calculate_ebn0_from_snr", "measure_encoding_throughput",
           "measure_decoding_throughput", "plot_ber_curves", "plot_comparison", "save_results"]
