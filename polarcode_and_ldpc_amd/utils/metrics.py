"""BER / FER / throughput metrics (src/utils/metrics.py:12-191).

Same formulas and return values as the reference.  The measure_* helpers keep
the reference's per-frame timing loop when handed reference-style objects, and
time one batched call when the object has `decode_batch` / `encode_batch`
(the GPU path of this package)."""
from __future__ import annotations

import time
from typing import Dict, List, Tuple

import numpy as np


def calculate_ber(original_bits: np.ndarray, decoded_bits: np.ndarray) -> float:
    """Fraction of differing bits (metrics.py:12-28)."""
    assert len(original_bits) == len(decoded_bits), "Bit sequences must have same length"
    n = len(original_bits)
    return float(np.sum(np.asarray(original_bits) != np.asarray(decoded_bits))) / n if n else 0.0


def calculate_fer(original_frames: List[np.ndarray], decoded_frames: List[np.ndarray]) -> float:
    """Fraction of frames with at least one error (metrics.py:31-52)."""
    assert len(original_frames) == len(decoded_frames), "Frame lists must have same length"
    n = len(original_frames)
    bad = sum(0 if np.array_equal(a, b) else 1 for a, b in zip(original_frames, decoded_frames))
    return bad / n if n else 0.0


def calculate_throughput(num_bits: int, elapsed_time: float) -> float:
    """Mbps = bits / seconds / 1e6; 0 for a non-positive time (metrics.py:55-69)."""
    return num_bits / elapsed_time / 1e6 if elapsed_time > 0 else 0.0


def _timing(total_bits: int, num_frames: int, elapsed: float) -> Dict[str, float]:
    return {"total_bits": total_bits, "num_frames": num_frames, "elapsed_time": elapsed,
            "throughput_mbps": calculate_throughput(total_bits, elapsed),
            "avg_time_per_frame": elapsed / num_frames if num_frames else 0.0}


def measure_encoding_throughput(encoder, num_frames: int = 1000) -> Dict[str, float]:
    """metrics.py:72-103: K info bits per frame, random messages."""
    K = encoder.K if hasattr(encoder, "K") else encoder.k
    msgs = np.random.randint(0, 2, (num_frames, K))
    t0 = time.time()
    if hasattr(encoder, "encode_batch") and not getattr(encoder, "use_crc", False):
        encoder.encode_batch(msgs)
    else:
        for m in msgs:
            encoder.encode(m)
    return _timing(num_frames * K, num_frames, time.time() - t0)


def measure_decoding_throughput(decoder, llr_inputs: List[np.ndarray]) -> Dict[str, float]:
    """metrics.py:106-135 (counts len(llr) bits per frame, as the reference)."""
    frames = len(llr_inputs)
    bits = frames * len(llr_inputs[0])
    t0 = time.time()
    if hasattr(decoder, "decode_batch"):
        decoder.decode_batch(np.stack(llr_inputs))
    else:
        for x in llr_inputs:
            decoder.decode(x)
    return _timing(bits, frames, time.time() - t0)


def calculate_ber_with_confidence(bit_errors: int, total_bits: int,
                                  confidence: float = 0.95) -> Tuple[float, float, float]:
    """(BER, lower, upper) Wilson score interval (metrics.py:138-167), with the
    reference's quantile (scipy's norm.ppf) and rounding (z ** 2 through pow)."""
    if total_bits == 0:
        return 0.0, 0.0, 0.0
    from scipy.stats import norm
    p = bit_errors / total_bits
    z = norm.ppf(1 - (1 - confidence) / 2)
    z2 = z ** 2
    den = 1 + z2 / total_bits
    mid = (p + z2 / (2 * total_bits)) / den
    half = z * np.sqrt(p * (1 - p) / total_bits + z2 / (4 * total_bits ** 2)) / den
    return p, max(0, mid - half), min(1, mid + half)


def calculate_snr_from_ebn0(ebn0_db: float, code_rate: float) -> float:
    return ebn0_db + 10 * np.log10(code_rate)


def calculate_ebn0_from_snr(snr_db: float, code_rate: float) -> float:
    return snr_db - 10 * np.log10(code_rate)
