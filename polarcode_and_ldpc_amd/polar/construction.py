"""Polar code construction (host side, one-off).

bhattacharyya_bounds / construct_polar_code return the reference's values
(src/polar/construction.py:11-48, :100-140).  Those indices are in Arikan
order; the SC/SCL decoders of the reference (and of this package) number bits
in natural order, so `construct_frozen_set(..., bit_reversed=True)` applies the
bit reversal that makes the set usable with them."""
from __future__ import annotations

from typing import Tuple

import numpy as np

from .utils import bit_reverse_indices


def bhattacharyya_bounds(N: int, snr_db: float) -> np.ndarray:
    n = int(np.log2(N))
    Z = np.array([np.exp(-(10 ** (snr_db / 10.0)))])
    for _ in range(n):
        nz = np.empty(2 * len(Z))
        nz[0::2] = 2 * Z - Z ** 2  # degraded channel
        nz[1::2] = Z ** 2          # upgraded channel
        Z = nz
    return Z


def construct_polar_code(N: int, K: int, method: str = "bhattacharyya", snr_db: float = 0.0
                         ) -> Tuple[np.ndarray, np.ndarray]:
    """(frozen, info) in the reference's order (NOT sorted, Arikan indexing)."""
    if method != "bhattacharyya":
        raise NotImplementedError("only the Bhattacharyya construction is provided")
    order = np.argsort(bhattacharyya_bounds(N, snr_db))
    return order[K:], order[:K]


def construct_frozen_set(N: int, K: int, snr_db: float = 2.0, bit_reversed: bool = True) -> np.ndarray:
    """Sorted frozen index set for the SC/SCL decoders (bit-reversed
    Bhattacharyya construction at design SNR snr_db)."""
    frozen, _ = construct_polar_code(N, K, "bhattacharyya", snr_db)
    if bit_reversed:
        frozen = bit_reverse_indices(int(np.log2(N)))[frozen]
    return np.sort(np.asarray(frozen, dtype=np.int64))
