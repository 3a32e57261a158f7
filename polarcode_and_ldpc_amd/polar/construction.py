"""Polar code construction (host side, one-off).

The reference's construction API (src/polar/construction.py): the
Bhattacharyya bounds (:11-48), its "gaussian approximation" recursion
(:51-97), construct_polar_code with its three methods, returning both index
sets sorted (:100-140), and calculate_channel_capacities (:143-174).  Every
function gives the reference's values (tests/test_host_api.py, fixtures made
by tests/golden/make_golden.py:job_host_api).

Those indices are in Arikan order; the SC/SCL decoders of the reference (and of
this package) number bits in natural order, so `construct_frozen_set(...,
bit_reversed=True)` applies the bit reversal that makes the set usable with
them."""
from __future__ import annotations

import math
from typing import Tuple

import numpy as np

from .utils import bit_reverse_indices


def _polarize(x0: float, n: int, bad, good) -> np.ndarray:
    """n levels of the channel-splitting recursion: child 2i = bad(x[i]),
    child 2i+1 = good(x[i]), element-wise (the reference's per-index loops)."""
    x = np.array([x0], dtype=np.float64)
    for _ in range(n):
        nx = np.empty(2 * len(x))
        nx[0::2] = bad(x)
        nx[1::2] = good(x)
        x = nx
    return x


def _sq(z: np.ndarray) -> np.ndarray:
    """z ** 2 as the reference's scalar `Z[i] ** 2` rounds it: libm pow(z, 2),
    which is 1 ulp off z * z for ~0.1 % of inputs (np.square is z * z)."""
    return np.array([math.pow(float(v), 2.0) for v in z])


def bhattacharyya_bounds(N: int, snr_db: float) -> np.ndarray:
    """Z of each bit channel, Z0 = exp(-SNR); degraded 2Z - Z^2, upgraded Z^2
    (construction.py:11-48).  Smaller is more reliable."""
    return _polarize(np.exp(-(10 ** (snr_db / 10.0))), int(np.log2(N)), lambda z: 2 * z - _sq(z), _sq)


def gaussian_approximation(N: int, snr_db: float) -> np.ndarray:
    """The reference's simplified "GA" mean recursion (construction.py:51-97):
    mu0 = 2 SNR; degraded child 0.9 mu below 10 (else mu), upgraded child 2 mu
    saturated at 100.  Larger is more reliable."""
    return _polarize(2.0 * 10 ** (snr_db / 10.0), int(np.log2(N)),
                     lambda m: np.where(m < 10, m * 0.9, m), lambda m: np.minimum(2 * m, 100.0))


def construct_polar_code(N: int, K: int, method: str = "bhattacharyya", snr_db: float = 0.0
                         ) -> Tuple[np.ndarray, np.ndarray]:
    """(frozen, info), both ascending (construction.py:100-140).

    "bhattacharyya": the K smallest Z; "gaussian_approximation": the first K of
    argsort(mu) reversed; any other method: the bit-reversal heuristic of
    generate_frozen_bits (the K largest bit-reversed indices).  Ties are broken
    by np.argsort exactly as the reference does (same call, same input)."""
    if method == "bhattacharyya":
        order = np.argsort(bhattacharyya_bounds(N, snr_db))
    elif method == "gaussian_approximation":
        order = np.argsort(gaussian_approximation(N, snr_db))[::-1]
    else:  # the K largest bit-reversed indices, sliced as the reference ([-K:], [:-K])
        order = np.argsort(bit_reverse_indices(int(np.log2(N))))
        return np.sort(order[:-K]), np.sort(order[-K:])
    return np.sort(order[K:]), np.sort(order[:K])


def calculate_channel_capacities(N: int, snr_db: float) -> np.ndarray:
    """1 - H2((1 - Z) / 2) per bit channel from the Bhattacharyya Z, 1 below
    Z = 1e-10 and 0 above 1 - 1e-10 (construction.py:143-174)."""
    Z = bhattacharyya_bounds(N, snr_db)
    cap = np.zeros(N)
    for i, z in enumerate(Z):  # scalar ufunc calls: the reference's rounding
        if z < 1e-10:
            cap[i] = 1.0
        elif z <= 1 - 1e-10:
            p = (1 - z) / 2
            if 0 < p < 1:
                cap[i] = 1 - (-p * np.log2(p) - (1 - p) * np.log2(1 - p))
    return cap


def construct_frozen_set(N: int, K: int, snr_db: float = 2.0, bit_reversed: bool = True) -> np.ndarray:
    """Sorted frozen index set for the SC/SCL decoders (bit-reversed
    Bhattacharyya construction at design SNR snr_db)."""
    frozen, _ = construct_polar_code(N, K, "bhattacharyya", snr_db)
    if bit_reversed:
        frozen = bit_reverse_indices(int(np.log2(N)))[frozen]
    return np.sort(np.asarray(frozen, dtype=np.int64))
