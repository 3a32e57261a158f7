"""Polar helpers (host side, NumPy): bit reversal, default frozen set, CRC,
polar transform.  Same results as the reference's src/polar/utils.py."""
from __future__ import annotations

from typing import Tuple

import numpy as np

CRC_POLYNOMIALS = {"CRC-8": 0x1D, "CRC-16": 0x1021, "CRC-24": 0x1864CFB}  # utils.py:99-103


def bit_reverse(n: int, num_bits: int) -> int:
    """n-bit reversal of n (src/polar/utils.py:11-26)."""
    return int(format(int(n), "0%db" % num_bits)[::-1], 2) if num_bits > 0 else 0


def bit_reverse_indices(num_bits: int) -> np.ndarray:
    """bit_reverse(i, num_bits) for i in range(2**num_bits), vectorised."""
    N = 1 << num_bits
    i = np.arange(N, dtype=np.int64)
    r = np.zeros(N, dtype=np.int64)
    for b in range(num_bits):
        r |= ((i >> b) & 1) << (num_bits - 1 - b)
    return r


def bit_reverse_array(arr: np.ndarray, num_bits: int) -> np.ndarray:
    """out[bit_reverse(i)] = arr[i] (src/polar/utils.py:29-45)."""
    out = np.zeros_like(arr)
    out[bit_reverse_indices(num_bits)[: len(arr)]] = arr
    return out


def generate_frozen_bits(N: int, K: int, channel_param: np.ndarray = None) -> Tuple[np.ndarray, np.ndarray]:
    """(frozen, info) index sets, both ascending (src/polar/utils.py:48-83).

    Default rule: the K positions whose bit-reversed index is largest are
    information bits (for K = N/2 these are the odd indices).  With
    channel_param, the K smallest values are information bits."""
    if channel_param is None:
        n = int(np.log2(N))
        order = np.argsort(bit_reverse_indices(n))
        info, frozen = order[-K:], order[:-K]
    else:
        order = np.argsort(channel_param)
        info, frozen = order[:K], order[K:]
    return np.sort(frozen), np.sort(info)


def _crc_value(bits, polynomial: str):
    if polynomial not in CRC_POLYNOMIALS:
        polynomial = "CRC-8"
    poly = CRC_POLYNOMIALS[polynomial]
    L = int(polynomial.split("-")[1])
    top, mask = 1 << (L - 1), (1 << L) - 1
    crc = 0
    for b in bits:  # bit-serial, MSB first
        crc ^= (int(b) & 1) << (L - 1)
        crc = ((crc << 1) ^ poly) if crc & top else (crc << 1)
        crc &= mask
    return crc, L


def crc_encode(data: np.ndarray, polynomial: str = "CRC-8") -> np.ndarray:
    """data followed by its CRC bits, MSB first (src/polar/utils.py:86-125)."""
    crc, L = _crc_value(data, polynomial)
    crc_bits = np.array([(crc >> s) & 1 for s in range(L - 1, -1, -1)], dtype=int)
    return np.concatenate([np.asarray(data), crc_bits])


def crc_check(data: np.ndarray, polynomial: str = "CRC-8") -> bool:
    """True when the CRC register of data (incl. its CRC) is zero
    (src/polar/utils.py:128-163)."""
    return _crc_value(data, polynomial)[0] == 0


def polar_transform(u: np.ndarray) -> np.ndarray:
    """x = u F^{(x)n} over GF(2), natural order, x[i] ^= x[i+s] for every stage
    (src/polar/utils.py:193-229).  Works on the last axis of a [.., N] array."""
    x = np.array(u, dtype=np.int64, copy=True) & 1
    N = x.shape[-1]
    s = 1
    while s < N:
        v = x.reshape(x.shape[:-1] + (N // (2 * s), 2, s))
        v[..., 0, :] ^= v[..., 1, :]
        s *= 2
    return x


def polar_transform_iterative(u: np.ndarray) -> np.ndarray:
    """The reference's single-vector transform (src/polar/utils.py:193-229):
    stage by stage x[i] = (x[i] + x[i+s]) % 2 on a copy of u, so u's dtype is
    kept and the entries that are never a left operand are not reduced mod 2
    (identical to polar_transform for 0/1 input)."""
    x = np.array(u, copy=True)
    N = len(x)
    s = 1
    while s < N:
        v = x.reshape(N // (2 * s), 2, s)
        v[:, 0, :] = (v[:, 0, :] + v[:, 1, :]) % 2
        s *= 2
    return x


def polar_transform_recursive(u: np.ndarray) -> np.ndarray:
    """The reference's recursive form (src/polar/utils.py:166-190):
    T(u) = [T((u1 + u2) % 2), T(u2)] over the halves u1, u2 -- evaluated top
    down (the widest butterfly first), so it returns the same values, dtype
    and unreduced entries as the recursion; a length-1 u is returned as is."""
    N = len(u)
    if N == 1:
        return u
    x = np.array(u, copy=True)
    h = N // 2
    while h >= 1:
        v = x.reshape(N // (2 * h), 2, h)
        v[:, 0, :] = (v[:, 0, :] + v[:, 1, :]) % 2
        h //= 2
    return x
