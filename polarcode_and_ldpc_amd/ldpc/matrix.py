"""Parity-check matrices (host side) and their CSR form.

mackay_construction reproduces the reference's H for a given seed
(src/ldpc/matrix.py:12-50: global np.random.seed, then one
np.random.choice(m, dv, replace=False) per column), so
LDPCEncoder(504, 252, dv=3, dc=6, seed=42)'s matrix is available offline.
regular_construction builds a (dv, dc)-regular H (every check has degree dc), the
kind Min-Sum needs (the reference's MSDecoder fails on degree-1 checks)."""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np


def dense_to_csr(H: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """CSR over rows of the entries equal to 1, ascending columns."""
    H = np.asarray(H)
    rows, cols = np.nonzero(H == 1)
    row_ptr = np.zeros(H.shape[0] + 1, dtype=np.int32)
    np.add.at(row_ptr, rows + 1, 1)
    return np.cumsum(row_ptr, dtype=np.int32), cols.astype(np.int32)


def csr_to_dense(row_ptr, col_idx, n: int) -> np.ndarray:
    m = len(row_ptr) - 1
    H = np.zeros((m, n), dtype=int)
    for c in range(m):
        H[c, col_idx[row_ptr[c]:row_ptr[c + 1]]] = 1
    return H


def mackay_construction(n: int, k: int, dv: int, dc: int, seed: Optional[int] = None) -> np.ndarray:
    m = n - k
    if dv * n != dc * m:
        raise ValueError(f"Degree constraint not satisfied: dv*n={dv*n} != dc*m={dc*m}")
    if seed is not None:
        np.random.seed(seed)
    H = np.zeros((m, n), dtype=int)
    for col in range(n):
        H[np.random.choice(m, dv, replace=False), col] = 1
    return H


def generate_ldpc_matrix(n: int, k: int, method: str = "mackay", dv: int = 3, dc: int = 6,
                         seed: Optional[int] = None) -> np.ndarray:
    """src/ldpc/matrix.py:53-91 (mackay / random)."""
    m = n - k
    if method == "mackay":
        if dv * n != dc * m:
            dc = (dv * n) // m
        return mackay_construction(n, k, dv, dc, seed)
    if method == "random":
        if seed is not None:
            np.random.seed(seed)
        return np.random.randint(0, 2, (m, n))
    raise ValueError(f"Unknown method: {method}")


def regular_construction(n: int, dv: int = 3, dc: int = 6, seed: int = 0) -> np.ndarray:
    """(dv, dc)-regular H by a seeded socket permutation without repeated edges."""
    assert (n * dv) % dc == 0
    m = n * dv // dc
    rng = np.random.RandomState(seed)
    while True:
        sockets = np.repeat(np.arange(m), dc)
        rng.shuffle(sockets)
        cols = sockets.reshape(n, dv)
        s = np.sort(cols, axis=1)
        if np.all(s[:, 1:] != s[:, :-1]):
            H = np.zeros((m, n), dtype=int)
            H[cols.ravel(), np.repeat(np.arange(n), dv)] = 1
            return H
