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


def peg_construction(n: int, k: int, dv: int) -> np.ndarray:
    """The reference's simplified progressive edge growth (matrix.py:94-132):
    column by column, dv times pick the least-loaded check not yet used by this
    column (first such check on ties)."""
    m = n - k
    H = np.zeros((m, n), dtype=int)
    load = np.zeros(m, dtype=np.int64)
    for col in range(n):
        used = np.zeros(m, dtype=bool)
        for _ in range(min(dv, m)):
            cand = np.where(used, np.iinfo(np.int64).max, load)
            r = int(np.argmin(cand))
            used[r] = True
            H[r, col] = 1
            load[r] += 1
    return H


def create_systematic_generator(H: np.ndarray):
    """(G [k, n], P) or (None, None) when the last m columns of H are singular
    over GF(2) (matrix.py:135-187)."""
    from .encoder import _systematic_generator
    return _systematic_generator(H)


def check_matrix_rank(H: np.ndarray) -> int:
    """np.linalg.matrix_rank, as the reference (real rank, not GF(2); matrix.py:190-200)."""
    return int(np.linalg.matrix_rank(H))


def calculate_girth(H: np.ndarray) -> int:
    """The reference returns a density-based estimate (matrix.py:203-225): 6 for
    density < 0.1, else 4."""
    m, n = H.shape
    return 6 if np.sum(H) / (m * n) < 0.1 else 4


def gf2_systematic_pair(H: np.ndarray):
    """A valid systematic code for any H over GF(2): (Hp, G) with Hp = H with its
    columns permuted so the message occupies positions 0..k-1 and G [n, k]
    (pyldpc's orientation: codeword = G @ message mod 2), k = n - rank_GF2(H).
    Used by the lib_wrappers substitute for the unavailable pyldpc."""
    A = (np.asarray(H) % 2).astype(np.uint8)
    m, n = A.shape
    pivots, r = [], 0
    for c in range(n - 1, -1, -1):  # parity checks on the right when possible
        if r == m:
            break
        nz = np.nonzero(A[r:, c])[0]
        if len(nz) == 0:
            continue
        p = r + nz[0]
        if p != r:
            A[[r, p]] = A[[p, r]]
        rows = np.nonzero(A[:, c])[0]
        A[rows[rows != r]] ^= A[r]
        pivots.append(c)
        r += 1
    piv_row = {c: i for i, c in enumerate(pivots)}
    info = [c for c in range(n) if c not in piv_row]
    parity = sorted(pivots)
    perm = np.array(info + parity)
    k = len(info)
    G = np.zeros((n, k), dtype=int)
    G[:k] = np.eye(k, dtype=int)
    for t, c in enumerate(parity):
        G[k + t] = A[piv_row[c], info]
    return np.asarray(H)[:, perm], G

