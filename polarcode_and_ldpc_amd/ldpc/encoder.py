"""LDPC encoder with the reference's API and outputs (src/ldpc/encoder.py:12-211).

Host side (it produces frames; it is not on the decode hot path).  The
reference's fallback for rank-deficient H, `_encode_direct` + `_solve_gf2`
(:97-187): Gaussian elimination picks its pivots from H2 alone, so all
right-hand sides share one elimination.
It is evaluated here for whole batches of messages at once (one elimination,
vectorised back-substitution) -- giving exactly the reference's
codewords, including the *invalid* ones it emits for the seed-42 (504, 252) H
(SURVEY.md §0 quirk 2), which is what benchmarks/throughput_test.py decodes.
`valid_generator` / `LDPCEncoder.encode_batch_device` add encoding into valid
codewords on the device (pl_gf2_encode).
"""
from __future__ import annotations

from typing import Optional

import numpy as np

from .matrix import generate_ldpc_matrix


def _systematic_generator(H: np.ndarray):
    """(G, P) or (None, None): src/ldpc/matrix.py:135-187 (GF(2) elimination on
    the last m columns)."""
    m, n = H.shape
    k = n - m
    W = (np.asarray(H) % 2).astype(np.uint8)
    for i in range(m):
        col = n - m + i
        nz = np.nonzero(W[i:, col])[0]
        if len(nz) == 0:
            return None, None
        p = i + nz[0]
        if p != i:
            W[[i, p]] = W[[p, i]]
        rows = np.nonzero(W[:, col])[0]
        rows = rows[rows != i]
        W[rows] ^= W[i]
    P = W[:, :k].astype(int)
    return np.hstack([np.eye(k, dtype=int), P.T]), P


def _solve_gf2_batch(A: np.ndarray, B: np.ndarray) -> np.ndarray:
    """The reference's _solve_gf2 (encoder.py:133-187) for many right-hand sides
    at once: A [m, n], B [m, r] -> X [n, r]."""
    m, n = A.shape
    aug = np.hstack([A.astype(np.uint8) & 1, B.astype(np.uint8) & 1])
    pivot_row = 0
    for col in range(n):
        if pivot_row >= m:
            break
        nz = np.nonzero(aug[pivot_row:, col])[0]
        if len(nz) == 0:
            continue
        p = pivot_row + nz[0]
        if p != pivot_row:
            aug[[pivot_row, p]] = aug[[p, pivot_row]]
        rows = np.nonzero(aug[:, col])[0]
        rows = rows[rows != pivot_row]
        aug[rows] ^= aug[pivot_row]
        pivot_row += 1
    # back-substitution exactly as the reference: x[i] = b ^ np.sum(a & x) with an
    # integer (not mod-2) sum, so x may leave {0, 1} (then so does the codeword)
    X = np.zeros((n, B.shape[1]), dtype=np.int64)
    for i in range(min(pivot_row, n) - 1, -1, -1):
        for row in range(i, m):
            if aug[row, i] == 1 and not aug[row, :i].any():
                X[i] = aug[row, n:].astype(np.int64) ^ (aug[row, i + 1:n, None].astype(np.int64) & X[i + 1:n]).sum(axis=0)
                break
    return X


def valid_generator(H: np.ndarray, k: Optional[int] = None):
    """A generator whose rows span the code of H: (G [k, n], info [k]).

    The reference's encoders (systematic G, or the direct-solving fallback for a
    rank-deficient H2, src/ldpc/encoder.py:56-131) emit non-codewords for the
    seed-42 (504, 252) H (rank 251, rank(H2) = 236).  Here H is brought to
    reduced row-echelon form over GF(2) with pivots taken from the right-most
    columns first (bit-packed rows, so n = 8192 takes seconds), the free columns
    carry the message -- the first k of them, as far left as possible, are the
    info positions `info` (codeword[info] = message; further free columns are
    0) -- and every pivot bit is the parity its reduced row prescribes.  H G^T =
    0 (mod 2) by construction.  k defaults to the code dimension n - rank(H).
    """
    Hb = (np.asarray(H) & 1).astype(np.uint8)
    m, n = Hb.shape
    nw = (n + 63) // 64
    W = np.zeros((m, nw * 64), np.uint8)
    W[:, :n] = Hb
    W = np.packbits(W.reshape(m, nw, 64)[:, :, ::-1], axis=2, bitorder="big").view(">u8")[:, :, 0].astype(np.uint64)
    # W[r, w] bit b = H[r, 64 w + b]
    pivots = []
    r = 0
    for c in range(n - 1, -1, -1):
        if r == m:
            break
        w, b = divmod(c, 64)
        col = (W[r:, w] >> np.uint64(b)) & np.uint64(1)
        nz = np.nonzero(col)[0]
        if len(nz) == 0:
            continue
        p = r + int(nz[0])
        if p != r:
            W[[r, p]] = W[[p, r]]
        hit = np.nonzero((W[:, w] >> np.uint64(b)) & np.uint64(1))[0]
        hit = hit[hit != r]
        W[hit] ^= W[r]
        pivots.append(c)
        r += 1
    R = ((W[:r, :, None] >> np.arange(64, dtype=np.uint64)[None, None, :]) & np.uint64(1)).astype(np.uint8)
    R = R.reshape(r, nw * 64)[:, :n]
    piv = np.array(pivots, dtype=np.int64)
    free = np.setdiff1d(np.arange(n), piv)
    kk = len(free) if k is None else int(k)
    if kk > len(free):
        raise ValueError("k = %d exceeds the code dimension %d" % (kk, len(free)))
    info = free[:kk]
    G = np.zeros((kk, n), dtype=np.uint8)
    G[np.arange(kk), info] = 1
    G[:, piv] = R[:, info].T
    return G, info


class LDPCEncoder:
    def __init__(self, n: int, k: int, H: Optional[np.ndarray] = None, G: Optional[np.ndarray] = None,
                 dv: int = 3, dc: int = 6, seed: Optional[int] = None):
        assert n > k > 0, "Invalid code parameters"
        self.n, self.k = n, k
        if H is None:
            self.m = n - k
            self.H = generate_ldpc_matrix(n, k, method="mackay", dv=dv, dc=dc, seed=seed)
        else:
            self.H = H
            assert H.shape[1] == n, f"H matrix must have {n} columns"
            self.m = H.shape[0]
            if n - self.m != k:  # encoder.py:50-51
                print(f"Warning: H implies k={n - self.m}, but k={k} was provided")
        if G is not None:
            if G.shape == (n, k):
                self.G = G.T
            elif G.shape == (k, n):
                self.G = G
            else:
                raise ValueError(f"G shape {G.shape} doesn't match (n,k)={n,k} or (k,n)={k,n}")
            self.P = None
            self.use_direct_solving = False
        else:
            self.G, self.P = _systematic_generator(self.H)
            self.use_direct_solving = self.G is None

    def encode(self, message: np.ndarray) -> np.ndarray:
        assert len(message) == self.k, f"Message length must be {self.k}"
        return self.encode_batch(np.asarray(message)[None, :])[0]

    def encode_batch(self, messages: np.ndarray) -> np.ndarray:
        msg = np.asarray(messages, dtype=np.int64) & 1
        if not self.use_direct_solving:
            return (msg @ self.G) % 2
        # _encode_direct (encoder.py:97-131): syndrome = H1 m mod 2, H2 p = syndrome
        syn = (msg @ (np.asarray(self.H[:, :self.k]).T)) % 2
        parity = _solve_gf2_batch(np.asarray(self.H[:, self.k:]), syn.T.astype(np.uint8)).T
        return np.hstack([msg, parity]).astype(int)

    # ---- valid codewords on the device (SURVEY §8 f row 3) -------------------
    def valid_generator(self):
        """(G [k, n], info positions [k]) of valid_generator(H, k), cached."""
        if getattr(self, "_valid", None) is None:
            self._valid = valid_generator(self.H, self.k)
        return self._valid

    @property
    def info_positions(self) -> np.ndarray:
        return self.valid_generator()[1]

    def encode_batch_device(self, messages, out=None):
        """Valid codewords for a batch of k-bit messages on the device
        (pl_gf2_encode): codeword[:, info_positions] = message.  messages: uint8
        [B, k] CUDA tensor or array; returns a uint8 [B, n] CUDA tensor."""
        import torch
        from .. import _native
        if getattr(self, "_g_dev", None) is None:
            G, _ = self.valid_generator()
            self._g_dev = torch.from_numpy(_native.pack_gf2_columns(G)).cuda()
        msg = messages if isinstance(messages, torch.Tensor) else torch.from_numpy(
            np.ascontiguousarray(np.asarray(messages), dtype=np.uint8))
        msg = msg.to(device="cuda", dtype=torch.uint8).contiguous()
        assert msg.dim() == 2 and msg.shape[1] == self.k, "messages must be [B, k]"
        cw = out if out is not None else torch.empty((msg.shape[0], self.n), dtype=torch.uint8, device="cuda")
        _native.gf2_encode(self._g_dev, self.k, self.n, msg, cw)
        return cw

    def _encode_direct(self, message: np.ndarray) -> np.ndarray:
        """One message through the direct-solving fallback (encoder.py:97-131)."""
        msg = np.asarray(message, dtype=np.int64) & 1
        syn = (np.asarray(self.H[:, :self.k]) @ msg) % 2
        return np.concatenate([msg, self._solve_gf2(np.asarray(self.H[:, self.k:]), syn)])

    def _solve_gf2(self, A: np.ndarray, b: np.ndarray) -> np.ndarray:
        """A x = b over GF(2) as the reference solves it (encoder.py:133-187)."""
        return _solve_gf2_batch(np.asarray(A), np.asarray(b).reshape(-1, 1))[:, 0]

    def verify_codeword(self, codeword: np.ndarray) -> bool:
        return bool(np.all((self.H @ codeword) % 2 == 0))

    def get_code_rate(self) -> float:
        """k / n (encoder.py:202-204)."""
        return self.k / self.n

    def get_parity_check_matrix(self) -> np.ndarray:
        """A copy of H (encoder.py:206-208)."""
        return self.H.copy()

    def __repr__(self) -> str:
        return f"LDPCEncoder(n={self.n}, k={self.k}, rate={self.get_code_rate():.3f})"
