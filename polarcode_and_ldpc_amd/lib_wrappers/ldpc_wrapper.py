"""LDPCLibWrapper substitute (src/lib_wrappers/ldpc_wrapper.py:18-140); see __init__."""
from __future__ import annotations

from typing import Optional

import numpy as np

from ..ldpc.matrix import gf2_systematic_pair, regular_construction


class LDPCLibWrapper:
    def __init__(self, n: int, k: int, dv: int = 3, dc: int = 6, seed: Optional[int] = None):
        assert n > k > 0, "Invalid code parameters: n > k > 0 required"
        assert dc >= dv, "Check degree dc must be >= variable degree dv"
        self.n, self.dv, self.dc, self.seed = n, dv, dc, seed
        H0 = regular_construction(n, dv, dc, seed=0 if seed is None else seed)
        self.H, self.G = gf2_systematic_pair(H0)
        self.k_actual = self.G.shape[1]
        if self.k_actual != k:
            print(f"Warning: Requested k={k}, but the GF(2) rank of H gives k={self.k_actual}")
        self.k = self.k_actual
        self.m = self.H.shape[0]
        self._dec = None

    def encode(self, message: np.ndarray) -> np.ndarray:
        assert len(message) == self.k, f"Message length must be {self.k}"
        return (self.G @ np.asarray(message, dtype=int)) % 2

    def decode(self, llr: np.ndarray, max_iter: int = 50) -> np.ndarray:
        """Message estimate: BP hard decision, first k positions (systematic)."""
        from ..ldpc.decoder import BPDecoder
        if self._dec is None or self._dec.max_iter != max_iter:
            self._dec = BPDecoder(self.H, max_iter=max_iter)
        return self._dec.decode(llr)[:self.k]

    def get_parity_check_matrix(self) -> np.ndarray:
        return self.H.copy()

    def get_generator_matrix(self) -> np.ndarray:
        return self.G.copy()

    def get_code_rate(self) -> float:
        return self.k / self.n

    def __repr__(self) -> str:
        return f"LDPCLibWrapper(n={self.n}, k={self.k}, dv={self.dv}, dc={self.dc}, offline substitute)"
