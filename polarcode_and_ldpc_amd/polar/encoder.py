"""Polar encoder (host side NumPy, batch-capable) with the reference's API
(src/polar/encoder.py:12-126).  The device encoder used by the Monte-Carlo
source is pl_polar_encode (channel.hip)."""
from __future__ import annotations

from typing import Optional

import numpy as np

from .utils import crc_encode, generate_frozen_bits, polar_transform


class PolarEncoder:
    def __init__(self, N: int, K: int, frozen_bits: Optional[np.ndarray] = None,
                 use_crc: bool = False, crc_polynomial: str = "CRC-8"):
        assert N > 0 and (N & (N - 1)) == 0, "N must be a power of 2"
        assert 0 < K < N, "K must be in range (0, N)"
        self.N, self.K, self.n = N, K, int(np.log2(N))
        self.use_crc, self.crc_polynomial = use_crc, crc_polynomial
        if use_crc:
            self.crc_len = int(crc_polynomial.split("-")[1])
            assert K > self.crc_len, f"K must be greater than CRC length ({self.crc_len})"
            self.K_data = K - self.crc_len
        else:
            self.crc_len, self.K_data = 0, K
        if frozen_bits is None:
            self.frozen_bits, self.info_bits = generate_frozen_bits(N, K)
        else:
            self.frozen_bits = frozen_bits
            self.info_bits = np.setdiff1d(np.arange(N), frozen_bits)
            assert len(self.info_bits) == K, "Number of info bits must equal K"
        self.frozen_values = np.zeros(len(self.frozen_bits), dtype=int)

    def encode(self, message: np.ndarray) -> np.ndarray:
        if self.use_crc:
            assert len(message) == self.K_data, f"Message length must be {self.K_data}"
            message = crc_encode(message, self.crc_polynomial)
        else:
            assert len(message) == self.K, f"Message length must be {self.K}"
        return self.encode_batch(np.asarray(message)[None, :])[0]

    def encode_batch(self, messages: np.ndarray) -> np.ndarray:
        """messages [B, K] (CRC already appended if used) -> codewords [B, N]."""
        m = np.asarray(messages, dtype=np.int64)
        u = np.zeros((m.shape[0], self.N), dtype=np.int64)
        u[:, self.info_bits] = m
        return polar_transform(u)

    def get_info_bits_positions(self) -> np.ndarray:
        return self.info_bits.copy()

    def get_frozen_bits_positions(self) -> np.ndarray:
        return self.frozen_bits.copy()

    def get_code_rate(self) -> float:
        return self.K / self.N

    def __repr__(self) -> str:
        crc = f", CRC={self.crc_polynomial}" if self.use_crc else ""
        return f"PolarEncoder(N={self.N}, K={self.K}, rate={self.get_code_rate():.3f}{crc})"
