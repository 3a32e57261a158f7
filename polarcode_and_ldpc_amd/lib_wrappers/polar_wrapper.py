"""PolarLibWrapper substitute (src/lib_wrappers/polar_wrapper.py:18-120); see __init__."""
from __future__ import annotations

import numpy as np

from ..polar.construction import construct_frozen_set
from ..polar.encoder import PolarEncoder


class PolarLibWrapper:
    def __init__(self, N: int, K: int, design_snr_db: float = 2.0):
        assert N > 0 and (N & (N - 1)) == 0, "N must be a power of 2"
        assert 0 < K < N, "K must be in (0, N)"
        self.N, self.K, self.design_snr_db = N, K, design_snr_db
        self.frozen_bits = construct_frozen_set(N, K, design_snr_db)
        self.info_bits = np.setdiff1d(np.arange(N), self.frozen_bits)
        self._enc = PolarEncoder(N, K, frozen_bits=self.frozen_bits)
        self._dec = None

    def encode(self, message: np.ndarray) -> np.ndarray:
        assert len(message) == self.K, f"Message length must be {self.K}"
        return self._enc.encode(np.asarray(message))

    def decode(self, llr: np.ndarray) -> np.ndarray:
        if self._dec is None:
            from ..polar.decoder import SCDecoder
            self._dec = SCDecoder(self.N, self.K, frozen_bits=self.frozen_bits)
        return self._dec.decode(llr)

    def get_code_rate(self) -> float:
        return self.K / self.N

    def get_frozen_bits_positions(self) -> np.ndarray:
        return self.frozen_bits.copy()

    def get_info_bits_positions(self) -> np.ndarray:
        return self.info_bits.copy()

    def __repr__(self) -> str:
        return f"PolarLibWrapper(N={self.N}, K={self.K}, design_snr={self.design_snr_db}dB, offline substitute)"
