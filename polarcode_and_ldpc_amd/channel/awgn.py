"""AWGN channel with the reference's API (src/channel/awgn.py:11-140).

The per-frame host methods keep the reference's exact behaviour (NumPy global
legacy RNG, so a caller's random stream is unchanged).  `llr_batch_device`
generates a whole batch of LLRs on the GPU (pl_awgn_llr: Philox4x32-10 keyed by
(seed, global frame index) + Box-Muller) -- statistically equivalent to the
reference's np.random.normal, not stream-identical.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch


class AWGNChannel:
    def __init__(self, snr_db: float, seed: int = None):
        self.snr_db = snr_db
        self.snr_linear = 10 ** (snr_db / 10.0)
        self.noise_std = np.sqrt(1.0 / (2.0 * self.snr_linear))  # Es/N0, no rate term (awgn.py:27-32)
        if seed is not None:
            np.random.seed(seed)

    def modulate_bpsk(self, bits: np.ndarray) -> np.ndarray:
        return 1.0 - 2.0 * bits.astype(float)

    def demodulate_bpsk_hard(self, symbols: np.ndarray) -> np.ndarray:
        return (symbols <= 0).astype(int)

    def symbols_to_llr(self, symbols: np.ndarray) -> np.ndarray:
        return 2.0 * symbols / (self.noise_std ** 2)

    def add_noise(self, symbols: np.ndarray) -> np.ndarray:
        return symbols + np.random.normal(0, self.noise_std, symbols.shape)

    def transmit(self, bits: np.ndarray, return_llr: bool = True) -> np.ndarray:
        received = self.add_noise(self.modulate_bpsk(bits))
        return self.symbols_to_llr(received) if return_llr else self.demodulate_bpsk_hard(received)

    def get_capacity(self) -> float:
        return 1.0 - np.log2(1.0 + np.exp(-self.snr_linear))

    def update_snr(self, snr_db: float):
        self.snr_db = snr_db
        self.snr_linear = 10 ** (snr_db / 10.0)
        self.noise_std = np.sqrt(1.0 / (2.0 * self.snr_linear))

    # ---- device batch path -------------------------------------------------
    def llr_batch_device(self, codewords: Optional[torch.Tensor], n: int, batch: int, seed: int,
                         frame_offset: int = 0, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """LLRs [batch, n] fp64 on the GPU for uint8 codewords [batch, n] (None =
        all-zero codeword).  Frame b uses noise stream (seed, frame_offset + b)."""
        from .. import _native
        _native.require_gpu()
        if out is None:
            out = torch.empty((batch, n), dtype=torch.float64, device="cuda")
        if codewords is not None:
            assert codewords.dtype == torch.uint8 and codewords.shape == (batch, n) and codewords.is_contiguous()
        _native.awgn_llr(codewords, n, batch, self.snr_db, seed, frame_offset, out)
        return out

    def __repr__(self) -> str:
        return f"AWGNChannel(SNR={self.snr_db:.2f}dB, noise_std={self.noise_std:.4f})"
