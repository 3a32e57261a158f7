"""Rayleigh fading channel with the reference's API (src/channel/fading.py:10-66).

`transmit` keeps the reference's exact host behaviour (NumPy global legacy RNG);
`llr_batch_device` produces a batch of LLRs on the GPU (pl_rayleigh_llr) --
statistically equivalent, not stream-identical."""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch


class RayleighFadingChannel:
    def __init__(self, snr_db: float, seed: int = None):
        self.snr_db = snr_db
        self.snr_linear = 10 ** (snr_db / 10.0)
        self.noise_std = np.sqrt(1.0 / (2.0 * self.snr_linear))
        if seed is not None:
            np.random.seed(seed)

    def transmit(self, bits: np.ndarray, return_llr: bool = True) -> np.ndarray:
        symbols = 1.0 - 2.0 * bits.astype(float)
        h_real = np.random.normal(0, 1 / np.sqrt(2), len(symbols))
        h_imag = np.random.normal(0, 1 / np.sqrt(2), len(symbols))
        h_mag = np.abs(h_real + 1j * h_imag)
        received = h_mag * symbols + np.random.normal(0, self.noise_std, len(symbols))
        if return_llr:
            return 2.0 * received * h_mag / (self.noise_std ** 2)
        return (received <= 0).astype(int)

    def llr_batch_device(self, codewords: Optional[torch.Tensor], n: int, batch: int, seed: int,
                         frame_offset: int = 0, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        from .. import _native
        _native.require_gpu()
        if out is None:
            out = torch.empty((batch, n), dtype=torch.float64, device="cuda")
        if codewords is not None:
            assert codewords.dtype == torch.uint8 and codewords.shape == (batch, n) and codewords.is_contiguous()
        _native.rayleigh_llr(codewords, n, batch, self.snr_db, seed, frame_offset, out)
        return out

    def __repr__(self) -> str:
        return f"RayleighFadingChannel(SNR={self.snr_db:.2f}dB)"
