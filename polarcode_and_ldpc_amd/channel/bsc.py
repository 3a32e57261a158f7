"""Binary symmetric channel with the reference's API (src/channel/bsc.py:10-52).

`transmit` keeps the reference's exact host behaviour (NumPy global legacy
RNG); `transmit_batch_device` flips a whole batch on the GPU (pl_bsc, Philox
keyed by (seed, global frame, bit)) -- statistically equivalent, not
stream-identical."""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch


class BSCChannel:
    def __init__(self, crossover_prob: float, seed: int = None):
        assert 0 <= crossover_prob <= 1, "Crossover probability must be in [0, 1]"
        self.crossover_prob = crossover_prob
        if seed is not None:
            np.random.seed(seed)

    def transmit(self, bits: np.ndarray) -> np.ndarray:
        flip_mask = np.random.random(len(bits)) < self.crossover_prob
        output = bits.copy()
        output[flip_mask] = 1 - output[flip_mask]
        return output.astype(int)

    def transmit_batch_device(self, codewords: Optional[torch.Tensor], n: int, batch: int, seed: int,
                              frame_offset: int = 0, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """uint8 [batch, n] on the GPU: codewords (None = all-zero) with each bit
        flipped with probability crossover_prob."""
        from .. import _native
        _native.require_gpu()
        if out is None:
            out = torch.empty((batch, n), dtype=torch.uint8, device="cuda")
        if codewords is not None:
            assert codewords.dtype == torch.uint8 and codewords.shape == (batch, n) and codewords.is_contiguous()
        _native.bsc(codewords, n, batch, self.crossover_prob, seed, frame_offset, out)
        return out

    def __repr__(self) -> str:
        return f"BSCChannel(crossover_prob={self.crossover_prob})"
