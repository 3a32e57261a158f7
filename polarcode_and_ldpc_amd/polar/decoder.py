"""Drop-in SCDecoder / SCLDecoder backed by the gfx950 HIP kernels.

Same constructors, attributes and `.decode(llr)` contract as the reference's
src/polar/decoder.py (SCDecoder :12-173, SCLDecoder :176-444); adds
`decode_batch` (host or device arrays) for batched decoding.  All decoding runs
in libpolarldpc.so (polar_tree.hip / polar_lane.hip); there is no CPU path.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from .. import _native
from .utils import generate_frozen_bits


class _PolarBase:
    _list_size = 0  # 0 = SC

    def _setup(self, N: int, K: int, frozen_bits):
        assert N > 0 and (N & (N - 1)) == 0, "N must be a power of 2"
        assert 0 < K < N, "K must be in (0, N)"
        self.N = N
        self.K = K
        self.n = int(np.log2(N))
        if frozen_bits is None:
            self.frozen_bits, self.info_bits = generate_frozen_bits(N, K)
        else:
            self.frozen_bits = np.array(frozen_bits, dtype=int)
            self.info_bits = np.setdiff1d(np.arange(N), self.frozen_bits)
        self.frozen_set = set(self.frozen_bits.tolist())
        mask = np.zeros(N, dtype=np.uint8)
        mask[self.frozen_bits] = 1
        self._frozen_mask = mask
        self._n_info = int(len(self.info_bits))
        self._plan = None

    @property
    def plan(self):
        if self._plan is None and self._n_info > 0:
            self._plan = _native.polar_plan(self.N, self._n_info, self._frozen_mask, self._list_size)
        return self._plan

    def decode(self, llr_input: np.ndarray) -> np.ndarray:
        """Decode one frame: channel LLRs [N] -> info bits [K'] (int64, ascending
        info index), K' = len(info_bits)."""
        llr_input = np.asarray(llr_input, dtype=np.float64)
        assert llr_input.shape == (self.N,), f"expected LLR shape ({self.N},), got {llr_input.shape}"
        return self.decode_batch(llr_input[None, :])[0]

    def decode_batch(self, llr, out: Optional[torch.Tensor] = None):
        """Decode a batch of frames.

        llr: np.ndarray [B, N] -> returns np.ndarray int64 [B, K'];
             torch.Tensor float64 [B, N] on the GPU -> returns a torch.uint8
             [B, K'] device tensor (written into `out` when given), asynchronously
             on the current stream.
        """
        if isinstance(llr, torch.Tensor) and llr.is_cuda:
            assert llr.dim() == 2 and llr.shape[1] == self.N, "expected LLR shape (B, %d)" % self.N
            if llr.dtype != torch.float64 or llr.stride(1) != 1:
                llr = llr.to(torch.float64).contiguous()
            if out is None:
                out = torch.empty((llr.shape[0], self._n_info), dtype=torch.uint8, device=llr.device)
            if self._n_info > 0 and llr.shape[0] > 0:
                self.plan.decode(llr, out)
            return out
        a = np.asarray(llr.cpu().numpy() if isinstance(llr, torch.Tensor) else llr, dtype=np.float64)
        assert a.ndim == 2 and a.shape[1] == self.N, "expected LLR shape (B, %d), got %s" % (self.N, a.shape)
        if self._n_info == 0 or a.shape[0] == 0:
            return np.zeros((a.shape[0], self._n_info), dtype=np.int64)
        _native.require_gpu()
        dev = torch.from_numpy(np.ascontiguousarray(a)).cuda()
        res = self.decode_batch(dev)
        return res.cpu().numpy().astype(np.int64)


class SCDecoder(_PolarBase):
    """Successive-cancellation decoder (src/polar/decoder.py:12-173)."""

    def __init__(self, N: int, K: int, frozen_bits: Optional[np.ndarray] = None):
        self._list_size = 0
        self._setup(N, K, frozen_bits)

    def __repr__(self) -> str:
        return f"SCDecoder(N={self.N}, K={self.K})"


class SCLDecoder(_PolarBase):
    """Successive-cancellation list decoder (src/polar/decoder.py:176-444).

    `use_crc` / `crc_polynomial` are stored and, as in the reference, do not
    change the decision (the reference never reads them: decoder.py:202-203,
    :259); CA-SCL selection is a separate, build-defined extension."""

    def __init__(self, N: int, K: int, list_size: int = 8, frozen_bits: Optional[np.ndarray] = None,
                 use_crc: bool = False, crc_polynomial: str = "CRC-8"):
        assert list_size >= 1
        self._list_size = int(list_size)
        self._setup(N, K, frozen_bits)
        self.L = int(list_size)
        self.use_crc = use_crc
        self.crc_polynomial = crc_polynomial

    def __repr__(self) -> str:
        return f"SCLDecoder(N={self.N}, K={self.K}, L={self.L}, use_crc={self.use_crc})"


class CASCLDecoder(SCLDecoder):
    """CRC-aided SCL (build-defined extension; the
    reference's SCLDecoder stores use_crc but never applies it).

    The list is decoded exactly as SCLDecoder; the output is the first path, in
    descending final-metric order (ties: lower list index), whose u_hat[info]
    passes crc_check (src/polar/utils.py:128-163); if none does, the argmax path
    (= SCLDecoder's answer).  The K information bits carry the message followed
    by its CRC, as PolarEncoder(use_crc=True) lays them out (encoder.py:74-78)."""

    def __init__(self, N: int, K: int, list_size: int = 8, frozen_bits: Optional[np.ndarray] = None,
                 crc_polynomial: str = "CRC-8"):
        super().__init__(N, K, list_size, frozen_bits, use_crc=True, crc_polynomial=crc_polynomial)
        from .utils import CRC_POLYNOMIALS
        name = crc_polynomial if crc_polynomial in CRC_POLYNOMIALS else "CRC-8"  # utils.py:104-105
        self.crc_len = int(name.split("-")[1])
        assert K > self.crc_len, f"K must be greater than CRC length ({self.crc_len})"
        self.plan.set_crc(self.crc_len, CRC_POLYNOMIALS[name])

    def __repr__(self) -> str:
        return f"CASCLDecoder(N={self.N}, K={self.K}, L={self.L}, crc={self.crc_polynomial})"

