"""Drop-in BPDecoder / MSDecoder backed by the gfx950 HIP kernel (ldpc.hip).

Same constructors, attributes and `.decode(llr)` contract as the reference's
src/ldpc/decoder.py (BPDecoder :11-205, MSDecoder :208-355), plus
`decode_batch` for host or device batches.  No CPU path.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from .. import _native
from .matrix import dense_to_csr


class _LdpcBase:
    _algo = _native.PL_LDPC_BP
    normalization = 1.0

    def _setup(self, H, max_iter, early_stop):
        self.H = H
        self.m, self.n = H.shape
        self.max_iter = max_iter
        self.early_stop = early_stop
        self._row_ptr, self._col_idx = dense_to_csr(H)  # entries == 1, ascending (decoder.py:43-47)
        deg = np.diff(self._row_ptr)
        self.check_degrees = deg
        self.var_neighbors = None  # the reference's Python adjacency lists are not materialised
        self._plan = None

    @property
    def plan(self):
        if self._plan is None:
            self._plan = _native.ldpc_plan(self._row_ptr, self._col_idx, self.n, self._algo, self.max_iter,
                                           self.early_stop, self.normalization)
        return self._plan

    def _check_runnable(self):
        pass

    def _run(self, llr, out=None, iters=None):
        """Device batch: llr fp64 [B, n] -> (bits uint8 [B, n], iters int32 [B])."""
        self._check_runnable()
        B = llr.shape[0]
        if out is None:
            out = torch.empty((B, self.n), dtype=torch.uint8, device=llr.device)
        if iters is None:
            iters = torch.empty((B,), dtype=torch.int32, device=llr.device)
        if B > 0:
            self.plan.decode(llr, out, iters)
        return out, iters

    def decode_batch(self, llr, out: Optional[torch.Tensor] = None, return_iterations: bool = False):
        if isinstance(llr, torch.Tensor) and llr.is_cuda:
            assert llr.dim() == 2 and llr.shape[1] == self.n, "LLR length must be %d" % self.n
            if llr.dtype != torch.float64 or llr.stride(1) != 1:
                llr = llr.to(torch.float64).contiguous()
            bits, its = self._run(llr, out)
            return (bits, its) if return_iterations else bits
        a = np.asarray(llr.cpu().numpy() if isinstance(llr, torch.Tensor) else llr, dtype=np.float64)
        assert a.ndim == 2 and a.shape[1] == self.n, "LLR length must be %d" % self.n
        if a.shape[0] == 0:
            z = np.zeros((0, self.n), dtype=np.int64)
            return (z, np.zeros(0, dtype=np.int64)) if return_iterations else z
        _native.require_gpu()
        bits, its = self._run(torch.from_numpy(np.ascontiguousarray(a)).cuda())
        b = bits.cpu().numpy().astype(np.int64)
        return (b, its.cpu().numpy().astype(np.int64)) if return_iterations else b


class BPDecoder(_LdpcBase):
    """Flooding sum-product decoder (src/ldpc/decoder.py:11-205)."""

    def __init__(self, H: np.ndarray, max_iter: int = 50, early_stop: bool = True):
        self._algo = _native.PL_LDPC_BP
        self._setup(H, max_iter, early_stop)

    def decode(self, llr: np.ndarray, return_iterations: bool = False):
        assert len(llr) == self.n, f"LLR length must be {self.n}"
        bits, its = self.decode_batch(np.asarray(llr, dtype=np.float64)[None, :], return_iterations=True)
        if return_iterations:
            return bits[0], int(its[0])
        return bits[0]

    def __repr__(self) -> str:
        return f"BPDecoder(n={self.n}, m={self.m}, max_iter={self.max_iter})"


class MSDecoder(_LdpcBase):
    """(Normalised) min-sum decoder (src/ldpc/decoder.py:208-355)."""

    def __init__(self, H: np.ndarray, max_iter: int = 50, normalization: float = 1.0, early_stop: bool = True):
        self._algo = _native.PL_LDPC_MS
        self.normalization = normalization
        self._setup(H, max_iter, early_stop)

    def _check_runnable(self):
        # the reference evaluates np.min over the other inputs of every check;
        # a degree-1 check makes that an empty reduction (decoder.py:282)
        if self.max_iter > 0 and np.any(self.check_degrees == 1):
            raise ValueError("zero-size array to reduction operation minimum which has no identity")

    def decode(self, llr: np.ndarray) -> np.ndarray:
        assert len(llr) == self.n, f"LLR length must be {self.n}"
        return self.decode_batch(np.asarray(llr, dtype=np.float64)[None, :])[0]

    def __repr__(self) -> str:
        return f"MSDecoder(n={self.n}, m={self.m}, max_iter={self.max_iter}, norm={self.normalization})"
