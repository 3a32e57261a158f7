"""Offline substitutes for src/lib_wrappers (PolarLibWrapper over `polarcodes`,
LDPCLibWrapper over `pyldpc`): neither library is installed here and neither is
on the decoder hot path.  They keep the wrappers'
constructors and methods so benchmarks/ber_simulation.py-style scripts run:

* PolarLibWrapper(N, K, design_snr_db): frozen set = the bit-reversed
  Bhattacharyya construction at design_snr_db (construct_frozen_set), the
  offline stand-in for polarcodes' Construct(); encode/decode use this
  package's PolarEncoder / SCDecoder (GPU).
* LDPCLibWrapper(n, k, dv, dc, seed): regular (dv, dc) H (regular_construction,
  the structure pyldpc.make_ldpc builds) made systematic over GF(2)
  (gf2_systematic_pair): message = codeword[:k], k = n - rank(H), as pyldpc.

The sets/matrices are NOT those the third-party libraries would produce
(parity unpinned: the libraries are absent); results obtained through them are
comparable with each other, not with the reference's published library curves."""
from .ldpc_wrapper import LDPCLibWrapper
from .polar_wrapper import PolarLibWrapper

__all__ = ["PolarLibWrapper", "LDPCLibWrapper"]
