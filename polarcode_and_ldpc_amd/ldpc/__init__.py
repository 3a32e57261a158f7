"""LDPC codes: drop-in BP / Min-Sum decoders (HIP) + parity-check matrices."""
from .decoder import BPDecoder, MSDecoder
from .encoder import LDPCEncoder
from .matrix import (csr_to_dense, dense_to_csr, generate_ldpc_matrix, mackay_construction,
                     regular_construction)

__all__ = ["BPDecoder", "MSDecoder", "LDPCEncoder", "dense_to_csr", "csr_to_dense", "generate_ldpc_matrix",
           "mackay_construction", "regular_construction"]
