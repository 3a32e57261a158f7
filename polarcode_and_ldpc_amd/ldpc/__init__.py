"""LDPC codes: drop-in BP / Min-Sum decoders (HIP) + parity-check matrices."""
from .decoder import BPDecoder, MSDecoder
from .encoder import LDPCEncoder, valid_generator
from .matrix import (calculate_girth, check_matrix_rank, create_systematic_generator, csr_to_dense, dense_to_csr,
                     generate_ldpc_matrix, gf2_systematic_pair, mackay_construction, peg_construction,
                     regular_construction)
from .utils import calculate_syndrome, check_syndrome, count_errors, create_tanner_graph, hamming_distance

__all__ = ["BPDecoder", "MSDecoder", "LDPCEncoder", "dense_to_csr", "csr_to_dense", "generate_ldpc_matrix",
           "mackay_construction", "regular_construction", "peg_construction", "create_systematic_generator",
           "check_matrix_rank", "calculate_girth", "gf2_systematic_pair", "create_tanner_graph", "check_syndrome",
           "calculate_syndrome", "count_errors", "hamming_distance"]
