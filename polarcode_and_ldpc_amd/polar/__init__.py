"""Polar codes: drop-in SC/SCL decoders (HIP) + host helpers."""
from .construction import (bhattacharyya_bounds, calculate_channel_capacities, construct_frozen_set,
                           construct_polar_code, gaussian_approximation)
from .decoder import CASCLDecoder, SCDecoder, SCLDecoder
from .encoder import PolarEncoder
from .utils import (bit_reverse, bit_reverse_array, crc_check, crc_encode, generate_frozen_bits, polar_transform,
                    polar_transform_iterative, polar_transform_recursive)

__all__ = ["SCDecoder", "SCLDecoder", "CASCLDecoder", "PolarEncoder", "construct_polar_code", "construct_frozen_set",
           "bhattacharyya_bounds", "gaussian_approximation", "calculate_channel_capacities", "generate_frozen_bits",
           "crc_encode", "crc_check", "bit_reverse", "bit_reverse_array", "polar_transform",
           "polar_transform_iterative", "polar_transform_recursive"]
