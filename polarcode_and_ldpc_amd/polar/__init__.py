"""Polar codes: drop-in SC/SCL decoders (HIP) + host helpers."""
from .construction import bhattacharyya_bounds, construct_frozen_set, construct_polar_code
from .decoder import CASCLDecoder, SCDecoder, SCLDecoder
from .encoder import PolarEncoder
from .utils import bit_reverse, crc_check, crc_encode, generate_frozen_bits, polar_transform

__all__ = ["SCDecoder", "SCLDecoder", "CASCLDecoder", "PolarEncoder", "construct_polar_code", "construct_frozen_set",
           "bhattacharyya_bounds", "generate_frozen_bits", "crc_encode", "crc_check", "bit_reverse",
           "polar_transform"]
