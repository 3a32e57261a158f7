"""polarcode_and_ldpc_amd -- MI355X-native batched Polar SC/SCL and LDPC BP/Min-Sum
decoders (hand-written HIP kernels for gfx950 behind a C-ABI), drop-in for the
decoder hot path of B1ear/PolarCode_and_LDPC.

Importing a decoder module loads libpolarldpc.so; there is no CPU fallback.
"""
__version__ = "0.1.0"
