"""Channel models (src/channel/): AWGN, BSC, Rayleigh fading -- host methods as
the reference, plus device batch generators."""
from .awgn import AWGNChannel
from .bsc import BSCChannel
from .fading import RayleighFadingChannel

__all__ = ["AWGNChannel", "BSCChannel", "RayleighFadingChannel"]
