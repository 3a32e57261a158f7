"""Channel models."""
from .awgn import AWGNChannel

__all__ = ["AWGNChannel"]
