from .NegativeSampling import NegativeSampling
from .Strategy import Strategy

__all__ = ["Strategy", "NegativeSampling"]
