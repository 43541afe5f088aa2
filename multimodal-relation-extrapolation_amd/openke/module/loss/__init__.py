from .Loss import Loss
from .MarginLoss import MarginLoss
from .SigmoidLoss import SigmoidLoss
from .SoftplusLoss import SoftplusLoss

__all__ = ["Loss", "MarginLoss", "SigmoidLoss", "SoftplusLoss"]
