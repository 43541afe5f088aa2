from .Tester import Tester
from .Trainer import Trainer

__all__ = ["Trainer", "Tester"]
