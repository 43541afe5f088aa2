from .ComplEx import ComplEx
from .DistMult import DistMult
from .Model import Model
from .RotatE import RotatE
from .TransE import TransE

__all__ = ["Model", "TransE", "DistMult", "ComplEx", "RotatE"]
