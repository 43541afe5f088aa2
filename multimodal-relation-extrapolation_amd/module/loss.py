"""MarginLoss / SigmoidLoss of the repo (module/loss.py:5-53); same API as the OpenKE ones."""
from openke.module.loss.MarginLoss import MarginLoss  # noqa: F401  (identical semantics, loss.py:5-28)
from openke.module.loss.SigmoidLoss import SigmoidLoss  # noqa: F401  (loss.py:30-53)
