"""MarginLoss / SigmoidLoss of the repo (module/loss.py:5-53).

The reference's module/loss.py repeats OpenKE's loss classes class for class
(openke/module/loss/MarginLoss.py, SigmoidLoss.py: same constructors, get_weights, forward,
predict), so both import paths resolve to one implementation here: the OpenKE mirror, whose
MarginLoss is what the fused negative-sampling kernel (mmre.ns, csrc/ns.hip) evaluates and
differentiates when module/NegativeSampling.py trains through it."""
from openke.module.loss.MarginLoss import MarginLoss  # noqa: F401  (loss.py:5-28)
from openke.module.loss.SigmoidLoss import SigmoidLoss  # noqa: F401  (loss.py:30-53)

__all__ = ["MarginLoss", "SigmoidLoss"]
