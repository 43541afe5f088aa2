"""openke -- drop-in mirror of the OpenKE-PyTorch API used by the reference
(/root/reference/OpenKE/openke), with every hot op routed through libmmre_hip.so:

    from openke.config import Trainer, Tester
    from openke.module.model import TransE, DistMult, ComplEx, RotatE
    from openke.module.loss import MarginLoss, SigmoidLoss, SoftplusLoss
    from openke.module.strategy import NegativeSampling
    from openke.data import TrainDataLoader, TestDataLoader
"""
