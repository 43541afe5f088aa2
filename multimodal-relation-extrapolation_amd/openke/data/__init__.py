from .TestDataLoader import TestDataLoader
from .TrainDataLoader import TrainDataLoader

__all__ = ["TrainDataLoader", "TestDataLoader"]
