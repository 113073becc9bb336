"""Model families trained through the parameter server."""
from .fm import FMConfig, FMTrainer
from .sparse_lr import SparseLRConfig, SparseLRTrainer
from .wide_deep import WideDeepConfig, WideDeepTrainer

__all__ = ["SparseLRConfig", "SparseLRTrainer", "WideDeepConfig", "WideDeepTrainer", "FMConfig",
           "FMTrainer"]
