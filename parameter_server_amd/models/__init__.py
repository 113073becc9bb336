"""Model families trained through the parameter server."""
from .sparse_lr import SparseLRConfig, SparseLRTrainer

__all__ = ["SparseLRConfig", "SparseLRTrainer"]
