"""Device ops: HIP kernels for gfx950 with host (C++ / PyTorch) reference paths."""
from .countmin import CountMinSketch
from .keymix import key_bits_for, mix, unmix
from .kv_table import InitRule, KVTable, UpdateRule
from .linear import (AUC_BINS, auc_from_hist, exact_auc, linear_backward, linear_forward,
                     linear_fwd_bwd)
from .localize import Localized, Localizer, localize_torch
from .native import core, hip_available, hipops

__all__ = [
    "CountMinSketch", "key_bits_for", "mix", "unmix", "InitRule", "KVTable", "UpdateRule",
    "AUC_BINS", "auc_from_hist", "exact_auc", "linear_backward", "linear_forward",
    "linear_fwd_bwd", "Localized",
    "Localizer", "localize_torch", "core", "hip_available", "hipops",
]
