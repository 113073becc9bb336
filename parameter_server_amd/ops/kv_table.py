"""HBM-resident open-addressing KV table for scalar linear models.

Python handle over the ``kv_*`` kernels (csrc/hip/kv_table.hip) with an
identical C++ host implementation (csrc/core/cpu_kernels.cc) for CPU tensors.
It is the MI355X-native replacement of the reference's per-server
``KVStore<Key, V, Entry, SGDState>`` (src/parameter/kv_store.h:28-80), whose
hash-map entries carry the optimizer (src/app/linear_method/async_sgd.h:71-124).

Slots are 32 bytes ``{u64 key | f32 w, z, n, acc | u32 cnt, flags}`` stored as an
``int64 [capacity, 4]`` tensor; keys are stored in the *mixed* key space.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from .native import core, hipops, is_gpu, ptr

EMPTY_KEY = -1  # 0xFFFF_FFFF_FFFF_FFFF as int64

ALGOS = {"sgd": 0, "standard": 0, "adagrad": 1, "ftrl": 2}
LR_TYPES = {"constant": 1, "decay": 2}
INIT_TYPES = {"zero": 0, "constant": 1, "gaussian": 2, "uniform": 3}


@dataclass
class UpdateRule:
    """Server-side per-key update (SGD / AdaGrad / FTRL-proximal with L1+L2).

    Mirrors reference LearningRate (learning_rate.h:15-22: CONSTANT=alpha,
    DECAY=alpha/(x+beta)) and ElasticNet::proximal (penalty.h:38-43).
    """

    algo: str = "ftrl"
    lr_type: str = "decay"
    alpha: float = 0.01
    beta: float = 10.0
    l1: float = 0.0
    l2: float = 0.0
    grad_scale: float = 1.0
    max_delta: float = 0.0

    def args(self):
        return (ALGOS[self.algo.lower()], LR_TYPES[self.lr_type.lower()], float(self.alpha),
                float(self.beta), float(self.l1), float(self.l2), float(self.grad_scale),
                float(self.max_delta))


@dataclass
class InitRule:
    """Reference ParameterInitConfig {ZERO, CONSTANT, GAUSSIAN, ...} (param.proto)."""

    type: str = "zero"
    value: float = 0.0
    std: float = 0.0
    seed: int = 0

    def args(self):
        return INIT_TYPES[self.type.lower()], float(self.value), float(self.std), int(self.seed) & ((1 << 64) - 1)


def next_pow2(x: int) -> int:
    return 1 << max(0, int(x - 1).bit_length())


class KVTable:
    def __init__(self, capacity: int, device="cpu", init: InitRule | None = None,
                 key_range: tuple[int, int] | None = None):
        """``key_range = (lo, hi)``: the (mixed) key range this shard owns; keys then get
        ORDERED home slots (see kv_table.hip home_slot) instead of hashed ones."""
        cap = next_pow2(max(64, int(capacity)))
        self.home_base, self.home_m = 0, 0
        self.key_range = (int(key_range[0]), int(key_range[1])) if key_range is not None else None
        if key_range is not None:
            lo, hi = int(key_range[0]), int(key_range[1])
            if hi > lo:
                self.home_base = lo
                self.home_m = ((1 << 64) - 1) // (hi - lo)
        self.capacity = cap
        self.device = torch.device(device)
        self.init = init or InitRule()
        self.slots = torch.empty((cap, 4), dtype=torch.int64, device=self.device)
        self.gpu = self.device.type == "cuda"
        if self.gpu:
            self._err = torch.zeros(1, dtype=torch.int32, device=self.device)
            # no per-wave insert counter on the hot path: one device atomic per wave on a
            # single address serialises (measured ~50 us of a 55 us resolve at 234k
            # keys); the occupancy comes from census() when it is needed
            self._inserted = None
            hipops().kv_init(self.slots)
        else:
            core().kv_init(ptr(self.slots), cap)
        self.num_inserted = 0  # host-side count (CPU path exact; GPU path lazily synced)

    # ------------------------------------------------------------------ pull
    def resolve(self, keys: torch.Tensor, insert: bool = True, with_w: bool = True,
                n_dev: torch.Tensor | None = None):
        """Lookup-or-insert mixed keys; returns (slot_idx int64, w float32 | None)."""
        keys = keys.contiguous()
        n = keys.numel()
        slot = torch.empty(n, dtype=torch.int64, device=keys.device)
        w = torch.empty(n, dtype=torch.float32, device=keys.device) if with_w else None
        it, iv, isd, seed = self.init.args()
        if self.gpu:
            hipops().kv_resolve(self.slots, keys, n_dev, slot, w, insert, it, iv, isd, seed,
                                self._err, self._inserted, self.home_base, self.home_m)
        else:
            ins, full = core().kv_resolve(ptr(self.slots), self.capacity, ptr(keys), n, ptr(slot),
                                          ptr(w), insert, it, iv, isd, seed, self.home_base,
                                          self.home_m)
            self.num_inserted += ins
            if full:
                raise RuntimeError("KVTable full: increase capacity")
        return slot, w

    def gather(self, slot_idx: torch.Tensor, field: int = 0, n_dev=None, out=None):
        n = slot_idx.numel()
        out = torch.empty(n, dtype=torch.float32, device=slot_idx.device) if out is None else out
        if self.gpu:
            hipops().kv_gather(self.slots, slot_idx, n_dev, out, field)
        else:
            core().kv_gather(ptr(self.slots), ptr(slot_idx), n, ptr(out), field)
        return out

    def set(self, slot_idx, w=None, z=None, n=None):
        if self.gpu:
            hipops().kv_set(self.slots, slot_idx, w, z, n)
        else:
            core().kv_set(ptr(self.slots), ptr(slot_idx), slot_idx.numel(), ptr(w), ptr(z), ptr(n))

    # ------------------------------------------------------------------ push
    def update(self, slot_idx: torch.Tensor, grad: torch.Tensor, rule: UpdateRule,
               stats: torch.Tensor | None = None, n_dev=None):
        """Apply one optimizer step per (unique-in-call) slot; stats += [dnnz, sum w^2, sum dw^2]."""
        if self.gpu:
            hipops().kv_update(self.slots, slot_idx, grad.contiguous(), n_dev, *rule.args(), stats)
        else:
            assert n_dev is None
            core().kv_update(ptr(self.slots), ptr(slot_idx), ptr(grad.contiguous()),
                             slot_idx.numel(), *rule.args(), ptr(stats))

    # ------------------------------------------------------------- inspection
    def census(self):
        """(occupied slots, nonzero weights)."""
        if self.gpu:
            c = hipops().kv_census(self.slots).cpu()
            return int(c[0]), int(c[1])
        return core().kv_census(ptr(self.slots), self.capacity)

    def check_ok(self):
        if self.gpu and int(self._err.item()) != 0:
            raise RuntimeError("KVTable full: increase capacity")

    def occupied(self, chunk: int = 1 << 27):
        """(mixed keys, w, z, n) of every occupied slot (device tensors). Scanned in
        chunks of slots: boolean-mask indexing over more than 2^31 elements overflows in
        torch, and a whole-table copy of a 2^31-slot table would take 32 GiB."""
        parts = []
        for a in range(0, self.capacity, chunk):
            sl = self.slots[a:a + chunk]
            keys = sl[:, 0]
            mask = keys != EMPTY_KEY
            vals = sl[:, 1:3].contiguous().view(torch.float32)  # w,z,n,acc
            parts.append((keys[mask], vals[mask, 0], vals[mask, 1], vals[mask, 2]))
        if len(parts) == 1:
            return parts[0]
        return tuple(torch.cat([p[i] for p in parts]) for i in range(4))

    def load(self, keys_mixed: torch.Tensor, w, z=None, n=None):
        slot, _ = self.resolve(keys_mixed.to(self.device), insert=True, with_w=False)
        self.set(slot, w.to(self.device).float().contiguous(),
                 None if z is None else z.to(self.device).float().contiguous(),
                 None if n is None else n.to(self.device).float().contiguous())
        self.check_ok()
        return slot

    def nbytes(self) -> int:
        return self.capacity * 32
