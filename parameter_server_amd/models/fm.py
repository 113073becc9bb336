"""Factorization machine on the sharded embedding table.

Reference: src/app/factor_machine/ — an unfinished sketch in the reference (the
worker pulls ``w`` with a tail filter and pushes the logistic gradient,
fm_worker.h:13-91; ``fm_server.h`` / ``fm_scheduler.h`` are missing and it is not
in the Makefile) plus the MATLAB model it was heading for (fm.m): second-order FM

    py = x.w + 1/2 sum_f [ (sum_i x_i v_if)^2 - sum_i x_i^2 v_if^2 ]

with logistic loss, L2 on w and V and AdaGrad on both. Here it is a complete
model on the same parameter-server machinery as wide & deep: a key owns a 32-B KV
slot (the linear weight ``w`` with its AdaGrad state) and a bf16 factor row ``v``
of k = ``embedding_dim`` at the same slot index (row-wise AdaGrad); one process per
GPU is a worker + shard; G > 1 pulls/pushes packed ``[v | w]`` records with one
all-to-all each way (``EmbeddingPS``).

Per step: localise -> pull rows + w -> expand X0 [B*S, k] -> ``fm_fwd_bwd`` (one
wavefront per example: s_f, q_f, margin, loss / accuracy / AUC, dX0 = p (x s - x^2
v)) -> per-key reduction of dX0 (CSC order) + L2 -> AdaGrad rows; wide gradient by
the sparse-LR segmented reduction -> AdaGrad (proximal L2) on w.
"""
from __future__ import annotations

import math
import time
from dataclasses import dataclass, field

import torch

from ..ops import embedding as E
from ..ops.keymix import key_bits_for
from ..ops.kv_table import UpdateRule, next_pow2
from ..ops.linear import AUC_BINS, accum_total, auc_from_hist, linear_backward, new_accum
from ..ops.localize import Localizer
from ..ops.native import hipops
from ..parallel.comm import Comm, LocalComm
from ..parallel.partition import KeyPartition
from .wide_deep import EmbeddingPS


@dataclass
class FMConfig:
    num_features: int = 10 ** 8
    embedding_dim: int = 16              # k (fm.m: 5; multiple of 8 for the row kernels)
    slots: int = 39                      # keys per example
    minibatch: int = 10000               # fm.m: m = 10000
    # eta_v (row-wise AdaGrad: the first step moves every coordinate by ~eta_v, and 741
    # slot pairs add up: .2 over-shoots; Criteo-shaped B = 16384, 50 steps: .2 -> loss
    # .613 AUC .741, .02 with eta_w = .05 -> .523 / .797, profiles/r3_train_sweep.log)
    emb_lr: float = 0.02
    emb_init_scale: float = 0.01         # sigma
    lambda_v: float = 10.0               # L2 on V (once per unique key and step, as fm.m)
    # linear weights: AdaGrad eta_w = .05 with L2 lambda_w = 1 (proximal form)
    wide: UpdateRule = field(default_factory=lambda: UpdateRule("adagrad", "constant", 0.05,
                                                                 1e-6, 0.0, 1.0))
    table_capacity: int = 0
    table_load: float = 0.5
    max_table_bytes: int = 96 << 30
    exchange: str = "padded"             # G > 1 on GPU: sync-free fixed rows | "exact"
    exchange_slack: float = 1.5
    exchange_capacity: int = 0
    compact_rows: bool = True            # 1 GPU: gather each unique key's row once per step
    # GPU key localisation (ops/localize.py): "sort" (deterministic order inside a key's
    # occurrence segment, so bitwise-reproducible gradient sums) or "part" (partition +
    # per-bucket LDS dedup, run order inside a segment set by atomics; B = 65536: 0.563
    # vs 0.587 ms / step, profiles/r2_asp_tail.log)
    localize: str = "sort"
    seed: int = 0


class FMTrainer(EmbeddingPS):
    def __init__(self, cfg: FMConfig, comm: Comm | None = None, device="cpu"):
        self.cfg = cfg
        self.comm = comm or LocalComm(device)
        self.G, self.rank = self.comm.world, self.comm.rank
        self.device = dev = torch.device(device)
        self.gpu = dev.type == "cuda"
        self.bits = key_bits_for(cfg.num_features)
        self.part = KeyPartition(self.bits, self.G)
        D, S, B = cfg.embedding_dim, cfg.slots, cfg.minibatch
        if D % 8 or D > 128:
            raise ValueError("embedding_dim must be a multiple of 8 and <= 128")
        per_slot = 32 + 2 * D + 5
        cap = cfg.table_capacity or next_pow2(int(math.ceil(cfg.num_features / self.G /
                                                            cfg.table_load)))
        cap = max(1024, min(cap, 1 << max(10, (cfg.max_table_bytes // per_slot).bit_length() - 1)))
        self.shard = E.EmbeddingShard(cap, D, dev, init_scale=cfg.emb_init_scale,
                                      seed=cfg.seed * 7919 + 17)
        self.max_nnz = B * S
        self.localizer = Localizer(self.max_nnz, self.bits, dev, mode=cfg.localize)
        self.coef = torch.empty(B, dtype=torch.float32, device=dev)
        self.metrics = new_accum(dev)
        self.stats = new_accum(dev)
        self.hist = torch.zeros(2 * AUC_BINS, dtype=torch.int32, device=dev)
        self.step_dev = torch.zeros(1, dtype=torch.int64, device=dev)
        if self.gpu:
            self.slot_buf = torch.empty(self.max_nnz, dtype=torch.int64, device=dev)
            self.w_buf = torch.empty(self.max_nnz, dtype=torch.float32, device=dev)
            self.dX0 = torch.empty(self.max_nnz, D, dtype=torch.bfloat16, device=dev)
            self.dE = torch.empty(self.max_nnz, D, dtype=torch.float32, device=dev)
            self.rows_u = torch.empty(self.max_nnz, D, dtype=torch.bfloat16, device=dev)
        self.step_count = 0
        self.examples = 0
        self.t0 = time.time()

    # ------------------------------------------------------------------ step
    def step(self, keys: torch.Tensor, labels: torch.Tensor, vals: torch.Tensor | None = None,
             loc=None):
        """One minibatch: ``keys`` [B*S] raw feature ids (row-major, S per example),
        ``labels`` [B] in {-1, +1} (or {0, 1}), optional feature values ``vals``."""
        cfg = self.cfg
        S, D = cfg.slots, cfg.embedding_dim
        B = labels.numel()
        nnz = B * S
        if keys.numel() != nnz:
            raise ValueError(f"expected {nnz} keys, got {keys.numel()}")
        loc = self.localizer(keys) if loc is None else loc
        if self.G == 1:
            if self.gpu:
                slot, w_wide = self.shard.resolve(loc.uniq, loc.n_uniq, self.slot_buf, self.w_buf)
            else:
                slot, w_wide = self.shard.resolve(loc.uniq[:loc.num_unique()])
            rows_src, rows_idx = self.shard.rows, slot
            if self.gpu and cfg.compact_rows:
                # each unique key's factor row gathered ONCE from the (huge, randomly
                # addressed) table into a compact L2-sized buffer; the per-occurrence
                # gathers of the forward then read that buffer
                hipops().emb_gather_rows(slot, self.shard.rows, self.rows_u, loc.n_uniq)
                rows_src, rows_idx = self.rows_u, None
            push = ("local", slot)
        else:
            rows_u, w_wide, push = self._pull(loc)
            rows_src, rows_idx = rows_u, None
        u_cap = nnz
        # narrow factors on the GPU: the forward gathers the rows itself (no [B*S, D] X0)
        gather = self.gpu and S <= 64 and D in (8, 16, 32)
        if not gather:
            X0 = E.expand(loc.local_col, nnz, rows_src, idx=rows_idx)
        if self.gpu:
            dX0 = self.dX0[:nnz]
            if gather:
                hipops().fm_fwd_bwd_gather(rows_src, rows_idx, vals, B, S, loc.local_col, w_wide,
                                           labels, self.coef, dX0, self.metrics, self.hist,
                                           AUC_BINS)
            else:
                hipops().fm_fwd_bwd(X0, vals, B, S, loc.local_col, w_wide, labels, self.coef,
                                    dX0, self.metrics, self.hist, AUC_BINS)
            dE = E.grad_reduce(loc, dX0, D, u_cap, out=self.dE)
            # pulled rows (G > 1) hold the U unique keys' rows only: no more than that
            l2_cap = u_cap if rows_idx is not None else min(u_cap, rows_src.shape[0])
            hipops().fm_l2(dE, rows_src, rows_idx, loc.n_uniq, l2_cap, cfg.lambda_v)
        else:
            dX0 = self._fwd_bwd_torch(X0, vals, B, S, loc.local_col, w_wide, labels)
            U = loc.num_unique()
            dE = E.grad_reduce(loc, dX0, D, U)
            v = (rows_src[rows_idx[:U]] if rows_idx is not None else rows_src[:U]).float()
            dE += cfg.lambda_v * v
        g_wide, _ = linear_backward(loc, self.coef[:B], B=B, width=S, vals=vals)
        self._push(loc, push, dE, g_wide)
        auc_from_hist(self.hist, self.metrics, self.step_dev)
        self.step_count += 1
        self.examples += B

    def _fwd_bwd_torch(self, X0, vals, B, S, local_col, w_wide, labels):
        """fm_fwd_bwd in PyTorch (CPU path and numerics reference)."""
        D = X0.shape[1]
        x = vals.float().reshape(B, S, 1) if vals is not None else torch.ones(B, S, 1)
        V = X0[:B * S].float().reshape(B, S, D)
        xv = x * V
        s = xv.sum(1)
        inter = 0.5 * (s * s - (xv * xv).sum(1)).sum(1)
        lc = local_col[:B * S].long().reshape(B, S)
        m = (w_wide[lc] * x[..., 0]).sum(1) + inter
        y = torch.where(labels[:B] > 0, 1.0, -1.0)
        ym = y * m
        c = -y * torch.sigmoid(-ym)
        self.coef[:B] = c
        dX = c[:, None, None] * (x * s[:, None, :] - x * x * V)
        self.metrics[0] += torch.nn.functional.softplus(-ym).double().sum()
        self.metrics[1] += ((y > 0) == (m > 0)).double().sum()
        self.metrics[2] += B
        nb = AUC_BINS
        pb = torch.clamp((torch.sigmoid(m) * nb).long(), 0, nb - 1)
        self.hist += torch.bincount(pb + torch.where(y > 0, nb, 0), minlength=2 * nb).to(
            self.hist.dtype)
        return dX.reshape(B * S, D).to(torch.bfloat16)

    # ------------------------------------------------------------------ eval
    def predict(self, keys: torch.Tensor, B: int) -> torch.Tensor:
        """Margins of B examples (no update; unseen keys contribute 0). G == 1."""
        if self.G != 1:
            raise NotImplementedError("predict() reads the local shard (G == 1)")
        from ..ops.keymix import mix

        S, D = self.cfg.slots, self.cfg.embedding_dim
        mk = mix(keys.to(self.device), self.bits)
        slot, w = self.shard.table.resolve(mk, insert=False)
        ok = slot >= 0
        V = torch.zeros(mk.numel(), D, device=self.device)
        V[ok] = self.shard.rows[slot[ok]].float()
        w = torch.where(ok, w, torch.zeros_like(w))
        V = V.reshape(B, S, D)
        s = V.sum(1)
        return w.reshape(B, S).sum(1) + 0.5 * (s * s - (V * V).sum(1)).sum(1)

    def progress(self, reset: bool = True) -> dict:
        self._xe_check()
        m = accum_total(self.metrics)[:8].clone()
        if self.G > 1:
            m = self.comm.all_reduce_(m.to(self.comm.device) if self.comm.backend == "nccl"
                                      else m.cpu())
        m = m.cpu()
        n = max(float(m[2]), 1.0)
        out = {"examples": float(m[2]), "loss": float(m[0]) / n,
               "accuracy": max(float(m[1]) / n, 1 - float(m[1]) / n) if m[2] > 0 else 0.0,
               "auc": float(m[3]) / max(float(m[4]), 1.0)}
        if reset:
            self.metrics.zero_()
        return out
