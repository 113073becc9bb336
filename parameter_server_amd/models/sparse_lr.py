"""Sparse logistic regression trained through the sharded HBM parameter server.

This is the MI355X-native counterpart of the reference's async-SGD linear
method (src/app/linear_method/async_sgd.h: AsyncSGDWorker::computeGradient
:241-289 and AsyncSGDServer with FTRL/SGD/AdaGrad entries :101-178,
MinibatchReader::read src/learner/sgd.h:131-150). One process per GPU; every
rank is a colocated worker (data shard ``rank``) and server shard (key range
``rank`` of the mixed key space).

One training step on a rank (all on the GPU, no host round trip when G == 1):
  localise      mix -> radix sort -> RLE  (unique keys, local cols, CSC order)
  [tail filter] CountMin insert/query of per-key counts, drop rare keys
  pull          G == 1: lookup-or-insert in the local HBM table;
                G  > 1 (exchange="padded", default): keys are sorted by owner ->
                fixed-capacity row per peer [keys(t) | grads(t-1)] with the
                counts in the row header -> equal-split all-to-all -> owner applies
                the pushes of t-1, then resolves the pulls of t -> all-to-all of
                weights. No host sync, so the step replays from HIP graphs between
                the two collectives (exchange="exact": count all-gather + sized
                all-to-all-v, one host sync per step)
  forward       Xw, loss, dL/dXw, accuracy, AUC histogram (one kernel)
  backward      segmented reduction over the CSC order -> grad per unique key
  push          G == 1: optimizer update at the cached slots (key caching: the
                push never re-sends or re-hashes keys);
                G  > 1: gradients ride the next step's exchange [FixingFloat nb-byte
                codes] -> owner applies one optimizer step per source row in rank
                order (reference semantics: one FTRL step per push message) or
                sums them first (``push_mode='aggregate'``, synchronous SGD).
"""
from __future__ import annotations

import math
import os
import time
from dataclasses import dataclass, field

import torch

from ..ops import fixing_float as ff
from ..ops.countmin import CountMinSketch
from ..ops.keymix import key_bits_for, unmix
from ..ops.kv_table import InitRule, KVTable, UpdateRule, next_pow2
from ..ops.linear import (AUC_BINS, HIST_STRIPES, accum_total, auc_from_hist, fused_update_ok,
                          linear_fwd_bwd, loss_id, new_accum)
from ..ops.localize import Localizer
from ..ops.native import hipops
from ..parallel.comm import Comm, LocalComm
from ..parallel.consistency import ExchangeSchedule, MergedSchedule, parse_consistency
from ..parallel.partition import KeyPartition
from ..utils.trace import enabled as trace_enabled
from ..utils.trace import trace_range


# tp_fwd_bwd_csr encodes an occurrence's row as its offset from the tile's first row in 19
# bits: minibatches of this many rows or more take the compact path
_CSR_MAX_ROWS = (1 << 19) - 1


def _same_workspace(a, b) -> bool:
    """Two localisations share device workspaces (the same Localizer buffer set)."""
    if a is b:
        return True
    ua, ub = getattr(a, "uniq", None), getattr(b, "uniq", None)
    return (isinstance(ua, torch.Tensor) and isinstance(ub, torch.Tensor) and ua.numel() > 0
            and ua.device == ub.device and ua.data_ptr() == ub.data_ptr())


@dataclass
class SparseLRConfig:
    num_features: int = 10 ** 9          # hashed feature space (keys in [0, N)); 0 = raw u64
    minibatch: int = 10000               # examples per worker step (reference SGDConfig.minibatch)
    max_nnz_per_example: int = 39
    loss: str = "logit"
    algo: str = "ftrl"                   # ftrl | adagrad | sgd
    lr_type: str = "decay"               # constant | decay
    alpha: float = 0.01
    beta: float = 10.0
    l1: float = 10.0
    l2: float = 1.0
    grad_scale: float = 1.0
    max_delta: float = 0.0               # per-update |dw| clip (trust region), 0 = off
    table_capacity: int = 0              # slots per shard (power of 2); 0 = auto
    table_load: float = 0.5              # auto capacity = num_features / G / load
    max_table_bytes: int = 96 << 30      # cap for the auto size (per GPU)
    init: InitRule = field(default_factory=InitRule)
    # ssp (lag >= 1) owner apply of the carried pushes: "post" = after the exchange's
    # pulls are resolved and the weights sent back (off the worker's critical path),
    # "pre" = before resolving them; same visibility (parallel/consistency.py)
    ssp_apply: str = "post"
    tail_feature_freq: int = 0           # keep keys seen > freq times (0 = off)
    countmin_n: float = 1e8
    countmin_k: int = 2
    consistency: str = "bsp"             # bsp | ssp:<tau> | asp
    push_mode: str = "sequential"        # sequential | aggregate
    localize: str = "auto"               # auto (= tp where supported, else sort) | tp | sort |
                                         # part (tp: <= 34-bit keys, part: <= 32-bit keys)
    fixing_float_bytes: int = 0          # 0 = off, else 1..7 bytes per pushed gradient
    # multi-GPU data plane: "padded" = fixed-capacity rows per peer with device-side
    # counts (no host sync, graph-replayable); "exact" = count exchange + sized
    # all-to-all-v (one host sync per step); "p2p" = one-sided peer-HBM pulls and
    # inbox pushes, no collective per step (asynchronous only, parallel/p2p.py)
    exchange: str = "padded"
    p2p_queue: int = 16                  # p2p: inbox entries per source (staleness bound)
    p2p_rounds: int = 2                  # p2p: inbox entries applied per source per step
    exchange_capacity: int = 0           # keys per peer per step; 0 = auto (first step)
    exchange_slack: float = 1.5          # auto capacity = slack * max per-peer count + 1024
    # padded exchange pipelining depth: pushes of step t ride the exchange of step
    # t + 1 + lag, so the exchanges of steps t+1 .. t+lag can run while step t
    # computes; the pull of step t then misses exactly the `lag` most recent steps of
    # pushes. -1 = from `consistency` (bsp -> 0, ssp:tau -> tau, asp -> 1)
    exchange_lag: int = -1
    asp_depth: int = 4                   # asp: exchanges whose push applies may be in flight
    # padded exchange with lag >= 1: ONE all-to-all per step carrying [keys(t+1) |
    # grads(t-d) | weights of keys(t)] (parallel/consistency.MergedSchedule) instead of
    # two (keys + grads, then weights). "auto": on for ssp:tau >= 2; "on" also for
    # ssp:1 (worker and exchange then serialise) and asp (staleness exactly 3); "off":
    # two collectives
    exchange_merge: str = "auto"
    seed: int = 0

    def update_rule(self) -> UpdateRule:
        return UpdateRule(self.algo, self.lr_type, self.alpha, self.beta, self.l1, self.l2,
                          self.grad_scale, self.max_delta)


# Per-algorithm server defaults for the pushed minibatch-SUM gradients (the reference's
# push format, async_sgd.h:263-289). FTRL-proximal is the reference CTR online config
# (example/linear/ctr/online_l1lr.conf: L1 10 / L2 1, DECAY alpha .01 beta 10). AdaGrad
# normalises by the accumulated gradient norm like FTRL, so the same step trains. Plain
# SGD takes the raw minibatch sum: a hot key's gradient is ~B x larger than a rare
# key's, and with G workers an owner applies up to G pushes of a key per step, so its
# step is 30x smaller (benchmarks/train_check.py, 65,536 x 39 Criteo-shaped, 50 steps:
# alpha .01 diverges at 1 GPU (loss 4.7); .001 trains at 1 GPU (0.556) but diverges with
# 8 asynchronous peers + 2-byte fixing-float (2.56); .0003 trains there (0.621, AUC .734);
# profiles/r3_train_sweep.log).
ALGO_DEFAULTS = {
    "ftrl": dict(lr_type="decay", alpha=0.01, beta=10.0, l1=10.0, l2=1.0, grad_scale=1.0,
                 max_delta=0.0),
    "adagrad": dict(lr_type="decay", alpha=0.01, beta=10.0, l1=10.0, l2=1.0, grad_scale=1.0,
                    max_delta=0.0),
    "sgd": dict(lr_type="decay", alpha=0.0003, beta=10.0, l1=10.0, l2=1.0, grad_scale=1.0,
                max_delta=0.0),
}


def algo_defaults(algo: str) -> dict:
    return dict(ALGO_DEFAULTS[algo.lower()])


class SparseLRTrainer:
    def __init__(self, cfg: SparseLRConfig, comm: Comm | None = None, device="cpu"):
        self.cfg = cfg
        self.comm = comm or LocalComm(device)
        self.G, self.rank = self.comm.world, self.comm.rank
        self.device = torch.device(device)
        self.gpu = self.device.type == "cuda"
        self.bits = key_bits_for(cfg.num_features)
        self.part = KeyPartition(self.bits, self.G)
        self.rule = cfg.update_rule()
        self.tau = parse_consistency(cfg.consistency)
        cap = cfg.table_capacity or self.auto_capacity(cfg, self.G, self.bits)
        # ordered home slots over this shard's mixed-key range: sorted unique keys then
        # walk the (up to 64 GB) table in increasing address order
        # (the loopback emulation's one rank owns every peer's range: order over all)
        self._loopback = getattr(self.comm, "backend", "") == "loopback"
        rng = ((self.part.range_of(0)[0], self.part.range_of(self.G - 1)[1]) if self._loopback
               else self.part.range_of(self.rank))
        self.table = KVTable(cap, self.device, cfg.init, key_range=rng)
        self.max_nnz = cfg.minibatch * cfg.max_nnz_per_example
        # tail filter (reference MinibatchReader::read, sgd.h:131-150): a CountMin sketch
        # partitioned by mixed-key range (ops/countmin.py), so the flat localiser's bucket
        # workgroups insert and query it inside their own launch
        self.filter = (CountMinSketch(int(cfg.countmin_n), cfg.countmin_k, self.device,
                                      key_bits=self.bits)
                       if cfg.tail_feature_freq > 0 else None)
        # 1 GPU: entry scan + optimizer update fused (PSAMD_FUSED_UPDATE=0: scan, then
        # kv_update); read once, not per step (host issue time)
        self._fused_update = os.environ.get("PSAMD_FUSED_UPDATE", "1") != "0"
        self._use_plans = os.environ.get("PSAMD_STEP_PLAN", "1") != "0"
        mode = cfg.localize
        # the flat layout (Localizer "tpf": fixed per-bucket regions, ops/localize.FlatLoc):
        # 1 GPU: the step's pull fused into the previous step's update (tpf_step); G > 1
        # on the padded exchange: owner rows packed straight from the bucket regions (G a
        # power of two dividing the bucket groups, tpf_exchange_ok). PSAMD_FLAT=0: "tp"
        flat_env = os.environ.get("PSAMD_FLAT", "1") != "0"
        self._flat_x = False  # G > 1: the padded exchange on the flat layout
        # (the tail filter runs inside the flat bucket kernel: tpf_filter_unit)
        if self.G == 1:
            flat_ok = self.gpu and self._fused_update and self._use_plans and flat_env
        else:
            flat_ok = self._flat_x = bool(
                self.gpu and flat_env and cfg.exchange == "padded"
                and self.bits <= 34 and hipops().tploc_supported(self.max_nnz, self.bits)
                and hipops().tpf_exchange_ok(self.max_nnz, self.bits, self.G))
        if mode == "auto":  # tile dedup + key-range buckets (Localizer falls back to sort
            mode = "tpf" if flat_ok else "tp"  # for > 34-bit keys or > 5.2 M keys)
        if mode == "tpf" and not flat_ok:
            mode = "tp"
        self._flat_x = self._flat_x and mode == "tpf"
        if cfg.tail_feature_freq > 0 and mode == "tp":
            mode = "sort"  # the tail filter needs per-key nnz counts (seg_start over nnz)
        # local columns on demand: the fused tp forward/backward reads the entry map
        self.localizer = self._new_localizer(mode)
        self.localize_mode = self.localizer.mode  # after the Localizer's fallbacks
        self._localizers = [self.localizer]  # + a second buffer set for prefetching (G > 1)
        self._compact = None  # flat mode: a "tp" Localizer for steps the flat path cannot run
        # flat mode: (id, generation) of the FlatLoc whose pull the previous step issued
        # ahead (fused into its update launch); valid for the very next step only
        self._pre = None
        dev = self.device
        self.metrics = new_accum(dev)  # [loss, correct, n, auc_sum, auc_n, ...] (striped)
        self.stats = new_accum(dev)    # [nnz delta, sum w^2, sum dw^2] (striped)
        self.hist = torch.zeros(HIST_STRIPES * 2 * AUC_BINS, dtype=torch.int32, device=dev)
        self.coef = torch.empty(cfg.minibatch, dtype=torch.float32, device=dev)
        self.step_dev = torch.zeros(1, dtype=torch.int64, device=dev)  # device step clock
        if self.gpu:
            self.slot_buf = torch.empty(self.max_nnz, dtype=torch.int64, device=dev)
            self.w_buf = torch.empty(self.max_nnz, dtype=torch.float32, device=dev)
            self.touched = None
        # multi-GPU: fuse push(t-1) into the pull exchange of step t (2 all-to-alls/step)
        if cfg.exchange not in ("padded", "exact", "p2p"):
            raise ValueError(f"exchange must be 'padded', 'exact' or 'p2p', not {cfg.exchange!r}")
        self.p2p = self.G > 1 and cfg.exchange == "p2p"
        if self.p2p and (not self.gpu or self.filter is not None
                         or cfg.push_mode == "aggregate" or not math.isinf(self.tau)):
            raise ValueError("exchange='p2p' is the asynchronous GPU data plane: consistency "
                             "'asp', no tail filter, sequential pushes")
        self.px = None  # PeerExchange (p2p, set up on the first step)
        self.padded = self.G > 1 and cfg.exchange == "padded"
        self.fused = (self.G > 1 and self.filter is None and cfg.fixing_float_bytes == 0
                      and not self.padded and not self.p2p)
        self.xc = None  # padded-exchange state (allocated on the first step)
        # consistency on the padded exchange: the pushes of step t ride exchange t+1+lag
        # and are applied before its pulls, so the pull of step t sees exactly the
        # pushes of steps <= t-1-lag (bsp: lag 0; ssp:tau: lag tau). asp: lag 1 and the
        # owner applies pushes on their own stream, which later pulls do not wait for
        # (only buffer reuse bounds it: async_depth exchanges in flight).
        self.sched = ExchangeSchedule(self.tau, cfg.exchange_lag, cfg.asp_depth,
                                      post=cfg.ssp_apply == "post")
        self.lag, self.asp, self.async_depth = self.sched.lag, self.sched.asp, self.sched.depth
        # rings of R exchange buffers indexed by step (>= 2: the exchange of step t+1
        # runs while the worker half of step t still reads its weights)
        self.R = self.sched.R
        if cfg.exchange_merge not in ("auto", "on", "off"):
            raise ValueError(f"exchange_merge must be auto / on / off, not {cfg.exchange_merge!r}")
        # (auto: ssp:tau >= 2, and asp for FTRL / AdaGrad, served on the merged exchange
        # with staleness exactly 3 (an admissible asp schedule; both train there at 8
        # emulated peers + fixing-float, tests/test_train_quality_gpu.py; config 4 FTRL FF 1 B
        # 0.1299 -> 0.1205 ms, profiles/r6_asp_merged.log). Plain SGD diverged at
        # staleness 3 (loss 1.03 after 50 steps) and at staleness 2 the merged exchange
        # serialises with the worker (0.143 vs 0.130 ms): asp SGD keeps the two-collective
        # exchange, whose owner applies run beside the pulls)
        asp_merge = math.isinf(self.tau) and cfg.algo.lower() in ("ftrl", "adagrad")
        self.merged = bool(
            self.padded and cfg.exchange_merge != "off"
            and self.tau > 0 and (cfg.exchange_merge == "on" or asp_merge
                                  or (not math.isinf(self.tau) and self.tau >= 2)))
        self.msched = None
        if self.merged:  # one collective per step (MergedSchedule)
            self.msched = MergedSchedule(self.tau, cfg.exchange_lag)
            self.lag, self.asp, self.async_depth = self.msched.lag, False, 0
            self.R = self.msched.R
        self._mx_pend = None      # sequential API: the minibatch whose worker half is due
        self._mx_next = None      # index of the next merged exchange (None: bootstrap due)
        self._mx_external = False  # exchanges issued by a caller's pipeline (bench.py)
        self._xt = 0  # padded steps computed (worker halves run)
        self._xx = 0  # padded exchanges issued (exchange halves run)
        self.pending = None
        self._prefetch = None
        self._coef_views = {}  # B -> self.coef[:B]
        self._plans = {}  # 1 GPU: native launch lists of the fused step (_step_plan)
        self.step_count = 0
        self.examples = 0
        self.comm_bytes = 0
        self.t0 = time.time()

    def prefill(self, count: int, chunk: int = 1 << 24, seed: int = 12345) -> int:
        """Insert ``count`` random keys of this shard's mixed-key range (zero state), so
        a benchmark can measure the populated-table regime (probe lengths, TLB / DRAM
        page behaviour of a large table) instead of an almost empty one. Returns the
        occupied slots afterwards. (Reference: KVStore grows its hash map with every
        new key, src/parameter/kv_store.h:37-57.)"""
        from ..ops.keymix import random_keys_in_range

        self._pre = None  # (a pull issued ahead would miss nothing here, but stay strict)
        # the table's own key range (the loopback emulation's one rank owns all G ranges)
        lo, hi = self.table.key_range or self.part.range_of(self.rank)
        g = torch.Generator(device=self.device).manual_seed(seed + self.rank)
        done = 0
        while done < count:
            n = min(chunk, count - done)
            mk = random_keys_in_range(lo, hi, n, g, self.device)
            self.table.resolve(mk, insert=True, with_w=False)
            done += n
        self.table.check_ok()
        return self.table.census()[0]

    @staticmethod
    def auto_capacity(cfg: SparseLRConfig, G: int, bits: int) -> int:
        n = cfg.num_features if cfg.num_features else (1 << 27)
        want = next_pow2(int(math.ceil(n / G / cfg.table_load)))
        cap_max = 1 << max(6, (cfg.max_table_bytes // 32).bit_length() - 1)
        return max(1024, min(want, cap_max))

    # ------------------------------------------------------------------ step
    def localize(self, keys: torch.Tensor, buf: int = 0, stage: int = 0):
        """Localise a minibatch into buffer set ``buf`` (0 or 1). Used to prefetch the
        next minibatch on a side stream while the current step waits for its
        exchange (``step(..., loc=..., prefetch=...)``). ``stage`` (flat layout + tail
        filter): 4 = tile + bucket, 3 = the filter (``Localizer``)."""
        while len(self._localizers) <= buf:
            self._localizers.append(self._new_localizer(self.localize_mode))
        return self._localizers[buf](keys, stage) if stage else self._localizers[buf](keys)

    def _new_localizer(self, mode: str) -> Localizer:
        """A localisation workspace of this trainer (flat: with the fused tail filter)."""
        tf = ((self.filter, self.cfg.tail_feature_freq)
              if self.filter is not None and mode == "tpf" else None)
        return Localizer(self.max_nnz, self.bits, self.device, mode=mode, lazy_cols=True,
                         sorted_keys=self._flat_x if mode == "tpf" else False, tail_filter=tf)

    def step(self, keys: torch.Tensor, labels: torch.Tensor, *, width: int | None = None,
             row_ptr: torch.Tensor | None = None, vals: torch.Tensor | None = None,
             rows: torch.Tensor | None = None, loc=None, prefetch=None, next_loc=None):
        """One minibatch: pull, forward, backward, push. ``keys`` are raw feature ids
        in CSR order (fixed ``width`` per row, or ``row_ptr``). ``loc``: an already
        localised minibatch (``localize``); ``prefetch``: called once the step's
        exchange counts are in flight and before the step blocks on them (multi-GPU),
        so the caller can enqueue the next minibatch's work on another stream.
        ``next_loc`` (1 GPU, flat layout): the NEXT minibatch, already localised; its
        pull runs in this step's update launch (after the update, in the same
        workgroups), and the next ``step(loc=next_loc)`` skips its own pull. The table
        is fully updated when this step's work completes either way."""
        pre, self._pre = self._pre, None  # a pull issued ahead serves the next step only
        if self.localize_mode == "tpf" and self.G == 1:
            B = labels.numel()
            width = width or (None if row_ptr is not None else self.cfg.max_nnz_per_example)
            if (row_ptr is None and rows is None and vals is None and prefetch is None
                    and (loc is None or getattr(loc, "flat", False))
                    and self._flat_ok(B, width, keys.numel() if loc is None else loc.nnz)):
                if loc is None:
                    loc = self.localizer(keys)
                self._flat_step(loc, labels, B, width, next_loc,
                                pre == (id(loc), loc.gen))
                return
            if (prefetch is None and B < _CSR_MAX_ROWS and (loc is None or getattr(loc, "flat", False))
                    and (row_ptr is not None or vals is not None)):
                # valued and / or variable-width rows: the same flat step with the CSR
                # fused forward + tile backward (tp_fwd_bwd_csr)
                if loc is None:
                    loc = self.localizer(keys)
                row_ptr, rows = self._csr_of(B, width, loc.nnz, row_ptr, rows, keys.device)
                self._flat_step_csr(loc, labels, B, row_ptr, rows, vals, next_loc,
                                    pre == (id(loc), loc.gen))
                return
            # not expressible on the flat layout (valued / variable-width rows): the same
            # keys through a compact "tp" localisation and the generic step below
            loc = self._compact_localizer()(keys)
        if self.p2p:
            if loc is None:
                loc = self.localizer(keys)
            return self._p2p_step(loc, labels, width, prefetch)
        if self.merged:
            return self._mx_step(keys, labels, width=width, row_ptr=row_ptr, vals=vals,
                                 rows=rows, loc=loc, prefetch=prefetch)
        if self.padded:
            if loc is None:
                with trace_range("localize"):
                    if self.localize_mode == "tpf" and (row_ptr is not None or rows is not None
                                                        or vals is not None):
                        loc = self._compact_localizer()(keys)  # (flat: fixed width only)
                    else:
                        loc = self.localizer(keys)
            segs = self.step_segments(keys, labels, width=width, row_ptr=row_ptr, vals=vals,
                                      rows=rows, loc=loc)
            for kind, fn in segs:
                if kind == "comm" and prefetch is not None:
                    prefetch()  # overlap the next minibatch with this step's exchange
                    prefetch = None
                fn()
            return
        B = labels.numel()
        if width is None and row_ptr is None:
            width = self.cfg.max_nnz_per_example
        if (self.G == 1 and self.gpu and self.filter is None and self._fused_update
                and self._use_plans and row_ptr is None and rows is None and vals is None and prefetch is None
                and not trace_enabled()):
            if loc is None:
                loc = self.localizer(keys)
            plan = self._step_plan(loc, labels, B, width)
            if plan is not None:  # resolve + fused forward/backward + fused scan/update
                plan.run()
                self.step_count += 1
                self.examples += B
                return
        if row_ptr is not None and rows is None:
            rows = self._csr_rows(row_ptr, keys.numel())
        if loc is None:
            with trace_range("localize"):
                loc = self.localizer(keys)
        self._prefetch = prefetch
        _pull = trace_range("pull")
        _pull.__enter__()
        if self.filter is not None:
            w_local, push = self._pull_filtered(loc)
        elif self.G == 1 and self.gpu:
            slot, w_local = self.slot_buf, self.w_buf
            it, iv, isd, seed = self.table.init.args()
            hipops().kv_resolve(self.table.slots, loc.uniq, loc.n_uniq, slot, w_local, True, it,
                                iv, isd, seed, self.table._err, self.table._inserted,
                                self.table.home_base, self.table.home_m)
            push = ("local", slot, loc.n_uniq)
        elif self.fused:
            w_local, push = self._exchange_fused(loc)
        else:
            w_local, push = self._pull(loc.uniq, loc.n_uniq)
        _pull.__exit__(None, None, None)
        if self._prefetch is not None:  # single-GPU / non-fused paths: no blocking point
            self._prefetch()
            self._prefetch = None
        _cmp = trace_range("compute")
        _cmp.__enter__()
        if push[0] == "local" and push[2] is not None and self._fused_update and fused_update_ok(
                loc, w_local, B=B, width=width or 0, row_ptr=row_ptr, rows=rows, vals=vals):
            # 1 GPU: the entry scan applies the FTRL / AdaGrad / SGD update and the AUC
            # epilogue itself (tp_seg_update)
            coef = self._coef_views.get(B)
            if coef is None:
                coef = self._coef_views[B] = self.coef[:B]
            linear_fwd_bwd(loc, w_local, labels, B=B, width=width, vals=vals, loss=self.cfg.loss,
                           coef=coef, metrics=self.metrics, hist=self.hist,
                           update=(self.table.slots, push[1], self.rule, self.stats,
                                   self.step_dev))
            _cmp.__exit__(None, None, None)
            self.step_count += 1
            self.examples += B
            return
        coef, grad = linear_fwd_bwd(loc, w_local, labels, B=B, width=width or 0, row_ptr=row_ptr,
                                    rows=rows, vals=vals, loss=self.cfg.loss, coef=self.coef[:B],
                                    metrics=self.metrics, hist=self.hist)
        _cmp.__exit__(None, None, None)
        _push = trace_range("push")
        _push.__enter__()
        if push[0] == "fused":
            # deferred: travels with the next step's pull exchange (see _exchange_fused)
            _, slot, send_c, recv_c, U, perm = push
            g_send = grad[:U].clone() if perm is None else grad[perm[:U].long()]
            self.pending = (slot, send_c, recv_c, g_send)
        else:
            folded = self._push(grad, push, fold_auc=True)
        _push.__exit__(None, None, None)
        if push[0] == "fused" or not folded:
            auc_from_hist(self.hist, self.metrics, self.step_dev)
        self.step_count += 1
        self.examples += B

    def _csr_rows(self, row_ptr: torch.Tensor, nnz: int) -> torch.Tensor:
        """Row id of every CSR position (int32)."""
        if self.gpu:
            rows = torch.empty(nnz, dtype=torch.int32, device=row_ptr.device)
            hipops().csr_rows(row_ptr, rows)
            return rows
        B = row_ptr.numel() - 1
        return torch.repeat_interleave(torch.arange(B, dtype=torch.int32),
                                       (row_ptr[1:] - row_ptr[:-1]).long())

    def _compact_localizer(self, buf: int = 0) -> Localizer:
        """Flat mode: the "tp" Localizer (workspace ``buf``) for minibatches the flat
        layout cannot express (valued or variable-width rows)."""
        if self._compact is None:
            self._compact = []
        while len(self._compact) <= buf:
            # (tail filter: "sort", whose segments count occurrences; tp's count entries)
            self._compact.append(self._new_localizer("sort" if self.filter is not None
                                                     else "tp"))
        return self._compact[buf]

    # ----------------------------------------------- flat 1-GPU step (Localizer "tpf")
    _FLAT_WIDTHS: dict = {}

    def _flat_ok(self, B: int, width, nnz: int) -> bool:
        """Fixed width with a fused forward/backward instance, binary features, nnz =
        B * width: the flat step applies (anything else takes the compact path)."""
        if not width or nnz != B * width or B >= (1 << 25):
            return False
        ok = self._FLAT_WIDTHS.get(width)
        if ok is None:
            ok = self._FLAT_WIDTHS[width] = bool(hipops().tp_fwd_bwd_supported(width))
        return ok

    def _flat_step(self, loc, labels, B: int, width: int, next_loc, pre: bool):
        """pull (unless issued ahead) -> fused forward + tile backward -> tpf_step: the
        update of this minibatch, then the pull of ``next_loc`` (same size) in the same
        launch. One native launch list per (buffers, labels, next buffers)."""
        plan, nxt = self.flat_plan(loc, labels, B, width, next_loc, pre)
        plan.run()
        self.flat_done(B, nxt)

    def _csr_of(self, B: int, width, nnz: int, row_ptr, rows, device):
        """(row_ptr, rows) of a minibatch: given, or a fixed width's arithmetic row_ptr
        (cached per shape); rows = the row of every occurrence (csr_rows)."""
        if row_ptr is None:
            key = ("rp", B, width)
            row_ptr = self._coef_views.get(key)
            if row_ptr is None:
                row_ptr = self._coef_views[key] = torch.arange(
                    0, (B + 1) * width, width, dtype=torch.int64, device=device)
        if rows is None:
            rows = self._rows_buf(nnz)
            if self.gpu:
                hipops().csr_rows(row_ptr, rows)
            else:
                rows.copy_(self._csr_rows(row_ptr, nnz))
        return row_ptr, rows

    def _rows_buf(self, nnz: int) -> torch.Tensor:
        rb = getattr(self, "_rows", None)
        if rb is None or rb.numel() < nnz:
            rb = self._rows = torch.empty(max(nnz, self.max_nnz), dtype=torch.int32,
                                          device=self.device)
        return rb[:nnz]

    def _flat_step_csr(self, loc, labels, B: int, row_ptr, rows, vals, next_loc, pre: bool):
        """The flat 1-GPU step for valued / variable-width rows: pull (unless issued
        ahead), the CSR fused forward + tile backward, then tpf_step (update of this
        minibatch + pull of ``next_loc``). Issued op by op: minibatch shapes vary."""
        nxt = next_loc if (next_loc is not None and getattr(next_loc, "flat", False)
                           and next_loc.nnz == loc.nnz and next_loc is not loc) else None
        H, tb = hipops(), self.table
        it, iv, isd, seed = tb.init.args()
        n, bits = loc.nnz, loc.bits
        common = (tb.slots, it, iv, isd, seed, tb._err, tb._inserted, tb.home_base, tb.home_m,
                  *self.rule.args(), self.stats)
        if not pre:
            H.tpf_step(n, bits, None, None, loc.bufs, loc.w_ent, *common, None, None, None)
        coef = self._coef_views.get(B)
        if coef is None:
            coef = self._coef_views[B] = self.coef[:B]
        H.tp_fwd_bwd_csr(loc.rep, loc.dcnt, None, n, row_ptr, rows, vals, loc.w_ent, labels, B,
                         loss_id(self.cfg.loss), coef, self.metrics, self.hist, AUC_BINS,
                         loc.psum, None, None, None, None, False)
        H.tpf_step(n, bits, loc.bufs, loc.psum, nxt.bufs if nxt is not None else None,
                   nxt.w_ent if nxt is not None else None, *common, self.hist, self.metrics,
                   self.step_dev)
        self.flat_done(B, nxt)

    def flat_done(self, B: int, nxt):
        """Host bookkeeping of a flat step whose launches were issued (``flat_plan``)."""
        if nxt is not None:
            self._pre = (id(nxt), nxt.gen)
        self.step_count += 1
        self.examples += B

    def flat_plan(self, loc, labels, B: int, width: int, next_loc, pre: bool, fb_record=None):
        """(LaunchList of one flat step, the next FlatLoc its update launch pulls or None);
        cached per (buffers, labels, next buffers). bench.py splices it into its native
        multi-stream iteration lists. ``fb_record``: an event recorded between the fused
        forward/backward and the step kernel (a preparation stream may wait for it)."""
        nxt = next_loc if (next_loc is not None and getattr(next_loc, "flat", False)
                           and next_loc.nnz == loc.nnz and next_loc is not loc) else None
        key = (id(loc), id(labels), B, width, loc.nnz, pre, id(nxt) if nxt is not None else 0,
               id(self.rule), id(self.table.init), id(fb_record))
        plan = self._plans.get(key)
        if plan is None:
            H, tb = hipops(), self.table
            it, iv, isd, seed = tb.init.args()
            n, bits = loc.nnz, loc.bits
            common = (tb.slots, it, iv, isd, seed, tb._err, tb._inserted, tb.home_base, tb.home_m,
                      *self.rule.args(), self.stats)
            plan = H.LaunchList()
            if not pre:  # this minibatch's pull on its own
                plan.add_tpf_step(n, bits, None, None, loc.bufs, loc.w_ent, *common, None, None,
                                  None)
            plan.add_tp_fwd_bwd(loc.rep, loc.dcnt, None, n, width, None, loc.w_ent, labels, B,
                                loss_id(self.cfg.loss), self.coef[:B], self.metrics, self.hist,
                                AUC_BINS, loc.psum, None, None, None, None, False)
            if fb_record is not None:
                plan.add_record(fb_record)
            plan.add_tpf_step(n, bits, loc.bufs, loc.psum,
                              nxt.bufs if nxt is not None else None,
                              nxt.w_ent if nxt is not None else None, *common, self.hist,
                              self.metrics, self.step_dev)
            if len(self._plans) >= 32:  # (callers passing fresh label tensors every step)
                self._plans.clear()
            self._plans[key] = plan
        return plan, nxt

    def prep_plan(self, buf: int, keys: torch.Tensor, labels: torch.Tensor, *, seed: int,
                  row0: int, row_step: int, num_features: int, alpha: float = 1.1, gate=None,
                  bucket_after=None, bucket_done=None):
        """Flat mode: a native launch list that generates the next synthetic minibatch of
        workspace ``buf`` (rows row0, row0 + row_step, ... on successive runs) and
        localises it (tile + flat bucket kernels): ONE host call per data preparation.
        ``gate``: an event the localisation waits for after the generator (bench.py: the
        training step's fused forward/backward, so the two LDS-heavy 1024-thread kernels
        do not share the CUs). ``bucket_after`` / ``bucket_done`` (tail filter): the
        filter kernel (CountMin insert + query + compaction, after the bucket kernel)
        waits for the previous minibatch's filter kernel and records its own, so sketch
        updates run in minibatch order while the generators, tile and bucket kernels of
        several preparations still overlap. Returns a callable -> the FlatLoc of
        ``buf``."""
        from ..ops.synthetic import CRITEO_1TB_CARDS, _set_cards

        if self.localize_mode != "tpf":
            raise ValueError("prep_plan needs the flat (tpf) localisation")
        while len(self._localizers) <= buf:
            self._localizers.append(self._new_localizer(self.localize_mode))
        lz = self._localizers[buf]
        f = lz.flat
        B = labels.numel()
        n = keys.numel()
        _set_cards(self.device, CRITEO_1TB_CARDS)
        H = hipops()
        plan = H.LaunchList()
        plan.add_criteo_gen(seed & ((1 << 64) - 1), row0, row_step, B, num_features, alpha, keys,
                            labels)
        if gate is not None:
            plan.add_wait(gate)
        if bucket_after is None and bucket_done is None:
            plan.add_localize_tpf(keys, n, self.bits, lz.ptemp, f.dcnt, f.rep, f.uniqf,
                                  f.ent_pos, f.ent_j, f.cnt, f.err, self._flat_x,
                                  filt=lz.filt_args())
        else:
            for stage in ((1, 2, 3) if lz.filt_args() is not None else (1, 2)):
                if stage == 3 and bucket_after is not None:
                    plan.add_wait(bucket_after)
                plan.add_localize_tpf(keys, n, self.bits, lz.ptemp, f.dcnt, f.rep, f.uniqf,
                                      f.ent_pos, f.ent_j, f.cnt, f.err, self._flat_x,
                                      filt=lz.filt_args(), stage=stage)
            if bucket_done is not None:
                plan.add_record(bucket_done)

        def run():
            plan.run()
            return done()

        def done():  # (host bookkeeping: also after the list ran inside another one)
            f.nnz = n
            f.gen += 1
            return f
        run.plan, run.done = plan, done
        return run

    def _step_plan(self, loc, labels, B: int, width: int):
        """The 1-GPU fused step (kv_resolve, tp_fwd_bwd, tp_seg_update: the same launches
        ``step`` issues one by one below) as a native ``LaunchList`` over the fixed
        workspaces of one localisation buffer and one label buffer: arguments are
        validated once, and a step is one host call (profiles/r3_s3_host_issue.log).
        None when the fused tp path does not apply to this minibatch."""
        t = loc.tile
        if t is None:
            return None
        # (object ids: a cached plan holds its tensors, so no other tensor takes their id)
        key = (id(t.rep), id(loc.uniq), id(labels), B, width, loc.nnz, id(self.rule),
               id(self.table.init))
        plan = self._plans.get(key)
        if plan is None:
            if not fused_update_ok(loc, self.w_buf, B=B, width=width):
                return None
            H, tb = hipops(), self.table
            it, iv, isd, seed = tb.init.args()
            plan = H.LaunchList()
            plan.add_kv_resolve(tb.slots, loc.uniq, loc.n_uniq, self.slot_buf, self.w_buf, True,
                                it, iv, isd, seed, tb._err, tb._inserted, tb.home_base, tb.home_m)
            coef = self.coef[:B]
            plan.add_tp_fwd_bwd(t.rep, t.dcnt, t.ent_uid, loc.nnz, width, None, self.w_buf, labels,
                                B, loss_id(self.cfg.loss), coef, self.metrics, self.hist,
                                AUC_BINS, t.psum, loc.pos_s, loc.segid, t.n_ent, loc.grad, False)
            plan.add_tp_seg_update(loc.pos_s, loc.segid, loc.nnz, t.n_ent, t.psum, loc.seg_start,
                                   loc.n_uniq, t.pieces, self.slot_buf, tb.slots,
                                   *self.rule.args(), self.stats, self.hist, self.metrics,
                                   self.step_dev)
            if len(self._plans) >= 16:  # (callers passing fresh label tensors every step)
                self._plans.clear()
            self._plans[key] = plan
        return plan

    # --------------------------------------------- padded exchange (G > 1, default)
    def idle_step(self):
        """A key-less step (multi-rank file-fed runs, app/gpu.py): a rank whose data ran
        out still joins the exchanges -- it owns a key range, so it resolves its peers'
        pulls, applies their pushes and ships its own last pushes -- without pulling,
        computing or pushing anything itself. Collective on the padded exchange; a no-op
        on one rank."""
        if self.G == 1:
            return
        if not self.padded:
            raise NotImplementedError("key-less steps need the padded exchange")
        if self.merged:
            return self._mx_step(None, None, idle=True)
        for _, fn in self.step_segments(None, None, idle=True):
            fn()

    def step_segments(self, keys: torch.Tensor, labels: torch.Tensor, *, width=None,
                      row_ptr=None, vals=None, rows=None, loc=None, step=None, next_loc=None,
                      idle: bool = False):
        """The step as an ordered list of ``(kind, fn)``: ``"compute"`` segments are
        pure device work on fixed buffers (capturable in a HIP graph per localisation
        buffer and ring position), ``"comm"`` segments are the two equal-split RCCL
        all-to-alls, ``"async"`` (ASP only) is the owner's push apply that pulls do
        not wait for, and ``"host"`` is the host bookkeeping. No segment reads anything
        back to the host, so a step is enqueued without waiting for the GPU.

          compute  owner-split the unique keys, pack [keys(t)] next to [grads(t-1-lag)]
          comm     all-to-all A
          compute  owner: apply the pushes of t-1-lag (one optimizer step per source,
                   rank order, all sources in one launch), then lookup-or-insert of
                   the pulled keys of t -> weights       [ASP / SSP post: resolve only]
          async    [ASP: apply the pushes of t-1-lag; the next pulls do not wait]
          comm     all-to-all B (weights back)
          post     [SSP post (lag >= 1): apply the pushes of t-lag carried by this
                   exchange; the worker does not wait for it, the next exchange does]
          compute  unpack weights, forward, backward, pack grads(t), AUC
          host     counters, overflow check

        Everything before the last compute segment is the exchange half, the rest the
        worker half (``EXCHANGE_SEGMENTS``); with lag >= 1 the exchange half of step
        t+1 may run while the worker half of step t computes (bench.py issues them on
        different streams). Buffers live in rings of ``self.R`` entries indexed by the
        absolute step ``step`` (default: the next step to compute); only ``step %
        self.R`` matters, so a graph captured for ring position j replays for every
        step t with t % R == j.
        """
        if not self.padded:
            return [("compute", lambda: self.step(keys, labels, width=width, row_ptr=row_ptr,
                                                  vals=vals, rows=rows, loc=loc,
                                                  next_loc=next_loc))]
        if idle:
            return self._idle_segments()
        if loc is None:
            loc = self.localizer(keys)
        B = labels.numel()
        if width is None and row_ptr is None:
            width = self.cfg.max_nnz_per_example
        flat = getattr(loc, "flat", False)
        csr = flat and (row_ptr is not None or vals is not None) and B < _CSR_MAX_ROWS
        if flat and not ((csr or (row_ptr is None and rows is None and vals is None
                                  and self._flat_ok(B, width, loc.nnz)))
                         and hipops().tpf_exchange_ok(loc.nnz, self.bits, self.G)):
            # not expressible on the flat layout: the same keys, localised compactly
            loc, flat = self._compact_localizer()(keys), False
        csr_args = None
        if flat and (row_ptr is not None or vals is not None):
            rp = row_ptr if row_ptr is not None else torch.arange(
                0, (B + 1) * width, width, dtype=torch.int64, device=loc.rep.device)
            rw = rows if rows is not None else torch.empty(loc.nnz, dtype=torch.int32,
                                                           device=loc.rep.device)
            csr_args = (rp, rw, vals)
        elif row_ptr is not None and rows is None:
            rows = (torch.empty(keys.numel(), dtype=torch.int32, device=keys.device) if self.gpu
                    else self._csr_rows(row_ptr, keys.numel()))
        if self.xc is None:
            self._xc_setup(loc)
        comm, xc = self.comm, self.xc
        t = self._xt if step is None else int(step)
        r = self.sched.ring(t)        # ring position of step t
        gb = self.sched.grad_ring(t)  # grads(t-1-lag) live here; keys(t) join them

        def finish():
            if flat:
                if csr_args is not None:  # the row of every occurrence, at replay time
                    hipops().csr_rows(csr_args[0], csr_args[1])
                return self._x_finish_flat(loc, labels, B, width, r, csr=csr_args)
            if row_ptr is not None and self.gpu:
                hipops().csr_rows(row_ptr, rows)
            self._x_finish(loc, labels, B, width, row_ptr, vals, rows, r)

        def host():
            self.step_count += 1
            self._xt += 1
            self.examples += B
            self._x_poll_overflow()

        def exchanged():
            self._xx += 1

        pack = (lambda: self._x_pack_keys_flat(loc, gb, r)) if flat else \
            (lambda: self._x_pack_keys(loc, gb, r))
        segs = [("compute", pack),
                ("comm", lambda: comm.all_to_all_fixed(xc.sends[gb], xc.recvs[r]))]
        if self.cfg.ssp_apply not in ("post", "pre"):
            raise ValueError(f"ssp_apply must be 'post' or 'pre', not {self.cfg.ssp_apply!r}")
        if self.asp:
            segs += [("compute", lambda: self._x_resolve(r)),
                     ("async", lambda: self._x_apply(r, gb))]
        elif self.sched.post:
            segs += [("compute", lambda: self._x_resolve(r))]
        else:
            segs += [("compute", lambda: (self._x_apply(r, gb), self._x_resolve(r)))]
        segs += [("comm", lambda: comm.all_to_all_fixed(xc.wsend, xc.wrecvs[r])),
                 ("host", exchanged)]
        if self.sched.post:  # the carried pushes, after the weights went back
            segs += [("post", lambda: self._x_apply(r, gb))]
        segs += [("compute", finish),
                 ("host", host)]
        return segs

    def _idle_segments(self):
        """step_segments of a key-less step: the same exchange half with no keys packed
        (the carried gradients still travel) and, for the worker half, no gradients of
        this step (its row's gradient count is cleared)."""
        if self.xc is None:
            self._xc_setup(None)
        comm, xc = self.comm, self.xc
        t = self._xt
        r, gb = self.sched.ring(t), self.sched.grad_ring(t)

        def clear(buf, keys, grads):
            if self.gpu:
                hipops().xchg_clear_counts(buf, xc.H, keys, grads)
                return
            for p in range(self.G):
                if keys:
                    buf[p * xc.H] = 0
                if grads:
                    buf[p * xc.H + 1] = 0

        def host():
            self.step_count += 1
            self._xt += 1
            self._x_poll_overflow()

        def exchanged():
            self._xx += 1

        segs = [("compute", lambda: clear(xc.sends[gb], True, False)),
                ("comm", lambda: comm.all_to_all_fixed(xc.sends[gb], xc.recvs[r]))]
        if self.asp:
            segs += [("compute", lambda: self._x_resolve(r)),
                     ("async", lambda: self._x_apply(r, gb))]
        elif self.sched.post:
            segs += [("compute", lambda: self._x_resolve(r))]
        else:
            segs += [("compute", lambda: (self._x_apply(r, gb), self._x_resolve(r)))]
        segs += [("comm", lambda: comm.all_to_all_fixed(xc.wsend, xc.wrecvs[r])),
                 ("host", exchanged)]
        if self.sched.post:
            segs += [("post", lambda: self._x_apply(r, gb))]
        segs += [("compute", lambda: clear(xc.sends[r], False, True)), ("host", host)]
        return segs

    # ------------------------------ merged exchange (one all-to-all per step, lag >= 1)
    def mx_exchange(self, s: int, next_loc=None, *, prepare=True):
        """The parts of merged exchange ``s`` (parallel/consistency.MergedSchedule) as a
        dict of callables, for a caller that orders them against other streams
        (bench.py) -- or run in order by ``_mx_step``:

          pack     keys(s+1) of ``next_loc`` into the send rows of exchange s (None: no
                   keys -- a drain or an idle rank)
          comm     the all-to-all (send rows hold grads(s-d) packed by worker s-d and the
                   weights resolved after exchange s-1)
          resolve  owner: lookup-or-insert keys(s+1) -> slots of pull step s+1, their
                   weights into the send rows of exchange s+1
          apply    owner: the pushes of step s-d (``post``: after resolve, else before)

        Everything is fixed device buffers (ring entries), so each part replays from a
        HIP graph captured for ring position s % R. ``prepare``: allocate the exchange
        rows on the first call (collective: agrees on the row capacity)."""
        if self.xc is None and prepare:
            self._xc_setup(next_loc)
        xc, ms, comm = self.xc, self.msched, self.comm
        R, d = ms.R, ms.d
        b, bn = s % R, (s + 1) % R
        send, recv = xc.sends[b], xc.recvs[b]
        flat = next_loc is not None and getattr(next_loc, "flat", False)

        def pack():
            if next_loc is None:
                self._mx_clear(send, keys=True)
            elif flat:
                self._x_pack_keys_flat(next_loc, b, bn)
            else:
                self._x_pack_keys(next_loc, b, bn)

        def resolve():
            self._x_resolve(b, bn, wout=self._mx_wview(xc.sends[bn]), wstride=xc.H)

        def apply():
            if s - d >= 0:
                self._x_apply(b, (s - d) % R)

        if xc.fused:  # resolve + apply of the owner in ONE launch (kv_owner_part)
            def owner():
                tb, ra = self.table, (s - d) % R
                it, iv, isd, seed = tb.init.args()
                gsrc, gstride = self._x_grads(b) if s - d >= 0 else (None, 0)
                ap = s - d >= 0
                hipops().kv_owner_part(
                    tb.slots, recv, xc.H, xc.C, xc.kw, xc.b0, xc.lgP, xc.slots[bn],
                    xc.pkeys[bn], xc.bnd[bn], self._mx_wview(xc.sends[bn]), it, iv, isd, seed,
                    tb._err, tb._inserted, tb.home_base, tb.home_m,
                    xc.slots[ra] if ap else None, xc.pkeys[ra] if ap else None, gsrc, gstride,
                    xc.bnd[ra] if ap else None, ms.post, *self.rule.args(), self.stats)

            return {"pack": pack, "comm": lambda: comm.all_to_all_fixed(send, recv),
                    "resolve": owner, "apply": lambda: None, "post": ms.post}
        return {"pack": pack, "comm": lambda: comm.all_to_all_fixed(send, recv),
                "resolve": resolve, "apply": apply, "post": ms.post}

    def mx_worker(self, u: int, loc, labels, *, width=None, row_ptr=None, vals=None, rows=None):
        """Worker half of step ``u`` on the merged exchange: weights read in place from
        the rows of exchange u, forward + backward, gradients into the send rows of
        exchange u+d (+ AUC epilogue). ``loc=None``: an idle step (no minibatch): only
        clears its gradient rows."""
        xc, ms = self.xc, self.msched
        R = ms.R
        b, bg = u % R, ms.grad_ring(u)
        if loc is None:
            return lambda: self._mx_clear(xc.sends[bg], grads=True)
        B = labels.numel()
        if width is None and row_ptr is None:
            width = self.cfg.max_nnz_per_example
        wsrc = self._mx_wview(xc.recvs[b])
        if getattr(loc, "flat", False):
            csr = None
            if row_ptr is not None or vals is not None:
                rw = rows if rows is not None else torch.empty(loc.nnz, dtype=torch.int32,
                                                               device=self.device)
                rp = row_ptr
                if rp is None:
                    rp = torch.arange(0, (B + 1) * width, width, dtype=torch.int64,
                                      device=self.device)
                csr = (rp, rw, vals)

            def fin_flat():
                if csr is not None:  # (rows: scratch, refilled from row_ptr)
                    hipops().csr_rows(csr[0], csr[1])
                self._x_finish_flat(loc, labels, B, width, b, send=xc.sends[bg], wsrc=wsrc,
                                    wstride=xc.H, csr=csr)
            return fin_flat

        def fin():
            if row_ptr is not None and self.gpu:
                hipops().csr_rows(row_ptr, rows)
            self._x_finish(loc, labels, B, width, row_ptr, vals, rows, b, send=xc.sends[bg],
                           wsrc=wsrc, wstride=xc.H)
        return fin

    def mx_done(self, B: int):
        """Host bookkeeping of one merged worker step."""
        self.step_count += 1
        self._xt += 1
        self.examples += B
        self._x_poll_overflow()

    def _mx_wview(self, buf: torch.Tensor) -> torch.Tensor:
        """The weight words of a row buffer, as floats from row 0's weight offset (row
        stride H)."""
        return buf.view(torch.float32)[self.xc.w0:]

    def _mx_clear(self, buf, keys: bool = False, grads: bool = False):
        if self.gpu:
            hipops().xchg_clear_counts(buf, self.xc.H, keys, grads)
            return
        for p in range(self.G):
            if keys:
                buf[p * self.xc.H] = 0
            if grads:
                buf[p * self.xc.H + 1] = 0

    def _mx_run_exchange(self, s: int, next_loc):
        parts = self.mx_exchange(s, next_loc)
        parts["pack"]()
        parts["comm"]()
        if parts["post"]:
            parts["resolve"]()
            parts["apply"]()
        else:
            parts["apply"]()
            parts["resolve"]()
        self._mx_next = s + 1

    def _mx_step(self, keys, labels, *, width=None, row_ptr=None, vals=None, rows=None,
                 loc=None, prefetch=None, idle: bool = False):
        """Sequential API on the merged exchange: step(u) issues exchange u-1, which
        carries keys(u), and then runs the worker half of step u-1 (its weights came
        with that exchange). So a call trains the PREVIOUS minibatch; ``flush()`` (and
        ``progress()``) trains the last one and applies every outstanding push. The
        minibatch tensors are captured (labels / row_ptr / vals copied).

        A caller-supplied ``loc`` lives in a workspace the caller refills (``localize(k,
        buf=...)``): the pending minibatch keeps a copy of its keys, and when the caller's
        localisation of this minibatch reused the pending one's workspace, the pending
        minibatch is localised again into a private workspace before its worker half.
        ``prefetch`` runs after that worker half is enqueued (it may refill the pending
        minibatch's workspace)."""
        cur = None
        pend = self._mx_pend
        if not idle:
            B = labels.numel()
            if width is None and row_ptr is None:
                width = self.cfg.max_nnz_per_example
            buf = self._xt + (pend is not None)  # step index of this minibatch
            flat_ok = (self.localize_mode == "tpf"
                       and ((row_ptr is not None or vals is not None) and B < _CSR_MAX_ROWS
                            or (rows is None and self._flat_ok(B, width, keys.numel())))
                       and hipops().tpf_exchange_ok(keys.numel(), self.bits, self.G))
            own = loc is None
            if own:
                loc = (self.localize(keys, buf=buf % 2) if flat_ok
                       else self._compact_localizer(buf % 2)(keys))
            if row_ptr is not None and rows is None:
                rows = (torch.empty(keys.numel(), dtype=torch.int32, device=keys.device)
                        if self.gpu else self._csr_rows(row_ptr, keys.numel()))
            cur = dict(loc=loc, labels=labels.clone(), width=width,
                       row_ptr=None if row_ptr is None else row_ptr.clone(),
                       vals=None if vals is None else vals.clone(), rows=rows, B=B,
                       keys=None if own else keys.clone(), flat=flat_ok)
            if pend is not None and not pend.get("idle") and pend.get("keys") is not None \
                    and _same_workspace(pend["loc"], loc):
                # the caller localised this minibatch over the pending one's workspace:
                # localise the pending keys again, into a workspace the caller never sees
                if self.filter is not None:  # (a second localisation would count twice)
                    raise ValueError(
                        "merged exchange + tail filter: the caller's localisation of this "
                        "minibatch reused the pending minibatch's workspace; use "
                        "localize(keys, buf=t % 2) or pass keys without loc")
                pend["loc"] = self._mx_private_loc(pend["keys"], pend["flat"])
        u = self._xt + (pend is not None)
        self._mx_run_exchange(u - 1, None if cur is None else cur["loc"])
        self._mx_finish_pending()
        self._mx_pend = cur if cur is not None else {"idle": True}
        if prefetch is not None:
            prefetch()

    def _mx_private_loc(self, keys, flat: bool):
        """Merged sequential API: a localisation in a workspace of the trainer's own (not
        reachable through ``localize``), for a pending minibatch whose caller-supplied
        workspace was refilled."""
        own = self.__dict__.setdefault("_mx_own", {})
        lz = own.get(flat)
        if lz is None:
            lz = own[flat] = (self._new_localizer(self.localize_mode) if flat
                              else self._new_localizer("sort" if self.filter is not None
                                                       else "tp"))
        return lz(keys)

    def _mx_finish_pending(self):
        p, self._mx_pend = self._mx_pend, None
        if p is None:
            return
        u = self._xt
        if p.get("idle"):
            self.mx_worker(u, None, None)()
            self.step_count += 1
            self._xt += 1
            return
        self.mx_worker(u, p["loc"], p["labels"], width=p["width"], row_ptr=p["row_ptr"],
                       vals=p["vals"], rows=p["rows"])()
        self.mx_done(p["B"])

    def mx_drain(self):
        """Apply every computed push that no issued exchange has carried yet: key-less
        exchanges for the remaining ring entries (collective; synchronises the device).
        Leaves the exchange ready for a fresh bootstrap."""
        if self.xc is None:
            return
        ms = self.msched
        if self.gpu:
            torch.cuda.synchronize(self.device)
        last = self._xt - 1  # last worker step whose gradients were packed
        s = self._mx_next if self._mx_next is not None else last + 1
        while s - ms.d <= last:
            b = s % ms.R
            send = self.xc.sends[b]
            self._mx_clear(send, keys=True)
            self.comm.all_to_all_fixed(send, self.xc.recvs[b])
            if s - ms.d >= 0:
                self._x_apply(b, (s - ms.d) % ms.R)
            self._mx_clear(send, grads=True)
            s += 1
        # exchanges s' < s that a new bootstrap may reuse carry no gradients any more
        for j in range(ms.R):
            self._mx_clear(self.xc.sends[j], keys=True, grads=True)
        self._mx_next = None
        if self.gpu:
            torch.cuda.synchronize(self.device)

    @property
    def EXCHANGE_SEGMENTS(self) -> int:  # step_segments()[:n] = exchange half
        return 6 if self.asp or self.sched.post else 5

    def consistency_desc(self) -> str:
        """The consistency the data plane actually enforces (reported by bench.py)."""
        if self.G == 1:
            return "bsp (1 shard: every pull sees every earlier push)"
        if self.p2p:
            return (f"asp-p2p (one-sided pulls from the owners' HBM and inbox pushes, no "
                    f"collective per step; owners apply at their own pace, a pusher waits "
                    f"only {self.cfg.p2p_queue} steps ahead of an owner)")
        if self.merged:
            ms = self.msched
            base = "asp (bounded here: " if ms.asp else f"ssp:{int(self.tau)} ("
            return (f"{base}pull of step t sees exactly the pushes of steps <= t-1-{ms.lag}; "
                    f"one all-to-all per step carrying keys(t+1), pushes(t-{ms.d}) and the "
                    f"weights of keys(t), owner apply {'after' if ms.post else 'before'} "
                    f"its resolve)")
        if not self.padded or self.lag == 0 and not self.asp:
            return "bsp (pull of step t sees every push of steps <= t-1)"
        if self.asp:
            return (f"asp (pushes applied asynchronously to pulls; pull of step t misses "
                    f">= {self.lag} and, bounded only by the {self.R}-entry ring, "
                    f"<= {self.lag + self.async_depth} steps of pushes)")
        return (f"ssp:{int(self.tau)} (pull of step t sees exactly the pushes of steps "
                f"<= t-1-{self.lag})")

    def _xc_setup(self, loc):
        """Allocate the fixed exchange rows. Capacity C (keys per peer per step) is the
        same on every rank: configured, or slack x the max per-peer count of the first
        minibatch over all ranks (collective; hashed keys split ~Binomial(U, 1/G),
        so the margin is many standard deviations)."""
        from types import SimpleNamespace

        cfg, G, dev, R = self.cfg, self.G, self.device, self.R
        C = int(cfg.exchange_capacity)
        if C <= 0 and loc is None:  # a key-less first step (idle_step): join with count 0
            cnt = torch.zeros(1, dtype=torch.float64)
            cnt = self.comm.all_reduce_(cnt.to(self.comm.device) if self.comm.backend == "nccl"
                                        else cnt, op="max")
            C = int(math.ceil(float(cnt.item()) * cfg.exchange_slack)) + 1024
        elif C <= 0 and getattr(loc, "flat", False):
            # keys per owner: the owner's buckets' unit counts (buckets [p * B/G, ...))
            g = hipops().tpf_groups(loc.nnz, loc.bits)
            # (tail filter: the unfiltered counts -- later minibatches keep more keys)
            cc = loc.cnt_pre if getattr(loc, "cnt_pre", None) is not None else loc.cnt
            c = cc[:4 * g].view(G, g // G, 4).to(torch.float64)
            cnt = (c[:, :, 0] + c[:, :, 2]).sum(1).max().reshape(1)
            cnt = self.comm.all_reduce_(cnt.to(self.comm.device) if self.comm.backend == "nccl"
                                        else cnt.cpu(), op="max")
            C = int(math.ceil(float(cnt.item()) * cfg.exchange_slack)) + 1024
        elif C <= 0:
            _, _, off, _ = self._owner_order(loc)
            cnt = (off[1:] - off[:-1]).max().to(torch.float64).reshape(1)
            cnt = self.comm.all_reduce_(cnt.to(self.comm.device) if self.comm.backend == "nccl"
                                        else cnt.cpu(), op="max")
            C = int(math.ceil(float(cnt.item()) * cfg.exchange_slack)) + 1024
        C = min(max(64, (C + 63) // 64 * 64), max(64, self.max_nnz))
        kw = 1 if self.bits <= 32 else 2
        nb = int(cfg.fixing_float_bytes)  # FixingFloat: nb-byte codes instead of f32
        gw = (C * nb + 3) // 4 if nb else C
        # the partitioned apply needs rows sorted by key and an ordered home (key range
        # -> partition)
        part_apply = (self.gpu and cfg.push_mode != "aggregate" and self.table.home_m != 0
                      and os.environ.get("PSAMD_OWNER_APPLY", "part") == "part")
        # ~G*C/512 partitions (~1-2 entries per thread of a 256-thread workgroup, rows
        # are ~2/3 full): a few workgroups per CU hide the chain of dependent loads each
        # one runs; many more (tiny ones) pay per-workgroup setup and stats atomics
        # (profiles/r2_owner_apply.log: 8 x 45120 entries, 2^9 -> 21 us, link pair 58 us)
        lgP = max(0, min(16, math.floor(math.log2(max(1, G * C // 512))))) if part_apply else -1
        if part_apply and os.environ.get("PSAMD_APPLY_LGP"):
            lgP = int(os.environ["PSAMD_APPLY_LGP"])
        # merged exchange: each row also carries the owner's weights answering the keys
        # the row's receiver sent in the previous exchange (word w0) and, for the owner's
        # one-launch resolve + apply (kv_owner_part), the bounds of its 2^lgP key-range
        # partitions over the row's keys (word b0, written by the sender's key pack)
        # (off by default: one launch of both halves measured the SUM of their kernel
        # times, 56.4 vs 22.3 + 34.4 us at 8 emulated peers, and it puts the apply on the
        # path to the next collective: 0.175 vs 0.155 ms / step, profiles/r5_owner_fused.log)
        fused = (self.merged and lgP >= 0
                 and os.environ.get("PSAMD_OWNER_FUSED", "0") == "1")
        w0 = 4 + C * kw + gw
        b0 = w0 + (C if self.merged else 0)
        H = (b0 + (((1 << lgP) + 1) if fused else 0) + 3) // 4 * 4
        z32 = lambda n, dt: torch.zeros(n, dtype=dt, device=dev)  # noqa: E731
        self.xc = SimpleNamespace(
            C=C, kw=kw, H=H, nb=nb, w0=w0, b0=b0, fused=fused,
            homes=self._owner_homes() if fused else None,
            # (+ the flat pack's per-workgroup min / max partials: 2 per bucket group)
            gstage=z32(G * C + 2 * 2048, torch.float32) if nb else None,
            gins=[z32(G * C, torch.float32) for _ in range(R)] if nb else None,
            # rings of R entries indexed by step: sends[j] holds grads(j) then keys(j+1+lag);
            # recvs[j] what exchange j received; slots[j] the owner's resolved slots of
            # pull step j (its push arrives lag+1 exchanges later)
            sends=[z32(G * H, torch.int32) for _ in range(R)],
            recvs=[z32(G * H, torch.int32) for _ in range(R)],
            slots=[torch.full((G * C,), -1, dtype=torch.int64, device=dev) for _ in range(R)],
            wsend=z32(G * C, torch.float32), wrecvs=[z32(G * C, torch.float32) for _ in range(R)],
            w_local=z32(self.max_nnz, torch.float32), ovf=z32(1, torch.int32),
            offs=[z32(G + 1, torch.int64) for _ in range(R)], curs=[None] * R,
            touched=torch.empty(G * C, dtype=torch.int64, device=dev) if self.gpu else None,
            n_touched=z32(1, torch.int32),
            # per-exchange chain scratch of the one-launch sequential push apply
            link=(torch.empty(next_pow2(2 * G * C), dtype=torch.int64, device=dev)
                  if self.gpu and lgP < 0 else None),
            nxt=torch.empty(G * C, dtype=torch.int32, device=dev) if self.gpu and lgP < 0 else None,
            # partitioned one-launch apply (kv_apply_part): the pull's keys and the
            # per-row bounds of 2^lgP key-range partitions, per ring entry
            lgP=lgP, pkeys=([torch.empty(G * C, dtype=torch.int64, device=dev) for _ in range(R)]
                            if lgP >= 0 else None),
            bnd=([torch.zeros(G * ((1 << lgP) + 1), dtype=torch.int32, device=dev)
                  for _ in range(R)] if lgP >= 0 else None),
            ovf_host=(torch.zeros(1, dtype=torch.int32, pin_memory=True) if self.gpu else None))

    def _owner_homes(self) -> torch.Tensor:
        """[G, 2] (base, m) of every owner's ordered home (KVTable key_range): the sender
        computes the owner's key-range partitions of its rows with them (the loopback
        emulation's one table owns every row)."""
        M = (1 << 64) - 1
        if self._loopback:
            hs = [(self.table.home_base, self.table.home_m)] * self.G
        else:
            hs = []
            for p in range(self.G):
                lo, hi = self.part.range_of(p)
                hs.append((lo, M // (hi - lo)) if hi > lo else (0, 0))
        s64 = lambda x: x - (1 << 64) if x >= (1 << 63) else x  # noqa: E731
        return torch.tensor([[s64(int(b)), s64(int(m))] for b, m in hs], dtype=torch.int64,
                            device=self.device)

    def _tail_filter(self, loc, ring: int):
        """Tail-feature filter on the padded exchange (reference MinibatchReader::read,
        src/learner/sgd.h:131-150): insert this minibatch's per-key occurrence counts
        into the worker's CountMin, keep the keys whose estimate > tail_feature_freq.
        Returns (kept keys in sorted order, kept -> unique id, device kept count);
        device-side compaction, no host sync, so the step stays graph-capturable.
        Filtered keys are neither pulled (w = 0) nor pushed."""
        U = loc.uniq.numel()
        freq = self.cfg.tail_feature_freq
        if not self.gpu:
            n = int(loc.n_uniq.reshape(-1)[0])
            self.filter.insert_segments(loc.uniq, loc.seg_start, loc.n_uniq)
            keep, _ = self.filter.query(loc.uniq[:n], freq)
            idx = torch.nonzero(keep, as_tuple=False).flatten().to(torch.int32)
            return (loc.uniq[:n][idx.long()].contiguous(), idx,
                    torch.tensor([idx.numel()], dtype=torch.int32))
        tf = getattr(self, "_tf", None)
        if tf is None or tf["keep"].numel() < U:
            i32 = lambda k: torch.empty(k, dtype=torch.int32, device=self.device)  # noqa: E731
            tf = self._tf = {"keep": i32(U), "incl": i32(U),
                             "keys": [torch.empty(U, dtype=torch.int64, device=self.device)
                                      for _ in range(self.R)],
                             "idx": [i32(U) for _ in range(self.R)],
                             "n": [torch.zeros(1, dtype=torch.int32, device=self.device)
                                   for _ in range(self.R)]}
        keep, incl = tf["keep"][:U], tf["incl"][:U]
        self.filter.insert_segments(loc.uniq, loc.seg_start, loc.n_uniq)
        hh = hipops()
        keep.zero_()
        hh.cm_query(self.filter.cells.view(torch.int32), self.filter.k, self.filter.vmax,
                    loc.uniq, loc.n_uniq, freq, keep, None)
        torch.cumsum(keep, 0, dtype=torch.int32, out=incl)
        kk, ki, nk = tf["keys"][ring], tf["idx"][ring], tf["n"][ring]
        hh.compact_kept(keep, incl, loc.n_uniq, ki, nk, None, loc.uniq, kk)
        return kk, ki, nk

    def _owner_order(self, loc, ring: int = 0):
        """(keys in owner order, perm owner-order -> unique id | None, off[G+1], count)."""
        if self.filter is not None and self.xc is not None:
            kk, ki, nk = self._tail_filter(loc, ring)
            off = self.xc.offs[ring]
            if self.gpu:
                hipops().owner_split(kk, nk, self.part.bounds_on(self.device), off)
            else:
                off = self.part.split_sorted(kk, nk)
            return kk, ki, off, nk
        if self.gpu:
            off = self.xc.offs[ring] if self.xc is not None else torch.empty(
                self.G + 1, dtype=torch.int64, device=self.device)
            hipops().owner_split(loc.uniq, loc.n_uniq, self.part.bounds_on(self.device), off)
            if self.xc is None:
                return loc.uniq, None, off, loc.n_uniq
            # the count the worker half reads later lives in the ring, not in the
            # localiser (a caller may refill that workspace before the worker half runs)
            nkr = getattr(self.xc, "nkr", None)
            if nkr is None or len(nkr) < self.R:
                nkr = self.xc.nkr = [torch.zeros(1, dtype=torch.int32, device=self.device)
                                     for _ in range(self.R)]
            nkr[ring].copy_(loc.n_uniq.reshape(-1)[:1])
            return loc.uniq, None, off, nkr[ring]
        return loc.uniq, None, self.part.split_sorted(loc.uniq, loc.n_uniq), loc.n_uniq

    def _x_pack_keys(self, loc, gb: int, r: int):
        xc = self.xc
        ukeys, perm, off, nkeys = self._owner_order(loc, r)
        xc.curs[r] = (perm, off, nkeys)
        send = xc.sends[gb]
        if self.gpu:
            hh = hipops()
            hh.xchg_pack_keys(ukeys, nkeys, off, xc.C, xc.kw, xc.H, send, xc.ovf,
                              homes=xc.homes, b0=xc.b0, lgP=max(xc.lgP, 0))
            if xc.nb:  # (FixingFloat push: no pack_grads launch to carry the flag)
                hh.xchg_publish(xc.ovf, xc.ovf_host)
            return
        H, C, kw = xc.H, xc.C, xc.kw
        for p in range(self.G):
            a, cnt = int(off[p]), int(off[p + 1] - off[p])
            c = min(cnt, C)
            send[p * H] = c
            xc.ovf += cnt - c
            k = ukeys[a:a + c]
            k32 = k.to(torch.int32) if kw == 1 else k.contiguous().view(torch.int32)
            send[p * H + 4:p * H + 4 + c * kw] = k32

    def _x_pack_keys_flat(self, loc, gb: int, r: int):
        """Flat layout: every bucket's (rank-sorted) keys straight into its owner's row."""
        xc = self.xc
        xc.curs[r] = None
        hh = hipops()
        hh.tpf_pack_keys(loc.nnz, loc.bits, self.G, loc.cnt, loc.uniqf, xc.C, xc.kw, xc.H,
                         xc.sends[gb], xc.ovf, homes=xc.homes, b0=xc.b0, lgP=max(xc.lgP, 0))
        # (the overflow flag reaches the host through tpf_pack_grads' extra workgroup,
        # fixing-float or not)

    def _x_finish_flat(self, loc, labels, B: int, width: int, r: int, send=None, wsrc=None,
                       wstride: int = 0, csr=None):
        """Flat layout, worker half: the pulled weights into tile-entry order, the flat
        fused forward + tile backward, every key's gradient (per-bucket fixed-point sums)
        into its owner's row of the next exchange [+ FixingFloat codes], AUC epilogue.
        (merged exchange: weights read in place from the received rows ``wsrc`` with row
        stride ``wstride``, gradients into ``send``.)"""
        xc, hh = self.xc, hipops()
        n, bits, G = loc.nnz, loc.bits, self.G
        send = xc.sends[r] if send is None else send
        hh.tpf_unpack_w(n, bits, G, loc.cnt, loc.ent_pos, loc.ent_j, xc.C,
                        xc.wrecvs[r] if wsrc is None else wsrc, loc.w_ent, wstride)
        coef = self._coef_views.get(B)
        if coef is None:
            coef = self._coef_views[B] = self.coef[:B]
        if csr is not None:  # (row_ptr, rows, vals): valued / variable-width rows
            hh.tp_fwd_bwd_csr(loc.rep, loc.dcnt, None, n, csr[0], csr[1], csr[2], loc.w_ent,
                              labels, B, loss_id(self.cfg.loss), coef, self.metrics, self.hist,
                              AUC_BINS, loc.psum, None, None, None, None, False)
        else:
            hh.tp_fwd_bwd(loc.rep, loc.dcnt, None, n, width, None, loc.w_ent, labels, B,
                          loss_id(self.cfg.loss), coef, self.metrics, self.hist, AUC_BINS,
                          loc.psum, None, None, None, None, False)
        hh.tpf_pack_grads(n, bits, G, loc.cnt, loc.ent_pos, loc.ent_j, xc.C, xc.kw, xc.H,
                          loc.psum, send, xc.gstage if xc.nb else None, self.hist, self.metrics,
                          self.step_dev, xc.ovf, xc.ovf_host)
        if xc.nb:
            seed = (self.cfg.seed * 7919 + 17) & ((1 << 64) - 1)
            hh.xchg_ff_encode(xc.gstage, xc.C, xc.kw, xc.H, xc.nb, seed, self.step_dev, send,
                              per=hh.tpf_groups(n, bits) // G)  # (the pack's partials)

    def _x_poll_overflow(self):
        """Raise at the first step whose exchange dropped keys (the device counter is
        published into pinned host memory by the pack kernel: no stream sync; on the
        GPU the check sees a pack that has completed, at most the pipeline depth
        behind). Dropped keys would have been pulled as 0 and their pushes lost."""
        xc = self.xc
        if xc.ovf_host is not None:
            # (a cached numpy view of the pinned word: ~0.1 us, vs a few us for a tensor
            # index, on the per-step host path of the merged pipelines)
            npv = getattr(xc, "ovf_np", None)
            if npv is None:
                npv = xc.ovf_np = xc.ovf_host.numpy()
            ovf = int(npv[0])
        else:
            ovf = int(xc.ovf.item())
        if ovf:
            raise RuntimeError(
                f"padded exchange overflow at step {self.step_count}: {ovf} keys exceeded the "
                f"per-peer capacity {xc.C} (pulled as 0, pushes dropped); set exchange_capacity "
                f"or exchange_slack higher, or exchange='exact'")

    def _x_grads(self, r: int):
        """Gradient source of the pushes received by exchange ``r``: (tensor, row stride)."""
        xc = self.xc
        if xc.nb:  # FixingFloat codes -> f32, one launch for all source rows
            self._x_ff_decode(r)
            return xc.gins[r], xc.C
        g0 = 4 + xc.C * xc.kw
        return xc.recvs[r].view(torch.float32)[g0:], xc.H

    def _x_apply(self, r: int, gb: int):
        """Owner: the pushes carried by exchange ``r`` (gradients of the pull step
        whose resolved slots are ``slots[gb]``), every source row in ONE launch pair
        with per-push semantics (source-rank order per key) or summed per key
        (``push_mode='aggregate'``)."""
        xc, G, H, C = self.xc, self.G, self.xc.H, self.xc.C
        pslot, recv = xc.slots[gb], xc.recvs[r]
        if self.gpu:
            hh = hipops()
            if xc.nb and self.cfg.push_mode != "aggregate" and xc.bnd is not None:
                # FixingFloat codes decoded inside the apply (no decode launch)
                hh.kv_apply_part(self.table.slots, pslot, xc.pkeys[gb], xc.gins[r], C, recv, H,
                                 C, xc.bnd[gb], xc.lgP, *self.rule.args(), self.stats,
                                 ff_nb=xc.nb, kw=xc.kw)
                return
            gsrc, gstride = self._x_grads(r)
            if self.cfg.push_mode == "aggregate":
                xc.n_touched.zero_()
                hh.kv_accumulate_rows(self.table.slots, pslot, gsrc, gstride, recv, H, C,
                                      xc.touched, xc.n_touched)
                hh.kv_apply_accumulated(self.table.slots, xc.touched, xc.n_touched,
                                        *self.rule.args(), self.stats)
            elif xc.bnd is not None:
                hh.kv_apply_part(self.table.slots, pslot, xc.pkeys[gb], gsrc, gstride, recv, H, C,
                                 xc.bnd[gb], xc.lgP, *self.rule.args(), self.stats)
            else:
                hh.kv_update_rows(self.table.slots, pslot, gsrc, gstride, recv, H, C, xc.link,
                                  xc.nxt, *self.rule.args(), self.stats)
            return
        rows = [recv[s * H:(s + 1) * H] for s in range(G)]
        if xc.nb:
            self._x_ff_decode(r)
            grads = [xc.gins[r][s * C:(s + 1) * C] for s in range(G)]
        else:
            g0 = 4 + C * xc.kw
            grads = [rows[s][g0:g0 + C].view(torch.float32) for s in range(G)]
        parts = []
        for s in range(G):
            ng = int(rows[s][1])
            if ng:
                parts.append((pslot[s * C:s * C + ng], grads[s][:ng]))
        self._apply_pushes(parts)

    def _x_resolve(self, r: int, rs: int | None = None, wout=None, wstride: int = 0):
        """Owner: lookup-or-insert the keys pulled by exchange ``r`` -> slots[rs] (default
        rs = r) and their weights -> ``wout`` (default wsend; row stride ``wstride``, 0 =
        C: the merged exchange writes them into the next send rows)."""
        xc, G, H, C, kw = self.xc, self.G, self.xc.H, self.xc.C, self.xc.kw
        recv = xc.recvs[r]
        rs = r if rs is None else rs
        wout = xc.wsend if wout is None else wout
        ws = wstride or C
        if self.gpu:
            it, iv, isd, seed = self.table.init.args()
            hipops().kv_resolve_rows(self.table.slots, recv, H, C, kw, xc.slots[rs], wout,
                                     True, it, iv, isd, seed, self.table._err,
                                     self.table._inserted, self.table.home_base,
                                     self.table.home_m,
                                     xc.pkeys[rs] if xc.bnd is not None else None,
                                     xc.bnd[rs] if xc.bnd is not None else None, max(xc.lgP, 0),
                                     wstride=ws)
            return
        for s in range(G):
            row = recv[s * H:(s + 1) * H]
            nk = int(row[0])
            if not nk:
                continue
            if kw == 1:
                req = row[4:4 + nk].to(torch.int64) & 0xFFFFFFFF
            else:
                req = row[4:4 + 2 * nk].contiguous().view(torch.int64)
            slot, w = self.table.resolve(req, insert=True)
            xc.slots[rs][s * C:s * C + nk] = slot
            wout[s * ws:s * ws + nk] = w

    def _x_finish(self, loc, labels, B, width, row_ptr, vals, rows, r: int, send=None,
                  wsrc=None, wstride: int = 0):
        xc = self.xc
        perm, off, n_uniq = xc.curs[r]
        wrecv = xc.wrecvs[r] if wsrc is None else wsrc
        send = xc.sends[r] if send is None else send  # grads(t) -> sends[t % R]
        ws = wstride or xc.C
        if self.gpu:
            w_local = xc.w_local[:loc.uniq.numel()]
            if self.filter is not None:
                w_local.zero_()  # filtered keys: w = 0
            hipops().xchg_unpack_w(wrecv, perm, n_uniq, off, xc.C, w_local, wstride=ws)
        else:
            w_local = torch.zeros(max(int(loc.n_uniq.reshape(-1)[0]), 1), dtype=torch.float32)
            for p in range(self.G):
                a, c = int(off[p]), min(int(off[p + 1] - off[p]), xc.C)
                dst = perm[a:a + c].long() if perm is not None else slice(a, a + c)
                w_local[dst] = wrecv[p * ws:p * ws + c]
        coef, grad = linear_fwd_bwd(loc, w_local, labels, B=B, width=width or 0, row_ptr=row_ptr,
                                    rows=rows, vals=vals, loss=self.cfg.loss, coef=self.coef[:B],
                                    metrics=self.metrics, hist=self.hist)
        H, C, kw = xc.H, xc.C, xc.kw
        if xc.nb:
            self._x_ff_pack(grad[:loc.uniq.numel()], perm, n_uniq, off, send)
        elif self.gpu:  # (+ the step's AUC epilogue in block 0: one launch less)
            hipops().xchg_pack_grads(grad[:loc.uniq.numel()], perm, n_uniq, off, C, kw, H, send,
                                     hist=self.hist, metrics=self.metrics,
                                     step_counter=self.step_dev, ovf=xc.ovf,
                                     ovf_host=xc.ovf_host)
            return
        else:
            for p in range(self.G):
                a, c = int(off[p]), min(int(off[p + 1] - off[p]), C)
                send[p * H + 1] = c
                g0 = p * H + 4 + C * kw
                g = grad[perm[a:a + c].long()] if perm is not None else grad[a:a + c]
                send[g0:g0 + c] = g.contiguous().view(torch.int32)
        auc_from_hist(self.hist, self.metrics, self.step_dev)

    def _x_ff_pack(self, grad, perm, n_uniq, off, send):
        """FixingFloat push (reference fixing_float.h:44-95): per owner row min/max,
        nb-byte stochastic-rounded codes; the device step clock varies the rounding
        bits across graph replays."""
        xc, H, C, kw, nb = self.xc, self.xc.H, self.xc.C, self.xc.kw, self.xc.nb
        seed = (self.cfg.seed * 7919 + 17) & ((1 << 64) - 1)
        if self.gpu:
            hipops().xchg_ff_pack_grads(grad, perm, n_uniq, off, C, kw, H, nb, seed,
                                        self.step_dev, send, xc.gstage)
            return
        for p in range(self.G):
            a, c = int(off[p]), min(int(off[p + 1] - off[p]), C)
            send[p * H + 1] = c
            g = grad[perm[a:a + c].long()] if perm is not None else grad[a:a + c]
            code, mm = ff.encode(g, nb, seed=seed + 1000003 * self.step_count + p)
            send[p * H + 2:p * H + 4] = mm.view(torch.int32)
            g0 = p * H + 4 + C * kw
            words = send[g0:g0 + (C * nb + 3) // 4].view(torch.uint8)
            words[:code.numel()] = code

    def _x_ff_decode(self, r: int):
        xc, H, C, kw, nb = self.xc, self.xc.H, self.xc.C, self.xc.kw, self.xc.nb
        recv, gin = xc.recvs[r], xc.gins[r]
        if self.gpu:
            hipops().xchg_ff_decode(recv, C, kw, H, nb, gin)
            return
        for s in range(self.G):
            row = recv[s * H:(s + 1) * H]
            n = int(row[1])
            if n:
                g0 = 4 + C * kw
                code = row[g0:g0 + (C * nb + 3) // 4].view(torch.uint8)[:n * nb]
                gin[s * C:s * C + n] = ff.decode(code, nb, row[2:4].view(torch.float32), n)

    def _x_flush(self):
        """Apply the gradients that no issued exchange has carried yet (keys-free
        exchanges, oldest first), so the shards hold every push issued so far.
        Collective."""
        xc = self.xc
        if self.gpu:  # exchange halves / async applies may still run on other streams
            torch.cuda.synchronize(self.device)
        # exchange s carried grads(s - 1 - lag); steps computed whose grads no issued
        # exchange has carried yet, oldest first
        for s in self.sched.pending(self._xx, self._xt):
            b = self.sched.ring(s)
            send, recv = xc.sends[b], xc.recvs[b]
            if self.gpu:
                hipops().xchg_clear_counts(send, xc.H, True, False)
            else:
                for p in range(self.G):
                    send[p * xc.H] = 0
            self.comm.all_to_all_fixed(send, recv)
            self._x_apply(b, b)
            if self.gpu:
                hipops().xchg_clear_counts(send, xc.H, False, True)
            else:
                for p in range(self.G):
                    send[p * xc.H + 1] = 0
        if self.gpu:
            torch.cuda.synchronize(self.device)
        self._x_check_overflow()

    def _x_check_overflow(self):
        xc = self.xc
        if xc is None:
            return
        ovf = int(xc.ovf.item())
        if ovf:
            raise RuntimeError(
                f"padded exchange overflow: {ovf} keys exceeded the per-peer capacity "
                f"{xc.C} (they were pulled as 0 and not pushed); set exchange_capacity "
                f"or exchange_slack higher, or exchange='exact'")


    # ------------------------------------------ one-sided peer exchange (G > 1, p2p)
    def _p2p_setup(self, loc):
        """Row geometry (C keys per owner row: slack x the largest per-owner count of the
        first minibatch over all ranks, like the padded exchange) and the IPC mappings."""
        from types import SimpleNamespace

        from ..parallel.p2p import PeerExchange

        cfg, G, dev = self.cfg, self.G, self.device
        off = torch.empty(G + 1, dtype=torch.int64, device=dev)
        hipops().owner_split(loc.uniq, loc.n_uniq, self.part.bounds_on(dev), off)
        C = int(cfg.exchange_capacity)
        if C <= 0:
            cnt = (off[1:] - off[:-1]).max().to(torch.float64).reshape(1)
            cnt = self.comm.all_reduce_(cnt if self.comm.backend == "nccl" else cnt.cpu(),
                                        op="max")
            C = int(math.ceil(float(cnt.item()) * cfg.exchange_slack)) + 1024
        C = min(max(64, (C + 63) // 64 * 64), max(64, self.max_nnz))
        kw = 1 if self.bits <= 32 else 2
        nb = int(cfg.fixing_float_bytes)  # FixingFloat pushes: nb-byte codes (padded layout)
        gw = (C * nb + 3) // 4 if nb else C
        H = (4 + C * kw + gw + 3) // 4 * 4
        i32 = lambda n: torch.zeros(n, dtype=torch.int32, device=dev)  # noqa: E731
        self.xc = SimpleNamespace(
            C=C, kw=kw, H=H, nb=nb, w0=None, b0=None, fused=False, homes=None, off=off,
            send=i32(G * H),
            gstage=torch.zeros(G * C, dtype=torch.float32, device=dev) if nb else None,
            wout=torch.zeros(G * C, dtype=torch.float32, device=dev),
            slot=torch.full((G * C,), -1, dtype=torch.int64, device=dev),
            w_local=torch.zeros(self.max_nnz, dtype=torch.float32, device=dev),
            a_slot=torch.full((G * C,), -1, dtype=torch.int64, device=dev),
            a_w=torch.zeros(G * C, dtype=torch.float32, device=dev),
            link=torch.empty(next_pow2(2 * G * C), dtype=torch.int64, device=dev),
            nxt=torch.empty(G * C, dtype=torch.int32, device=dev), ovf=i32(1),
            ovf_host=torch.zeros(1, dtype=torch.int32, pin_memory=True))
        self.px = PeerExchange(self.comm, self.table, C, kw, H, dev, Q=cfg.p2p_queue, nb=nb)

    def _p2p_step(self, loc, labels, width, prefetch=None):
        """One asynchronous step: pack this minibatch's keys per owner, pull them
        one-sided (own row: lookup-or-insert), forward + backward, pack the gradients
        next to the keys, apply the own row locally, post the peer rows into the
        owners' inboxes, and apply whatever the peers have posted here so far."""
        if self.xc is None:
            self._p2p_setup(loc)
        xc, hh, G, r = self.xc, hipops(), self.G, self.rank
        C, kw, H = xc.C, xc.kw, xc.H
        B = labels.numel()
        width = width or self.cfg.max_nnz_per_example
        self.px.wait_own()  # (the previous own-row update has read send / slot / gstage)
        hh.owner_split(loc.uniq, loc.n_uniq, self.part.bounds_on(self.device), xc.off)
        hh.xchg_pack_keys(loc.uniq, loc.n_uniq, xc.off, C, kw, H, xc.send, xc.ovf)
        if xc.nb:  # (FixingFloat: no pack_grads launch to publish the overflow flag)
            hh.xchg_publish(xc.ovf, xc.ovf_host)
        self.px.lookup(xc.send, xc.wout, xc.slot)
        if prefetch is not None:  # the next minibatch's preparation overlaps this step
            prefetch()
        U = loc.uniq.numel()
        w_local = xc.w_local[:U]
        hh.xchg_unpack_w(xc.wout, None, loc.n_uniq, xc.off, C, w_local)
        _, grad = linear_fwd_bwd(loc, w_local, labels, B=B, width=width, loss=self.cfg.loss,
                                 coef=self.coef[:B], metrics=self.metrics, hist=self.hist)
        if xc.nb:
            # FixingFloat codes for the peers (reference async_sgd.h:273-277); the own row
            # is decoded from its codes too, as the padded exchange decodes every recv row
            # (the reference quantises every push through its filter)
            seed = (self.cfg.seed * 7919 + 17) & ((1 << 64) - 1)
            hh.xchg_ff_pack_grads(grad[:U], None, loc.n_uniq, xc.off, C, kw, H, xc.nb, seed,
                                  self.step_dev, xc.send, xc.gstage)
            g_own = xc.gstage[r * C:(r + 1) * C]
            hh.xchg_ff_decode(xc.send[r * H:(r + 1) * H], C, kw, H, xc.nb, g_own)
            auc_from_hist(self.hist, self.metrics, self.step_dev)
        else:
            hh.xchg_pack_grads(grad[:U], None, loc.n_uniq, xc.off, C, kw, H, xc.send,
                               hist=self.hist, metrics=self.metrics, step_counter=self.step_dev,
                               ovf=xc.ovf, ovf_host=xc.ovf_host)
            g_own = xc.send.view(torch.float32)[r * H + 4 + C * kw:r * H + 4 + C * kw + C]
        self.px.own_update(xc.slot[r * C:(r + 1) * C], g_own, xc.send[r * H + 1:r * H + 2],
                           self.rule, self.stats)
        self.px.post(xc.send)
        self.px.check_fatal()
        self.px.apply(self.rule, self.stats, xc.a_slot, xc.a_w, xc.link, xc.nxt,
                      rounds=self.cfg.p2p_rounds)
        self.step_count += 1
        self.examples += B
        if int(xc.ovf_host[0]):
            raise RuntimeError(f"p2p exchange overflow: keys exceeded the per-owner row "
                               f"capacity {C}; set exchange_capacity or exchange_slack higher")

    # ------------------------------------------------------- fused exchange (G > 1)
    def _exchange_fused(self, loc):
        """One step of the multi-GPU data plane with 2 all-to-alls instead of 3:

        A: per peer [keys(t) | grads(t-1)] packed as int32 words (keys are u32 when
           the mixed key space has <= 32 bits, else 2 words) -> the owner first
           applies the pushes of step t-1 (one optimizer step per source, rank
           order), THEN resolves the pulls of step t, so every pull sees all pushes
           up to t-1 (same order of operations as the unfused path: BSP results);
        B: weights back.
        The per-peer counts of both directions come from ONE all-gather of the
        G x G count matrix (the only host synchronisation of the step)."""
        uniq, n_uniq = loc.uniq, loc.n_uniq
        G, dev = self.G, uniq.device
        kw = 1 if self.bits <= 32 else 2
        perm = None
        off = self.part.split_sorted(uniq, n_uniq)
        send_t = (off[1:] - off[:-1]).to(torch.int64)
        M_dev = self.comm.all_gather_counts(send_t, to_host=False)
        if self._prefetch is not None:  # overlap the next minibatch with this sync
            self._prefetch()
            self._prefetch = None
        M = M_dev.cpu()                                  # [G src, G dst], host
        send_t = M[self.rank].tolist()
        recv_t = M[:, self.rank].tolist()
        U = int(sum(send_t))
        if self.pending is not None:
            slot_p, send_p, recv_p, g_p = self.pending
        else:
            slot_p, send_p, recv_p, g_p = None, [0] * G, [0] * G, None
        keys = uniq[:U]
        k32 = keys.to(torch.int32) if kw == 1 else keys.contiguous().view(torch.int32)
        g32 = g_p.view(torch.int32) if g_p is not None else None
        pieces, ks, gs = [], 0, 0
        for p in range(G):
            pieces.append(k32[ks * kw:(ks + send_t[p]) * kw])
            ks += send_t[p]
            if g32 is not None:
                pieces.append(g32[gs:gs + send_p[p]])
                gs += send_p[p]
        sendbuf = torch.cat(pieces) if pieces else torch.empty(0, dtype=torch.int32, device=dev)
        ssz = [kw * send_t[p] + send_p[p] for p in range(G)]
        rsz = [kw * recv_t[s] + recv_p[s] for s in range(G)]
        recv = self.comm.all_to_all_v(sendbuf, ssz, rsz)
        kparts, gparts, a = [], [], 0
        for s in range(G):
            kparts.append(recv[a:a + kw * recv_t[s]])
            a += kw * recv_t[s]
            n = recv_p[s]
            if n and slot_p is not None:
                gparts.append((slot_p[s], recv[a:a + n].view(torch.float32)))
            a += n
        self._apply_pushes(gparts)  # pushes of step t-1 first ...
        rk = torch.cat(kparts)
        if kw == 1:
            req = rk.to(torch.int64) & 0xFFFFFFFF
        else:
            req = rk.view(torch.int64)
        slot, w = self.table.resolve(req, insert=True)  # ... then the pulls of step t
        slots_by_src, a = [], 0
        for s in range(G):
            slots_by_src.append(slot[a:a + recv_t[s]])
            a += recv_t[s]
        w_back = self.comm.all_to_all_v(w, recv_t, send_t)
        if perm is not None:  # back to unique-id order
            w_local = torch.empty_like(w_back)
            w_local[perm[:U].long()] = w_back
            w_back = w_local
        return w_back, ("fused", slots_by_src, send_t, recv_t, U, perm)

    def _apply_pushes(self, parts):
        """parts: [(slots, grads)] per source in rank order."""
        if not parts:
            return
        if self.cfg.push_mode == "aggregate":
            self._apply_aggregated(torch.cat([p[0] for p in parts]),
                                   torch.cat([p[1] for p in parts]).contiguous())
            return
        for slot, g in parts:  # one optimizer step per push message, in rank order
            self.table.update(slot, g.contiguous(), self.rule, self.stats)

    def flush(self):
        """Apply the deferred pushes of the last step (fused / padded multi-GPU modes).
        Collective."""
        if self.p2p:
            if self.px is not None:
                xc = self.xc
                self.px.drain(self.rule, self.stats, xc.a_slot, xc.a_w, xc.link, xc.nxt)
            return
        if self.merged:
            if self._mx_external:
                return  # a caller's pipeline owns the in-flight exchanges (mx_drain)
            if self._mx_pend is not None:  # the last minibatch: exchange without keys
                self._mx_run_exchange(self._xt, None)
                self._mx_finish_pending()
            self.mx_drain()
            self._x_check_overflow()
            return
        if self.padded:
            if self.xc is not None:
                self._x_flush()
            return
        if not self.fused or self.pending is None:
            return
        slot_p, send_p, recv_p, g_p = self.pending
        self.pending = None
        g_in = self.comm.all_to_all_v(g_p, send_p, recv_p)
        parts, a = [], 0
        for s in range(self.G):
            n = recv_p[s]
            if n:
                parts.append((slot_p[s], g_in[a:a + n]))
            a += n
        self._apply_pushes(parts)

    # ---------------------------------------------------------------- pull/push
    def _pull(self, uniq: torch.Tensor, n_uniq: torch.Tensor):
        """Pull weights of sorted unique mixed keys; returns (w_local, push handle)."""
        if self.G == 1:
            U = int(n_uniq.item())
            keys = uniq[:U]
            slot, w = self.table.resolve(keys, insert=True)
            return w, ("local", slot, None)
        off = self.part.split_sorted(uniq, n_uniq).cpu()
        U = int(off[-1])
        send_counts = (off[1:] - off[:-1])
        recv_counts = self.comm.exchange_counts(send_counts).cpu()
        req = self.comm.all_to_all_v(uniq[:U], send_counts.tolist(), recv_counts.tolist())
        slot, w = self.table.resolve(req, insert=True)
        w_back = self.comm.all_to_all_v(w, recv_counts.tolist(), send_counts.tolist())
        return w_back, ("dist", slot, send_counts, recv_counts, U)

    def _pull_filtered(self, loc):
        """Tail-feature filter on the generic paths (reference MinibatchReader::read,
        sgd.h:140-148): insert per-key counts into the worker's CountMin, pull only keys
        whose estimated count > tail_feature_freq; filtered keys get w = 0, no push. (The
        flat layout filters inside its bucket kernel instead, tpf_filter_unit.) GPU, one
        shard: device-side compaction and counts, no host sync."""
        if not (self.gpu and self.G == 1):
            U = loc.num_unique()
            uniq = loc.uniq[:U]
            cnt = (loc.seg_start[1:U + 1] - loc.seg_start[:U]).clamp(max=255).to(torch.uint8)
            self.filter.insert(uniq, cnt)
            keep, _ = self.filter.query(uniq, self.cfg.tail_feature_freq)
            kept_idx = torch.nonzero(keep, as_tuple=False).flatten()
            w_kept, push = self._pull(uniq[kept_idx].contiguous(),
                                      torch.tensor([kept_idx.numel()], dtype=torch.int32,
                                                   device=uniq.device))
            w_local = torch.zeros(loc.grad.numel(), dtype=torch.float32, device=uniq.device)
            w_local[kept_idx] = w_kept
            return w_local, ("filtered", kept_idx, push)
        U = loc.uniq.numel()  # (workspace length; the live count stays on the device)
        pf = getattr(self, "_pf", None)
        if pf is None or pf["w"].numel() < U + 1:
            pf = self._pf = {"w": torch.empty(U + 1, dtype=torch.float32, device=self.device),
                             "wk": torch.empty(U, dtype=torch.float32, device=self.device)}
        kk, ki, nk = self._tail_filter(loc, 0)  # kept keys, kept -> unique id, kept count
        ki[:U].masked_fill_(torch.arange(U, device=self.device) >= nk.long(), U)  # tail -> dummy
        slot, wk = self.slot_buf, pf["wk"][:U]
        it, iv, isd, seed = self.table.init.args()
        hipops().kv_resolve(self.table.slots, kk, nk, slot, wk, True, it, iv, isd, seed,
                            self.table._err, self.table._inserted, self.table.home_base,
                            self.table.home_m)
        w_local = pf["w"][:U + 1]
        w_local.zero_()
        w_local.index_copy_(0, ki[:U].long(), wk)  # (kept tail past nk lands on the dummy U)
        return w_local[:U], ("filtered_dev", ki[:U], slot, nk)

    def _push(self, grad: torch.Tensor, push, fold_auc: bool = False) -> bool:
        """Apply a push; True when the step's AUC epilogue rode along (``fold_auc``: the
        1-GPU KV update's block 0 turns the histogram into metrics, one launch less)."""
        kind = push[0]
        if kind == "filtered_dev":  # gradients of the kept keys, in kept order (no host sync)
            _, ki, slot, nk = push
            g = torch.cat([grad[:ki.numel()], grad.new_zeros(1)])[ki.long()]
            if fold_auc:
                hipops().kv_update(self.table.slots, slot, g, nk, *self.rule.args(), self.stats,
                                   hist=self.hist, metrics=self.metrics,
                                   step_counter=self.step_dev)
                return True
            hipops().kv_update(self.table.slots, slot, g, nk, *self.rule.args(), self.stats)
            return False
        if kind == "filtered":
            kept_idx, inner = push[1], push[2]
            g = grad[kept_idx].contiguous()
            return self._push(g, inner)
        if kind == "local":
            slot, n_dev = push[1], push[2]
            if n_dev is not None:  # (the slot workspace is sized for the largest batch)
                slot = slot[:grad.numel()]
            if n_dev is None:
                self.table.update(slot, grad[:slot.numel()], self.rule, self.stats)
                return False
            if fold_auc:
                hipops().kv_update(self.table.slots, slot, grad, n_dev, *self.rule.args(),
                                   self.stats, hist=self.hist, metrics=self.metrics,
                                   step_counter=self.step_dev)
                return True
            hipops().kv_update(self.table.slots, slot, grad, n_dev, *self.rule.args(),
                               self.stats)
            return False
        _, slot, send_counts, recv_counts, U = push
        g = grad[:U].contiguous()
        nb = self.cfg.fixing_float_bytes
        if nb:
            code, mm = ff.encode(g, nb, seed=self.cfg.seed * 7919 + self.step_count)
            mm_all = self.comm.all_to_all_v(mm.repeat(self.G), [2] * self.G, [2] * self.G)
            code_in = self.comm.all_to_all_v(code, (send_counts * nb).tolist(),
                                             (recv_counts * nb).tolist())
            parts, a = [], 0
            for s in range(self.G):
                n = int(recv_counts[s])
                parts.append(ff.decode(code_in[a * nb:(a + n) * nb], nb, mm_all[2 * s:2 * s + 2], n))
                a += n
            g_in = torch.cat(parts) if parts else torch.empty(0, device=g.device)
        else:
            g_in = self.comm.all_to_all_v(g, send_counts.tolist(), recv_counts.tolist())
        if self.cfg.push_mode == "aggregate":
            self._apply_aggregated(slot, g_in)
            return
        a = 0
        for s in range(self.G):  # one optimizer step per push message, in rank order
            n = int(recv_counts[s])
            if n:
                self.table.update(slot[a:a + n], g_in[a:a + n], self.rule, self.stats)
            a += n

    def _apply_aggregated(self, slot: torch.Tensor, g_in: torch.Tensor):
        if self.gpu:
            if self.touched is None or self.touched.numel() < slot.numel():
                self.touched = torch.empty(max(slot.numel(), 1024), dtype=torch.int64,
                                           device=self.device)
                self.n_touched = torch.zeros(1, dtype=torch.int32, device=self.device)
            self.n_touched.zero_()
            H = hipops()
            H.kv_accumulate(self.table.slots, slot, g_in, None, self.touched, self.n_touched)
            H.kv_apply_accumulated(self.table.slots, self.touched[:slot.numel()], self.n_touched,
                                   *self.rule.args(), self.stats)
            return
        valid = slot >= 0
        s, inv = torch.unique(slot[valid], return_inverse=True)
        g = torch.zeros(s.numel(), dtype=torch.float32).index_add_(0, inv, g_in[valid])
        self.table.update(s, g, self.rule, self.stats)

    # ------------------------------------------------------------ reporting
    def check_ok(self, collective: bool | None = None):
        """Host sync: raise if any device-side capacity was exceeded since the start --
        the table (full: a key could not be inserted), a localisation workspace (a tile
        or bucket overflowed its LDS hash or its fixed entry region: the step kernels
        would have dropped those occurrences' gradients and read stale weights) or the
        padded exchange rows. All error words are sticky, so a check at any later point
        still sees an overflow. Called by ``progress()`` and by bench.py after timing
        (same fail-loudly rule as the exchange overflow, ``_x_poll_overflow``).

        With G > 1 (``collective`` default) the three error classes are max-all-reduced
        first, so every rank raises together: a rank-local raise would leave its peers
        blocked in their next collective until the communicator timeout."""
        if not self.gpu:
            return
        lzs = [lz for lz in list(self._localizers) + list(self._compact or [])
               + list(getattr(self, "_mx_own", {}).values())
               if getattr(lz, "err", None) is not None]
        words = [self.table._err] + [lz.err for lz in lzs]
        if self.xc is not None and getattr(self.xc, "ovf", None) is not None:
            words.append(self.xc.ovf)
        v = torch.cat([w.reshape(-1)[:1].to(torch.int64) for w in words])
        nl = len(lzs)
        # [table full, OR-ish (max) of the localisation error bits, exchange overflow]
        summary = torch.stack([v[0], v[1:1 + nl].max() if nl else v[0] * 0,
                               v[-1] if len(words) > 1 + nl else v[0] * 0])
        if collective is None:
            collective = self.G > 1
        if collective:
            summary = self.comm.all_reduce_(
                summary.to(self.comm.device) if self.comm.backend == "nccl" else summary.cpu(),
                op="max")
        tab, loc_e, ovf = summary.cpu().tolist()
        local = v.cpu().tolist()
        if tab:
            raise RuntimeError("KVTable full: increase table_capacity (keys were not inserted)")
        if loc_e:
            bad = [lz.mode for lz, e in zip(lzs, local[1:1 + nl]) if e]
            mode = bad[0] if bad else "tpf/tp (on a peer rank)"
            raise RuntimeError(
                f"localize_{mode} overflow (error bits {loc_e:#x}): a tile or bucket "
                f"exceeded its LDS hash / entry region, so some occurrences were dropped "
                f"from the step; the minibatch is too skewed for the {mode} layout "
                f"(PSAMD_FLAT=0 or localize='sort')")
        if ovf:
            raise RuntimeError(
                f"exchange overflow: {ovf} keys exceeded the per-peer capacity {self.xc.C}; "
                f"set exchange_capacity or exchange_slack higher, or exchange='exact'")

    def progress(self, reset: bool = True) -> dict:
        """Merged progress across ranks (reference ISGDScheduler::showProgress, sgd.h:45-80).
        Collective when G > 1 (also applies deferred pushes). Raises on a device-side
        overflow (``check_ok``) instead of reporting a silently corrupted run."""
        self.flush()
        self.check_ok()
        m = torch.cat([accum_total(self.metrics)[:8], accum_total(self.stats)[:3]])
        if self.G > 1:
            m = self.comm.all_reduce_(m.to(self.comm.device) if self.comm.backend == "nccl"
                                      else m.cpu())
        m = m.cpu()
        n = max(float(m[2]), 1.0)
        out = {
            "examples": float(m[2]),
            "loss": float(m[0]) / n,
            # reference Evaluation::accuracy folds to max(acc, 1-acc) (evaluation.h:61)
            "accuracy": max(float(m[1]) / n, 1.0 - float(m[1]) / n) if m[2] > 0 else 0.0,
            "auc": float(m[3]) / max(float(m[4]), 1.0),
            "nnz_w": float(m[8]),
            "updt_ratio": math.sqrt(float(m[10])) / math.sqrt(max(float(m[9]), 1e-20)),
        }
        if reset:
            self.metrics.zero_()
            self.stats.view(-1, 16)[:, 1:].zero_()  # keep the cumulative nnz column
        return out

    # ------------------------------------------------------------ checkpoint
    def save_model(self, prefix: str, node_id: str | None = None) -> str:
        """Reference checkpoint layout: ``<prefix>_<NodeID>`` with one ``key\\tweight``
        line per non-zero weight (src/parameter/kv_store.h:63-73)."""
        from ..utils.checkpoint import write_text_model

        self.flush()

        keys, w, _, _ = self.table.occupied()
        raw = unmix(keys, self.bits)
        path = f"{prefix}_{node_id or f'S{self.rank}'}"
        write_text_model(path, raw.cpu(), w.cpu())
        return path

    def state_dict(self) -> dict:
        self.flush()
        keys, w, z, n = self.table.occupied()
        return {"keys": unmix(keys, self.bits).cpu(), "w": w.cpu(), "z": z.cpu(), "n": n.cpu(),
                "step": self.step_count, "bits": self.bits, "rank": self.rank, "world": self.G}

    def load_state_dict(self, sd: dict):
        from ..ops.keymix import mix

        self._pre = None  # the table changes under any pull issued ahead
        keys = mix(sd["keys"].to(self.device), self.bits)
        own = self.part.owner_of(keys) == self.rank
        self.table.load(keys[own], sd["w"].to(self.device)[own], sd["z"].to(self.device)[own],
                        sd["n"].to(self.device)[own])
        self.step_count = int(sd.get("step", 0))
