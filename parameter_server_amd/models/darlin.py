"""Darlin: L1-regularised logistic regression by block coordinate descent, MI355X-native.

Reference algorithm (PS v1 "Darlin"):
* scheduler  src/app/linear_method/darlin.h:32-132 — passes over shuffled
  feature blocks (prior groups first in pass 0), bounded block delay tau, KKT
  filter threshold ``violation / num_ex * ratio``, convergence when the relative
  objective <= epsilon twice with a KKT reset in between;
* worker     darlin.h:297-502 — block gradient (G, U), dual update;
* server     darlin.h:175-265 — aggregates G, U of all workers, proximal Newton
  coordinate step with trust region + KKT filter, evaluation;
* framework  src/learner/bcd.h — data loading, tail-feature filtering and key
  localisation (preprocessData :324-465), block division (:78-122).

MI355X design (one process per GPU, every rank = worker + server):
* preprocessing builds, per feature group, the GLOBAL sorted list of kept keys
  (tail filter with exact counts summed at owner ranks, then an all-gather), so
  every rank's training matrix is ONE CSC over a global column space and a
  feature block is a contiguous column range;
* per block: HIP gradient kernel -> ONE fp64 all-reduce of [G; U] over RCCL
  (replaces the push to servers and their ``KVBufferedVector`` sum) -> every
  rank applies the identical coordinate update to its replica of the block
  (replaces the server update AND the weight pull) -> HIP margin update;
* bounded delay: the gradient of block i only waits for the dual updates of
  blocks <= i - tau - 1, so with tau >= 1 the all-reduce of block i-1 is in
  flight (on RCCL's stream) while block i's gradient runs;
* state in HBM: w, delta (fp64) and the active set (uint8) per global column,
  margins ym (fp64) per local example.

Semantic differences (documented): tail filtering uses exact counts instead of a
CountMin sketch (the sketch only over-counts, so the reference keeps a superset);
a KKT-filtered weight stays 0 and is re-activated by a KKT reset (the reference
server leaves it NaN forever, darlin.h:228-231 + 223-246).
"""
from __future__ import annotations

import math
import os
import random
import sys
import time
from collections import deque
from dataclasses import dataclass, field

import numpy as np
import torch

from ..data.slot_reader import SlotData, merge_slot_info
from ..ops import bcd
from ..ops.native import hipops
from ..parallel.comm import Comm, LocalComm
from ..parallel.partition import even_divide

SIGN = -(1 << 63)


def _flip(keys_u64: np.ndarray) -> np.ndarray:
    """uint64 -> int64 whose signed order is the unsigned order."""
    return (keys_u64.astype(np.uint64) ^ np.uint64(1 << 63)).view(np.int64)


def _unflip(k: np.ndarray) -> np.ndarray:
    return k.view(np.uint64) ^ np.uint64(1 << 63)


@dataclass
class DarlinConfig:
    l1: float = 1.0                 # penalty.lambda(0)
    eta: float = 1.0                # learning_rate.alpha
    delta_init: float = 1.0         # [PS.LM.delta_init_value]
    delta_max: float = 5.0          # [PS.LM.delta_max_value]
    kkt_ratio: float = 10.0         # [PS.LM.kkt_filter_threshold_ratio]
    block_ratio: float = 4.0        # feature_block_ratio
    random_order: bool = True       # random_feature_block_order
    prior_groups: tuple = ()        # prior_fea_group
    prior_iters: int = 5            # num_iter_for_prior_fea_group
    tau: int = 0                    # max_block_delay
    max_pass: int = 10              # max_pass_of_data
    epsilon: float = 1e-4
    tail_freq: int = 0              # tail_feature_freq
    init_w: float = 0.0             # init_w (ZERO / CONSTANT)
    seed: int = 0
    host_preprocess: bool = False   # GPU trainer: build the CSC with numpy instead (reference)
    # G > 1, per block: "on" = reduce-scatter [G | U] to the owners of the block's
    # slices + all-gather dw (3 x ncols x 8 B over the links, 2 collectives), "off" = one
    # all-reduce of [G | U] and the identical update on every rank (4 x ncols x 8 B, 1
    # collective), "auto" = sharded for blocks of >= shard_min_cols columns (bandwidth-
    # bound), all-reduce below (latency-bound)
    shard_server: str = "auto"
    shard_min_cols: int = 1 << 16
    # fused row pass: tau_i = 1 / (1 + exp(ym_i)) in fp32 (bcd.hip rp_tau; the G / U sums
    # stay fp64 / fixed point). Off = fp64 exp, the mode the CPU-parity tests pin.
    tau32: bool = False

    @classmethod
    def from_lm(cls, lm, seed: int = 0) -> "DarlinConfig":
        d = lm.darlin
        lam = list(lm.penalty.__getattr__("lambda")) or [1.0]
        init = 0.0
        if d.has("init_w") and d.init_w.type == "CONSTANT":
            init = float(d.init_w.constant)
        return cls(l1=float(lam[0]), eta=float(lm.learning_rate.alpha),
                   delta_init=float(d.ext("delta_init_value")),
                   delta_max=float(d.ext("delta_max_value")),
                   kkt_ratio=float(d.ext("kkt_filter_threshold_ratio")),
                   block_ratio=float(d.feature_block_ratio),
                   random_order=bool(d.random_feature_block_order),
                   prior_groups=tuple(d.prior_fea_group), prior_iters=int(d.num_iter_for_prior_fea_group),
                   tau=int(d.max_block_delay), max_pass=int(d.max_pass_of_data),
                   epsilon=float(d.epsilon), tail_freq=int(d.tail_feature_freq), init_w=init,
                   seed=seed)


# narrow blocks of at most this many entries: gradient and coordinate update in one
# launch of a few workgroups (one rank)
_SMALL_ROWS_BLOCK = 1 << 18


_FUSED_W = int(os.environ.get("PSAMD_BCD_FUSED_W", "0"))  # (A/B pin of the fused grid)


def _hot_piece(entries: int) -> int:
    """Entries per piece of a hot column in the chunked gradient: ~2048 pieces per block
    (256 .. 4096), so a block of a few 100 k entries is not a few dozen waves each
    walking 4096 dependent gathers (CTR-log groups: 44.7 us per wide block at 4096)."""
    if os.environ.get("PSAMD_BCD_HOT"):  # (A/B pin)
        return int(os.environ["PSAMD_BCD_HOT"])
    want = max(1, entries // 2048)
    return int(min(4096, max(256, 1 << (want - 1).bit_length())))


def divide_feature_blocks(info: dict, ratio: float) -> list[tuple[int, int, int]]:
    """[(group, key_begin, key_end)] — reference BCDScheduler::divideFeatureBlocks
    (src/learner/bcd.h:78-106): a group with nnz_per_row > 1 is split into
    ceil(nnz_per_row * ratio) even key ranges of [min_key, max_key)."""
    out = []
    for g in sorted(info["slots"]):
        if g == 0:
            continue
        s = info["slots"][g]
        npr = s["nnz_ele"] / max(s["nnz_ex"], 1)
        n = max(int(math.ceil(npr * ratio)), 1) if npr > 1 + 1e-6 else 1
        for i in range(n):
            a, b = even_divide(s["min_key"], s["max_key"], n, i)
            if b > a:
                out.append((g, a, b))
    return out


def block_orders(blocks, cfg: DarlinConfig, rng: random.Random):
    """(blk_order, prior_blk_order) — bcd.h:108-121."""
    blk = list(range(len(blocks)))
    prior = []
    for g in cfg.prior_groups:
        tmp = [k for k, b in enumerate(blocks) if b.group == g]
        if not tmp:
            continue
        for _ in range(cfg.prior_iters):
            if cfg.random_order:
                rng.shuffle(tmp)
            prior.extend(tmp)
    return blk, prior


@dataclass
class Block:
    group: int
    key_begin: int
    key_end: int
    c0: int
    c1: int
    p0: int
    p1: int
    chunks: object = None  # device work list of the chunked gradient kernel (GPU)
    gu: object = None      # device [G | U] buffer of the block (GPU)
    busy: bool = False     # gu holds a launched, not yet consumed gradient
    unique_rows: bool = False  # no example has two entries in the block (dual w/o atomics)
    row_mode: bool = False     # narrow block: row-order gradient (bcd.grad_rows)
    fx_k: int = 0              # its fixed-point scale 2^k
    dcol: object = None        # dense per-example layout (bcd.dense_rows) for the row pass
    dval: object = None
    kenc: object = None        # wide block: hot / cold encoded layout (bcd.hot_layout)
    hcols: object = None       # ... its LDS hot slot -> column map
    chunks_cold: object = None  # ... and the chunk list of its cold columns
    part2: object = None       # narrow block: its gradient's segment sums (1 rank)
    few_rows: bool = False     # wide block w/o dense layout on < half of the examples
    dw: object = None          # small narrow block: dw of its fused update (bcd.grad_rows)

    @property
    def ncols(self):
        return self.c1 - self.c0


@dataclass
class BCDProgress:
    objective: float = 0.0
    relative_obj: float = 0.0
    nnz_w: int = 0
    violation: float = 0.0
    nnz_active_set: int = 0
    total_time: float = 0.0
    busy_time: list = field(default_factory=list)


class DarlinTrainer:
    """Darlin BCD on one rank (GPU or CPU tensors); ``comm`` spans all ranks."""

    def __init__(self, data: SlotData, cfg: DarlinConfig, comm: Comm | None = None,
                 device="cpu", verbose: bool = False):
        self.cfg = cfg
        self.comm = comm or LocalComm(device)
        self.G = self.comm.world
        self.rank = self.comm.rank
        self.device = torch.device(device)
        self.verbose = verbose
        self.rng = random.Random(cfg.seed)
        # sharded server (see DarlinConfig.shard_server); both block paths keep the
        # replicas of w / delta / active bitwise equal, so they mix freely
        if cfg.shard_server not in ("auto", "on", "off"):
            raise ValueError(f"shard_server must be auto / on / off, got {cfg.shard_server!r}")
        self.shard = self.G > 1 and cfg.shard_server != "off" and \
            getattr(self.comm, "backend", None) in ("nccl", "gloo")
        t0 = time.time()
        self._preprocess(data)
        self.preprocess_time = time.time() - t0
        self.progress: list[BCDProgress] = []
        self.kkt_thr = 1e20

    # ------------------------------------------------------------ preprocess
    def _global_info(self, data: SlotData) -> dict:
        infos = self.comm.all_gather_obj(data.info()) if self.G > 1 else [data.info()]
        return merge_slot_info(infos)

    def _group_keys(self, gid: int, uniq: np.ndarray, cnt: np.ndarray, info_g) -> np.ndarray:
        """Global sorted (flipped) key list of group ``gid`` after the tail filter."""
        freq = self.cfg.tail_freq
        if self.G == 1:
            return uniq[cnt > freq] if freq > 0 else uniq
        # owner = even split of the group's (flipped) key range; counts summed at owners
        lo = int(_flip(np.array([info_g["min_key"]], np.uint64))[0])
        hi = int(_flip(np.array([info_g["max_key"] - 1], np.uint64))[0]) + 1
        bounds = np.array([even_divide(lo, hi, self.G, r)[0] for r in range(1, self.G)], np.int64)
        owner = np.searchsorted(bounds, uniq, side="right")
        sc = np.bincount(owner, minlength=self.G).astype(np.int64)
        comm = self.comm
        rc = comm.exchange_counts(torch.from_numpy(sc)).cpu().numpy()
        rk = self._a2a(uniq, sc, rc)
        rn = self._a2a(cnt.astype(np.int64), sc, rc)
        if rk.size:
            u, inv = np.unique(rk, return_inverse=True)
            tot = np.bincount(inv, weights=rn.astype(np.float64)).astype(np.int64)
            kept = u[tot > freq] if freq > 0 else u
        else:
            kept = np.zeros(0, np.int64)
        # all-gather of the owners' kept lists (owner ranges are ordered -> sorted)
        n = np.array([kept.size] * self.G, np.int64)
        rcnt = comm.exchange_counts(torch.from_numpy(n)).cpu().numpy()
        return self._a2a(np.tile(kept, self.G), n, rcnt)

    def _a2a(self, x: np.ndarray, sc, rc) -> np.ndarray:
        t = torch.from_numpy(np.ascontiguousarray(x))
        if getattr(self.comm, "backend", "") == "nccl":
            t = t.to(self.comm.device)
        return self.comm.all_to_all_v(t, sc, rc).cpu().numpy()

    def _preprocess(self, data: SlotData):
        cfg = self.cfg
        sync = (lambda: torch.cuda.synchronize(self.device)) if self.device.type == "cuda" \
            else (lambda: None)
        t0 = time.time()
        if self.device.type == "cuda" and not getattr(cfg, "host_preprocess", False):
            col, row, val, colptr, base, nkeys = self._build_csc_gpu(data)
        else:
            col, row, val, colptr, base, nkeys = self._build_csc_host(data)
        sync()
        t1 = time.time()
        self._finish_preprocess(data, col, row, val, colptr, base, nkeys)
        sync()
        self.prep_times = {"csc": t1 - t0, "blocks_and_row_copies": time.time() - t1}

    def _build_csc_host(self, data: SlotData):
        """Reference-shaped host preprocessing (numpy): per group np.unique, tail filter,
        searchsorted column map, stable argsort CSR -> CSC (bcd.h:324-465,
        sparse_matrix.h:186-241). The GPU path (``_build_csc_gpu``) produces the same
        arrays bit for bit."""
        self.info = self._global_info(data)
        self.num_ex = int(self.info["num_ex"])
        rows = data.rows
        if rows >= (1 << 31):
            raise ValueError("a rank holds at most 2^31-1 examples")
        self.rows = rows
        gids = sorted(g for g in self.info["slots"] if g != 0)
        cols, rws, vals = [], [], []
        self.group_keys: dict[int, np.ndarray] = {}   # flipped, sorted
        self.group_base: dict[int, int] = {}
        base = 0
        valued = any(data.groups.get(g, (None, None, None))[2] is not None for g in gids)
        for g in gids:
            if g in data.groups:
                off, keys, v = data.groups[g]
            else:
                off, keys, v = np.zeros(rows + 1, np.int64), np.zeros(0, np.uint64), None
            kf = _flip(keys)
            uniq, inv, cnt = np.unique(kf, return_inverse=True, return_counts=True)
            gk = self._group_keys(g, uniq, cnt, self.info["slots"][g])
            self.group_keys[g] = gk
            self.group_base[g] = base
            # local nnz -> global column (drop tail-filtered keys)
            pos = np.searchsorted(gk, uniq)
            hit = (pos < gk.size) & (gk[np.minimum(pos, max(gk.size - 1, 0))] == uniq) \
                if gk.size else np.zeros(uniq.size, bool)
            ucol = np.where(hit, pos + base, -1)
            c = ucol[inv]
            r = np.repeat(np.arange(rows, dtype=np.int64), np.diff(off))
            keep = c >= 0
            cols.append(c[keep])
            rws.append(r[keep])
            if valued:
                vals.append((np.ones(keys.size, np.float32) if v is None else v)[keep])
            base += gk.size
        if base >= (1 << 31):
            raise ValueError("at most 2^31-1 global columns")
        col = np.concatenate(cols) if cols else np.zeros(0, np.int64)
        row = np.concatenate(rws) if rws else np.zeros(0, np.int64)
        order = np.argsort(col, kind="stable")  # CSR -> CSC (reference toColMajor)
        col, row = col[order], row[order]
        val = np.concatenate(vals)[order] if valued else None
        colptr = np.zeros(base + 1, np.int64)
        np.cumsum(np.bincount(col, minlength=base), out=colptr[1:])
        dev = self.device
        col = torch.from_numpy(col.astype(np.int32)).to(dev)
        row = torch.from_numpy(row.astype(np.int32)).to(dev)
        val = None if val is None else torch.from_numpy(val.astype(np.float32)).to(dev)
        return col, row, val, colptr, base, len(gids)

    # -------------------------------------------------------- GPU preprocess
    def _group_tensors(self, data: SlotData, g: int):
        """(offsets int64, keys int64 (raw uint64 bits), vals f32 | None) of group g on
        the device; numpy groups are uploaded, device tensors used as they are."""
        dev = self.device
        off, keys, v = data.groups[g]
        def up(x, dt):
            if isinstance(x, torch.Tensor):
                return x.to(dev, dt)
            return torch.from_numpy(np.ascontiguousarray(x)).to(dev, dt, non_blocking=False)
        k = keys if isinstance(keys, torch.Tensor) else torch.from_numpy(
            np.ascontiguousarray(keys).view(np.int64))
        return up(off, torch.int64), k.to(dev, torch.int64), \
            (None if v is None else up(v, torch.float32))

    def _sort_unique(self, keys: torch.Tensor, end_bit: int):
        """Own radix sort (primitives.hip) + fused run-length encode (localize.hip) of
        raw uint64 keys < 2^end_bit: (sorted unique keys, segment starts, positions in
        key order (stable), 1-based segment id of every sorted position)."""
        H = hipops()
        n = keys.numel()
        dev = keys.device
        i32 = lambda m: torch.empty(m, dtype=torch.int32, device=dev)  # noqa: E731
        temp = torch.empty(max(1, H.sort_pairs_temp_bytes(n, end_bit)), dtype=torch.uint8,
                           device=dev)
        hs = torch.empty_like(keys)
        pos = torch.arange(n, dtype=torch.int32, device=dev)
        pos_s = i32(n)
        H.sort_pairs(temp, keys, hs, pos, pos_s, n, end_bit)
        flags, segid, local_col = i32(n), i32(n), i32(n)
        uniq = torch.empty(n, dtype=torch.int64, device=dev)
        seg_start = i32(n + 1)
        n_uniq = torch.zeros(1, dtype=torch.int32, device=dev)
        scan_temp = torch.empty(max(1, H.scan_temp_bytes(n)), dtype=torch.uint8, device=dev)
        H.rle(hs, pos_s, n, flags, segid, scan_temp, uniq, seg_start, local_col, n_uniq, None,
              None)
        U = int(n_uniq.item())
        return uniq[:U], seg_start[:U + 1].to(torch.int64), pos_s, segid

    def _group_keys_dev(self, uf: torch.Tensor, cnt: torch.Tensor, info_g) -> torch.Tensor:
        """Device twin of ``_group_keys``: global sorted (flipped) kept keys of a group;
        G > 1 sums the counts at owner ranks (all-to-all-v) and all-gathers the kept
        lists (owner ranges are ordered, so the concatenation is sorted)."""
        freq = self.cfg.tail_freq
        if self.G == 1:
            return uf[cnt > freq] if freq > 0 else uf
        comm, dev = self.comm, self.device
        lo = int(_flip(np.array([info_g["min_key"]], np.uint64))[0])
        hi = int(_flip(np.array([info_g["max_key"] - 1], np.uint64))[0]) + 1
        bounds = torch.tensor([even_divide(lo, hi, self.G, r)[0] for r in range(1, self.G)],
                              dtype=torch.int64, device=dev)
        owner = torch.searchsorted(bounds, uf, right=True)
        sc = torch.bincount(owner, minlength=self.G).to(torch.int64)
        rc = comm.exchange_counts(sc).cpu()
        scl = sc.cpu()
        rk = comm.all_to_all_v(uf.contiguous(), scl.tolist(), rc.tolist()).to(dev)
        rn = comm.all_to_all_v(cnt.contiguous(), scl.tolist(), rc.tolist()).to(dev)
        if rk.numel():
            raw = rk ^ SIGN  # back to raw uint64 bits for the unsigned sort
            end_bit = max(1, int(info_g["max_key"] - 1).bit_length())
            u, seg, pos_s, segid = self._sort_unique(raw, end_bit)
            tot = torch.zeros(u.numel(), dtype=torch.int64, device=dev)
            tot.index_add_(0, segid[:rk.numel()].to(torch.int64) - 1, rn[pos_s[:rk.numel()].long()])
            uf2 = u ^ SIGN
            kept = uf2[tot > freq] if freq > 0 else uf2
        else:
            kept = torch.zeros(0, dtype=torch.int64, device=dev)
        n = torch.full((self.G,), kept.numel(), dtype=torch.int64)
        rcnt = comm.exchange_counts(n).cpu()
        return comm.all_to_all_v(kept.repeat(self.G), n.tolist(), rcnt.tolist()).to(dev)

    def _build_csc_gpu(self, data: SlotData):
        """CSC of the rank's examples over the global column space, on the device:
        per group one own radix sort + run-length encode of the keys (the sorted order
        IS the group's CSC order: columns ascending, rows ascending inside a column,
        so no separate transpose), tail filter on the device counts, global column
        map by a device searchsorted; only the kept key lists and the column pointer
        come back to the host (block division, model output). Same arrays as
        ``_build_csc_host`` bit for bit (tests/test_darlin_gpu.py)."""
        dev = self.device
        H = hipops()
        rows = data.rows
        if rows >= (1 << 31):
            raise ValueError("a rank holds at most 2^31-1 examples")
        self.rows = rows
        gt = {g: self._group_tensors(data, g) for g in sorted(data.groups)}
        # ExampleInfo on the device: unsigned min / max via the flipped order
        loc = {0: {"min_key": 0, "max_key": 1, "nnz_ele": rows, "nnz_ex": rows}}
        for g, (off, k, _) in gt.items():
            if k.numel() == 0:
                continue
            mn, mx = torch.aminmax(k ^ SIGN)
            ne = int((off[1:] > off[:-1]).sum().item())
            mn, mx = int(mn.item()) + (1 << 63), int(mx.item()) + (1 << 63)  # unflip
            loc[g] = {"min_key": mn, "max_key": mx + 1,
                      "nnz_ele": int(k.numel()), "nnz_ex": ne}
        local_info = {"num_ex": rows, "slots": loc}
        infos = self.comm.all_gather_obj(local_info) if self.G > 1 else [local_info]
        self.info = merge_slot_info(infos)
        self.num_ex = int(self.info["num_ex"])
        gids = sorted(g for g in self.info["slots"] if g != 0)
        valued = any(gt.get(g, (None, None, None))[2] is not None for g in gids)
        self.group_keys, self.group_base = {}, {}
        cols, rws, vals, counts = [], [], [], []
        base = 0
        for g in gids:
            off, k, v = gt.get(g, (None, torch.zeros(0, dtype=torch.int64, device=dev), None))
            n = k.numel()
            info_g = self.info["slots"][g]
            if n:
                end_bit = max(1, int(info_g["max_key"] - 1).bit_length())
                uniq, seg, pos_s, segid = self._sort_unique(k, end_bit)
                uf = uniq ^ SIGN
                cnt = seg[1:] - seg[:-1]
            else:
                uf = torch.zeros(0, dtype=torch.int64, device=dev)
                cnt = torch.zeros(0, dtype=torch.int64, device=dev)
            gk = self._group_keys_dev(uf, cnt, info_g)
            self.group_keys[g] = gk.cpu().numpy()
            self.group_base[g] = base
            ccount = torch.zeros(gk.numel(), dtype=torch.int64, device=dev)
            if n and gk.numel():
                p = torch.searchsorted(gk, uf)
                pc = p.clamp(max=gk.numel() - 1)
                hit = (p < gk.numel()) & (gk[pc] == uf)
                ucol = torch.where(hit, p + base, torch.full_like(p, -1))
                ccount.index_add_(0, pc[hit], cnt[hit])
                rows_of = torch.empty(n, dtype=torch.int32, device=dev)
                H.csr_rows(off, rows_of)
                ps = pos_s[:n].long()
                ck = ucol[segid[:n].long() - 1]
                keep = ck >= 0
                cols.append(ck[keep].to(torch.int32))
                rws.append(rows_of[ps][keep])
                if valued:
                    vv = torch.ones(n, dtype=torch.float32, device=dev) if v is None else v
                    vals.append(vv[ps][keep])
            counts.append(ccount)
            base += gk.numel()
        if base >= (1 << 31):
            raise ValueError("at most 2^31-1 global columns")
        col = torch.cat(cols) if cols else torch.zeros(0, dtype=torch.int32, device=dev)
        row = torch.cat(rws) if rws else torch.zeros(0, dtype=torch.int32, device=dev)
        val = (torch.cat(vals) if vals else torch.zeros(0, dtype=torch.float32, device=dev)) \
            if valued else None
        colptr = np.zeros(base + 1, np.int64)
        if base:
            colptr[1:] = torch.cumsum(torch.cat(counts), 0).cpu().numpy()
        return col, row, val, colptr, base, len(gids)

    def _finish_preprocess(self, data, col, row, val, colptr, base, ngroups):
        cfg = self.cfg
        dev = self.device
        self.num_cols = base
        self.colptr = colptr
        self.col, self.row, self.val = col, row, val
        self.y = torch.from_numpy(np.where(data.labels > 0, 1.0, -1.0).astype(np.float32)).to(dev)
        self.nnz = int(col.numel())
        # blocks: key ranges -> global column ranges
        self.blocks: list[Block] = []
        for g, a, b in divide_feature_blocks(self.info, cfg.block_ratio):
            gk = self.group_keys[g]
            fa = int(_flip(np.array([a], np.uint64))[0])
            fb = int(_flip(np.array([b - 1], np.uint64))[0])
            c0 = self.group_base[g] + int(np.searchsorted(gk, fa, side="left"))
            c1 = self.group_base[g] + int(np.searchsorted(gk, fb, side="right"))
            blk = Block(g, a, b, c0, c1, int(colptr[c0]), int(colptr[c1]))
            if dev.type == "cuda":
                blk.chunks = torch.from_numpy(bcd.build_chunks(
                    colptr, c0, c1, hot=_hot_piece(blk.p1 - blk.p0))).to(dev)
                # persistent [G | U], zeroed by the update that consumes it
                blk.gu = torch.zeros(2 * (c1 - c0), dtype=torch.float64, device=dev)
            self.blocks.append(blk)
        self.blk_order, self.prior_order = block_orders(self.blocks, cfg, self.rng)
        # row-sorted copy of every block's entries for the dual update: each example
        # has ~1 entry per block, so its margin update walks ym sequentially
        # (coalesced, uncontended atomics) instead of gathering it in column order
        self.col_r, self.row_r, self.val_r = self.col, self.row, self.val
        # fused row pass (bcd.rowpass): a block's dual update runs inside the next
        # block's gradient pass over dense per-example layouts (PSAMD_DARLIN_FUSE=0: the
        # separate kernels, for A/B)
        self.fuse_rows = dev.type == "cuda" and os.environ.get("PSAMD_DARLIN_FUSE", "1") != "0"
        self._pending_dual = None
        # workgroups of the row-order gradient and row pass and their partial-sum buffer
        self.rows_W = int(os.environ.get("PSAMD_BCD_W", "256"))
        rows_max = hipops().bcd_rows_max_cols() if dev.type == "cuda" else 0
        # (+ the row pass's segment sums behind the partials; hot-column passes of wide
        # blocks use fewer workgroups, rows_W_hot: their per-workgroup setup and partials
        # cover 2048 columns)
        # (256 = one workgroup per CU for both: 2.84 ms / pass vs 3.10 at 768 narrow,
        # 3.06 / 3.36 at 192 / 320 hot; profiles/r3_darlin_rowpass.log)
        self.rows_W_hot = int(os.environ.get("PSAMD_BCD_WHOT", "256"))
        nseg = hipops().bcd_part_segments() if dev.type == "cuda" else 0
        self.rows_part = (torch.empty((max(self.rows_W, self.rows_W_hot) + nseg) * 2 *
                                      max(rows_max, 1),
                                      dtype=torch.int64, device=dev)
                          if dev.type == "cuda" else None)
        # wide blocks: packed per-example gradient factors (bcd.grad rowq)
        self.rowq = (torch.empty(2 * self.rows, dtype=torch.float64, device=dev)
                     if dev.type == "cuda" else None)
        if dev.type == "cuda" and self.nnz:
            self.col_r, self.row_r = torch.empty_like(self.col), torch.empty_like(self.row)
            self.val_r = None if self.val is None else torch.empty_like(self.val)
            for blk in self.blocks:
                p0, p1 = blk.p0, blk.p1
                if p1 <= p0:
                    continue
                rs, perm = torch.sort(self.row[p0:p1], stable=True)
                # one entry per example and feature group (slot data): the dual
                # update needs no atomics
                blk.unique_rows = bool((rs[1:] != rs[:-1]).all()) if p1 - p0 > 1 else True
                self.row_r[p0:p1] = rs
                self.col_r[p0:p1] = self.col[p0:p1][perm]
                if self.val is not None:
                    self.val_r[p0:p1] = self.val[p0:p1][perm]
                # narrow blocks: gradient in row order too (sequential ym / y reads)
                if 0 < blk.ncols <= rows_max:
                    vmax = 1.0 if self.val is None else float(self.val[p0:p1].abs().max())
                    blk.row_mode = True
                    blk.fx_k = bcd.fixed_point_shift(p1 - p0, vmax)
                # dense per-example layout (4 B per example) for the fused row pass:
                # blocks with one entry per example covering >= 1/4 of the examples
                if self.fuse_rows and blk.unique_rows and 4 * (p1 - p0) >= self.rows:
                    blk.dcol, blk.dval = bcd.dense_rows(self.row_r, self.col_r, self.val_r,
                                                        p0, p1, blk.c0, self.rows)
                    # wide block: its hottest columns summed in LDS by the row pass, the
                    # cold ones by the chunked kernel (random per-entry gathers only for
                    # the cold share)
                    if not blk.row_mode and blk.chunks is not None:
                        hl = bcd.hot_layout(blk.dcol, colptr, blk.c0, blk.c1, nhot=rows_max)
                        if hl is not None:
                            blk.kenc, blk.hcols, cold, nh = hl
                            blk.chunks_cold = torch.from_numpy(cold).to(dev)
                            vmax = 1.0 if self.val is None else float(self.val[p0:p1].abs().max())
                            blk.fx_k = bcd.fixed_point_shift(nh, vmax)
                # wide block without a dense layout on < half of the examples (CTR-log
                # groups: ~1/15): its gradient gathers ym / y per entry instead of packing
                # rowq first (4 M examples, 17.5 us; even packing its own examples only,
                # bcd.grad urows=, 8.4 us, cost more than it saved: 19.1-19.6 vs 18.1 ms per
                # pass, profiles/r5_darlin_groups.log)
                if not blk.row_mode and blk.dcol is None:
                    blk.few_rows = 2 * torch.unique_consecutive(rs).numel() < self.rows
        # model state (replicated per rank) and margins
        f64 = torch.float64
        self.w = torch.full((base,), float(cfg.init_w), dtype=f64, device=dev)
        self.delta = torch.full((base,), float(cfg.delta_init), dtype=f64, device=dev)
        self.active = torch.ones(base, dtype=torch.uint8, device=dev)
        self.ym = torch.zeros(self.rows, dtype=f64, device=dev)
        if cfg.init_w != 0 and base:
            bcd.dual(self.col, self.row, self.val, 0, self.nnz, 0, base, self.w, self.y, self.ym)
        self.vio = torch.zeros(1, dtype=torch.int64, device=dev)
        # last-workgroup counter of the fused gradient + update (reset by the kernel)
        self._upd_ctr = torch.zeros(1, dtype=torch.int32, device=dev)
        # owned column share for the server-side statistics
        self.own = even_divide(0, base, self.G, self.rank)
        if self.verbose and self.rank == 0:
            print(f"Darlin: {self.num_ex} examples, {base} features in {ngroups} groups, "
                  f"{len(self.blocks)} blocks", file=sys.stderr)

    # -------------------------------------------------------------- one pass
    def _sharded(self, b: Block) -> bool:
        return self.shard and (self.cfg.shard_server == "on"
                               or b.ncols >= self.cfg.shard_min_cols)

    def _dual(self, b: Block, dw):
        """Dual update of block b: deferred into the next gradient's row pass when b has a
        dense layout (the next kernel touching the margins is always that gradient or a
        flush), else now."""
        self._flush_dual()
        if b.dcol is not None:
            self._pending_dual = (b, dw)
            return
        bcd.dual(self.col_r, self.row_r, self.val_r, b.p0, b.p1, b.c0, b.ncols, dw, self.y,
                 self.ym, b.unique_rows)

    def _defer_sums(self, b: Block, persistent: bool) -> bool:
        """Narrow dense block on one rank, launched into its persistent buffers: its row
        pass leaves the segment sums in b.part2 and the coordinate update adds them (one
        launch less per block; G / U never materialise). The same predicate is evaluated
        at launch and at finish."""
        return (persistent and self.G == 1 and b.row_mode and b.dcol is not None
                and not self._sharded(b))

    def _fused_update(self, b: Block, persistent: bool) -> bool:
        """Small narrow block without a dense layout, one rank, persistent buffers: its
        row-order gradient applies the coordinate update in its last workgroup (dw kept
        in b.dw for the dual update at finish: the block's columns belong to no other
        block, so the earlier update changes nothing). Same predicate at launch and
        finish."""
        return (persistent and self.G == 1 and b.row_mode and b.dcol is None
                and not self._sharded(b) and b.p1 - b.p0 <= _SMALL_ROWS_BLOCK)

    def _flush_dual(self):
        """Apply a deferred dual update on its own (before anything else reads ym)."""
        if self._pending_dual is None:
            return
        j, dw = self._pending_dual
        self._pending_dual = None
        bcd.rowpass(self.ym, self.y, self.delta, self.active, jcol=j.dcol, jval=j.dval,
                    jdw=dw, jncols=j.ncols)

    def _grad(self, b: Block, G, U, zeroed: bool):
        """Block gradient into G / U: row order for narrow blocks, the load-balanced
        column-order kernel otherwise. With a dense layout the pending dual update of
        the previous block runs in the same row pass."""
        if b.dcol is not None and (b.row_mode or b.chunks is not None):
            jd = {}
            if self._pending_dual is not None:
                j, dw = self._pending_dual
                self._pending_dual = None
                jd = dict(jcol=j.dcol, jval=j.dval, jdw=dw, jncols=j.ncols)
            if b.row_mode:
                p2 = None
                if self._defer_sums(b, zeroed):  # the update reads the segment sums itself
                    if b.part2 is None:
                        b.part2 = torch.empty(hipops().bcd_part_segments() * 2 * b.ncols,
                                              dtype=torch.int64, device=self.device)
                    p2 = b.part2
                bcd.rowpass(self.ym, self.y, self.delta, self.active, kcol=b.dcol, kval=b.dval,
                            c0=b.c0, ncols=b.ncols, k2=b.fx_k, W=self.rows_W,
                            part=self.rows_part, G=G, U=U, part2=p2, tau32=self.cfg.tau32, **jd)
                return
            if b.hcols is not None:  # hot columns in LDS, cold ones column by column
                if not zeroed:  # (the reduce stores the hot sums before the chunk pass)
                    G.zero_()
                    U.zero_()
                bcd.rowpass(self.ym, self.y, self.delta, self.active, kcol=b.kenc, kval=b.dval,
                            c0=b.c0, ncols=b.ncols, k2=b.fx_k, W=self.rows_W_hot,
                            part=self.rows_part, G=G, U=U, rowq=self.rowq, hcols=b.hcols, tau32=self.cfg.tau32, **jd)
                bcd.grad(self.col, self.row, self.val, b.p0, b.p1, b.c0, b.ncols, self.ym,
                         self.y, self.delta, self.active, G, U, chunks=b.chunks_cold,
                         zeroed=True, rowq=self.rowq, rowq_ready=True)
                return
            bcd.rowpass(self.ym, self.y, self.delta, self.active, kcol=b.dcol, kval=b.dval,
                        c0=b.c0, ncols=b.ncols, rowq=self.rowq, tau32=self.cfg.tau32, **jd)
            bcd.grad(self.col, self.row, self.val, b.p0, b.p1, b.c0, b.ncols, self.ym, self.y,
                     self.delta, self.active, G, U, chunks=b.chunks, zeroed=zeroed,
                     rowq=self.rowq, rowq_ready=True)
            return
        self._flush_dual()
        if self._fused_update(b, zeroed):
            # small narrow block: gradient + coordinate update in one launch of a few
            # workgroups (no 256-workgroup partials pass, no reduce, no update launch)
            if b.part2 is None:
                b.part2 = torch.zeros(2 * b.ncols, dtype=torch.int64, device=self.device)
                b.dw = torch.empty(b.ncols, dtype=torch.float64, device=self.device)
            c = self.cfg
            # (8 workgroups for a ~60 k-entry block: 17.3 ms per pass vs 18.1 at 4, 18.2 at
            # ~15, 18.1 at 32, 20.6 at 64; profiles/r5_darlin_groups.log)
            W = _FUSED_W or max(8, min(32, (b.p1 - b.p0) // 8192))
            bcd.grad_rows(self.col_r, self.row_r, self.val_r, b.p0, b.p1, b.c0, b.ncols, self.ym,
                          self.y, self.delta, self.active, G, U, b.part2, W, b.fx_k,
                          upd=dict(w=self.w, dw=b.dw, vio=self.vio, counter=self._upd_ctr,
                                   eta=c.eta, lam=c.l1, delta_max=c.delta_max,
                                   kkt_thr=self.kkt_thr))
            return
        if b.row_mode:
            bcd.grad_rows(self.col_r, self.row_r, self.val_r, b.p0, b.p1, b.c0, b.ncols, self.ym,
                          self.y, self.delta, self.active, G, U, self.rows_part, self.rows_W,
                          b.fx_k)
            return
        bcd.grad(self.col, self.row, self.val, b.p0, b.p1, b.c0, b.ncols, self.ym, self.y,
                 self.delta, self.active, G, U, chunks=b.chunks, zeroed=zeroed,
                 rowq=self.rowq if b.chunks is not None and not b.few_rows else None)

    def _launch(self, b: Block):
        if self._sharded(b):
            return self._launch_sharded(b)
        # the block's persistent [G | U] unless a previous launch of the same block is
        # still in flight (a prior block re-launched within the delay window)
        zeroed = b.gu is not None and not b.busy
        GU = b.gu if zeroed else torch.empty(2 * b.ncols, dtype=torch.float64, device=self.device)
        if zeroed:
            b.busy = True
        G, U = GU[:b.ncols], GU[b.ncols:]
        self._grad(b, G, U, zeroed)
        work = self.comm.all_reduce_async(GU) if self.G > 1 else None
        return (b, GU, work, zeroed)

    def _finish(self, item):
        if self._sharded(item[0]):
            return self._finish_sharded(item)
        b, GU, work, persistent = item
        if work is not None:
            work.wait()
        G, U = GU[:b.ncols], GU[b.ncols:]
        c = self.cfg
        if self._fused_update(b, persistent):  # (updated by its gradient launch)
            b.busy = False
            self._dual(b, b.dw)
            return
        p2 = b.part2 if self._defer_sums(b, persistent) else None
        dw, _ = bcd.update(b.c0, b.ncols, G, U, self.w, self.delta, self.active, c.eta, c.l1,
                           c.delta_max, self.kkt_thr, vio=self.vio, consume=persistent,
                           part2=p2, k2=b.fx_k)
        if persistent:
            b.busy = False
        self._dual(b, dw)

    # ---- sharded server (G > 1): rank r owns the r-th even slice of every block
    def _own_slice(self, b: Block) -> tuple[int, int, int]:
        """(m, own0, own1): the block's slice width m = ceil(ncols / G) and this rank's
        columns [own0, own1) relative to c0 (empty past ncols)."""
        m = -(-b.ncols // self.G)
        j0 = min(self.rank * m, b.ncols)
        return m, j0, min(j0 + m, b.ncols)

    def _launch_sharded(self, b: Block):
        """Worker half of a block: gradient into a [G | U] padded to G equal slices,
        then two reduce-scatters over RCCL: every owner receives the sums of its slice
        only (the reference's push of G, U to the servers of the block's key range,
        darlin.h:318-354, each server summing what its workers pushed)."""
        m, _, _ = self._own_slice(b)
        P = m * self.G
        dev = self.device
        GU = torch.zeros(2 * P, dtype=torch.float64, device=dev)
        self._grad(b, GU[:b.ncols], GU[P:P + b.ncols], True)
        mine = torch.empty(2 * m, dtype=torch.float64, device=dev)
        w1 = self.comm.reduce_scatter_async(mine[:m], GU[:P])
        w2 = self.comm.reduce_scatter_async(mine[m:], GU[P:])
        return (b, mine, (w1, w2))

    def _finish_sharded(self, item):
        """Server half on the owner's slice (the coordinate update of darlin.h:206-246
        with NaN marks for KKT-filtered columns), one all-gather of the block's dw (the
        workers' pull of the new weights), then every rank replays the other owners'
        updates on its replica and applies the dual update."""
        b, mine, works = item
        for wk in works:
            wk.wait()
        m, j0, j1 = self._own_slice(b)
        c = self.cfg
        dwo = torch.zeros(m, dtype=torch.float64, device=self.device)
        bcd.update(b.c0 + j0, j1 - j0, mine[:m], mine[m:], self.w, self.delta, self.active,
                   c.eta, c.l1, c.delta_max, self.kkt_thr, dw=dwo, vio=self.vio,
                   nan_filtered=True)
        dw = torch.empty(m * self.G, dtype=torch.float64, device=self.device)
        self.comm.all_gather_into_async(dw, dwo).wait()
        bcd.replica(b.c0, b.ncols, j0, j1, dw, self.w, self.delta, self.active, c.delta_max)
        self._dual(b, dw)

    def run_pass(self, it: int, reset_kkt: bool = False) -> BCDProgress:
        cfg = self.cfg
        order = list(self.blk_order)
        if cfg.random_order:
            self.rng.shuffle(order)
        nprior = 0
        if it == 0:
            order = list(self.prior_order) + order
            nprior = len(self.prior_order)
        if reset_kkt:
            self.active.fill_(1)
        self.vio.zero_()  # kkt threshold set at the first block of the pass: violation_ = 0
        t0 = time.time()
        inflight: deque = deque()
        for i, k in enumerate(order):
            tau = 0 if i < nprior else cfg.tau  # prior blocks: zero delay (darlin.h:86-88)
            while inflight and inflight[0][0] <= i - tau - 1:
                self._finish(inflight.popleft()[1])
            inflight.append((i, self._launch(self.blocks[k])))
        while inflight:
            self._finish(inflight.popleft()[1])
        prog = self.evaluate()
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        busy = time.time() - t0
        prog.busy_time = [busy]
        prev = self.progress[-1].objective if self.progress else None
        prog.relative_obj = 1.0 if prev is None else prev / prog.objective - 1
        prog.total_time = (self.progress[-1].total_time if self.progress else 0.0) + busy
        self.progress.append(prog)
        return prog

    def evaluate(self) -> BCDProgress:
        """Objective = sum_i log(1+exp(-ym_i)) + l1 * ||w||_1 (darlin.h:248-265, 504-511)."""
        self._flush_dual()
        obj = bcd.objective(self.ym)
        st = bcd.server_stats(self.w, self.active, self.own[0], self.own[1])
        vio = self.vio.view(torch.float64)
        if self.G > 1:
            buf = torch.cat([obj, st])
            self.comm.all_reduce_(buf)
            v = vio.clone()
            self.comm.all_reduce_(v, op="max")
            obj, st, vio = buf[:1], buf[1:], v
        h = torch.cat([obj, st, vio]).cpu().tolist()
        return BCDProgress(objective=h[0] + self.cfg.l1 * h[1], nnz_w=int(h[2]),
                           nnz_active_set=int(h[3]), violation=h[4])

    def train(self, printer=None) -> list[BCDProgress]:
        """The scheduler loop of darlin.h:50-126."""
        cfg = self.cfg
        reset = False
        for it in range(cfg.max_pass):
            prog = self.run_pass(it, reset_kkt=reset)
            if printer is not None:
                printer(it, prog, self)
            self.kkt_thr = prog.violation / max(self.num_ex, 1) * cfg.kkt_ratio
            rel = prog.relative_obj
            if 0 < rel <= cfg.epsilon:
                if reset:
                    break
                reset = True
            else:
                reset = False
        return self.progress

    # ------------------------------------------------------------ model I/O
    def model(self) -> tuple[np.ndarray, np.ndarray]:
        """(raw uint64 keys, fp64 weights) of all global columns, group by group."""
        keys = np.concatenate([_unflip(self.group_keys[g]) for g in sorted(self.group_keys)]) \
            if self.group_keys else np.zeros(0, np.uint64)
        return keys, self.w.cpu().numpy()

    def save_model(self, prefix: str, node_id: str | None = None) -> str:
        """Text ``key\\tw`` of the non-zero weights in this rank's server key range
        (reference BCDServer::saveModel, src/learner/bcd.h:251-272; server s owns
        Range::all().evenDivide(S, s), src/system/postmaster.cc:17-31)."""
        from ..utils.checkpoint import write_text_model

        keys, w = self.model()
        lo, hi = even_divide(0, 1 << 64, self.G, self.rank)
        ku = keys.astype(np.uint64)
        m = (ku >= np.uint64(lo)) & ((ku < np.uint64(hi)) if hi < (1 << 64) else True)
        m &= (w != 0) & ~np.isnan(w)
        path = f"{prefix}_{node_id or f'S{self.rank}'}"
        write_text_model(path, ku[m], w[m])
        return path


# ----------------------------------------------------------------- printing
def show_progress(it: int, prog: BCDProgress, trainer: DarlinTrainer, out=sys.stderr):
    """The three tables of darlin.h:136-156 / bcd.h:146-178."""
    if it == 0:
        out.write("     |        training        |  sparsity |      KKT filter     |    time (sec.)\n")
        out.write("iter |  objective    relative |     |w|_0 | threshold  #activet |(app:min max) total\n")
        out.write(" ----+------------------------+-----------+---------------------+-----------------\n")
    bt = prog.busy_time or [0.0]
    dt = prog.total_time - (trainer.progress[-2].total_time if len(trainer.progress) > 1 else 0)
    out.write(f"{it:4d} | {prog.objective:.5e}  {prog.relative_obj:.3e} |{prog.nnz_w:10d} "
              f"| {trainer.kkt_thr:.1e} {prog.nnz_active_set:11d} "
              f"|{min(bt):6.1f}{max(bt):6.1f}{dt:6.1f}\n")
    out.flush()
