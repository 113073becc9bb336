"""Wide & deep CTR model on a sharded embedding table (BASELINE.json config 5).

Not a reference model: the reference only *declares* dense value blocks
(KVVector with k values per key, src/parameter/kv_vector.h:13-100; SArray
segments); BASELINE.json names "embedding table 10^9 x 128 sharded across
8 x 288 GB HBM, dense-block push/pull + MFMA GEMM" as a target workload.

Per rank (one process per GPU):
* embedding shard (model parallel): key -> 32-B KV slot (wide weight w + FTRL
  state, the sparse-LR table) and a bf16 row of D at the same slot index, with
  row-wise AdaGrad (``ops.embedding.EmbeddingShard``); keys are mixed and
  range-partitioned like the sparse-LR keys;
* minibatch: localise the B x S keys (sort / RLE kernels), pull [row | w] for
  the unique keys (G > 1: ONE all-to-all of packed 65-word records each way),
  expand to X0 [B, S*D] (bf16), MLP (S*D -> hidden... -> 1, ReLU) on the bf16
  MFMA GEMM with fused bias/ReLU epilogues, wide margin + deep logit in one head
  kernel (logistic loss, accuracy, AUC histogram, head gradients);
* backward: input / weight gradients on the same GEMM (ReLU masks fused, split-K
  weight gradients), embedding gradients reduced per unique key in CSC order,
  wide gradients by the sparse-LR segmented reduction; push [bf16 grad row |
  wide grad] to the owners, which apply AdaGrad rows + FTRL wide weights;
* dense MLP (data parallel): fp32 master weights in one flat buffer, ONE RCCL
  all-reduce of the flat gradient per step, fused Adam writing the bf16 copy.
"""
from __future__ import annotations

import math
import os
import time
from dataclasses import dataclass, field

import torch

from ..ops import embedding as E
from ..ops import gemm as GM
from ..ops.keymix import key_bits_for, mix, unmix
from ..ops.kv_table import UpdateRule, next_pow2
from ..ops.linear import AUC_BINS, accum_total, auc_from_hist, linear_backward, new_accum
from ..ops.localize import Localizer
from ..ops.native import hipops
from ..parallel.comm import Comm, LocalComm
from ..parallel.partition import KeyPartition


@dataclass
class WideDeepConfig:
    num_features: int = 10 ** 9          # hashed key space (whole job)
    embedding_dim: int = 128
    slots: int = 39                      # keys per example (Criteo: 13 int + 26 categorical)
    hidden: tuple = (1024, 512, 256)
    minibatch: int = 16384               # per rank
    emb_lr: float = 0.05                 # row-wise AdaGrad
    emb_init_scale: float = 0.01
    mlp_lr: float = 1e-3                 # Adam
    wide: UpdateRule = field(default_factory=lambda: UpdateRule("ftrl", "decay", 0.05, 1.0,
                                                                 0.5, 1.0))
    table_capacity: int = 0              # slots per rank (0 = auto)
    table_load: float = 0.5
    max_table_bytes: int = 160 << 30     # HBM budget of one shard (slots + rows)
    gemm: str = "auto"                   # auto (measured per product) | mfma | hipblaslt
    overlap_wgrad: bool = True           # GPU: weight-gradient GEMMs on a side stream
    exchange: str = "padded"             # G > 1 on GPU: sync-free fixed rows | "exact"
    exchange_slack: float = 1.5          # padded row capacity = slack x first max + 1024
    exchange_capacity: int = 0           # explicit per-peer capacity (0 = from slack)
    localize: str = "sort"               # GPU key localisation: "sort" (deterministic) | "part"
    seed: int = 0


class EmbeddingPS:
    """Sparse side shared by the embedding models (wide & deep, factorization
    machine): pull [bf16 row | wide weight] records of a minibatch's unique keys
    from their owners and push [row gradient | wide gradient] back, one packed
    all-to-all each way. Needs ``shard``, ``part``, ``comm``, ``G``, ``gpu``,
    ``stats`` and ``cfg.{embedding_dim, emb_lr, wide}`` on the host class."""

    # one-shard GPU step, PSAMD_WD_FUSE=1: the wide gradient rides along the embedding
    # gradient reduction and the wide slot update along the row update. Fewer kernels, but
    # the step measured 0.963-0.971 vs 0.956-0.958 ms with separate passes on one box
    # (the weight-gradient side stream sets the pace; profiles/r4_wide_deep_fusion_ab.log),
    # so the separate passes stay the default
    _fuse = os.environ.get("PSAMD_WD_FUSE", "0") == "1"
    _defer_reduce = os.environ.get("PSAMD_WD_DEFER_REDUCE", "0") == "1"

    def localize(self, keys: torch.Tensor, buf: int = 0):
        """Localise a minibatch into workspace ``buf`` (buffer 0 = the step's own), so
        the next minibatch can be prepared on a side stream while a step trains
        (``step(..., loc=...)``)."""
        locs = self.__dict__.setdefault("_localizers", [self.localizer])
        while len(locs) <= buf:
            locs.append(Localizer(self.max_nnz, self.bits, self.device,
                                  mode=getattr(self.cfg, "localize", "sort")))
        return locs[buf](keys)

    # ------------------------------------------------------------ checkpoint
    _dense_state: tuple = ()  # replicated dense tensors saved with the shard

    def state_dict(self) -> dict:
        """Resume snapshot of this rank: the shard's keys (raw ids, so a snapshot reloads
        under any world size), wide FTRL state, embedding rows + AdaGrad accumulators,
        the replicated dense state and the step counter. Write with
        ``utils.checkpoint.save_snapshot``; merge ranks with ``merge_state_dicts``.
        (The reference has no resume path: src/parameter/kv_store.h:63-73 only writes
        the text model; src/app/factor_machine has no checkpoint at all.)"""
        if self.gpu:
            torch.cuda.synchronize(self.device)
        self._xe_check()  # a dropped pull / push must not be written as a valid state
        st = self.shard.state()
        sd = {"keys": unmix(st.pop("mkeys"), self.bits).cpu()}
        sd.update({k: v.cpu() for k, v in st.items()})
        for name in self._dense_state:
            sd[name] = getattr(self, name).detach().cpu()
        sd.update(step=self.step_count, examples=int(self.examples), bits=self.bits,
                  rank=self.rank, world=self.G, dim=self.cfg.embedding_dim,
                  model=type(self).__name__, wide_rule=self._wide_rule_tag())
        return sd

    _SHARD_KEYS = ("keys", "w", "z", "n", "rows", "acc", "cnt")

    def _wide_rule_tag(self) -> str:
        r = self.cfg.wide
        return f"{r.algo}/{r.lr_type}"

    @staticmethod
    def merge_state_dicts(sds: list) -> dict:
        """Concatenate per-rank snapshots (key-disjoint shards; dense state and counters
        are replicated, taken from the first)."""
        out = dict(sds[0])
        for k in EmbeddingPS._SHARD_KEYS:
            if k in out:
                out[k] = torch.cat([sd[k] for sd in sds])
        return out

    def load_state_dict(self, sd: dict, chunk: int = 1 << 24) -> None:
        """Load the keys this rank owns (any world size wrote ``sd``) and the dense state.

        Ownership is decided on the host (mix + owner_of have CPU paths) and only the
        owned slice travels to the device, ``chunk`` keys at a time: a merged snapshot of
        a 1e9 x 128 table (~256 GB of rows) never has to fit on one GPU."""
        if int(sd["bits"]) != self.bits or int(sd["dim"]) != self.cfg.embedding_dim:
            raise ValueError(f"snapshot bits/dim {sd['bits']}/{sd['dim']} != "
                             f"{self.bits}/{self.cfg.embedding_dim}")
        model = sd.get("model")
        if model is not None and str(model) != type(self).__name__:
            raise ValueError(f"snapshot of a {model}, not a {type(self).__name__}")
        rule = sd.get("wide_rule")
        if rule is not None and str(rule) != self._wide_rule_tag():
            raise ValueError(f"snapshot wide rule {rule} != {self._wide_rule_tag()}")
        if rule is None or "cnt" not in sd:
            if self.cfg.wide.algo.lower() in ("sgd", "standard") and \
                    self.cfg.wide.lr_type.lower() == "decay":
                raise ValueError("snapshot has no update counts; a decaying SGD wide rule "
                                 "cannot resume from it")
        keys = sd["keys"].cpu()
        for a in range(0, keys.numel(), chunk):
            mk = mix(keys[a:a + chunk].contiguous(), self.bits)
            own = torch.nonzero(self.part.owner_of(mk) == self.rank).flatten()
            if own.numel() == 0:
                continue
            vals = [sd[k][a:a + chunk][own].to(self.device) for k in ("w", "z", "n", "rows", "acc")]
            cnt = sd["cnt"][a:a + chunk][own].to(self.device) if "cnt" in sd else None
            self.shard.load_state(mk[own].to(self.device), *vals, cnt=cnt)
        for name in self._dense_state:
            getattr(self, name).copy_(sd[name].to(self.device))
        if "param" in self._dense_state:
            self.param16.copy_(self.param.to(torch.bfloat16))
        self.step_count = int(sd.get("step", 0))
        if hasattr(self, "step_dev"):  # the device step clock Adam reads
            self.step_dev.fill_(self.step_count)
        self.examples = int(sd.get("examples", 0))

    def prefill(self, count: int, chunk: int = 1 << 23, seed: int = 12345) -> int:
        """Insert ``count`` random keys of this shard's mixed-key range with initialised
        rows (the populated-table regime of a long run); returns the occupied slots."""
        from ..ops.keymix import random_keys_in_range

        # the table's own key range (the loopback emulation's one rank owns all G ranges)
        lo, hi = self.shard.table.key_range or self.part.range_of(self.rank)
        g = torch.Generator(device=self.device).manual_seed(seed + self.rank)
        done = 0
        while done < count:
            n = min(chunk, count - done)
            mk = random_keys_in_range(lo, hi, n, g, self.device)
            self.shard.resolve(mk)
            done += n
        self.shard.table.check_ok()
        return self.shard.table.census()[0]

    # ------------------------------------------------------------ exchange (G > 1)
    _xe = None  # padded-exchange state (GPU, G > 1)

    def _padded(self) -> bool:
        return self.gpu and self.G > 1 and getattr(self.cfg, "exchange", "padded") == "padded"

    def _xe_setup(self, off):
        """Per-peer capacity C agreed by all ranks (slack x the largest per-peer count of
        the first minibatch + 1024, a multiple of 8) and the fixed exchange buffers."""
        from types import SimpleNamespace

        cfg, G, dev = self.cfg, self.G, self.device
        cnt = (off[1:] - off[:-1]).max().reshape(1).to(torch.int64)
        cnt = cnt if self.comm.backend == "nccl" else cnt.cpu()
        m = int(self.comm.all_reduce_(cnt, op="max").item())
        C = getattr(cfg, "exchange_capacity", 0) or \
            int(math.ceil(m * getattr(cfg, "exchange_slack", 1.5))) + 1024
        C = (C + 7) // 8 * 8
        kw = 1 if self.bits <= 32 else 2
        D = cfg.embedding_dim
        H, Q = (4 + C * kw + 1 + 3) // 4 * 4, C * (D // 2) + C  # row geometry of exchange.hip
        i32 = dict(dtype=torch.int32, device=dev)
        self._xe = SimpleNamespace(
            C=C, kw=kw, H=H, Q=Q, D=D,
            send_k=torch.zeros(G * H, **i32), recv_k=torch.zeros(G * H, **i32),
            slot=torch.full((G * C,), -1, dtype=torch.int64, device=dev),
            w=torch.zeros(G * C, dtype=torch.float32, device=dev),
            rec_s=torch.zeros(G * Q, **i32), rec_r=torch.zeros(G * Q, **i32),
            grad_s=torch.zeros(G * Q, **i32), grad_r=torch.zeros(G * Q, **i32),
            ovf=torch.zeros(1, **i32),
            rows_u=torch.zeros(self.max_nnz, D, dtype=torch.bfloat16, device=dev),
            w_u=torch.zeros(self.max_nnz, dtype=torch.float32, device=dev))

    def _xe_check(self):
        if self._xe is not None:
            ovf = int(self._xe.ovf.item())
            if ovf:
                raise RuntimeError(
                    f"padded exchange overflow: {ovf} keys exceeded the per-peer capacity "
                    f"{self._xe.C} (pulled as zero rows, not pushed); set exchange_capacity "
                    f"or exchange_slack higher, or exchange='exact'")

    def _pull_padded(self, loc):
        """Sync-free pull (no sizes on the host): pack keys into fixed rows of C ->
        equal-split all-to-all -> owner: one resolve / row-init / record-gather launch
        for all G rows -> all-to-all of [row | w] records -> unpack in key order."""
        off = self.part.split_sorted(loc.uniq, loc.n_uniq)
        if self._xe is None:
            self._xe_setup(off)
        xe, hh, tb = self._xe, hipops(), self.shard.table
        hh.xchg_pack_keys(loc.uniq, loc.n_uniq, off, xe.C, xe.kw, xe.H, xe.send_k, xe.ovf)
        self.comm.all_to_all_fixed(xe.send_k, xe.recv_k)
        it, iv, isd, seed = tb.init.args()
        hh.kv_resolve_rows(tb.slots, xe.recv_k, xe.H, xe.C, xe.kw, xe.slot, xe.w, True, it, iv,
                           isd, seed, tb._err, tb._inserted, tb.home_base, tb.home_m)
        hh.emb_padded_serve(xe.recv_k, xe.H, xe.C, xe.kw, xe.slot, xe.w, self.shard.rows,
                            self.shard.inited, self.shard.seed, self.shard.init_scale, xe.rec_s)
        self.comm.all_to_all_fixed(xe.rec_s, xe.rec_r)
        hh.emb_unpack_records(xe.rec_r, xe.C, off, loc.n_uniq, xe.rows_u, xe.w_u)
        return xe.rows_u, xe.w_u, ("padded", off)

    def _push_padded(self, loc, off, dE, g_wide):
        """[dE | wide grad] into the owners' rows -> all-to-all -> one row-wise AdaGrad and
        one wide update per source row (rank order), counts read on the device."""
        cfg, xe = self.cfg, self._xe
        C, D, Q, H = xe.C, xe.D, xe.Q, xe.H
        hipops().emb_pack_grads(dE, g_wide, off, loc.n_uniq, C, xe.grad_s)
        self.comm.all_to_all_fixed(xe.grad_s, xe.grad_r)
        for s in range(self.G):
            chunk = xe.grad_r[s * Q:(s + 1) * Q]
            g16 = chunk[:C * (D // 2)].view(torch.bfloat16).view(C, D)
            gw = chunk[C * (D // 2):].view(torch.float32)
            n_dev = xe.recv_k[s * H:s * H + 1]  # keys this source pulled (its row header)
            slot_s = xe.slot[s * C:(s + 1) * C]
            self.shard.update_rows(slot_s, grad16=g16, lr=cfg.emb_lr, n_dev=n_dev)
            self.shard.update_wide(slot_s, gw, cfg.wide, self.stats, n_dev=n_dev)

    def _pull(self, loc):
        """Owner split -> keys all-to-all -> resolve + gather [row | w] -> records back."""
        if self._padded():
            return self._pull_padded(loc)
        D = self.cfg.embedding_dim
        U = loc.num_unique()
        off = self.part.split_sorted(loc.uniq, loc.n_uniq).cpu()
        send = (off[1:] - off[:-1]).tolist()
        recv = self.comm.exchange_counts(torch.tensor(send, dtype=torch.int64)).cpu().tolist()
        rk = self.comm.all_to_all_v(loc.uniq[:U].contiguous(), send, recv)
        slot, w = self.shard.resolve(rk)
        rec = self._pack(self.shard.gather_rows(slot), w)
        back = self.comm.all_to_all_v(rec, recv, send)
        rows_u, w_u = self._unpack(back, D)
        return rows_u, w_u, ("dist", slot, send, recv, U)

    @staticmethod
    def _pack(rows16: torch.Tensor, w32: torch.Tensor) -> torch.Tensor:
        """[n, D] bf16 + [n] f32 -> [n, D/2 + 1] int32 records (one all-to-all)."""
        n, D = rows16.shape
        rec = torch.empty(n, D // 2 + 1, dtype=torch.int32, device=rows16.device)
        rec[:, :D // 2] = rows16.contiguous().view(torch.int32).view(n, D // 2)
        rec[:, D // 2] = w32.contiguous().view(torch.int32)
        return rec

    @staticmethod
    def _unpack(rec: torch.Tensor, D: int):
        n = rec.shape[0]
        rows16 = rec[:, :D // 2].contiguous().view(torch.bfloat16).view(n, D)
        w32 = rec[:, D // 2].contiguous().view(torch.float32)
        return rows16, w32

    def _push(self, loc, push, dE, g_wide):
        cfg = self.cfg
        if push[0] == "local":
            slot = push[1]
            n_dev = loc.n_uniq if self.gpu else None
            if self.gpu and not self._fuse:
                self.shard.update_rows(slot, grad=dE, lr=cfg.emb_lr, n_dev=n_dev)
                hipops().kv_update(self.shard.table.slots, slot, g_wide, n_dev,
                                   *cfg.wide.args(), self.stats)
            elif self.gpu:
                # rows (AdaGrad) and wide slots (cfg.wide) of the same keys in ONE pass
                hipops().emb_update(slot, n_dev, dE, None, self.shard.rows, self.shard.acc,
                                    cfg.emb_lr, 1e-8, self.shard.table.slots, g_wide,
                                    list(cfg.wide.args()), self.stats)
            else:
                U = loc.num_unique()
                self.shard.update_rows(slot[:U], grad=dE[:U], lr=cfg.emb_lr)
                self.shard.update_wide(slot[:U], g_wide[:U], cfg.wide, self.stats)
            return
        if push[0] == "padded":
            self._push_padded(loc, push[1], dE, g_wide)
            return
        _, slot, send, recv, U = push
        D = cfg.embedding_dim
        rec = self._pack(dE[:U].to(torch.bfloat16), g_wide[:U])
        got = self.comm.all_to_all_v(rec, send, recv)
        g16, gw = self._unpack(got, D)
        a = 0
        for s in range(self.G):  # one update per source (slots unique within a source)
            n = recv[s]
            if n:
                self.shard.update_rows(slot[a:a + n], grad16=g16[a:a + n], lr=cfg.emb_lr)
                self.shard.update_wide(slot[a:a + n], gw[a:a + n].contiguous(), cfg.wide,
                                       self.stats)
            a += n


class WideDeepTrainer(EmbeddingPS):
    _dense_state = ("param", "m", "v")  # MLP params + Adam moments

    def __init__(self, cfg: WideDeepConfig, comm: Comm | None = None, device="cpu"):
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
        # ---- dense MLP: flat fp32 params / grads / Adam state, bf16 copy for the GEMMs
        dims = [S * D] + list(cfg.hidden)
        shapes = []
        for i in range(len(cfg.hidden)):
            shapes += [(dims[i + 1], dims[i]), (dims[i + 1],)]
        shapes += [(dims[-1],), (1,)]  # head w, b
        sizes = [math.prod(s) for s in shapes]
        P = sum(sizes)
        self.param = torch.zeros(P, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(P, dtype=torch.float32, device=dev)
        self.m = torch.zeros(P, dtype=torch.float32, device=dev)
        self.v = torch.zeros(P, dtype=torch.float32, device=dev)
        self.param16 = torch.zeros(P, dtype=torch.bfloat16, device=dev)
        gen = torch.Generator().manual_seed(cfg.seed + 1)  # identical on every rank
        views, gviews, v16, off = [], [], [], 0
        for s, n in zip(shapes, sizes):
            views.append(self.param[off:off + n].view(s))
            gviews.append(self.grad[off:off + n].view(s))
            v16.append(self.param16[off:off + n].view(s))
            off += n
        for i in range(len(cfg.hidden)):
            views[2 * i].copy_(E.xavier(dims[i + 1], dims[i], gen).to(dev))
        views[-2].copy_((torch.rand(dims[-1], generator=gen) * 2 - 1).to(dev) / math.sqrt(dims[-1]))
        self.param16.copy_(self.param.to(torch.bfloat16))
        nl = len(cfg.hidden)
        self.W = [views[2 * i] for i in range(nl)]
        self.b = [views[2 * i + 1] for i in range(nl)]
        self.W16 = [v16[2 * i] for i in range(nl)]
        self.b16 = [v16[2 * i + 1] for i in range(nl)]
        self.dW = [gviews[2 * i] for i in range(nl)]
        self.db = [gviews[2 * i + 1] for i in range(nl)]
        self.w_head, self.b_head = views[-2], views[-1]
        self.dw_head, self.db_head = gviews[-2], gviews[-1]
        self.dims = dims
        self.num_params = P
        # ---- buffers / metrics
        self.coef = torch.empty(B, dtype=torch.float32, device=dev)
        self.metrics = new_accum(dev)
        self.stats = new_accum(dev)
        self.hist = torch.zeros(2 * AUC_BINS, dtype=torch.int32, device=dev)
        self.step_dev = torch.zeros(1, dtype=torch.int64, device=dev)
        if self.gpu:
            self.slot_buf = torch.empty(self.max_nnz, dtype=torch.int64, device=dev)
            self.w_buf = torch.empty(self.max_nnz, dtype=torch.float32, device=dev)
            self.dE = torch.empty(self.max_nnz, D, dtype=torch.float32, device=dev)
        self._side = torch.cuda.Stream(dev) if self.gpu else None
        self.step_count = 0
        self.examples = 0
        self.t0 = time.time()

    # ------------------------------------------------------------------ step
    def step(self, keys: torch.Tensor, labels: torch.Tensor, loc=None):
        """One minibatch (``keys`` [B*S] raw feature ids, row-major; ``labels`` [B];
        ``loc``: its localisation from ``localize`` if already prepared)."""
        cfg, dev = self.cfg, self.device
        S, D = cfg.slots, cfg.embedding_dim
        B = labels.numel()
        nnz = B * S
        if keys.numel() != nnz:
            raise ValueError(f"expected {nnz} keys, got {keys.numel()}")
        loc = self.localizer(keys) if loc is None else loc
        # ---------------- pull rows + wide weights of the unique keys
        if self.G == 1:
            if self.gpu:
                slot, w_wide = self.shard.resolve(loc.uniq, loc.n_uniq, self.slot_buf, self.w_buf)
            else:
                slot, w_wide = self.shard.resolve(loc.uniq[:loc.num_unique()])
            X0 = E.expand(loc.local_col, nnz, self.shard.rows, idx=slot)
            push = ("local", slot)
        else:
            rows_u, w_wide, push = self._pull(loc)
            X0 = E.expand(loc.local_col, nnz, rows_u)
        X0 = X0.view(B, S * D)
        # ---------------- MLP forward
        acts = [X0]
        for i in range(len(cfg.hidden)):
            acts.append(GM.linear_forward(acts[-1], self.W16[i], self.b[i], relu=True,
                                          backend=cfg.gemm, bias16=self.b16[i]))
        # ---------------- head (wide + deep), loss, metrics, head grads
        # (the flat gradient is zero here: allocated zeroed, and Adam zeroes it once read)
        H = acts[-1]
        dH = torch.empty_like(H)
        L = len(cfg.hidden)
        E.head(H, self.w_head, self.b_head, w_wide, loc.local_col, S, labels, self.coef, dH,
               self.dw_head, self.db_head, self.metrics, self.hist, AUC_BINS,
               db_h=self.db[L - 1])
        # ---------------- MLP backward: ReLU masks and the bias gradient of the
        # layer below fused into the dX GEMMs (grads zeroed at the step start, so the
        # weight-gradient GEMMs accumulate with beta 1: no zeroing pass of their own,
        # which on the side stream waited ~128 us for CUs behind the dX GEMM)
        # The weight gradient of layer i and the input gradient of layer i both read
        # dH only, so on the GPU the weight gradients run on a side stream next to the
        # input-gradient chain and the sparse push (GEMMs that each use part of the
        # chip overlap); the side stream joins before the dense all-reduce / Adam.
        side = self._side if self.gpu and cfg.overlap_wgrad else None
        main = torch.cuda.current_stream(dev) if side is not None else None
        # PSAMD_WD_DEFER_REDUCE=1: the split-K reduces of the weight gradients wait at the
        # end of the side stream, so layer 0's weight-gradient GEMM follows layer 1's at once
        # instead of queueing behind a memory-bound reduce that the input-gradient GEMM starves
        deferred = [] if side is not None and self._defer_reduce else None
        for i in reversed(range(L)):
            if side is not None:
                side.wait_stream(main)
                with torch.cuda.stream(side):
                    GM.linear_weight_grad(dH, acts[i], out=self.dW[i], beta=1.0,
                                          backend=cfg.gemm, deferred=deferred)
                dH.record_stream(side)
                acts[i].record_stream(side)
            else:
                GM.linear_weight_grad(dH, acts[i], out=self.dW[i], beta=1.0, backend=cfg.gemm)
            mask = acts[i] if i > 0 else None
            dH = GM.linear_input_grad(dH, self.W16[i], mask=mask, backend=cfg.gemm,
                                      colsum=self.db[i - 1] if i > 0 else None)
        dX0 = dH  # [B, S*D]
        # ---------------- sparse gradients
        u_cap = nnz
        if self.gpu and self._fuse and E.grad_wide_fused(D, True) and loc.grad is not None:
            # the wide gradient (same segments) in the same pass over the CSC entries
            dE = E.grad_reduce(loc, dX0, D, u_cap, out=self.dE, coef=self.coef[:B], width=S,
                               g_wide=loc.grad)
            g_wide = loc.grad
        else:
            if self.gpu:
                dE = E.grad_reduce(loc, dX0, D, u_cap, out=self.dE)
            else:
                dE = E.grad_reduce(loc, dX0, D, loc.num_unique())
            g_wide, _ = linear_backward(loc, self.coef[:B], B=B, width=S)
        self._push(loc, push, dE, g_wide)
        if deferred:
            with torch.cuda.stream(side):
                for fn in deferred:
                    fn()
        if side is not None:
            main.wait_stream(side)
        # ---------------- dense update: one all-reduce, fused Adam
        if self.G > 1:
            self.comm.all_reduce_(self.grad)
        self.step_count += 1
        # bias corrections from the device step clock (advanced by auc_from_hist below),
        # so the whole step can replay from a HIP graph
        E.adam(self.param, self.grad, self.m, self.v, lr=cfg.mlp_lr, step=self.step_count,
               gscale=1.0 / (B * self.G), p16=self.param16,
               step_dev=self.step_dev if self.gpu else None, zero_grad=True)
        auc_from_hist(self.hist, self.metrics, self.step_dev)
        self.examples += B

    # ------------------------------------------------------------ progress
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
