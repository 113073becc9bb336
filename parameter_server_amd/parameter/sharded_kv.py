"""GPU key-value push/pull API: ``KVWorker`` / ``KVServer`` over RCCL (ps.h parity).

Reference user API (src/ps.h, src/parameter/shared_parameter.h:17-40,
kv_vector.h:45-100): ``ts = pull(keys)`` / ``ts = push(keys, vals)`` return a
timestamp, ``wait(ts)`` blocks until the operation finished, values are merged
key-ordered, servers own contiguous key ranges.

MI355X design (one process per GPU, every rank = worker + server shard):
* keys are mixed by the bijective ``KeyMix`` and range-partitioned in the mixed
  space (balanced shards for any key distribution); a request is deduplicated,
  grouped by owner and moved with ONE ``all_to_all_v`` (RCCL over xGMI), the
  owner resolves / updates its HBM table, and a second ``all_to_all_v`` returns
  pulled values;
* operations are SPMD: every rank issues the same sequence of push/pull calls
  (possibly with empty key lists) — the RCCL analogue of the reference's
  "every worker talks to every server" message rounds;
* calls run on the worker's own HIP stream and return immediately; ``wait(ts)``
  makes the caller's stream wait on the op's event (no host sync) and returns
  the pulled values aligned with the request keys;
* server-side push semantics: ``"add"`` (KVVector PLUS, kv_vector.h:70-75),
  ``"assign"``, or an optimizer ``UpdateRule`` (SGD / AdaGrad / FTRL,
  kv_store.h:47-57 + async_sgd.h:71-124).
"""
from __future__ import annotations

import torch

from ..ops.keymix import mix, unmix
from ..ops.kv_table import InitRule, KVTable, UpdateRule
from ..parallel.comm import Comm, LocalComm
from ..parallel.partition import KeyPartition

ADD = UpdateRule("sgd", "constant", alpha=1.0)  # applied to -v: w -= 1 * (-v)  ==  w += v


class KVServer:
    """One rank's shard of a scalar-valued table in HBM."""

    def __init__(self, capacity: int, device, rule="add", init: InitRule | None = None):
        self.table = KVTable(capacity, device, init)
        self.rule = rule
        self.stats = torch.zeros(3, dtype=torch.float64, device=device)

    def get(self, mkeys: torch.Tensor) -> torch.Tensor:
        _, w = self.table.resolve(mkeys, insert=True)
        return w

    def put(self, mkeys: torch.Tensor, vals: torch.Tensor):
        slot, _ = self.table.resolve(mkeys, insert=True, with_w=False)
        if self.rule == "assign":
            self.table.set(slot, vals.float().contiguous())
            return
        if self.rule == "add":
            self.table.update(slot, (-vals.float()).contiguous(), ADD, self.stats)
            return
        self.table.update(slot, vals.float().contiguous(), self.rule, self.stats)

    def dump(self):
        """(raw uint64-as-int64 keys, values) of this shard."""
        k, w, _, _ = self.table.occupied()
        return k, w


class KVWorker:
    """``pull`` / ``push`` / ``wait`` against all shards (this rank's server included)."""

    def __init__(self, comm: Comm | None = None, device="cpu", *, capacity: int = 1 << 20,
                 rule="add", key_bits: int = 64, init: InitRule | None = None):
        self.device = torch.device(device)
        self.comm = comm or LocalComm(self.device)
        self.G, self.rank = self.comm.world, self.comm.rank
        self.bits = key_bits
        self.part = KeyPartition(key_bits, self.G)
        self.server = KVServer(capacity, self.device, rule, init)
        self.gpu = self.device.type == "cuda"
        self.stream = torch.cuda.Stream(self.device) if self.gpu else None
        self._ts = 0
        self._done: dict[int, tuple] = {}

    # ------------------------------------------------------------- helpers
    def _dedup(self, keys: torch.Tensor):
        mk = mix(keys.to(self.device, torch.int64).contiguous(), self.bits)
        # sorted unique in the signed order of the mixed keys (owner ranges are
        # contiguous in it: KeyPartition bounds are monotone in int64 order)
        uniq, inv = torch.unique(mk, sorted=True, return_inverse=True)
        return uniq, inv

    def _route(self, uniq: torch.Tensor):
        owner = self.part.owner_of(uniq)
        send = torch.bincount(owner, minlength=self.G).to(torch.int64)
        order = torch.argsort(owner, stable=True)
        return order, send

    def _exchange(self, x: torch.Tensor, send, recv):
        if self.G == 1:
            return x
        return self.comm.all_to_all_v(x.contiguous(), send.tolist(), recv.tolist())

    def _run(self, fn):
        self._ts += 1
        ts = self._ts
        if self.gpu:
            self.stream.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(self.stream):
                out = fn()
                ev = torch.cuda.Event()
                ev.record(self.stream)
            self._done[ts] = (out, ev)
        else:
            self._done[ts] = (fn(), None)
        return ts

    # ----------------------------------------------------------------- API
    def pull(self, keys: torch.Tensor) -> int:
        """Values of ``keys`` (any order, duplicates allowed) -> timestamp."""

        def op():
            uniq, inv = self._dedup(keys)
            order, send = self._route(uniq)
            req = uniq[order]
            recv = self.comm.exchange_counts(send).cpu() if self.G > 1 else send.cpu()
            rk = self._exchange(req, send.cpu(), recv)
            vals = self.server.get(rk)
            back = self._exchange(vals, recv, send.cpu())
            by_uniq = torch.empty_like(back)
            by_uniq[order] = back
            return by_uniq[inv]

        return self._run(op)

    def push(self, keys: torch.Tensor, vals: torch.Tensor) -> int:
        """Send ``vals`` for ``keys``; duplicates are summed before the server op."""

        def op():
            uniq, inv = self._dedup(keys)
            v = torch.zeros(uniq.numel(), dtype=torch.float32, device=self.device)
            v.index_add_(0, inv, vals.to(self.device, torch.float32).reshape(-1))
            order, send = self._route(uniq)
            recv = self.comm.exchange_counts(send).cpu() if self.G > 1 else send.cpu()
            rk = self._exchange(uniq[order], send.cpu(), recv)
            rv = self._exchange(v[order], send.cpu(), recv)
            self.server.put(rk, rv)
            return None

        return self._run(op)

    def wait(self, ts: int):
        """Block the caller's stream until op ``ts`` finished; pulled values or None."""
        out, ev = self._done.pop(ts)
        if ev is not None:
            torch.cuda.current_stream(self.device).wait_event(ev)
        return out

    def barrier(self):
        if self.gpu:
            torch.cuda.current_stream(self.device).wait_stream(self.stream)
        self.comm.barrier()

    # ---------------------------------------------------------- inspection
    def shard_items(self):
        """(raw keys, values) held by this rank's server shard."""
        mk, w = self.server.dump()
        return unmix(mk, self.bits), w
