"""GPU key-value push/pull API: ``KVWorker`` / ``KVServer`` over RCCL (ps.h parity).

Reference user API (src/ps.h:18-50, src/parameter/shared_parameter.h:17-40,
kv_vector.h:45-100): ``ts = pull(keys)`` / ``ts = push(keys, vals)`` return a
timestamp without blocking, ``wait(ts)`` completes the operation, a key carries
``k`` values (``KVVector<K, V>`` with ``k`` values per key), values are merged
key-ordered on the servers, servers own contiguous key ranges, and a pull may be
served before the pushes of the last ``tau`` steps are applied (bounded delay,
src/app/linear_method/darlin.h:81-91, src/system/executor.cc:170-177).

MI355X design (one process per GPU, every rank = worker + server shard):

* a call's keys are localised on the device by the same kernels as the trainers
  (``ops.localize``: mix -> radix sort -> run-length encode; sorted unique mixed
  keys, CSC order and the per-occurrence unique id), split by owner range on the
  device (``KeyPartition.split_sorted``) and packed into FIXED rows of C keys per
  peer with the live count in the row header (``exchange.hip``); a push row also
  carries the k values of every unique key, the duplicates of the call summed in
  CSC order (``kvv_pack_vals``);
* ONE equal-split all-to-all (RCCL over xGMI) moves the rows; the owner resolves all
  G source rows in one launch (``kv_resolve_rows``: lookup-or-insert, InitRule for
  new keys) and then serves (``kvv_serve``: gather the value rows) or merges
  (``kvv_apply``: PLUS with float atomics over all rows in one launch, ASSIGN in
  rank order; or one optimizer step per source row in rank order for an
  ``UpdateRule`` on scalar values, ``kv_update_rows``); a pull's records come back
  with a second all-to-all and ``kvv_unpack`` scatters them to request order;
* nothing of a call is read back on the host: a peer row holds C keys, sized to a
  peer's SHARE of the most keys one call may carry (``max_keys``): keys are mixed
  (KeyMix) before the range split, so a call's unique keys spread ~Binomial(U, 1/G)
  over the owners and C = ``peer_slack`` x max_keys / G + 6 standard deviations
  (the reference slices a message to each server's key range,
  src/system/message.h:120-159; a fixed row of max_keys per peer would move G x the
  live payload over xGMI). A row that would overflow keeps its first C keys and the
  excess is counted on the device; the count is published to pinned host memory
  (no stream sync) and the next call, ``wait`` or ``check`` of THAT rank raises on it
  (its peers then stop at their next collective, within the collective timeout
  PSAMD_COMM_TIMEOUT); ``flush`` checks collectively, so every rank raises together
  (``peer_capacity=max_keys`` makes overflow impossible). The whole op runs on the
  worker's own HIP stream and ``push`` / ``pull`` return at once; ``wait(ts)``
  orders the caller's stream after the op (no host sync);
* operations are SPMD: every rank issues the same sequence of push / pull calls
  (possibly with different or empty key lists) — the RCCL analogue of the
  reference's "every worker messages every server" rounds.

Consistency (``consistency=`` ``"bsp"`` | ``"ssp:tau"`` | ``"asp"``): the owner keeps
the received push rows of the last ``tau`` pushes pending and applies a push only
when ``tau`` newer pushes have arrived, so a pull issued after the P-th push sees
exactly the pushes 1 .. P - tau of every worker. What enforces this is the SPMD
order of the collectives: push P of every worker rides the same all-to-all, so when
the owner applies it, it holds every worker's push P. The ``VectorClock`` records
the applied pushes per worker for ``staleness()`` and asserts the bound; it is
bookkeeping that the collective order makes true, not a gate that could block.
``bsp`` is tau = 0. ``asp`` applies each push on a separate apply stream as soon as
it arrives and no pull waits for it (a pull sees whatever has landed).
``flush()`` applies everything pending.

Key caching (reference KeyCachingFilter, src/filter/key_caching.h:6-76: the sender
hashes a key list into a signature and, when the receiver already holds the list of
that signature, sends the values only): ``h = register_keys(keys)`` is a collective
call that localises the keys once, sends them to the owners once, and keeps the
localisation on the worker and the resolved slots of every source row on the owners.
``pull(h)`` then needs no request exchange at all (the owners serve their cached
slots straight into the one value all-to-all) and ``push(h, vals)`` sends key-less
rows ``[hdr | values]``. The device key signature (``ops.fixing_float.key_signature``)
deduplicates registrations: registering a key list whose signature every rank already
holds, under the SAME handle on every rank, returns the existing handle. Handle calls are SPMD like every other call (every
rank passes its handle of the same ``register_keys`` call).

Server-side push semantics: ``"add"`` (KVVector PLUS, kv_vector.h:70-75),
``"assign"``, or an optimizer ``UpdateRule`` (SGD / AdaGrad / FTRL, scalar values,
kv_store.h:47-57 + async_sgd.h:71-124).
"""
from __future__ import annotations

import math
from collections import deque

import torch

from ..ops.keymix import unmix
from ..ops.kv_table import EMPTY_KEY, InitRule, KVTable, UpdateRule
from ..ops.localize import Localizer, localize_torch
from ..ops.native import hipops
from ..parallel.comm import Comm, LocalComm
from ..parallel.consistency import INF, VectorClock, parse_consistency
from ..parallel.partition import KeyPartition

ADD, ASSIGN = 0, 1


class KeyHandle:
    """A registered key list (``KVWorker.register_keys``): the worker's localisation
    (unique-id per request position, duplicates' CSC order, per-owner offsets) and the
    owner's resolved slots of every source row, cached for key-less push / pull."""

    def __init__(self, hid: int, n: int, signature: int):
        self.id, self.n, self.signature = hid, n, signature
        self.loc = None    # worker: localisation of the key list
        self.off = None    # worker: per-owner offsets of its unique keys [G + 1]
        self.slot = None   # owner: resolved slots of every source row [G * C] (GPU)
        self.hdr = None    # owner: received row headers [G * 4] (live counts, GPU)
        self.rows = None   # owner (CPU path): [(slots, count)] per source row
        self.live = True

    def __repr__(self):
        return f"KeyHandle(id={self.id}, n={self.n}, signature={self.signature:#018x})"


class KVServer:
    """One rank's shard: the KV table (key index; scalar value + optimizer state in
    its slots) and, for ``add`` / ``assign``, a ``[capacity, k]`` fp32 value block at
    the slot index (the layout of the embedding shards)."""

    def __init__(self, capacity: int, device, rule="add", init: InitRule | None = None,
                 dim: int = 1, key_range=None):
        self.table = KVTable(capacity, device, init, key_range=key_range)
        self.rule = rule
        self.dim = int(dim)
        self.device = torch.device(device)
        self.stats = torch.zeros(3, dtype=torch.float64, device=self.device)
        self.vals = None
        if not isinstance(rule, UpdateRule):
            if rule not in ("add", "assign"):
                raise ValueError(f"rule must be 'add', 'assign' or an UpdateRule, not {rule!r}")
            if init is not None and init.type.lower() != "zero":
                raise ValueError("add / assign values start at zero (KVVector semantics); "
                                 "InitRule needs an UpdateRule")
            self.vals = torch.zeros(self.table.capacity, self.dim, dtype=torch.float32,
                                    device=self.device)
        elif self.dim != 1:
            raise ValueError("an optimizer UpdateRule updates scalar values (dim = 1)")

    @property
    def op(self) -> int | None:
        return None if isinstance(self.rule, UpdateRule) else (ADD if self.rule == "add" else ASSIGN)

    def dump(self):
        """(mixed keys, values [n, dim]) of this shard."""
        keys = self.table.slots[:, 0]
        mask = keys != EMPTY_KEY
        if self.vals is None:
            k, w, _, _ = self.table.occupied()
            return k, w.reshape(-1, 1)
        return keys[mask], self.vals[mask]


class KVWorker:
    """``pull`` / ``push`` / ``wait`` against all shards (this rank's server included)."""

    def __init__(self, comm: Comm | None = None, device="cpu", *, capacity: int = 1 << 20,
                 rule="add", key_bits: int = 64, init: InitRule | None = None, dim: int = 1,
                 max_keys: int = 1 << 20, consistency="bsp", peer_capacity: int = 0,
                 peer_slack: float = 1.2):
        self.device = torch.device(device)
        self.comm = comm or LocalComm(self.device)
        self.G, self.rank = self.comm.world, self.comm.rank
        self.bits = int(key_bits)
        self.dim = k = int(dim)
        self.part = KeyPartition(self.bits, self.G)
        self.server = KVServer(capacity, self.device, rule, init, k)
        self.gpu = self.device.type == "cuda"
        self.tau = parse_consistency(consistency)
        self.asp = math.isinf(self.tau)
        self.consistency = "asp" if self.asp else ("bsp" if self.tau == 0 else f"ssp:{int(self.tau)}")
        self.clock = VectorClock(self.G, self.tau)
        # fixed exchange geometry: C keys per peer row, a peer's share of the most keys
        # one call carries (slack x mean + 6 sigma of the binomial split), <= max_keys
        self.max_keys = int(max_keys)
        C = int(peer_capacity)
        if C <= 0:
            mean = self.max_keys / self.G
            C = int(math.ceil(peer_slack * mean + 6 * math.sqrt(mean) + 64))
        C = max(8, min(C, self.max_keys))
        C = (C + 7) // 8 * 8
        kw = 1 if self.bits <= 32 else 2
        self.C, self.kw = C, kw
        self.Hk = (4 + C * kw + 1 + 3) // 4 * 4          # pull rows: header + keys
        self.Hp = (4 + C * kw + C * k + 3) // 4 * 4       # push rows: + k values per key
        self.Hv = (4 + C * k + 3) // 4 * 4                # key-less push rows (registered keys)
        self._ts = 0
        self._pushes = 0          # pushes issued (the worker's step clock)
        self._done: dict[int, tuple] = {}
        self._pending: deque = deque()  # (push index, received rows, handle) not yet applied
        self._handles: list[KeyHandle] = []  # registered key lists, in registration order
        G, dev = self.G, self.device
        if self.gpu:
            self.stream = torch.cuda.Stream(self.device)
            self.apply_stream = torch.cuda.Stream(self.device) if self.asp else None
            self.loc = Localizer(self.max_keys, self.bits, dev)
            i32 = dict(dtype=torch.int32, device=dev)
            self.send_k, self.recv_k = torch.zeros(G * self.Hk, **i32), torch.zeros(G * self.Hk, **i32)
            self.send_p = torch.zeros(G * self.Hp, **i32)
            self.slot = torch.empty(G * C, dtype=torch.int64, device=dev)
            self.w = torch.empty(G * C, dtype=torch.float32, device=dev)
            self.rec_s = torch.empty(G * C * k, dtype=torch.float32, device=dev)
            self.rec_r = torch.empty(G * C * k, dtype=torch.float32, device=dev)
            self.off1 = torch.zeros(2, dtype=torch.int64, device=dev)
            # keys dropped by a full peer row (device counter + pinned host mirror)
            self.ovf = torch.zeros(1, dtype=torch.int32, device=dev)
            self.ovf_host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
            # apply-side scratch (the apply stream's own under asp)
            self.a_slot = torch.empty(G * C, dtype=torch.int64, device=dev)
            self.a_w = torch.empty(G * C, dtype=torch.float32, device=dev)
            if self.server.op is None:
                from ..ops.kv_table import next_pow2

                self.link = torch.empty(next_pow2(2 * G * C), dtype=torch.int64, device=dev)
                self.nxt = torch.empty(G * C, dtype=torch.int32, device=dev)
        else:
            self.stream = self.apply_stream = None
            self.ovf = torch.zeros(1, dtype=torch.int32)
            self.ovf_host = self.ovf

    # ------------------------------------------------------------- helpers
    def check(self, sync: bool = False, collective: bool = False) -> None:
        """Raise if a call dropped keys because a peer row was full. The pack kernels
        publish the device count to pinned host memory (seen once they completed);
        ``sync=True`` waits for the worker's stream first; ``collective=True`` (every
        rank calls it) takes the largest count of all ranks over the host channel, so
        all ranks raise together instead of the others waiting in their next collective."""
        if sync and self.gpu:
            self.stream.synchronize()
        n = int(self.ovf_host[0])
        if collective and self.G > 1:
            n = max(self.comm.host_gather_obj(n))
        if n:
            raise RuntimeError(
                f"KVWorker exchange overflow: {n} keys exceeded the per-peer row capacity "
                f"{self.C} (max_keys {self.max_keys}, {self.G} shards); those keys were not "
                f"pulled / pushed. Pass a larger peer_capacity (max_keys makes overflow "
                f"impossible) or peer_slack")

    def _pack_keys(self, loc, off, H, send):
        hh = hipops()
        hh.xchg_pack_keys(loc.uniq, loc.n_uniq, off, self.C, self.kw, H, send, self.ovf)
        hh.xchg_publish(self.ovf, self.ovf_host)

    def _keys(self, keys: torch.Tensor) -> torch.Tensor:
        keys = keys.to(self.device, torch.int64).reshape(-1).contiguous()
        if keys.numel() > self.max_keys:
            raise ValueError(f"{keys.numel()} keys in one call > max_keys {self.max_keys}")
        return keys

    def _localize(self, keys):
        if keys.numel() == 0:
            return None
        return self.loc(keys) if self.gpu else localize_torch(keys, self.bits)

    def _offsets(self, loc):
        if self.G == 1:
            if self.gpu:
                hipops().kvv_single_off(loc.n_uniq, self.off1)
                return self.off1
            return torch.tensor([0, loc.uniq.numel()], dtype=torch.int64)
        return self.part.split_sorted(loc.uniq, loc.n_uniq)

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

    # ------------------------------------------------- row packing (CPU path)
    def _cpu_pack_keys(self, loc, off, H, send):
        send.zero_()
        if loc is None:
            return
        for p in range(self.G):
            a, b = int(off[p]), int(off[p + 1])
            if b - a > self.C:  # full row: keep the first C keys, count the rest
                self.ovf += b - a - self.C
                b = a + self.C
            base = p * H
            send[base] = b - a
            ks = loc.uniq[a:b]
            if self.kw == 2:
                send[base + 4:base + 4 + 2 * (b - a)] = ks.contiguous().view(torch.int32)
            else:
                send[base + 4:base + 4 + (b - a)] = (ks & 0xFFFFFFFF).to(torch.int32)

    def _cpu_row_keys(self, recv, s, H):
        base = s * H
        n = int(recv[base])
        if self.kw == 2:
            return recv[base + 4:base + 4 + 2 * n].contiguous().view(torch.int64)
        return recv[base + 4:base + 4 + n].to(torch.int64) & 0xFFFFFFFF

    def _row_vals(self, buf, s, H, n=None):
        """Float view of source row s's value region ([C, k])."""
        C, k = self.C, self.dim
        v = buf.view(torch.float32)[s * H + 4 + C * self.kw:s * H + 4 + C * self.kw + C * k]
        v = v.view(C, k)
        return v if n is None else v[:n]

    # ----------------------------------------------------------------- API
    def register_keys(self, keys: torch.Tensor) -> KeyHandle:
        """Collective: register a key list for key-less push / pull (key caching).
        Localises the keys once and resolves them at their owners (inserting new keys
        with the InitRule), keeping both sides' results. A list whose device signature
        and length every rank has registered before returns that handle (one host read
        of the signature: a setup call, not a per-step one)."""
        from ..ops.fixing_float import key_signature

        self._local_check()
        keys = self._keys(keys)
        sig = key_signature(keys) if keys.numel() else 0
        old = next((h for h in self._handles
                    if h.live and h.signature == sig and h.n == keys.numel()), None)
        hit = old is not None
        if self.G > 1:
            # reuse only when every rank holds the list under the SAME handle: owners
            # apply key-less rows against the cached slots of their own handle, so a
            # crossed match (rank A's list X is handle 0, rank B's is handle 1) would
            # land values on the wrong keys. min(id) == max(id) >= 0 over all ranks.
            hid = float(old.id) if hit else -1.0
            t = torch.tensor([hid, -hid], dtype=torch.float64,
                             device=self.device if getattr(self.comm, "backend", "") == "nccl"
                             else "cpu")
            t = self.comm.all_reduce_(t, op="max").cpu()
            hit = float(t[0]) == -float(t[1]) and float(t[0]) >= 0
        if hit:
            return old
        h = KeyHandle(len(self._handles), keys.numel(), sig)
        self._handles.append(h)

        def op():
            self._register(keys, h)

        self.wait(self._run(op))
        # (a setup call: a full row would break the handle for good; collective like the
        # registration itself, so every rank raises together)
        self.check(sync=True, collective=True)
        return h

    def release(self, h: KeyHandle) -> None:
        """Drop a registered key list's cached state (collective in effect: call it on
        every rank with the same handle). Pushes of ``h`` still pending under SSP keep
        the owner-side slots until they are applied (``_drain`` frees them then)."""
        h.live = False
        h.loc = h.off = None
        if not any(e[2] is h for e in self._pending):
            h.slot = h.hdr = h.rows = None

    def _register(self, keys, h: KeyHandle):
        C, H, G = self.C, self.Hk, self.G
        loc = self._localize(keys)
        tb = self.server.table
        n = keys.numel()
        if self.gpu:
            hh = hipops()
            if loc is None:
                hh.xchg_clear_counts(self.send_k, G, H, True, True)
            else:
                off = self._offsets(loc)
                self._pack_keys(loc, off, H, self.send_k)
                h.off = off.clone()
                h.loc = (loc.local_col[:n].clone(), loc.pos_s[:n].clone(),
                         loc.seg_start[:n + 1].clone(), loc.n_uniq.clone())
            self.comm.all_to_all_fixed(self.send_k, self.recv_k)
            it, iv, isd, seed = tb.init.args()
            slot = torch.empty(G * C, dtype=torch.int64, device=self.device)
            hh.kv_resolve_rows(tb.slots, self.recv_k, H, C, self.kw, slot, self.w, True, it, iv,
                               isd, seed, tb._err, tb._inserted, tb.home_base, tb.home_m)
            h.slot = slot
            h.hdr = self.recv_k.view(G, H)[:, :4].contiguous().reshape(-1)
            return
        off = self._offsets(loc) if loc is not None else None
        send, recv = torch.zeros(G * H, dtype=torch.int32), torch.empty(G * H, dtype=torch.int32)
        self._cpu_pack_keys(loc, off, H, send)
        self.comm.all_to_all_fixed(send, recv)
        h.loc, h.off = loc, off
        h.rows = []
        for s in range(G):
            rk = self._cpu_row_keys(recv, s, H)
            slot = tb.resolve(rk, insert=True, with_w=False)[0] if rk.numel() else None
            h.rows.append((slot, rk.numel()))

    def _check_handle(self, h: KeyHandle):
        if not h.live or h.id >= len(self._handles) or self._handles[h.id] is not h:
            raise ValueError(f"{h!r} is not a live handle of this worker")

    def pull(self, keys) -> int:
        """Values of ``keys`` (any order, duplicates allowed; or a ``KeyHandle`` from
        ``register_keys``) -> timestamp; ``wait`` returns ``[n]`` (dim 1) or ``[n, dim]``
        float32 values in request order."""
        self._local_check()
        if isinstance(keys, KeyHandle):
            self._check_handle(keys)
            if not self.clock.admissible(self._pushes):
                raise AssertionError("pull admitted before the pushes it must see were applied")
            h = keys
            return self._run(lambda: self._pull_cached(h))
        keys = self._keys(keys)
        # after P pushes (indices 0 .. P-1) the pull is step P: it must see pushes
        # 0 .. P-1-tau of every worker
        if not self.clock.admissible(self._pushes):
            raise AssertionError("pull admitted before the pushes it must see were applied")

        def op():
            return self._pull(keys)

        return self._run(op)

    def _pull(self, keys):
        k, C, H, G = self.dim, self.C, self.Hk, self.G
        n = keys.numel()
        loc = self._localize(keys)
        out = torch.zeros(n, k, dtype=torch.float32, device=self.device)
        srv, tb = self.server, self.server.table
        if self.gpu:
            hh = hipops()
            if loc is None:
                hh.xchg_clear_counts(self.send_k, G, H, True, True)
            else:
                off = self._offsets(loc)
                self._pack_keys(loc, off, H, self.send_k)
            self.comm.all_to_all_fixed(self.send_k, self.recv_k)
            it, iv, isd, seed = tb.init.args()
            hh.kv_resolve_rows(tb.slots, self.recv_k, H, C, self.kw, self.slot, self.w, True, it,
                               iv, isd, seed, tb._err, tb._inserted, tb.home_base, tb.home_m)
            if srv.vals is None:
                rec = self.w
            else:
                hh.kvv_serve(self.recv_k, H, C, self.slot, srv.vals, self.rec_s)
                rec = self.rec_s
            self.comm.all_to_all_fixed(rec, self.rec_r)
            if loc is not None:
                hh.kvv_unpack(self.rec_r, C, k, off, loc.local_col, out)
        else:
            off = self._offsets(loc) if loc is not None else None
            send, recv = torch.zeros(G * H, dtype=torch.int32), torch.empty(G * H, dtype=torch.int32)
            self._cpu_pack_keys(loc, off, H, send)
            self.comm.all_to_all_fixed(send, recv)
            rec_s = torch.zeros(G * C * k, dtype=torch.float32)
            for s in range(G):
                rk = self._cpu_row_keys(recv, s, H)
                if rk.numel() == 0:
                    continue
                slot, w = tb.resolve(rk, insert=True)
                vals = w.reshape(-1, 1) if srv.vals is None else srv.vals[slot]
                rec_s[s * C * k:(s * C + rk.numel()) * k] = vals.reshape(-1)
            rec_r = torch.empty_like(rec_s)
            self.comm.all_to_all_fixed(rec_s, rec_r)
            if loc is not None:
                u = loc.local_col.to(torch.int64)
                p = torch.searchsorted(off[1:], u, right=True)
                i = u - off[p]
                out = rec_r.view(G * C, k)[p * C + i.clamp(max=C - 1)]
                out[i >= C] = 0.0  # dropped by a full row (counted in ovf)
        return out.reshape(-1) if k == 1 else out

    def _pull_cached(self, h: KeyHandle):
        """Pull of a registered key list: no request rows; every owner serves the
        cached slots of every source row into the value all-to-all."""
        k, C, G = self.dim, self.C, self.G
        srv, tb = self.server, self.server.table
        out = torch.zeros(h.n, k, dtype=torch.float32, device=self.device)
        if self.gpu:
            hh = hipops()
            if srv.vals is None:
                hh.kv_serve_w(h.hdr, 4, C, h.slot, tb.slots, self.rec_s)
            else:
                hh.kvv_serve(h.hdr, 4, C, h.slot, srv.vals, self.rec_s)
            self.comm.all_to_all_fixed(self.rec_s, self.rec_r)
            if h.loc is not None:
                hh.kvv_unpack(self.rec_r, C, k, h.off, h.loc[0], out)
        else:
            rec_s = torch.zeros(G * C * k, dtype=torch.float32)
            for s, (slot, cnt) in enumerate(h.rows):
                if not cnt:
                    continue
                vals = (tb.gather(slot, 0).reshape(-1, 1) if srv.vals is None else srv.vals[slot])
                rec_s[s * C * k:(s * C + cnt) * k] = vals.reshape(-1)
            rec_r = torch.empty_like(rec_s)
            self.comm.all_to_all_fixed(rec_s, rec_r)
            if h.loc is not None:
                u = h.loc.local_col.to(torch.int64)
                p = torch.searchsorted(h.off[1:], u, right=True)
                i = u - h.off[p]
                out = rec_r.view(G * C, k)[p * C + i.clamp(max=C - 1)]
                out[i >= C] = 0.0
        return out.reshape(-1) if k == 1 else out

    def push(self, keys, vals: torch.Tensor) -> int:
        """Send ``vals`` (``[n]`` or ``[n, dim]``) for ``keys`` (or a ``KeyHandle``:
        key-less rows against the owners' cached slots); duplicates are summed before
        the server op. Returns the timestamp."""
        self._local_check()
        if isinstance(keys, KeyHandle):
            self._check_handle(keys)
            h = keys
            vals = vals.to(self.device, torch.float32).reshape(h.n, self.dim).contiguous()
            p = self._pushes
            self._pushes += 1
            return self._run(lambda: self._push_cached(h, vals, p))
        keys = self._keys(keys)
        vals = vals.to(self.device, torch.float32).reshape(keys.numel(), self.dim).contiguous()
        p = self._pushes  # 0-based push index (the worker's step clock)
        self._pushes += 1

        def op():
            return self._push(keys, vals, p)

        return self._run(op)

    def _push(self, keys, vals, p):
        k, C, H, G = self.dim, self.C, self.Hp, self.G
        loc = self._localize(keys)
        if self.gpu:
            hh = hipops()
            if loc is None:
                hh.xchg_clear_counts(self.send_p, G, H, True, True)
            else:
                off = self._offsets(loc)
                self._pack_keys(loc, off, H, self.send_p)
                hh.kvv_pack_vals(vals, k, loc.pos_s, loc.seg_start, loc.n_uniq, off, C, self.kw, H,
                                 self.send_p)
            recv = torch.empty(G * H, dtype=torch.int32, device=self.device)
            self.comm.all_to_all_fixed(self.send_p, recv)
        else:
            off = self._offsets(loc) if loc is not None else None
            send, recv = torch.zeros(G * H, dtype=torch.int32), torch.empty(G * H, dtype=torch.int32)
            self._cpu_pack_keys(loc, off, H, send)
            if loc is not None:
                # duplicates summed in CSC order (the kernel's order)
                u = torch.zeros(loc.uniq.numel(), k, dtype=torch.float32)
                u.index_add_(0, loc.local_col.to(torch.int64), vals)
                for q in range(G):
                    a, b = int(off[q]), int(off[q + 1])
                    b = min(b, a + C)
                    self._row_vals(send, q, H)[:b - a] = u[a:b]
            self.comm.all_to_all_fixed(send, recv)
        self._pending.append((p, recv, None))
        self._drain(keep=0 if self.asp else int(self.tau))
        # the vector clock is the gate: every worker's pushes through P - tau applied
        assert self.asp or self.clock.min_clock() >= p - int(self.tau)
        return None

    def _push_cached(self, h: KeyHandle, vals, p):
        k, C, H, G = self.dim, self.C, self.Hv, self.G
        if self.gpu:
            hh = hipops()
            send = torch.zeros(G * H, dtype=torch.int32, device=self.device)
            if h.loc is not None:
                _, pos_s, seg_start, n_uniq = h.loc
                hh.kvv_pack_vals(vals, k, pos_s, seg_start, n_uniq, h.off, C, 0, H, send)
            recv = torch.empty(G * H, dtype=torch.int32, device=self.device)
            self.comm.all_to_all_fixed(send, recv)
        else:
            send, recv = torch.zeros(G * H, dtype=torch.int32), torch.empty(G * H, dtype=torch.int32)
            if h.loc is not None:
                u = torch.zeros(h.loc.uniq.numel(), k, dtype=torch.float32)
                u.index_add_(0, h.loc.local_col.to(torch.int64), vals)
                for q in range(G):
                    a, b = int(h.off[q]), int(h.off[q + 1])
                    b = min(b, a + C)
                    send[q * H] = b - a
                    send.view(torch.float32)[q * H + 4:q * H + 4 + (b - a) * k] = u[a:b].reshape(-1)
            self.comm.all_to_all_fixed(send, recv)
        self._pending.append((p, recv, h))
        self._drain(keep=0 if self.asp else int(self.tau))
        assert self.asp or self.clock.min_clock() >= p - int(self.tau)
        return None

    def _drain(self, keep: int):
        """Apply pending pushes until at most ``keep`` remain (oldest first); every
        applied push advances every worker's vector clock (SPMD: push p of all workers
        rides the same exchange)."""
        while len(self._pending) > keep:
            p, recv, h = self._pending.popleft()
            apply = self._apply if h is None else (lambda r, h=h: self._apply_cached(r, h))
            if self.apply_stream is not None:
                cur = torch.cuda.current_stream(self.device)
                self.apply_stream.wait_stream(cur)
                recv.record_stream(self.apply_stream)
                with torch.cuda.stream(self.apply_stream):
                    apply(recv)
            else:
                apply(recv)
            for w in range(self.G):
                self.clock.tick(w, p)
            if h is not None and not h.live and not any(e[2] is h for e in self._pending):
                h.slot = h.hdr = h.rows = None  # released with pushes still pending

    def _apply(self, recv):
        srv, tb = self.server, self.server.table
        C, H, G = self.C, self.Hp, self.G
        if self.gpu:
            hh = hipops()
            it, iv, isd, seed = tb.init.args()
            hh.kv_resolve_rows(tb.slots, recv, H, C, self.kw, self.a_slot, self.a_w, True, it, iv,
                               isd, seed, tb._err, tb._inserted, tb.home_base, tb.home_m)
            if srv.op is None:
                grad = recv.view(torch.float32)[4 + C * self.kw:]
                hh.kv_update_rows(tb.slots, self.a_slot, grad, H, recv, H, C, self.link, self.nxt,
                                  *srv.rule.args(), srv.stats)
            else:
                hh.kvv_apply(recv, H, C, self.kw, self.a_slot, srv.vals, srv.op)
            return
        for s in range(G):  # source rows in rank order
            rk = self._cpu_row_keys(recv, s, H)
            if rk.numel() == 0:
                continue
            v = self._row_vals(recv, s, H, rk.numel())
            slot, _ = tb.resolve(rk, insert=True, with_w=False)
            if srv.op is None:
                tb.update(slot, v[:, 0].contiguous(), srv.rule, srv.stats)
                continue
            ok = ~torch.isnan(v)
            if srv.op == ADD:
                srv.vals[slot] += torch.where(ok, v, torch.zeros_like(v))
            else:
                srv.vals[slot] = torch.where(ok, v, srv.vals[slot])

    def _apply_cached(self, recv, h: KeyHandle):
        """Owner merge of key-less rows against the cached slots of their source rows."""
        srv, tb = self.server, self.server.table
        C, H, G, k = self.C, self.Hv, self.G, self.dim
        if self.gpu:
            hh = hipops()
            if srv.op is None:
                hh.kv_update_rows(tb.slots, h.slot, recv.view(torch.float32)[4:], H, recv, H, C,
                                  self.link, self.nxt, *srv.rule.args(), srv.stats)
            else:
                hh.kvv_apply(recv, H, C, 0, h.slot, srv.vals, srv.op)
            return
        for s, (slot, cnt) in enumerate(h.rows):  # source rows in rank order
            n = int(recv[s * H])
            if not cnt or not n:
                continue
            v = recv.view(torch.float32)[s * H + 4:s * H + 4 + n * k].view(n, k)
            if srv.op is None:
                tb.update(slot[:n], v[:, 0].contiguous(), srv.rule, srv.stats)
                continue
            ok = ~torch.isnan(v)
            if srv.op == ADD:
                srv.vals[slot[:n]] += torch.where(ok, v, torch.zeros_like(v))
            else:
                srv.vals[slot[:n]] = torch.where(ok, v, srv.vals[slot[:n]])

    def wait(self, ts: int):
        """Order the caller's stream after op ``ts``; pulled values (or None).

        One process (G == 1 or the loopback emulation): an overflow published by a
        completed pack raises here. With peer processes the check is deferred to the
        next collective check (``flush()`` / ``barrier()``), where every rank raises
        together: a rank-local raise here would leave the peers blocked in their next
        all-to-all until the communicator timeout."""
        out = self._wait_nocheck(ts)
        self._local_check()
        return out

    def _local_check(self):
        """The non-collective overflow check of push / pull / wait: only where no peer
        process waits in a collective (one rank, or the loopback emulation)."""
        if self.G == 1 or getattr(self.comm, "backend", "") == "loopback":
            self.check()

    def _wait_nocheck(self, ts: int):
        out, ev = self._done.pop(ts)
        if ev is not None:
            torch.cuda.current_stream(self.device).wait_event(ev)
        return out

    def flush(self):
        """Apply every pending push (end of a training phase). Collective: the overflow
        check after the drain takes the largest count of all ranks, so every rank raises
        together (a rank-local check first would let one rank raise while its peers wait
        for it in the host gather)."""
        def op():
            self._drain(keep=0)

        out = self._wait_nocheck(self._run(op))
        self.check(sync=True, collective=True)
        return out

    def barrier(self):
        """Collective: the caller's stream after every issued op, then the overflow
        check of all ranks (every rank raises together)."""
        if self.gpu:
            cur = torch.cuda.current_stream(self.device)
            cur.wait_stream(self.stream)
            if self.apply_stream is not None:
                cur.wait_stream(self.apply_stream)
        self.comm.barrier()
        self.check(sync=True, collective=True)

    def staleness(self) -> int:
        """Pushes a pull issued now would miss (0 for bsp, <= tau for ssp)."""
        return self.clock.staleness(self._pushes)

    # ---------------------------------------------------------- inspection
    def shard_items(self):
        """(raw keys, values) held by this rank's server shard (values ``[n]`` for dim 1)."""
        if self.gpu:
            torch.cuda.current_stream(self.device).wait_stream(self.stream)
            if self.apply_stream is not None:
                torch.cuda.current_stream(self.device).wait_stream(self.apply_stream)
        mk, v = self.server.dump()
        return unmix(mk, self.bits), (v.reshape(-1) if self.dim == 1 else v)


__all__ = ["KVWorker", "KVServer", "KeyHandle", "INF"]
