"""One-sided peer-HBM exchange: asynchronous SGD without per-step collectives.

The reference's async-SGD worker pulls and pushes without ever waiting for another
worker (src/app/linear_method/async_sgd.h:219-238) and a server applies each push as
it arrives (src/parameter/kv_store.h:47-57). The default multi-GPU data plane here is
SPMD: every push / pull rides an RCCL all-to-all, so one slow rank stalls all of
them. ``PeerExchange`` is the straggler-tolerant alternative (SURVEY §7.4 option b):
at setup every rank exports its KV shard, its push inbox and its applied counters
as IPC handles (``hipIpcGetMemHandle``; one host all-gather), and maps its peers'.
Then, per step and without any collective (kernels in csrc/hip/p2p.hip):

* pull: the keys owned by peer p are probed straight in p's table over xGMI
  (read only; a key not inserted yet reads as its init value);
* push: the rows of this step (keys + gradients per owner) are written into each
  owner's inbox ring, entry ``[self][seq % Q]``, and published by a sequence word;
* apply: each owner, at its own pace, applies the ready inbox entries of every
  source (one entry per source per round, per-push semantics in rank order) with
  the table kernels of the padded exchange, and publishes its applied counters.

A pusher waits (bounded device spin) only when it is ``Q`` steps ahead of what an
owner has applied from it: the staleness bound of this mode. Between ranks there is
no lock step, so a slow rank delays only the application of its own pushes.

A second, documented source of staleness: a peer's one-sided lookup reads the owner's
table (ordinary coarse-grained HBM, mapped over xGMI) while the owner's apply kernels
write it. A remote read returns the slot's weight as of some point during the owner's
update stream -- before or after any given in-flight apply, and never torn (the
weight is one aligned 32-bit word; a key being inserted reads as its init value until
its weight is published, ``kv_slot.cuh publish_init`` / ``published_w``). So a pull
sees every push the owner had finished applying when the lookup kernel ran, plus
possibly some it was applying: asynchronous SGD semantics (the reference's servers
answer pulls between pushes the same way, kv_store.h:37-57), not a bounded-delay
guarantee -- use the padded exchange with ``ssp:tau`` for that.

Rows use the padded exchange's layout, so FixingFloat pushes (nb-byte codes with the
row's min / max in the header; reference fixing_float.h:44-95) travel as they do there
and the owner decodes them before the update. The inbox (entries + a separate area of
sequence words) and the applied counters are FINE-GRAINED device memory: another GPU
writes / reads them while kernels run (``PSAMD_P2P_FINE=0``: ordinary coarse-grained
allocations, for A/B). A push that gives up waiting for ring space is fatal at once:
the post publishes the error word into pinned host memory and ``check_fatal`` raises
(its sequence number is consumed, so that owner would otherwise wait for it forever).
Host-side bookkeeping (handle exchange, drain counts) goes over a gloo group, never
through a device-synchronising RCCL object collective. The owner side (the own row's
update and the inbox applies) runs on a stream of its own, so a rank whose post waits
for a peer's ring space still applies that peer's posts: two ranks with full rings
toward each other cannot block each other. Every update of this rank's table must
therefore go through ``own_update`` (serialised with the applies on that stream; a
``kv_update`` on another stream would race them on the same slots), and the next
step's writes of the buffers it reads wait for ``wait_own``.

Validated on one MI355X with several processes sharing the GPU (real IPC mappings,
the same kernels); the xGMI path itself needs a multi-GPU node.
"""
from __future__ import annotations

import time

import torch

from ..ops.native import hipops


def _u64_to_i64(x: int) -> int:
    x &= (1 << 64) - 1
    return x - (1 << 64) if x >= (1 << 63) else x


def _fine_i32(n: int, dev, fine: bool):
    """n zeroed int32 words: fine-grained device memory, or (fine=False) torch's."""
    if fine:
        return hipops().fine_empty(4 * n).view(torch.int32)
    return torch.zeros(n, dtype=torch.int32, device=dev)


class PeerExchange:
    def __init__(self, comm, table, C: int, kw: int, H: int, device, Q: int = 16,
                 spin_us: int = 5_000_000, nb: int = 0):
        import os

        self.comm, self.table = comm, table
        self.G, self.rank = comm.world, comm.rank
        self.C, self.kw, self.H, self.Q = int(C), int(kw), int(H), int(Q)
        self.nb = int(nb)  # FixingFloat bytes per pushed gradient (0: f32)
        self.spin = int(spin_us)  # give-up time of a push waiting for inbox space
        self.device = dev = torch.device(device)
        G, H, Q = self.G, self.H, self.Q
        i32 = dict(dtype=torch.int32, device=dev)
        self.fine = os.environ.get("PSAMD_P2P_FINE", "1") != "0"
        # [source][Q][H] entries, then [source][Q] sequence words (0 = empty)
        self.inbox = _fine_i32(G * Q * H + G * Q, dev, self.fine)
        self.applied = _fine_i32(G, dev, self.fine)   # last sequence applied per source
        self.stage = torch.zeros(G * H, **i32)
        self.gdec = torch.zeros(G * C, dtype=torch.float32, device=dev) if self.nb else None
        self.ready = torch.zeros(G, **i32)
        self.ok = torch.zeros(G, **i32)
        self.err = torch.zeros(1, **i32)
        self.err_host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        self.total = torch.zeros(1, dtype=torch.int64, device=dev)  # entries applied
        self.seq = 0                                  # pushes posted by this rank
        # the owner side runs on its own stream: a post spinning for ring space on a peer
        # never blocks this rank's applies (which free the peer's posts to it), so two
        # ranks waiting on each other's rings always make progress
        self.astream = torch.cuda.Stream(dev) if dev.type == "cuda" else None
        self.ev_own = torch.cuda.Event() if dev.type == "cuda" else None
        hh = hipops()
        cap = table.capacity
        lg = (cap - 1).bit_length()
        geom = [int(cap - 1), int(table.home_base), int(table.home_m), 64 - lg]
        mine = {"slots": hh.ipc_export(table.slots), "inbox": hh.ipc_export(self.inbox),
                "applied": hh.ipc_export(self.applied), "geom": geom}
        allh = comm.host_gather_obj(mine)
        self._opened = []
        tabs, rings, applieds = [], [], []
        for p, h in enumerate(allh):
            if p == self.rank:
                sp, ip, ap = table.slots.data_ptr(), self.inbox.data_ptr(), self.applied.data_ptr()
            else:
                sp, ip, ap = (self._open(h["slots"]), self._open(h["inbox"]),
                              self._open(h["applied"]))
            tabs += [sp] + [_u64_to_i64(v) for v in h["geom"]]
            rings.append(ip)
            applieds.append(ap)
        self.tabs = torch.tensor(tabs, dtype=torch.int64).to(dev)
        self.rings = torch.tensor(rings, dtype=torch.int64).to(dev)
        self.applieds = torch.tensor(applieds, dtype=torch.int64).to(dev)

    def _open(self, handle: bytes) -> int:
        ptr = hipops().ipc_import(handle)
        off = int.from_bytes(handle[64:72], "little", signed=True)
        self._opened.append((ptr, off))
        return ptr

    # ------------------------------------------------------------------ step
    def lookup(self, send, wout, slot_out):
        """Weights of every row's keys: own row resolved with insert (slots ->
        ``slot_out[self*C:]``), peer rows probed in the peers' tables."""
        it, iv, isd, seed = self.table.init.args()
        hipops().p2p_lookup_rows(self.tabs, self.G, self.rank, send, self.H, self.C, self.kw,
                                 wout, slot_out, it, iv, isd, seed, self.table._err,
                                 self.table._inserted)

    def post(self, send):
        """Write the peer rows of ``send`` (keys + gradients) into the owners' inboxes."""
        self.seq += 1
        hipops().p2p_post(send, self.H, self.C, self.kw, self.nb, self.G, self.rank, self.seq,
                          self.Q, self.rings, self.applieds, self.ok, self.err, self.err_host,
                          self.spin)

    def check_fatal(self):
        """No sync: raise if a completed post gave up waiting for ring space (published
        into pinned host memory by the post's last kernel; seen at most the stream's
        depth after it happened)."""
        if int(self.err_host[0]):
            raise RuntimeError(
                f"p2p exchange: a push waited {self.spin / 1e6:g} s for an owner's inbox space "
                f"and gave up (that owner stopped applying); its gradients are lost")

    def own_update(self, slot, grad, count, rule, stats):
        """This rank's own row of a step (resolved slots, gradients, live count) applied
        on the owner stream, after the current stream's work so far; ``ev_own`` marks
        its end (the next step's packs wait for it before reusing the buffers)."""
        if self.astream is None:
            hipops().kv_update(self.table.slots, slot, grad, count, *rule.args(), stats)
            return
        self.astream.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(self.astream):
            hipops().kv_update(self.table.slots, slot, grad, count, *rule.args(), stats)
            self.ev_own.record(self.astream)

    def wait_own(self):
        """Order the current stream after the last ``own_update``."""
        if self.ev_own is not None:
            torch.cuda.current_stream(self.device).wait_event(self.ev_own)

    def apply(self, rule, stats, slots_scratch, wscratch, link, nxt, rounds: int = 1):
        """Owner: apply up to ``rounds`` ready inbox entries per source (on the owner
        stream: independent of this rank's own posts)."""
        if self.astream is None:
            return self._apply(rule, stats, slots_scratch, wscratch, link, nxt, rounds)
        with torch.cuda.stream(self.astream):
            self._apply(rule, stats, slots_scratch, wscratch, link, nxt, rounds)

    def _apply(self, rule, stats, slots_scratch, wscratch, link, nxt, rounds: int = 1):
        hh, tb = hipops(), self.table
        G, H, C = self.G, self.H, self.C
        it, iv, isd, seed = tb.init.args()
        for _ in range(rounds):
            hh.p2p_gather(self.inbox, self.applied, G, self.rank, self.Q, H, C, self.kw, self.nb,
                          self.stage, self.ready)
            hh.kv_resolve_rows(tb.slots, self.stage, H, C, self.kw, slots_scratch, wscratch, True,
                               it, iv, isd, seed, tb._err, tb._inserted, tb.home_base, tb.home_m,
                               None, None, 0)
            if self.nb:  # FixingFloat codes -> f32 (rows not ready decode 0 gradients)
                hh.xchg_ff_decode(self.stage, C, self.kw, H, self.nb, self.gdec)
                g, gstride = self.gdec, C
            else:
                g, gstride = self.stage.view(torch.float32)[4 + C * self.kw:], H
            hh.kv_update_rows(tb.slots, slots_scratch, g, gstride, self.stage, H, C, link, nxt,
                              *rule.args(), stats)
            hh.p2p_commit(self.applied, self.ready, G, self.total)

    def check(self):
        """Host sync: raise if a push gave up waiting for ring space (a peer stopped
        applying for ``spin_us``)."""
        if int(self.err.item()):
            raise RuntimeError("p2p exchange: a push timed out waiting for an owner's inbox "
                               "space (that owner stopped applying)")

    def drain(self, rule, stats, slots_scratch, wscratch, link, nxt, timeout: float = 120.0):
        """Collective at the end of training: apply every push every rank posted. The
        posted counts go over the host (gloo) channel: an RCCL object all-gather would
        synchronise this rank's stream first, and a post still waiting for ring space on a
        peer that only frees it while draining would then stall both sides until the
        spin gives up."""
        posted = self.comm.host_gather_obj(self.seq)
        want = torch.tensor(posted, dtype=torch.int32)
        want[self.rank] = 0
        t0 = time.time()
        while True:
            if self.astream is not None:  # (never behind this rank's own spinning posts)
                self.astream.synchronize()
                with torch.cuda.stream(self.astream):
                    got = self.applied.cpu()
            else:
                got = self.applied.cpu()
            got[self.rank] = 0
            if bool((got >= want).all()):
                break
            if time.time() - t0 > timeout:
                raise RuntimeError(f"p2p drain: applied {got.tolist()} of {want.tolist()}")
            self.apply(rule, stats, slots_scratch, wscratch, link, nxt)
        torch.cuda.synchronize(self.device)
        self.check()
        self.comm.barrier()

    def close(self):
        torch.cuda.synchronize(self.device)
        for ptr, off in self._opened:
            hipops().ipc_close(ptr, off)
        self._opened = []
