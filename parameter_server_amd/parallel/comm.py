"""Data-plane communicator: variable-size all-to-all over RCCL (xGMI) or gloo.

The reference moves every push/pull as ZeroMQ point-to-point messages through
per-process send/recv threads (src/system/van.cc:117-223). On an MI355X node
every rank is a colocated worker + server shard and a push or pull step is ONE
grouped all-to-all-v (``torch.distributed.all_to_all_single`` -> RCCL
``ncclSend/ncclRecv`` in a group, one direct xGMI link per peer pair), preceded by
a tiny all-to-all of the per-peer element counts.

Device ordering. The training pipeline issues collectives from several HIP
streams (the exchange half of step t runs on preparation stream t % 3). A
synchronous ProcessGroupNCCL collective launches its RCCL kernel on the CALLER's
stream, so two collectives of the one communicator issued from two streams could
be in flight at once, and the ranks could then pair up different operations.
Every collective here is therefore chained on the device: it waits for the
completion event of the previous collective of this communicator (whatever stream
that ran on) and records its own, so the device order of the collectives is their
host issue order on every rank. The key packs, applies and resolves around them
still overlap freely. Asynchronous collectives (reduce-scatter / all-gather of the
Darlin and wide-and-deep servers) run on one communicator stream inside the same
chain.

Failing fast. ``init_from_env`` sets a collective timeout (PSAMD_COMM_TIMEOUT
seconds, default 180); a collective that a stalled or dead peer never joins
raises (gloo) or is aborted by the ProcessGroupNCCL watchdog (RCCL), so the job
exits non-zero instead of hanging. The reference has no such bound: a dead peer
stalls its Executor forever (src/system/executor.cc:160-166). ``Comm.last_op``
names the last collective issued (for bench.py's stall report).
"""
from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist

from ..utils.trace import count_traffic


def comm_timeout() -> datetime.timedelta:
    return datetime.timedelta(seconds=float(os.environ.get("PSAMD_COMM_TIMEOUT", "180")))


def nccl_options():
    """ProcessGroupNCCL options. PSAMD_NCCL_HIGH_PRIO=1 puts the communicator's
    internal stream at high priority. Off by default: the 8-peer loopback measured
    0.140-0.147 ms/step with it vs 0.139-0.140 without, and the collectives of the
    data plane are synchronous (they run on the caller's stream, where the option
    does nothing); the real multi-GPU effect is unmeasured."""
    try:
        opts = dist.ProcessGroupNCCL.Options()
    except (AttributeError, RuntimeError):
        return None
    opts.is_high_priority_stream = os.environ.get("PSAMD_NCCL_HIGH_PRIO", "0") == "1"
    try:
        opts._timeout = comm_timeout()
    except (AttributeError, TypeError):
        pass
    return opts


_OPS = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}


class _Done:
    def wait(self):
        return True


class _ChainedWork:
    """Handle of an asynchronous chained collective: ``wait()`` orders the current
    stream after it (no host block)."""

    def __init__(self, ev):
        self.ev = ev

    def wait(self):
        torch.cuda.current_stream().wait_event(self.ev)
        return True


def _a2a_equal(recv: torch.Tensor, send: torch.Tensor, group=None) -> None:
    """Equal-split all-to-all straight on the c10d ProcessGroup (the per-step data
    plane: skips the Python wrapper's per-call checks, ~1/3 of its host time); the
    work's wait() orders the caller's stream after the collective, no host block."""
    pg = group if group is not None else dist.distributed_c10d._get_default_group()
    opts = dist.AllToAllOptions()
    opts.asyncOp = False
    work = pg.alltoall_base(recv, send, [], [], opts)
    if work is not None:  # (ProcessGroupNCCL returns None for a synchronous op)
        work.wait()


class _DeviceChain:
    """Total device order of one communicator's collectives (see the module doc).
    ``run(name, fn)`` runs ``fn`` (a synchronous collective on the current stream)
    after the previous chained collective and records its completion;
    ``run_async`` runs it on the communicator stream and returns a handle."""

    def __init__(self, device):
        self.device = torch.device(device)
        # PSAMD_COMM_CHAIN=0: no device ordering (A/B of its host cost only; unsafe
        # with collectives issued from several streams)
        self.on = self.device.type == "cuda" and os.environ.get("PSAMD_COMM_CHAIN", "1") != "0"
        self.ev = None           # completion of the last chained collective
        self._cs = None          # communicator stream of the asynchronous collectives
        self.n = 0
        self.last = None

    def _note(self, name):
        self.n += 1
        self.last = name

    def run(self, name, fn):
        self._note(name)
        if not self.on or torch.cuda.is_current_stream_capturing():
            # (a collective captured into a HIP graph: the replay of that graph is what
            # gets ordered, by wait() before it and mark() after it)
            return fn()
        cur = torch.cuda.current_stream(self.device)
        if self.ev is not None:
            cur.wait_event(self.ev)
        out = fn()
        if self.ev is None:
            self.ev = torch.cuda.Event()
        # (re-recording one event is safe: a wait enqueued earlier is bound to the
        # record that preceded it)
        self.ev.record(cur)
        return out

    def wait(self, stream):
        """``stream`` waits for the last chained collective (before replaying a graph
        that contains collectives)."""
        if self.on and self.ev is not None:
            stream.wait_event(self.ev)

    def mark(self, stream, n: int = 1):
        """The work just issued on ``stream`` (a graph replay holding ``n``
        collectives) is now the last chained collective."""
        self.n += n
        self.last = "graph"
        if not self.on:
            return
        if self.ev is None:
            self.ev = torch.cuda.Event()
        self.ev.record(stream)

    def run_async(self, name, fn, tensors=()):
        self._note(name)
        if not self.on:
            fn()
            return _Done()
        if self._cs is None:
            self._cs = torch.cuda.Stream(self.device)
        cur = torch.cuda.current_stream(self.device)
        self._cs.wait_stream(cur)
        if self.ev is not None:
            self._cs.wait_event(self.ev)
        with torch.cuda.stream(self._cs):
            fn()
        for t in tensors:  # the caller's buffers are in use on the communicator stream
            t.record_stream(self._cs)
        done = torch.cuda.Event()
        done.record(self._cs)
        self.ev = done
        return _ChainedWork(done)


class Comm:
    rank = 0
    world = 1
    chain = None

    @property
    def last_op(self) -> str:
        """'<name> #<n>' of the last collective issued (stall diagnostics)."""
        c = self.chain
        return f"{c.last} #{c.n}" if c is not None and c.n else "none"

    def exchange_counts(self, send_counts: torch.Tensor) -> torch.Tensor:
        return send_counts.clone()

    def all_to_all_v(self, send: torch.Tensor, send_counts, recv_counts) -> torch.Tensor:
        return send

    def all_to_all_fixed(self, send: torch.Tensor, recv: torch.Tensor) -> torch.Tensor:
        """Equal-split all-to-all into a preallocated ``recv`` (chunk p of ``send`` goes
        to rank p). No host-side sizes, so it can sit between graph replays with no
        device->host sync."""
        recv.copy_(send)
        return recv

    def all_gather_counts(self, counts: torch.Tensor, to_host: bool = True) -> torch.Tensor:
        """[world, world] int64 matrix (row r = counts sent by rank r); on the host
        unless ``to_host=False`` (then the caller syncs when it needs the values)."""
        m = counts.reshape(1, -1)
        return m.cpu() if to_host else m

    def all_reduce_(self, t: torch.Tensor, op="sum") -> torch.Tensor:
        return t

    def all_reduce_async(self, t: torch.Tensor, op="sum"):
        """Start an in-place all-reduce; returns a handle whose ``wait()`` orders the
        current stream after it (RCCL runs it on its own stream meanwhile)."""
        return _Done()

    def reduce_scatter_async(self, out: torch.Tensor, inp: torch.Tensor):
        """Start ``out = sum over ranks of chunk[rank] of inp`` (``inp`` holds ``world``
        equal chunks of ``out.numel()``); ``wait()`` orders the current stream after it."""
        out.copy_(inp[:out.numel()])
        return _Done()

    def all_gather_into_async(self, out: torch.Tensor, inp: torch.Tensor):
        """Start ``out = cat over ranks of inp``; ``wait()`` as above."""
        out[:inp.numel()].copy_(inp)
        return _Done()

    def all_gather_obj(self, obj):
        return [obj]

    def host_gather_obj(self, obj):  # (host-only channel; see DistComm)
        return self.all_gather_obj(obj)

    def barrier(self):
        pass

    def bytes_moved(self) -> int:
        return 0


class LocalComm(Comm):
    """Single rank: identity exchanges."""

    def __init__(self, device="cpu"):
        self.device = torch.device(device)


class LoopbackComm(Comm):
    """Emulated ``world``-rank group inside ONE process (rank 0): every exchange
    returns the local buffer, so the rank also plays the owner of every peer's key
    range. Used to measure on one GPU the per-rank device work of an N-GPU step
    (G exchange rows, G per-source owner updates, the row-wise resolve) without
    the collectives; a benchmarking aid, not a training mode."""

    backend = "loopback"

    def __init__(self, world: int, device="cpu", comm_stream: bool = True, group=None):
        self.world = int(world)
        self.rank = 0
        self.device = torch.device(device)
        # group: a real 1-rank process group (nccl = RCCL) that carries every exchange,
        # so the emulation runs RCCL's kernels, streams and work-completion waits
        self.group = group
        # model ProcessGroupNCCL's stream structure: the collective runs on the
        # communicator's own stream, ordered after the caller's stream and before
        # the caller's next work (so the emulation sees the same number of streams)
        self._cs = (torch.cuda.Stream(self.device) if comm_stream and self.device.type == "cuda"
                    else None)
        # the real communicator's device chain (rehearsed on the 1-rank RCCL loopback)
        self.chain = _DeviceChain(self.device if group is not None else "cpu")

    def all_to_all_fixed(self, send: torch.Tensor, recv: torch.Tensor) -> torch.Tensor:
        if self.group is not None:
            self.chain.run("all_to_all_fixed", lambda: _a2a_equal(recv, send, self.group))
            return recv
        if self._cs is None:
            recv.copy_(send)
            return recv
        cur = torch.cuda.current_stream(self.device)
        self._cs.wait_stream(cur)
        with torch.cuda.stream(self._cs):
            recv.copy_(send)
        cur.wait_stream(self._cs)
        return recv

    def all_gather_counts(self, counts: torch.Tensor, to_host: bool = True) -> torch.Tensor:
        m = counts.reshape(1, -1).expand(self.world, -1)
        return m.cpu() if to_host else m

    def all_reduce_(self, t: torch.Tensor, op="sum") -> torch.Tensor:
        if self.group is not None and t.is_cuda:
            self.chain.run("all_reduce", lambda: dist.all_reduce(t, op=_OPS[op], group=self.group))
        return t

    def barrier(self):
        if self.group is not None:
            self.chain.run("barrier", lambda: dist.barrier(group=self.group,
                                                           device_ids=[self.device.index or 0]))


def nccl_loopback(world: int, device) -> LoopbackComm:
    """Emulated ``world``-rank exchange whose collectives run through a real 1-rank
    RCCL communicator (rehearses the NCCL code path on a 1-GPU box: RCCL refuses two
    ranks on one device)."""
    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if "MASTER_PORT" not in os.environ:
            import socket

            with socket.socket() as s:
                s.bind(("127.0.0.1", 0))
                os.environ["MASTER_PORT"] = str(s.getsockname()[1])
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device(device),
                                pg_options=nccl_options(), timeout=comm_timeout())
    return LoopbackComm(world, device, comm_stream=False, group=dist.group.WORLD)


class DistComm(Comm):
    """torch.distributed process group (nccl = RCCL on ROCm, or gloo on CPU)."""

    def __init__(self, device=None, group=None):
        assert dist.is_initialized(), "init_process_group first"
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.backend = dist.get_backend(group)
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self._sent = 0
        # device order of the collectives (RCCL on GPU tensors); gloo only counts
        self.chain = _DeviceChain(self.device if self.backend == "nccl" else "cpu")

    def exchange_counts(self, send_counts: torch.Tensor) -> torch.Tensor:
        sc = send_counts.to(torch.int64)
        if self.backend == "nccl" and not sc.is_cuda:
            sc = sc.to(self.device)
        elif self.backend == "gloo" and sc.is_cuda:
            sc = sc.cpu()
        rc = torch.empty_like(sc)
        self.chain.run("exchange_counts",
                       lambda: dist.all_to_all_single(rc, sc.contiguous(), group=self.group))
        count_traffic("all_to_all_counts", 8 * (sc.numel() - 1), 8 * (sc.numel() - 1))
        return rc

    def all_to_all_v(self, send: torch.Tensor, send_counts, recv_counts) -> torch.Tensor:
        sc = [int(x) for x in send_counts]
        rc = [int(x) for x in recv_counts]
        staged = self.backend == "gloo" and send.is_cuda  # rehearsal mode: GPU ranks over gloo
        src = send.cpu() if staged else send
        out = torch.empty((sum(rc),) + tuple(send.shape[1:]), dtype=send.dtype,
                          device=src.device)
        self.chain.run("all_to_all_v", lambda: dist.all_to_all_single(
            out, src.contiguous(), output_split_sizes=rc, input_split_sizes=sc, group=self.group))
        if staged:
            out = out.to(send.device)
        row = send.element_size() * max(1, send[0:1].numel())
        sent, got = row * (sum(sc) - sc[self.rank]), row * (sum(rc) - rc[self.rank])
        self._sent += sent
        count_traffic("all_to_all", sent, got)
        return out

    def all_to_all_fixed(self, send: torch.Tensor, recv: torch.Tensor) -> torch.Tensor:
        assert send.numel() == recv.numel() and send.numel() % self.world == 0
        if self.backend == "gloo" and send.is_cuda:  # rehearsal mode: staged through host
            out = torch.empty(recv.shape, dtype=recv.dtype)
            self.chain.run("all_to_all_fixed",
                           lambda: dist.all_to_all_single(out, send.cpu(), group=self.group))
            recv.copy_(out)
        else:
            self.chain.run("all_to_all_fixed", lambda: _a2a_equal(recv, send, self.group))
        b = send.numel() * send.element_size() * (self.world - 1) // self.world
        self._sent += b
        count_traffic("all_to_all_fixed", b, b)
        return recv

    def all_gather_counts(self, counts: torch.Tensor, to_host: bool = True) -> torch.Tensor:
        c = counts.to(torch.int64).reshape(-1).contiguous()
        if self.backend == "nccl":
            c = c.to(self.device)
        elif c.is_cuda:
            c = c.cpu()
        out = torch.empty(self.world * c.numel(), dtype=torch.int64, device=c.device)
        self.chain.run("all_gather_counts",
                       lambda: dist.all_gather_into_tensor(out, c, group=self.group))
        count_traffic("all_gather", 8 * c.numel(), 8 * c.numel() * (self.world - 1))
        out = out.reshape(self.world, -1)
        return out.cpu() if to_host else out

    def _count_reduce(self, t: torch.Tensor) -> None:
        # ring all-reduce: each rank sends/receives 2 (G-1)/G of the buffer
        b = t.numel() * t.element_size() * 2 * (self.world - 1) // max(1, self.world)
        count_traffic("all_reduce", b, b)

    def all_reduce_(self, t: torch.Tensor, op="sum") -> torch.Tensor:
        self._count_reduce(t)
        if self.backend == "gloo" and t.is_cuda:
            h = t.cpu()
            self.chain.run("all_reduce", lambda: dist.all_reduce(h, op=_OPS[op], group=self.group))
            t.copy_(h)
            return t
        self.chain.run("all_reduce", lambda: dist.all_reduce(t, op=_OPS[op], group=self.group))
        return t

    def all_reduce_async(self, t: torch.Tensor, op="sum"):
        if self.backend == "gloo" and t.is_cuda:  # rehearsal mode: synchronous, staged
            self.all_reduce_(t, op)
            return _Done()
        self._count_reduce(t)
        if self.backend == "gloo":
            return dist.all_reduce(t, op=_OPS[op], group=self.group, async_op=True)
        return self.chain.run_async(
            "all_reduce", lambda: dist.all_reduce(t, op=_OPS[op], group=self.group), (t,))

    def reduce_scatter_async(self, out: torch.Tensor, inp: torch.Tensor):
        n = out.numel()
        assert inp.numel() == n * self.world
        b = n * out.element_size() * (self.world - 1)
        count_traffic("reduce_scatter", b, b)
        if self.backend == "gloo":  # gloo has no reduce-scatter: all-reduce, keep own chunk
            h = inp.detach().to("cpu", copy=True)
            self.chain.run("reduce_scatter", lambda: dist.all_reduce(h, group=self.group))
            out.copy_(h[self.rank * n:(self.rank + 1) * n])
            return _Done()
        return self.chain.run_async(
            "reduce_scatter", lambda: dist.reduce_scatter_tensor(out, inp, group=self.group),
            (out, inp))

    def all_gather_into_async(self, out: torch.Tensor, inp: torch.Tensor):
        assert out.numel() == inp.numel() * self.world
        b = inp.numel() * inp.element_size() * (self.world - 1)
        count_traffic("all_gather", b, b)
        if self.backend == "gloo" and inp.is_cuda:  # rehearsal mode: staged through host
            h = torch.empty(out.shape, dtype=out.dtype)
            self.chain.run("all_gather",
                           lambda: dist.all_gather_into_tensor(h, inp.cpu(), group=self.group))
            out.copy_(h)
            return _Done()
        if self.backend == "gloo":
            return dist.all_gather_into_tensor(out, inp, group=self.group, async_op=True)
        return self.chain.run_async(
            "all_gather", lambda: dist.all_gather_into_tensor(out, inp, group=self.group),
            (out, inp))

    def all_gather_obj(self, obj):
        out = [None] * self.world
        self.chain.run("all_gather_obj", lambda: dist.all_gather_object(out, obj, group=self.group))
        return out

    def host_gather_obj(self, obj):
        """All-gather of a small picklable object over a gloo group: host only, no device
        synchronisation (an RCCL object collective stages through the device stream).
        Collective; the first call creates the gloo group on every rank."""
        if self.backend == "gloo":
            return self.all_gather_obj(obj)
        if getattr(self, "_hgroup", None) is None:
            ranks = dist.get_process_group_ranks(self.group) if self.group is not None else None
            self._hgroup = dist.new_group(ranks=ranks, backend="gloo")
        out = [None] * self.world
        dist.all_gather_object(out, obj, group=self._hgroup)
        return out

    def barrier(self):
        if self.backend == "nccl":
            self.chain.run("barrier", lambda: dist.barrier(group=self.group,
                                                           device_ids=[self.device.index or 0]))
        else:
            self.chain.run("barrier", lambda: dist.barrier(group=self.group))

    def bytes_moved(self) -> int:
        return self._sent


def init_from_env(device_type: str = "cuda", backend: str | None = None):
    """Initialise torch.distributed from torchrun env vars; returns (Comm, device)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if device_type == "cuda":
        # PSAMD_DIST_BACKEND=gloo + more ranks than GPUs = rehearsal of the multi-rank
        # GPU protocol on a 1-GPU box (exchanges staged through host memory).
        ndev = max(1, torch.cuda.device_count())
        torch.cuda.set_device(local_rank % ndev)
        device = torch.device("cuda", local_rank % ndev)
    else:
        device = torch.device("cpu")
    if world <= 1:
        return LocalComm(device), device
    if not dist.is_initialized():
        backend = backend or os.environ.get("PSAMD_DIST_BACKEND") or (
            "nccl" if device_type == "cuda" else "gloo")
        kw = {}
        if backend == "nccl":
            kw["device_id"] = device
            kw["pg_options"] = nccl_options()
        dist.init_process_group(backend=backend, timeout=comm_timeout(), **kw)
    return DistComm(device), device
