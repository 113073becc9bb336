"""One-sided peer-HBM exchange (parallel/p2p.py, csrc/hip/p2p.hip): several ranks on
one GPU bootstrap over gloo and map each other's shards / inboxes through real IPC
handles, then move data with no collective per step.

* transport: known gradients for known keys, SGD with a constant step and no
  penalty (linear in the pushes): after the drain every key's weight must be
  -alpha x the sum of every rank's pushes, whatever order the owners applied them in;
* training: asynchronous FTRL through the trainer's p2p mode learns (loss < ln 2).
"""
import math
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _transport_worker(rank, world, port, out_dir, steps, Q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from parameter_server_amd.ops.kv_table import KVTable, UpdateRule, next_pow2
    from parameter_server_amd.parallel.comm import DistComm
    from parameter_server_amd.parallel.p2p import PeerExchange
    from parameter_server_amd.parallel.partition import KeyPartition

    dev = torch.device("cuda", 0)
    comm = DistComm(dev)
    bits = 30
    part = KeyPartition(bits, world)
    table = KVTable(1 << 14, dev, key_range=part.range_of(rank))
    C, kw = 256, 1
    H = (4 + C * kw + C + 3) // 4 * 4
    px = PeerExchange(comm, table, C, kw, H, dev, Q=Q)
    rule = UpdateRule("sgd", "constant", 0.5, 0.0, 0.0, 0.0)
    G = world
    stats = torch.zeros(3, dtype=torch.float64, device=dev)
    send = torch.zeros(G * H, dtype=torch.int32, device=dev)
    wout = torch.zeros(G * C, dtype=torch.float32, device=dev)
    slot = torch.full((G * C,), -1, dtype=torch.int64, device=dev)
    a_slot = torch.full((G * C,), -1, dtype=torch.int64, device=dev)
    a_w = torch.zeros(G * C, dtype=torch.float32, device=dev)
    link = torch.empty(next_pow2(2 * G * C), dtype=torch.int64, device=dev)
    nxt = torch.empty(G * C, dtype=torch.int32, device=dev)
    # every owner's 40 keys (the same on every rank): the first 40 keys of its range
    keys = {p: [part.range_of(p)[0] + 7 * i for i in range(40)] for p in range(G)}
    rng = np.random.default_rng(100 + rank)
    sent = {}
    for t in range(steps):
        sh = torch.zeros(G * H, dtype=torch.int32)
        for p in range(G):
            n = int(rng.integers(1, 41))
            ks = sorted(rng.choice(keys[p], size=n, replace=False).tolist())
            gs = rng.standard_normal(n).astype(np.float32)
            sh[p * H] = n
            sh[p * H + 1] = n
            sh[p * H + 4:p * H + 4 + n] = torch.tensor(ks, dtype=torch.int64).to(torch.int32)
            sh.view(torch.float32)[p * H + 4 + C * kw:p * H + 4 + C * kw + n] = torch.from_numpy(gs)
            for k, g in zip(ks, gs):
                sent[(p, k)] = sent.get((p, k), 0.0) + float(g)
        px.wait_own()  # (the previous own-row update has read send / slot)
        send.copy_(sh.to(dev))
        px.lookup(send, wout, slot)
        g_own = send.view(torch.float32)[rank * H + 4 + C:rank * H + 4 + 2 * C]
        # the own row on the owner stream, serialised with the peer applies (a kv_update
        # on this stream would race them on the same slots)
        px.own_update(slot[rank * C:(rank + 1) * C], g_own, send[rank * H + 1:rank * H + 2],
                      rule, stats)
        px.post(send)
        px.apply(rule, stats, a_slot, a_w, link, nxt, rounds=1)
    px.drain(rule, stats, a_slot, a_w, link, nxt)
    mine = keys[rank]
    slot_m, w_m = table.resolve(torch.tensor(mine, dtype=torch.int64, device=dev), insert=False)
    torch.save({"sent": sent, "keys": mine, "w": w_m.cpu(), "slot": slot_m.cpu(),
                "total": int(px.total.item())}, os.path.join(out_dir, f"t{rank}.pt"))
    px.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,steps,Q", [(2, 12, 4), (3, 9, 16)])
def test_p2p_transport_applies_every_push(tmp_path, world, steps, Q):
    mp.spawn(_transport_worker, args=(world, _port(), str(tmp_path), steps, Q), nprocs=world,
             join=True)
    res = [torch.load(tmp_path / f"t{r}.pt", weights_only=False) for r in range(world)]
    for owner, r in enumerate(res):
        exp = {}
        for src in res:
            for (p, k), g in src["sent"].items():
                if p == owner:
                    exp[k] = exp.get(k, 0.0) + g
        for k, w, s in zip(r["keys"], r["w"].tolist(), r["slot"].tolist()):
            if k in exp:
                assert s >= 0
                assert w == pytest.approx(-0.5 * exp[k], rel=1e-4, abs=1e-4)
        # every peer entry applied exactly once (steps per source, own row local)
        assert r["total"] == steps * (world - 1)


def _train_worker(rank, world, port, out_dir, init="zero", nb=0):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from parameter_server_amd.models import SparseLRConfig, SparseLRTrainer
    from parameter_server_amd.ops.kv_table import InitRule
    from parameter_server_amd.ops.synthetic import criteo_batch
    from parameter_server_amd.parallel.comm import DistComm

    dev = torch.device("cuda", 0)
    B = 8192
    cfg = SparseLRConfig(num_features=10 ** 8, minibatch=B, table_capacity=1 << 22,
                         consistency="asp", exchange="p2p", seed=rank, fixing_float_bytes=nb,
                         init=InitRule(init, 0.0, 0.01 if init == "gaussian" else 0.0, 3))
    tr = SparseLRTrainer(cfg, DistComm(dev), dev)
    for t in range(40):
        k, lab = criteo_batch(B, seed=1000 + rank, row0=t * B, num_features=cfg.num_features,
                              device=dev)
        tr.step(k, lab, width=39)
        if t == 19:
            tr.progress(reset=True)
    p = tr.progress(reset=True)
    occ, nnz = tr.table.census()
    torch.save({"p": p, "occ": occ, "desc": tr.consistency_desc(), "fine": tr.px.fine},
               os.path.join(out_dir, f"p{rank}.pt"))
    tr.px.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,init,nb", [(2, "zero", 0), (2, "gaussian", 1), (3, "zero", 2)])
def test_p2p_trainer_trains(tmp_path, world, init, nb):
    """Asynchronous FTRL over the one-sided exchange trains, also with non-zero initial
    weights (a peer's lookup may race the owner's insert: it must see the init value,
    never an unpublished 0) and with FixingFloat pushes (1 or 2 bytes per gradient)."""
    mp.spawn(_train_worker, args=(world, _port(), str(tmp_path), init, nb), nprocs=world,
             join=True)
    res = [torch.load(tmp_path / f"p{r}.pt", weights_only=False) for r in range(world)]
    for r in res:
        assert r["p"]["loss"] < math.log(2) and r["p"]["auc"] > 0.65, r["p"]
        assert r["occ"] > 0
        assert r["desc"].startswith("asp-p2p")
        assert r["fine"]  # inbox / applied counters in fine-grained memory


def _stall_worker(rank, world, port, out_dir):
    """Rank 1 never applies; rank 0 keeps posting to it with a short give-up time and
    must fail at the first post that gave up, not train on with lost pushes."""
    import time

    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from parameter_server_amd.ops.kv_table import KVTable
    from parameter_server_amd.parallel.comm import DistComm
    from parameter_server_amd.parallel.p2p import PeerExchange
    from parameter_server_amd.parallel.partition import KeyPartition

    dev = torch.device("cuda", 0)
    comm = DistComm(dev)
    part = KeyPartition(30, world)
    table = KVTable(1 << 12, dev, key_range=part.range_of(rank))
    C, kw, Q = 64, 1, 2
    H = (4 + C * kw + C + 3) // 4 * 4
    px = PeerExchange(comm, table, C, kw, H, dev, Q=Q, spin_us=200_000)
    send = torch.zeros(world * H, dtype=torch.int32, device=dev)
    send[1 * H] = 1  # one key for the owner, rank 1
    send[1 * H + 1] = 1
    send[1 * H + 4] = int(part.range_of(1)[0])
    msg, t0 = "", time.time()
    if rank == 0:
        try:
            for _ in range(Q + 3):
                px.post(send)
                torch.cuda.synchronize()
                px.check_fatal()
        except RuntimeError as e:
            msg = str(e)
    dt = time.time() - t0
    with open(os.path.join(out_dir, f"s{rank}.txt"), "w") as f:
        f.write(f"{dt}\n{msg}")
    dist.barrier()
    px.close()
    dist.destroy_process_group()


def test_p2p_push_timeout_is_fatal_at_once(tmp_path):
    mp.spawn(_stall_worker, args=(2, _port(), str(tmp_path)), nprocs=2, join=True)
    dt, msg = (tmp_path / "s0.txt").read_text().split("\n", 1)
    assert "gave up" in msg, msg
    assert float(dt) < 10.0  # the first post past the ring (Q = 2) waits 0.2 s, then raises
