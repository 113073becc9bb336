"""Wide & deep on the sharded embedding table: CPU single rank learns; 2 ranks over
gloo keep identical dense replicas and shard the table."""
import socket

import pytest
import torch
import torch.multiprocessing as mp

from parameter_server_amd.models.wide_deep import WideDeepConfig, WideDeepTrainer
from parameter_server_amd.ops.synthetic import criteo_batch

CFG = dict(num_features=1 << 20, embedding_dim=16, hidden=(64, 32), minibatch=256,
           table_capacity=1 << 15, emb_lr=0.05, mlp_lr=3e-3)


def test_wide_deep_cpu_learns():
    tr = WideDeepTrainer(WideDeepConfig(**CFG))
    first = last = None
    for s in range(40):
        k, l = criteo_batch(256, seed=5, row0=s * 256, num_features=CFG["num_features"],
                            cards=[300] * 26)
        tr.step(k, l)
        if s == 9:
            first = tr.progress()
        if s == 39:
            last = tr.progress()
    assert last["loss"] < first["loss"] - 0.03
    assert last["auc"] > 0.7


def test_pack_unpack_records():
    rows = torch.randn(5, 16).to(torch.bfloat16)
    w = torch.randn(5)
    rec = WideDeepTrainer._pack(rows, w)
    assert rec.shape == (5, 9) and rec.dtype == torch.int32
    r2, w2 = WideDeepTrainer._unpack(rec, 16)
    assert torch.equal(r2, rows) and torch.equal(w2, w)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist

    from parameter_server_amd.parallel.comm import DistComm

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    tr = WideDeepTrainer(WideDeepConfig(**CFG), DistComm("cpu"), "cpu")
    for s in range(12):
        k, l = criteo_batch(256, seed=11 + rank, row0=s * 256, num_features=CFG["num_features"],
                            cards=[300] * 26)
        tr.step(k, l)
    p = tr.progress()
    occ, _ = tr.shard.table.census()
    q.put((rank, p, tr.param.detach().numpy().copy(), occ))  # numpy: no fd sharing
    dist.barrier()
    dist.destroy_process_group()


def test_wide_deep_two_ranks_gloo():
    port = _port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=240) for _ in ps], key=lambda r: r[0])
    for p in ps:
        p.join(timeout=60)
    assert (res[0][2] == res[1][2]).all()  # dense replicas identical after all-reduce
    assert res[0][1]["examples"] == 2 * 12 * 256
    assert 0.3 < res[0][1]["loss"] < 0.75
    assert res[0][3] > 0 and res[1][3] > 0  # both shards hold rows
