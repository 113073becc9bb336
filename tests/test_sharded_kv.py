"""KVWorker / KVServer push-pull API (ps.h parity) on one rank and over gloo."""
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from parameter_server_amd.ops.kv_table import UpdateRule
from parameter_server_amd.parameter.sharded_kv import KVWorker


def test_single_rank_add_assign_and_optimizer():
    kv = KVWorker(device="cpu", capacity=1 << 12)
    keys = torch.tensor([5, 1, 5, -(1 << 63) + 7, 42], dtype=torch.int64)
    kv.wait(kv.push(keys, torch.tensor([1.0, 2.0, 3.0, 4.0, 5.0])))
    out = kv.wait(kv.pull(torch.tensor([5, 42, 1, 999, -(1 << 63) + 7], dtype=torch.int64)))
    assert out.tolist() == [4.0, 5.0, 2.0, 0.0, 4.0]  # duplicates summed, unknown -> 0
    kv2 = KVWorker(device="cpu", capacity=1 << 10, rule="assign")
    kv2.wait(kv2.push(torch.tensor([3, 4]), torch.tensor([7.0, 8.0])))
    kv2.wait(kv2.push(torch.tensor([3]), torch.tensor([1.5])))
    assert kv2.wait(kv2.pull(torch.tensor([4, 3]))).tolist() == [8.0, 1.5]
    kv3 = KVWorker(device="cpu", rule=UpdateRule("sgd", "constant", alpha=0.5))
    kv3.wait(kv3.push(torch.tensor([9]), torch.tensor([2.0])))
    assert kv3.wait(kv3.pull(torch.tensor([9]))).tolist() == [-1.0]
    k, v = kv.shard_items()
    # pull inserts unknown keys (KVStore::getValue uses map operator[], kv_store.h:37-45)
    assert sorted(k.tolist()) == sorted([5, 1, 42, 999, -(1 << 63) + 7])


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
    kv = KVWorker(DistComm("cpu"), "cpu", capacity=1 << 14)
    rng = np.random.default_rng(rank)
    keys = torch.from_numpy(rng.integers(0, 500, 300)).to(torch.int64)
    vals = torch.from_numpy(rng.normal(0, 1, 300)).float()
    t = kv.push(keys, vals)
    kv.wait(t)
    kv.barrier()
    allk = torch.arange(500, dtype=torch.int64)
    got = kv.wait(kv.pull(allk))
    sk, sv = kv.shard_items()
    q.put((rank, got.numpy(), sk.numel()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_multi_rank_push_pull(world):
    port = _port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=120) for _ in ps], key=lambda r: r[0])
    for p in ps:
        p.join(timeout=30)
    exp = np.zeros(500)
    for r in range(world):
        rng = np.random.default_rng(r)
        k = rng.integers(0, 500, 300)
        v = rng.normal(0, 1, 300).astype(np.float32)
        np.add.at(exp, k, v)
    for _, got, _ in res:
        np.testing.assert_allclose(got, exp, rtol=1e-5, atol=1e-5)
    assert sum(r[2] for r in res) == 500  # every key lives on exactly one shard
    assert all(r[2] > 0 for r in res)     # and the shards are balanced-ish


@pytest.mark.gpu
def test_kvworker_gpu_single_rank():
    kv = KVWorker(device="cuda", capacity=1 << 14)
    keys = torch.randint(0, 1 << 40, (5000,), device="cuda")
    vals = torch.randn(5000, device="cuda")
    kv.wait(kv.push(keys, vals))
    got = kv.wait(kv.pull(keys))
    uk, inv = torch.unique(keys, return_inverse=True)
    exp = torch.zeros(uk.numel(), device="cuda").index_add_(0, inv, vals)[inv]
    torch.testing.assert_close(got, exp, rtol=1e-5, atol=1e-5)
