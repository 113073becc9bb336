"""KVWorker / KVServer push-pull API (ps.h parity) on one rank and over gloo:
k values per key, non-blocking timestamps, bounded-delay consistency (BSP / SSP(tau) /
ASP) checked against a protocol simulation of the reference's semantics
(src/parameter/kv_vector.h:45-100, src/app/linear_method/darlin.h:81-91)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from parameter_server_amd.ops.kv_table import UpdateRule
from parameter_server_amd.parameter.sharded_kv import KVWorker


def test_single_rank_add_assign_and_optimizer():
    kv = KVWorker(device="cpu", capacity=1 << 12, max_keys=64)
    keys = torch.tensor([5, 1, 5, -(1 << 63) + 7, 42], dtype=torch.int64)
    kv.wait(kv.push(keys, torch.tensor([1.0, 2.0, 3.0, 4.0, 5.0])))
    out = kv.wait(kv.pull(torch.tensor([5, 42, 1, 999, -(1 << 63) + 7], dtype=torch.int64)))
    assert out.tolist() == [4.0, 5.0, 2.0, 0.0, 4.0]  # duplicates summed, unknown -> 0
    kv2 = KVWorker(device="cpu", capacity=1 << 10, rule="assign", max_keys=64)
    kv2.wait(kv2.push(torch.tensor([3, 4]), torch.tensor([7.0, 8.0])))
    kv2.wait(kv2.push(torch.tensor([3]), torch.tensor([1.5])))
    assert kv2.wait(kv2.pull(torch.tensor([4, 3]))).tolist() == [8.0, 1.5]
    kv3 = KVWorker(device="cpu", rule=UpdateRule("sgd", "constant", alpha=0.5), max_keys=64)
    kv3.wait(kv3.push(torch.tensor([9]), torch.tensor([2.0])))
    assert kv3.wait(kv3.pull(torch.tensor([9]))).tolist() == [-1.0]
    k, v = kv.shard_items()
    # pull inserts unknown keys (KVStore::getValue uses map operator[], kv_store.h:37-45)
    assert sorted(k.tolist()) == sorted([5, 1, 42, 999, -(1 << 63) + 7])


def test_single_rank_vector_values_and_nan_skip():
    kv = KVWorker(device="cpu", capacity=1 << 10, dim=4, max_keys=64)
    keys = torch.tensor([3, 8, 3])
    v = torch.arange(12, dtype=torch.float32).reshape(3, 4)
    t1 = kv.push(keys, v)
    t2 = kv.pull(torch.tensor([8, 3, 77]))
    got = kv.wait(t2)   # waited out of order: the pull is still after the push
    kv.wait(t1)
    assert got.shape == (3, 4)
    assert got[0].tolist() == v[1].tolist()
    assert got[1].tolist() == (v[0] + v[2]).tolist()
    assert got[2].tolist() == [0.0] * 4
    nan = torch.full((1, 4), float("nan"))
    kv.wait(kv.push(torch.tensor([8]), nan))  # SparseFilter mark: no value
    assert kv.wait(kv.pull(torch.tensor([8])))[0].tolist() == v[1].tolist()
    with pytest.raises(ValueError):
        kv.push(torch.arange(65), torch.zeros(65, 4))


@pytest.mark.parametrize("tau", [0, 1, 2])
def test_single_rank_ssp_delays_pushes_by_tau(tau):
    kv = KVWorker(device="cpu", capacity=1 << 10, max_keys=16, consistency=f"ssp:{tau}"
                  if tau else "bsp")
    key = torch.tensor([11])
    seen = []
    for i in range(1, 6):
        kv.wait(kv.push(key, torch.tensor([float(i)])))
        seen.append(kv.wait(kv.pull(key)).item())
        assert kv.staleness() == min(i, tau)
    exp = [sum(range(1, max(0, p - tau) + 1)) for p in range(1, 6)]
    assert seen == exp
    kv.flush()
    assert kv.wait(kv.pull(key)).item() == 15.0


# ------------------------------------------------------------------ multi-rank
OPS = ["push", "pull", "push", "push", "pull", "push", "pull", "pull", "push", "pull"]
NK, K = 400, 4


def _batch(rank, i, dim):
    rng = np.random.default_rng(1000 * rank + i)
    n = int(rng.integers(0, 160))  # some calls carry few keys
    keys = rng.integers(0, NK, n)
    vals = rng.normal(0, 1, (n, dim)).astype(np.float32)
    return keys, vals


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir, consistency, dim, device):
    import torch.distributed as dist

    from parameter_server_amd.parallel.comm import DistComm

    torch.set_num_threads(1)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    dev = torch.device(device)
    kv = KVWorker(DistComm(dev), dev, capacity=1 << 12, dim=dim, max_keys=512,
                  consistency=consistency, key_bits=32 if dim == 4 else 64)
    pulls, ts_pull = [], []
    allk = torch.arange(NK, dtype=torch.int64)
    for i, op in enumerate(OPS):
        if op == "push":
            keys, vals = _batch(rank, i, dim)
            kv.push(torch.from_numpy(keys).to(dev), torch.from_numpy(vals).to(dev))
        else:
            ts_pull.append(kv.pull(allk.to(dev)))
    for t in reversed(ts_pull):  # timestamps waited in any order
        pulls.append(kv.wait(t).cpu().numpy())
    pulls.reverse()
    kv.barrier()
    sk, _ = kv.shard_items()
    torch.save({"pulls": pulls, "nkeys": int(sk.numel())}, os.path.join(out_dir, f"kv{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def _simulate(world, tau, dim):
    """Reference semantics: a pull issued after P pushes sees, for every key, the sum
    of all workers' pushes 1 .. P - tau (duplicates within a push summed)."""
    table = np.zeros((NK, dim))
    pushes, out, applied = [], [], 0
    for i, op in enumerate(OPS):
        if op == "push":
            d = np.zeros((NK, dim))
            for r in range(world):
                keys, vals = _batch(r, i, dim)
                np.add.at(d, keys, vals)
            pushes.append(d)
        else:
            while applied < len(pushes) - tau:
                table += pushes[applied]
                applied += 1
            out.append(table.copy())
    return out


def _run(tmp_path, world, consistency, dim, device="cpu"):
    port = _port()
    mp.spawn(_worker, args=(world, port, str(tmp_path), consistency, dim, device), nprocs=world,
             join=True)
    return [torch.load(tmp_path / f"kv{r}.pt", weights_only=False) for r in range(world)]


@pytest.mark.parametrize("world,consistency", [(2, "bsp"), (3, "bsp"), (2, "ssp:1"),
                                               (3, "ssp:2"), (2, "ssp:4")])
def test_gloo_multi_rank_vector_push_pull_consistency(tmp_path, world, consistency):
    tau = 0 if consistency == "bsp" else int(consistency.split(":")[1])
    res = _run(tmp_path, world, consistency, K)
    exp = _simulate(world, tau, K)
    for r in res:
        assert len(r["pulls"]) == len(exp)
        for got, e in zip(r["pulls"], exp):
            np.testing.assert_allclose(got, e, rtol=1e-5, atol=1e-5)
    assert sum(r["nkeys"] for r in res) == NK  # every key lives on exactly one shard
    assert all(r["nkeys"] > 0 for r in res)


def test_gloo_scalar_asp_sees_at_least_bsp_lower_bound(tmp_path):
    """ASP on CPU applies each push at arrival (so equals BSP there); the GPU applies on
    its own stream. Scalar values, 64-bit keys."""
    res = _run(tmp_path, 2, "asp", 1)
    exp = _simulate(2, 0, 1)
    for r in res:
        for got, e in zip(r["pulls"], exp):
            np.testing.assert_allclose(got, e[:, 0], rtol=1e-5, atol=1e-5)


# ------------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("dim,bits", [(1, 64), (4, 32), (16, 64)])
def test_kvworker_gpu_single_rank(dim, bits):
    kv = KVWorker(device="cuda", capacity=1 << 14, dim=dim, key_bits=bits, max_keys=8192)
    keys = torch.randint(0, 1 << 30, (5000,), device="cuda")
    keys[::7] = keys[0]  # a hot key
    vals = torch.randn(5000, dim, device="cuda")
    kv.wait(kv.push(keys, vals))
    got = kv.wait(kv.pull(keys))
    uk, inv = torch.unique(keys, return_inverse=True)
    exp = torch.zeros(uk.numel(), dim, device="cuda").index_add_(0, inv, vals)[inv]
    torch.testing.assert_close(got.reshape(-1, dim), exp, rtol=1e-4, atol=1e-4)
    k, v = kv.shard_items()
    assert k.numel() == uk.numel()


@pytest.mark.gpu
def test_kvworker_gpu_optimizer_rule_and_ssp():
    rule = UpdateRule("sgd", "constant", alpha=0.5)
    kv = KVWorker(device="cuda", rule=rule, max_keys=1024, consistency="ssp:1")
    key = torch.tensor([123456789], device="cuda")
    seen = []
    for i in range(1, 5):
        kv.push(key, torch.tensor([float(i)], device="cuda"))
        seen.append(kv.wait(kv.pull(key)).item())
    # w = -0.5 * sum of the pushes applied: 1 push late
    assert seen == [0.0, -0.5, -1.5, -3.0]


@pytest.mark.gpu
def test_kvworker_gpu_two_rank_rehearsal(tmp_path):
    """Two ranks on the one GPU over gloo (exchanges staged through host memory): the
    device localise / pack / resolve / serve / apply / unpack path of G = 2."""
    res = _run(tmp_path, 2, "ssp:1", K, device="cuda")
    exp = _simulate(2, 1, K)
    for r in res:
        for got, e in zip(r["pulls"], exp):
            np.testing.assert_allclose(got, e, rtol=1e-4, atol=1e-4)
    assert sum(r["nkeys"] for r in res) == NK


def test_hello_world_gpu_app_two_ranks_cpu():
    import subprocess
    import sys

    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node=2", "--master-addr=127.0.0.1",
                        f"--master-port={_port()}", "-m",
                        "parameter_server_amd.app.hello_world_gpu", "--cpu"],
                       capture_output=True, text=True, timeout=180, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    import re

    vals = {int(k): float(v) for k, v in re.findall(r"rank 0: key (\d+): ([-0-9.e]+)", r.stdout)}
    assert vals == {0: 0.0, 1: 0.1, 2: 0.2, 3: 0.3, 4: 0.8, 5: 0.5}


# ----------------------------------------------- row sizing / overflow / registration
def test_rows_sized_to_peer_share():
    """8 shards, 2^20 keys x 16 values per call: a peer row carries ~1/8 of the keys,
    so the bytes on the wire of a push + pull stay within 1.5 x the live payload."""
    from parameter_server_amd.parallel.comm import LoopbackComm

    G, n, k = 8, 1 << 20, 16
    kv = KVWorker(LoopbackComm(G), "cpu", dim=k, max_keys=n, key_bits=64, capacity=1 << 10)
    assert kv.C < 1.25 * n / G
    push_wire = G * kv.Hp * 4          # push rows: header + keys + values
    pull_wire = G * kv.Hk * 4 + G * kv.C * k * 4  # request rows + value records
    live = n * (kv.kw * 4 + k * 4) + n * (kv.kw * 4) + n * k * 4
    assert push_wire + pull_wire <= 1.5 * live, (push_wire + pull_wire) / live


def test_skewed_keys_overflow_raises():
    """Keys that all mix into owner 0's range overflow its row: the excess is counted
    and the next call fails loudly instead of silently dropping keys."""
    from parameter_server_amd.ops.keymix import unmix
    from parameter_server_amd.parallel.comm import LoopbackComm

    G, n = 4, 4096
    kv = KVWorker(LoopbackComm(G), "cpu", dim=1, max_keys=n, key_bits=64, capacity=1 << 14)
    ok = unmix(torch.arange(100, dtype=torch.int64), 64)  # fits in a row
    kv.wait(kv.push(ok, torch.ones(100)))
    np.testing.assert_allclose(kv.wait(kv.pull(ok)).numpy(), 1.0)
    bad = unmix(torch.arange(n, dtype=torch.int64), 64)   # all owned by shard 0
    assert int(kv.part.owner_of(torch.arange(n, dtype=torch.int64)).max()) == 0
    with pytest.raises(RuntimeError, match="overflow"):  # (wait() checks: CPU pack is done)
        kv.wait(kv.push(bad, torch.ones(n)))
        kv.pull(ok)


def _cross_worker(rank, world, port, out_dir):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from parameter_server_amd.parallel.comm import DistComm

    kv = KVWorker(DistComm("cpu"), "cpu", capacity=1 << 12, max_keys=256)
    X = torch.arange(0, 50, dtype=torch.int64)
    Y = torch.arange(1000, 1040, dtype=torch.int64)
    first, second = (X, Y) if rank == 0 else (Y, X)
    h0 = kv.register_keys(first)
    h1 = kv.register_keys(second)
    hx = kv.register_keys(X)  # rank 0: X is handle 0, rank 1: handle 1 -> must not reuse
    kv.wait(kv.push(hx, torch.full((50,), float(rank + 1))))
    got = kv.wait(kv.pull(X)).numpy()
    torch.save({"ids": (h0.id, h1.id, hx.id), "got": got}, os.path.join(out_dir, f"x{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_crossed_registration_gets_new_handle(tmp_path):
    port = _port()
    mp.spawn(_cross_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    res = [torch.load(tmp_path / f"x{r}.pt", weights_only=False) for r in range(2)]
    assert res[0]["ids"] == res[1]["ids"] == (0, 1, 2)
    for r in res:  # every key got both ranks' pushes: 1 + 2
        np.testing.assert_allclose(r["got"], 3.0)


def _ovf_worker(rank, world, port, out_dir):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from parameter_server_amd.ops.keymix import unmix
    from parameter_server_amd.parallel.comm import DistComm

    n = 2048
    kv = KVWorker(DistComm("cpu"), "cpu", capacity=1 << 14, max_keys=n, key_bits=64)
    # rank 0 overflows its row to owner 0; rank 1 pushes keys that fit
    keys = unmix(torch.arange(n if rank == 0 else 64, dtype=torch.int64), 64)
    kv.push(keys, torch.ones(keys.numel()))
    raised = False
    try:
        kv.flush()
    except RuntimeError as e:
        raised = "overflow" in str(e)
    torch.save({"raised": raised}, os.path.join(out_dir, f"o{rank}.pt"))
    dist.destroy_process_group()


def _ovf_wait_worker(rank, world, port, out_dir):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from parameter_server_amd.ops.keymix import unmix
    from parameter_server_amd.parallel.comm import DistComm

    n = 2048
    kv = KVWorker(DistComm("cpu"), "cpu", capacity=1 << 14, max_keys=n, key_bits=64)
    keys = unmix(torch.arange(n if rank == 0 else 64, dtype=torch.int64), 64)
    waited = True
    try:  # rank 0's push overflows; its wait() must not raise alone
        kv.wait(kv.push(keys, torch.ones(keys.numel())))
        kv.wait(kv.pull(keys[:64]))  # the peers' next collective still completes
    except RuntimeError:
        waited = False
    raised = False
    try:
        kv.barrier()
    except RuntimeError as e:
        raised = "overflow" in str(e)
    torch.save({"waited": waited, "raised": raised}, os.path.join(out_dir, f"w{rank}.pt"))
    dist.destroy_process_group()


def test_gloo_wait_overflow_deferred_to_collective_check(tmp_path):
    """with peer processes wait() defers the overflow check, and the next
    collective check (barrier / flush) raises on EVERY rank."""
    port = _port()
    mp.spawn(_ovf_wait_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    res = [torch.load(tmp_path / f"w{r}.pt", weights_only=False) for r in range(2)]
    assert all(r["waited"] for r in res), res
    assert all(r["raised"] for r in res), res


def test_gloo_flush_overflow_raises_on_every_rank(tmp_path):
    """flush() must not run a rank-local overflow check before its collective
    one, or the overflowing rank raises alone and its peers hang in the host gather."""
    port = _port()
    mp.spawn(_ovf_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    res = [torch.load(tmp_path / f"o{r}.pt", weights_only=False) for r in range(2)]
    assert all(r["raised"] for r in res), res


@pytest.mark.gpu
def test_skewed_keys_overflow_raises_gpu():
    """Device path: the pack kernel counts the dropped keys and publishes the count to
    pinned host memory; flush() (sync) raises."""
    from parameter_server_amd.ops.keymix import unmix
    from parameter_server_amd.parallel.comm import LoopbackComm

    G, n = 4, 4096
    kv = KVWorker(LoopbackComm(G, "cuda"), "cuda", dim=1, max_keys=n, key_bits=64,
                  capacity=1 << 14)
    ok = unmix(torch.arange(100, dtype=torch.int64), 64).cuda()
    kv.wait(kv.push(ok, torch.ones(100, device="cuda")))
    np.testing.assert_allclose(kv.wait(kv.pull(ok)).cpu().numpy(), 1.0)
    kv.flush()
    bad = unmix(torch.arange(n, dtype=torch.int64), 64).cuda()
    with pytest.raises(RuntimeError, match="overflow"):  # at wait() once the pack completed,
        kv.wait(kv.push(bad, torch.ones(n, device="cuda")))  # else at the collective flush
        kv.flush()
