"""Registered key lists on the KVWorker data plane (key caching, reference
src/filter/key_caching.h:6-76): key-less pushes / request-free pulls against the
owners' cached slots give the same values as the keyed calls, the signature dedupes
registrations, and mixed handle / keyed call sequences keep BSP / SSP semantics
across ranks (gloo) and on the GPU."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from parameter_server_amd.ops.kv_table import UpdateRule
from parameter_server_amd.parameter.sharded_kv import KeyHandle, KVWorker


def test_single_rank_handle_matches_keyed_calls():
    kv = KVWorker(device="cpu", capacity=1 << 12, dim=3, max_keys=64)
    keys = torch.tensor([5, 1, 5, -(1 << 63) + 7, 42], dtype=torch.int64)
    h = kv.register_keys(keys)
    assert isinstance(h, KeyHandle) and h.n == 5
    assert kv.register_keys(keys.clone()) is h          # same signature -> same handle
    assert kv.register_keys(keys.flip(0)) is not h      # order matters (position-dependent)
    v = torch.arange(15, dtype=torch.float32).reshape(5, 3)
    kv.wait(kv.push(h, v))
    got_h = kv.wait(kv.pull(h))
    got_k = kv.wait(kv.pull(keys))
    assert torch.equal(got_h, got_k)
    assert got_h[0].tolist() == (v[0] + v[2]).tolist()  # duplicates summed
    kv.release(h)
    with pytest.raises(ValueError):
        kv.pull(h)


def test_single_rank_handle_optimizer_rule():
    rule = UpdateRule("sgd", "constant", alpha=0.5)
    kv = KVWorker(device="cpu", rule=rule, max_keys=16)
    h = kv.register_keys(torch.tensor([9, 3]))
    kv.wait(kv.push(h, torch.tensor([2.0, -4.0])))
    assert kv.wait(kv.pull(h)).tolist() == [-1.0, 2.0]
    kv.wait(kv.push(torch.tensor([3]), torch.tensor([2.0])))  # keyed push, same slot
    assert kv.wait(kv.pull(h)).tolist() == [-1.0, 1.0]


# ------------------------------------------------------------------ multi-rank
NK = 300
# (op, which): "hpush"/"hpull" use the rank's registered list, "push"/"pull" plain keys
OPS = ["hpush", "hpull", "push", "hpush", "pull", "hpush", "hpull", "push", "hpull", "pull"]


def _hkeys(rank):
    rng = np.random.default_rng(77 + rank)
    return rng.integers(0, NK, 90 + 20 * rank)  # duplicates included


def _batch(rank, i, dim, n=None):
    rng = np.random.default_rng(1000 * rank + i)
    if n is None:
        n = int(rng.integers(0, 120))
        keys = rng.integers(0, NK, n)
    else:
        keys = _hkeys(rank)
    return keys, rng.normal(0, 1, (len(keys), dim)).astype(np.float32)


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
                  consistency=consistency, key_bits=32 if dim > 1 else 64)
    hk = torch.from_numpy(_hkeys(rank)).to(dev)
    h = kv.register_keys(hk)
    assert kv.register_keys(hk) is h
    allk = torch.arange(NK, dtype=torch.int64, device=dev)
    outs = []
    for i, op in enumerate(OPS):
        if op in ("push", "hpush"):
            keys, vals = _batch(rank, i, dim, n=0 if op == "hpush" else None)
            v = torch.from_numpy(vals).to(dev)
            kv.push(h if op == "hpush" else torch.from_numpy(keys).to(dev), v)
        else:
            outs.append((op, kv.pull(h if op == "hpull" else allk)))
    res = [(op, kv.wait(t).cpu().numpy()) for op, t in outs]
    kv.barrier()
    torch.save({"pulls": res}, os.path.join(out_dir, f"kc{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def _simulate(world, tau, dim, rank):
    table = np.zeros((NK, dim))
    pushes, out, applied = [], [], 0
    for i, op in enumerate(OPS):
        if op in ("push", "hpush"):
            d = np.zeros((NK, dim))
            for r in range(world):
                keys, vals = _batch(r, i, dim, n=0 if op == "hpush" else None)
                np.add.at(d, keys, vals)
            pushes.append(d)
        else:
            while applied < len(pushes) - tau:
                table += pushes[applied]
                applied += 1
            out.append(table[_hkeys(rank)].copy() if op == "hpull" else table.copy())
    return out


def _run(tmp_path, world, consistency, dim, device="cpu"):
    port = _port()
    mp.spawn(_worker, args=(world, port, str(tmp_path), consistency, dim, device), nprocs=world,
             join=True)
    return [torch.load(tmp_path / f"kc{r}.pt", weights_only=False) for r in range(world)]


def _check(res, world, tau, dim, tol):
    for rank, r in enumerate(res):
        exp = _simulate(world, tau, dim, rank)
        assert len(r["pulls"]) == len(exp)
        for (op, got), e in zip(r["pulls"], exp):
            np.testing.assert_allclose(got.reshape(e.shape[0], -1), e.reshape(e.shape[0], -1),
                                       rtol=tol, atol=tol, err_msg=op)


@pytest.mark.parametrize("world,consistency,dim", [(2, "bsp", 4), (3, "bsp", 1),
                                                   (2, "ssp:2", 1), (3, "ssp:1", 4)])
def test_gloo_handles_mixed_with_keyed_calls(tmp_path, world, consistency, dim):
    tau = 0 if consistency == "bsp" else int(consistency.split(":")[1])
    _check(_run(tmp_path, world, consistency, dim), world, tau, dim, 1e-5)


# ------------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("dim,bits", [(1, 64), (8, 32)])
def test_kvworker_gpu_handle_single_rank(dim, bits):
    kv = KVWorker(device="cuda", capacity=1 << 14, dim=dim, key_bits=bits, max_keys=8192)
    keys = torch.randint(0, 1 << 30, (5000,), device="cuda")
    keys[::7] = keys[0]
    h = kv.register_keys(keys)
    assert kv.register_keys(keys.clone()) is h
    vals = torch.randn(5000, dim, device="cuda")
    kv.wait(kv.push(h, vals))
    kv.wait(kv.push(keys, vals))  # keyed push onto the same slots
    got = kv.wait(kv.pull(h))
    uk, inv = torch.unique(keys, return_inverse=True)
    exp = 2 * torch.zeros(uk.numel(), dim, device="cuda").index_add_(0, inv, vals)[inv]
    torch.testing.assert_close(got.reshape(-1, dim), exp, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(kv.wait(kv.pull(keys)), got)


@pytest.mark.gpu
def test_kvworker_gpu_handle_optimizer_rule_ssp():
    rule = UpdateRule("sgd", "constant", alpha=0.5)
    kv = KVWorker(device="cuda", rule=rule, max_keys=1024, consistency="ssp:1")
    h = kv.register_keys(torch.tensor([123456789, 5], device="cuda"))
    seen = []
    for i in range(1, 5):
        kv.push(h, torch.tensor([float(i), 1.0], device="cuda"))
        seen.append(kv.wait(kv.pull(h)).tolist())
    assert [s[0] for s in seen] == [0.0, -0.5, -1.5, -3.0]
    assert [s[1] for s in seen] == [0.0, -0.5, -1.0, -1.5]


@pytest.mark.gpu
def test_kvworker_gpu_handles_two_rank_rehearsal(tmp_path):
    """Two ranks on the one GPU over gloo: device register / key-less pack / cached serve
    and apply at G = 2."""
    _check(_run(tmp_path, 2, "ssp:1", 4, device="cuda"), 2, 1, 4, 1e-4)
