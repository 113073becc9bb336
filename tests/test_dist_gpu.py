"""Multi-rank GPU protocol rehearsal on a single GPU: 2 ranks share cuda:0 and
exchange through gloo (host-staged). Exercises the exact multi-GPU code path of the
trainer (owner split, count exchange, all-to-all-v pull/push, per-source updates)
with the HIP kernels, and checks it against the single-process protocol reference."""
import os
import sys

sys.path.insert(0, os.path.dirname(__file__))

import pytest
import torch
import torch.multiprocessing as mp

from test_dist_gloo import _free_port, _reference

pytestmark = pytest.mark.gpu


def _gpu_worker(rank, world, port, out_dir, cfg_kw, steps, pipelined=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), PSAMD_DIST_BACKEND="gloo")
    import torch.distributed as dist

    from parameter_server_amd.models import SparseLRConfig, SparseLRTrainer
    from parameter_server_amd.ops.synthetic import criteo_batch
    from parameter_server_amd.parallel.comm import init_from_env

    comm, dev = init_from_env("cuda")
    cfg = SparseLRConfig(**cfg_kw)
    tr = SparseLRTrainer(cfg, comm, dev)
    assert tr.localize_mode == cfg.localize or cfg.localize == "auto", tr.localize_mode
    B = cfg.minibatch
    batches = [criteo_batch(B, seed=100 + rank, row0=s * B, num_features=cfg.num_features,
                            cards=[200] * 26) for s in range(steps)]
    batches = [(k.to(dev), l.to(dev)) for k, l in batches]
    if not pipelined:
        for k, l in batches:
            tr.step(k, l)
    elif pipelined == "buf0":  # every minibatch localised into the default workspace
        for k, l in batches:
            tr.step(k, l, loc=tr.localize(k))
    else:  # bench.py's multi-GPU loop: localise t+1 on a side stream during step t
        side = torch.cuda.Stream(dev)

        def produce(t):
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                return tr.localize(batches[t][0], buf=t % 2)

        loc = produce(0)
        for t in range(steps):
            torch.cuda.current_stream(dev).wait_stream(side)
            nxt = {}
            pf = (lambda t=t: nxt.setdefault("loc", produce(t + 1))) if t + 1 < steps else None
            tr.step(batches[t][0], batches[t][1], loc=loc, prefetch=pf)
            loc = nxt.get("loc")
    torch.cuda.synchronize()
    p = tr.progress()
    tr.table.check_ok()
    torch.save({"progress": p, "state": tr.state_dict()}, os.path.join(out_dir, f"g{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("ff_bytes,pipelined,exchange,localize",
                         [(0, False, "padded", "sort"), (0, False, "exact", "sort"),
                          (3, False, "padded", "sort"), (3, False, "exact", "sort"),
                          (0, True, "padded", "sort"),
                          (0, True, "exact", "sort"), (0, False, "padded", "tp"),
                          (0, False, "padded", "tpf"), (3, False, "padded", "tpf"),
                          (0, True, "padded", "tpf")])
def test_two_rank_gpu_protocol_matches_reference(tmp_path, ff_bytes, pipelined, exchange,
                                                 localize):
    cfg_kw = dict(num_features=1 << 20, minibatch=128, table_capacity=1 << 15, l1=0.5,
                  fixing_float_bytes=ff_bytes, exchange=exchange, localize=localize)
    port = _free_port()
    mp.spawn(_gpu_worker, args=(2, port, str(tmp_path), cfg_kw, 4, pipelined), nprocs=2,
             join=True)
    res = [torch.load(tmp_path / f"g{r}.pt", weights_only=False) for r in range(2)]
    merged = {}
    for r in res:
        for k, w in zip(r["state"]["keys"].tolist(), r["state"]["w"].tolist()):
            assert k not in merged
            merged[k] = w
    ref = _reference(cfg_kw, 4, 2)
    assert merged.keys() == ref.keys()
    tol = 1e-5 if ff_bytes == 0 else 2e-3
    assert max(abs(merged[k] - ref[k]) for k in ref) < tol


@pytest.mark.parametrize("pattern", ["side", "buf0"])
@pytest.mark.parametrize("localize", ["tpf", "tp"])
def test_merged_exchange_caller_localisations(tmp_path, pattern, localize):
    """ssp:2 runs the merged one-collective exchange, whose sequential API trains the
    PREVIOUS minibatch on each step() call. Caller-supplied localisations (the
    prefetch-on-a-side-stream pattern over 2 workspaces, and every minibatch in the
    default workspace) must not corrupt the pending minibatch: same weights as the
    stale-pull protocol reference at lag 2."""
    cfg_kw = dict(num_features=1 << 20, minibatch=128, table_capacity=1 << 15, l1=0.5,
                  consistency="ssp:2", localize=localize)
    port = _free_port()
    mp.spawn(_gpu_worker, args=(2, port, str(tmp_path), cfg_kw, 6, pattern), nprocs=2,
             join=True)
    res = [torch.load(tmp_path / f"g{r}.pt", weights_only=False) for r in range(2)]
    merged = {}
    for r in res:
        for k, w in zip(r["state"]["keys"].tolist(), r["state"]["w"].tolist()):
            merged[k] = w
    ref = _reference(cfg_kw, 6, 2, lag=2)
    assert merged.keys() == ref.keys()
    assert max(abs(merged[k] - ref[k]) for k in ref) < 1e-5


@pytest.mark.parametrize("exchange,consistency,world", [
    ("padded", "ssp:4", 2), ("exact", "ssp:4", 2), ("padded", "ssp:1", 2), ("padded", "asp", 2),
    ("padded", "ssp:4", 4)])
def test_bench_two_rank_rehearsal_json(tmp_path, exchange, consistency, world):
    """bench.py's multi-GPU path (padded: graph-replayed compute segments around the
    exchanges, post / tail owner applies, ssp:4 the merged one-collective exchange;
    exact: pipelined count-sized exchange) under torchrun, 2 (or 4) ranks on one GPU
    over gloo (every rank must issue its collectives in the same order, or the run
    hangs); checks the one-line JSON contract."""
    import json
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PSAMD_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", "bench.py", "--gpus",
           str(world), "--steps", "4", "--warmup", "2", "--minibatch", "4096", "--num-features",
           "1e8", "--exchange", exchange, "--consistency", consistency]
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == world and out["steps"] == 4
    assert out["config"]["global_batch"] == 4096 * world
    if exchange == "padded" and consistency == "ssp:4":  # exchange_merge "auto": one collective
        assert out["config"]["ssp_apply"] == "merged"
        assert out["config"]["collectives_per_step"] == 1
    assert out["value"] > 0 and 0.3 < out["train"]["loss"] < 1.0
    assert out["config"]["hip_graph"] == (exchange == "padded")


@pytest.mark.parametrize("exchange,ff", [("padded", 0), ("padded", 3), ("exact", 0)])
def test_two_rank_gpu_aggregate_push_matches_reference(tmp_path, exchange, ff):
    """push_mode="aggregate": one launch accumulates every source row into the slots,
    one launch applies the summed gradient (KVBufferedVector semantics)."""
    from test_dist_gloo import _reference_aggregate

    cfg_kw = dict(num_features=1 << 20, minibatch=128, table_capacity=1 << 15, l1=0.5,
                  push_mode="aggregate", exchange=exchange, fixing_float_bytes=ff)
    port = _free_port()
    mp.spawn(_gpu_worker, args=(2, port, str(tmp_path), cfg_kw, 4, False), nprocs=2, join=True)
    res = [torch.load(tmp_path / f"g{r}.pt", weights_only=False) for r in range(2)]
    merged = {}
    for r in res:
        for k, w in zip(r["state"]["keys"].tolist(), r["state"]["w"].tolist()):
            merged[k] = w
    ref = _reference_aggregate(cfg_kw, 4, 2)
    assert merged.keys() == ref.keys()
    tol = 1e-5 if ff == 0 else 2e-3
    assert max(abs(merged[k] - ref[k]) for k in ref) < tol
