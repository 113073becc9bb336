"""Resume snapshots of the embedding models (EmbeddingPS.state_dict / load_state_dict):
a run restored from a safetensors snapshot continues exactly like the uninterrupted
run, and a snapshot taken by 2 ranks (key-disjoint shards) merges and reloads into 1."""
import pytest
import torch

from parameter_server_amd.models.fm import FMConfig, FMTrainer
from parameter_server_amd.models.wide_deep import WideDeepConfig, WideDeepTrainer
from parameter_server_amd.ops.synthetic import criteo_batch
from parameter_server_amd.utils.checkpoint import load_snapshot, save_snapshot

NF = 1 << 20
FM_CFG = dict(num_features=NF, embedding_dim=8, minibatch=128, table_capacity=1 << 15,
              emb_lr=0.05, lambda_v=0.1)
WD_CFG = dict(num_features=NF, embedding_dim=8, minibatch=64, hidden=[32, 16],
              table_capacity=1 << 15)


def _batch(B, s, dev="cpu"):
    return criteo_batch(B, seed=9, row0=s * B, num_features=NF, cards=[300] * 26, device=dev)


def _table(tr):
    sd = tr.state_dict()
    o = torch.argsort(sd["keys"])
    return {k: sd[k][o] for k in ("keys", "w", "z", "n", "rows", "acc")}, sd


@pytest.mark.parametrize("kind,dev", [("fm", "cpu"), ("wd", "cpu"),
                                      pytest.param("fm", "cuda", marks=pytest.mark.gpu),
                                      pytest.param("wd", "cuda", marks=pytest.mark.gpu)])
def test_resume_matches_uninterrupted(kind, dev, tmp_path):
    make = ((lambda: FMTrainer(FMConfig(**FM_CFG), device=dev)) if kind == "fm"
            else (lambda: WideDeepTrainer(WideDeepConfig(**WD_CFG), device=dev)))
    B = (FM_CFG if kind == "fm" else WD_CFG)["minibatch"]
    a = make()
    for s in range(3):
        a.step(*_batch(B, s, dev))
    path = str(tmp_path / "snap.safetensors")
    save_snapshot(path, a.state_dict())
    b = make()
    b.load_state_dict(load_snapshot(path))
    assert b.step_count == a.step_count == 3
    for s in range(3, 5):
        a.step(*_batch(B, s, dev))
        b.step(*_batch(B, s, dev))
    ta, sa = _table(a)
    tb, sb = _table(b)
    assert torch.equal(ta["keys"], tb["keys"])
    for k in ("w", "z", "n", "acc"):
        torch.testing.assert_close(ta[k], tb[k], rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(ta["rows"].float(), tb["rows"].float(), rtol=1e-2, atol=1e-3)
    if kind == "wd":
        torch.testing.assert_close(sa["param"], sb["param"], rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(sa["v"], sb["v"], rtol=1e-5, atol=1e-8)


def test_two_rank_snapshot_reloads_into_one():
    """Split one rank's state into 2 key-disjoint halves (what 2 shards save), merge,
    reload: the restored shard holds exactly the same keys and values."""
    a = FMTrainer(FMConfig(**FM_CFG))
    for s in range(2):
        a.step(*_batch(128, s))
    sd = a.state_dict()
    half = torch.arange(sd["keys"].numel()) % 2 == 0
    parts = [{**sd, **{k: sd[k][m] for k in ("keys", "w", "z", "n", "rows", "acc")}}
             for m in (half, ~half)]
    b = FMTrainer(FMConfig(**FM_CFG))
    b.load_state_dict(FMTrainer.merge_state_dicts(parts))
    ta, _ = _table(a)
    tb, _ = _table(b)
    assert torch.equal(ta["keys"], tb["keys"])
    assert torch.equal(ta["rows"], tb["rows"]) and torch.equal(ta["w"], tb["w"])
    with pytest.raises(ValueError):
        WideDeepTrainer(WideDeepConfig(**dict(WD_CFG, embedding_dim=16))).load_state_dict(sd)


def _reload_worker(rank, world, port, snap, out_dir):
    import os

    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from parameter_server_amd.parallel.comm import init_from_env

    comm, dev = init_from_env("cpu")
    tr = FMTrainer(FMConfig(**FM_CFG), comm, dev)
    tr.load_state_dict(load_snapshot(snap), chunk=97)  # several host chunks
    torch.save(tr.state_dict(), os.path.join(out_dir, f"s{rank}.pt"))
    dist.destroy_process_group()


def test_one_rank_snapshot_reloads_into_two_ranks(tmp_path):
    """A 1-rank snapshot loaded by 2 gloo ranks: the shards are key-disjoint, together
    hold every key, and carry the saved values (ownership decided on the host)."""
    import socket

    import torch.multiprocessing as mp

    a = FMTrainer(FMConfig(**FM_CFG))
    for s in range(2):
        a.step(*_batch(128, s))
    snap = str(tmp_path / "one.safetensors")
    save_snapshot(snap, a.state_dict())
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.spawn(_reload_worker, args=(2, port, snap, str(tmp_path)), nprocs=2, join=True)
    shards = [torch.load(tmp_path / f"s{r}.pt", weights_only=True) for r in range(2)]
    k0, k1 = set(shards[0]["keys"].tolist()), set(shards[1]["keys"].tolist())
    assert k0 and k1 and not (k0 & k1)
    ta, _ = _table(a)
    assert k0 | k1 == set(ta["keys"].tolist())
    merged = FMTrainer.merge_state_dicts(shards)
    o = torch.argsort(merged["keys"])
    for k in ("w", "z", "n", "rows", "acc", "cnt"):
        assert torch.equal(merged[k][o], a.state_dict()[k][torch.argsort(a.state_dict()["keys"])]), k


def test_snapshot_refuses_other_model():
    a = FMTrainer(FMConfig(**FM_CFG))
    a.step(*_batch(128, 0))
    sd = a.state_dict()
    wd = WideDeepTrainer(WideDeepConfig(**dict(WD_CFG, embedding_dim=FM_CFG["embedding_dim"])))
    with pytest.raises(ValueError, match="FMTrainer"):
        wd.load_state_dict(sd)
