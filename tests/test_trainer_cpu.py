import os

import torch

from parameter_server_amd.models import SparseLRConfig, SparseLRTrainer
from parameter_server_amd.ops.synthetic import criteo_batch
from parameter_server_amd.utils.checkpoint import load_snapshot, read_text_models, save_snapshot


def _train(cfg, steps=15, B=256, seed=1):
    tr = SparseLRTrainer(cfg)
    for s in range(steps):
        k, l = criteo_batch(B, seed=seed, row0=s * B, num_features=cfg.num_features,
                            cards=[300] * 26)
        tr.step(k, l)
    return tr


def test_loss_decreases_cpu():
    cfg = SparseLRConfig(num_features=10 ** 6, minibatch=256, table_capacity=1 << 15, l1=1.0)
    tr = SparseLRTrainer(cfg)
    losses = []
    for s in range(30):
        k, l = criteo_batch(256, seed=2, row0=s * 256, num_features=10 ** 6, cards=[300] * 26)
        tr.step(k, l)
        if s % 10 == 9:
            losses.append(tr.progress()["loss"])
    assert losses[-1] < losses[0]


def test_tail_filter_drops_rare_keys():
    cfg = SparseLRConfig(num_features=10 ** 6, minibatch=256, table_capacity=1 << 15,
                         tail_feature_freq=2, countmin_n=1 << 16)
    tr = _train(cfg, steps=5)
    cfg0 = SparseLRConfig(num_features=10 ** 6, minibatch=256, table_capacity=1 << 15)
    tr0 = _train(cfg0, steps=5)
    assert tr.table.census()[0] < tr0.table.census()[0]


def test_text_checkpoint_layout(tmp_path):
    cfg = SparseLRConfig(num_features=10 ** 6, minibatch=256, table_capacity=1 << 15, l1=0.1)
    tr = _train(cfg)
    path = tr.save_model(str(tmp_path / "model" / "ctr_online"))
    assert path.endswith("ctr_online_S0") and os.path.exists(path)
    lines = open(path).read().strip().split("\n")
    k, v = lines[0].split("\t")
    assert int(k) < 10 ** 6 and float(v) != 0
    m = read_text_models(str(tmp_path / "model" / "ctr_online.*"))
    sd = tr.state_dict()
    nz = {kk: ww for kk, ww in zip(sd["keys"].tolist(), sd["w"].tolist()) if ww != 0}
    assert set(m) == set(nz)
    assert all(abs(m[kk] - nz[kk]) < 1e-6 for kk in m)


def test_snapshot_resume_equivalence(tmp_path):
    cfg = SparseLRConfig(num_features=10 ** 6, minibatch=256, table_capacity=1 << 15, l1=0.1)
    a = _train(cfg, steps=10)
    save_snapshot(str(tmp_path / "snap.safetensors"), a.state_dict())
    b = SparseLRTrainer(cfg)
    b.load_state_dict(load_snapshot(str(tmp_path / "snap.safetensors")))
    assert b.step_count == 10
    for tr in (a, b):
        for s in range(10, 13):
            k, l = criteo_batch(256, seed=1, row0=s * 256, num_features=10 ** 6, cards=[300] * 26)
            tr.step(k, l)
    sa, sb = a.state_dict(), b.state_dict()
    da = dict(zip(sa["keys"].tolist(), sa["w"].tolist()))
    db = dict(zip(sb["keys"].tolist(), sb["w"].tolist()))
    assert da.keys() == db.keys()
    assert max(abs(da[k] - db[k]) for k in da) < 1e-6


def test_aggregate_push_mode_cpu():
    cfg = SparseLRConfig(num_features=10 ** 6, minibatch=128, table_capacity=1 << 15,
                         push_mode="aggregate")
    tr = _train(cfg, steps=3, B=128)
    assert tr.table.census()[0] > 0


def test_p2p_exchange_is_asp_gpu_only():
    """exchange='p2p' (one-sided peer-HBM data plane) is the asynchronous GPU mode: a
    CPU run or a synchronous consistency is refused up front."""
    import pytest

    from parameter_server_amd.models import SparseLRConfig, SparseLRTrainer
    from parameter_server_amd.parallel.comm import LoopbackComm

    for cons in ("asp", "bsp"):
        cfg = SparseLRConfig(num_features=1 << 20, minibatch=64, table_capacity=1 << 12,
                             consistency=cons, exchange="p2p")
        with pytest.raises(ValueError, match="p2p"):
            SparseLRTrainer(cfg, LoopbackComm(2), "cpu")
