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


def _gpu_worker(rank, world, port, out_dir, cfg_kw, steps):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), PSAMD_DIST_BACKEND="gloo")
    import torch.distributed as dist

    from parameter_server_amd.models import SparseLRConfig, SparseLRTrainer
    from parameter_server_amd.ops.synthetic import criteo_batch
    from parameter_server_amd.parallel.comm import init_from_env

    comm, dev = init_from_env("cuda")
    cfg = SparseLRConfig(**cfg_kw)
    tr = SparseLRTrainer(cfg, comm, dev)
    B = cfg.minibatch
    for s in range(steps):
        k, l = criteo_batch(B, seed=100 + rank, row0=s * B, num_features=cfg.num_features,
                            cards=[200] * 26)
        tr.step(k.to(dev), l.to(dev))
    torch.cuda.synchronize()
    p = tr.progress()
    tr.table.check_ok()
    torch.save({"progress": p, "state": tr.state_dict()}, os.path.join(out_dir, f"g{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("ff_bytes", [0, 3])
def test_two_rank_gpu_protocol_matches_reference(tmp_path, ff_bytes):
    cfg_kw = dict(num_features=1 << 20, minibatch=128, table_capacity=1 << 15, l1=0.5,
                  fixing_float_bytes=ff_bytes)
    port = _free_port()
    mp.spawn(_gpu_worker, args=(2, port, str(tmp_path), cfg_kw, 4), nprocs=2, join=True)
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
