"""FM HIP kernels (fm.hip) vs the PyTorch step on the same data, and a GPU run
that learns."""
import pytest
import torch

from parameter_server_amd.models.fm import FMConfig, FMTrainer
from parameter_server_amd.ops.synthetic import criteo_batch

pytestmark = pytest.mark.gpu
CFG = dict(num_features=1 << 20, embedding_dim=16, minibatch=512, table_capacity=1 << 16,
           emb_lr=0.05, lambda_v=0.5)


def test_fm_gpu_matches_cpu():
    cpu = FMTrainer(FMConfig(**CFG))
    gpu = FMTrainer(FMConfig(**CFG), device="cuda")
    for s in range(3):
        k, l = criteo_batch(512, seed=2, row0=s * 512, num_features=CFG["num_features"],
                            cards=[300] * 26)
        cpu.step(k, l)
        gpu.step(k.cuda(), l.cuda())
    torch.cuda.synchronize()
    pc, pg = cpu.progress(), gpu.progress()
    assert abs(pc["loss"] - pg["loss"]) < 2e-3, (pc, pg)
    kc, wc, _, _ = cpu.shard.table.occupied()
    kg, wg, _, _ = gpu.shard.table.occupied()
    oc, og = torch.argsort(kc), torch.argsort(kg.cpu())
    assert torch.equal(kc[oc], kg.cpu()[og])
    assert torch.allclose(wc[oc], wg.cpu()[og], atol=2e-3)


def test_fm_gpu_vals_and_learning():
    tr = FMTrainer(FMConfig(**CFG), device="cuda")
    losses = []
    for s in range(30):
        k, l = criteo_batch(512, seed=4, row0=s * 512, num_features=CFG["num_features"],
                            cards=[300] * 26, device="cuda")
        tr.step(k, l, vals=torch.ones(k.numel(), device="cuda"))
        if s % 10 == 9:
            losses.append(tr.progress()["loss"])
    assert losses[-1] < losses[0]
