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


@pytest.mark.parametrize("D,S,with_vals", [(16, 39, False), (8, 39, True), (32, 64, True),
                                           (16, 5, True), (48, 39, True)])
def test_fm_kernel_matches_torch(D, S, with_vals):
    """fm_fwd_bwd (lane-per-position kernel for D <= 32, S <= 64; the feature-lane
    kernel otherwise) against the PyTorch forward/backward of the same inputs."""
    from parameter_server_amd.ops.linear import AUC_BINS, accum_total, new_accum
    from parameter_server_amd.ops.native import hipops

    B, U = 1000, 700
    g = torch.Generator().manual_seed(D + S)
    X0 = (torch.randn(B * S, D, generator=g) * 0.3).to(torch.bfloat16)
    vals = torch.rand(B * S, generator=g) + 0.5 if with_vals else None
    lc = torch.randint(0, U, (B * S,), generator=g, dtype=torch.int32)
    w = torch.randn(U, generator=g) * 0.1
    y = torch.where(torch.rand(B, generator=g) < 0.4, 1.0, -1.0)
    ref = FMTrainer(FMConfig(**dict(CFG, embedding_dim=D, slots=S, minibatch=B)))
    dref = ref._fwd_bwd_torch(X0, vals, B, S, lc, w, y)
    coef = torch.empty(B, device="cuda")
    dX0 = torch.empty(B * S, D, dtype=torch.bfloat16, device="cuda")
    met = new_accum("cuda")
    hist = torch.zeros(2 * AUC_BINS, dtype=torch.int32, device="cuda")
    hipops().fm_fwd_bwd(X0.cuda(), None if vals is None else vals.cuda(), B, S, lc.cuda(),
                        w.cuda(), y.cuda(), coef, dX0, met, hist, AUC_BINS)
    torch.testing.assert_close(coef.cpu(), ref.coef[:B], rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(dX0.float().cpu(), dref.float(), rtol=2e-2, atol=1e-3)
    m = accum_total(met).cpu()
    assert abs(float(m[0]) - float(ref.metrics[0])) < 1e-3 * B
    assert float(m[2]) == B
    assert abs(int((hist.cpu() - ref.hist).abs().sum())) <= 4


@pytest.mark.parametrize("D,with_idx,with_vals", [(16, True, False), (8, False, True),
                                                  (32, True, True)])
def test_fm_kernel_gather_matches_expanded(D, with_idx, with_vals):
    """fm_fwd_bwd_gather (rows read through local_col / idx, no expanded X0) against the
    PyTorch forward/backward of the explicitly expanded rows; idx entries of -1 (key
    not resolved) read as zero rows, like emb_expand."""
    from parameter_server_amd.ops.linear import AUC_BINS, accum_total, new_accum
    from parameter_server_amd.ops.native import hipops

    B, S, U, R = 1000, 39, 700, 900
    g = torch.Generator().manual_seed(D + 7)
    rows = (torch.randn(R, D, generator=g) * 0.3).to(torch.bfloat16)
    idx = torch.randint(0, R, (U,), generator=g) if with_idx else None
    if idx is not None:
        idx[::50] = -1
    vals = torch.rand(B * S, generator=g) + 0.5 if with_vals else None
    lc = torch.randint(0, U, (B * S,), generator=g, dtype=torch.int32)
    w = torch.randn(U, generator=g) * 0.1
    y = torch.where(torch.rand(B, generator=g) < 0.4, 1.0, -1.0)
    r = lc.long() if idx is None else idx[lc.long()]
    X0 = torch.where((r >= 0)[:, None], rows[r.clamp(min=0)], torch.zeros((), dtype=rows.dtype))
    ref = FMTrainer(FMConfig(**dict(CFG, embedding_dim=D, slots=S, minibatch=B)))
    dref = ref._fwd_bwd_torch(X0, vals, B, S, lc, w, y)
    coef = torch.empty(B, device="cuda")
    dX0 = torch.empty(B * S, D, dtype=torch.bfloat16, device="cuda")
    met = new_accum("cuda")
    hist = torch.zeros(2 * AUC_BINS, dtype=torch.int32, device="cuda")
    hipops().fm_fwd_bwd_gather(rows.cuda(), None if idx is None else idx.cuda(),
                               None if vals is None else vals.cuda(), B, S, lc.cuda(), w.cuda(),
                               y.cuda(), coef, dX0, met, hist, AUC_BINS)
    torch.testing.assert_close(coef.cpu(), ref.coef[:B], rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(dX0.float().cpu(), dref.float(), rtol=2e-2, atol=1e-3)
    m = accum_total(met).cpu()
    assert abs(float(m[0]) - float(ref.metrics[0])) < 1e-3 * B
    assert float(m[2]) == B
