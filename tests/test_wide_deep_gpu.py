"""Embedding / wide & deep HIP kernels (csrc/hip/embedding.hip) vs the PyTorch
reference, and the GPU trainer vs the CPU trainer."""
import numpy as np
import pytest
import torch

from parameter_server_amd.models.wide_deep import WideDeepConfig, WideDeepTrainer
from parameter_server_amd.ops import embedding as E
from parameter_server_amd.ops.localize import Localizer, localize_torch
from parameter_server_amd.ops.synthetic import criteo_batch

pytestmark = pytest.mark.gpu


def test_shard_init_gather_update_match_cpu():
    D, cap = 128, 1 << 12
    keys = torch.randint(0, 1 << 40, (3000,), dtype=torch.int64).unique()
    sc, sg = E.EmbeddingShard(cap, D, "cpu", seed=3), E.EmbeddingShard(cap, D, "cuda", seed=3)
    slc, _ = sc.resolve(keys)
    slg, _ = sg.resolve(keys.cuda())  # concurrent inserts may place keys differently
    assert slg.unique().numel() == keys.numel()
    rc, rg = sc.gather_rows(slc), sg.gather_rows(slg)  # rows in request-key order
    # identical counter-based init stream (fp32 transcendental ulps may move a bf16 rounding)
    torch.testing.assert_close(rg.cpu().float(), rc.float(), rtol=1e-2, atol=1e-4)
    assert rc.float().std().item() == pytest.approx(0.01, rel=0.1)
    sg.rows[slg] = rc.cuda()  # identical starting rows per key
    g = torch.randn(keys.numel(), D)
    sc.update_rows(slc, grad=g, lr=0.1)
    sg.update_rows(slg, grad=g.cuda(), lr=0.1)
    torch.testing.assert_close(sg.gather_rows(slg).cpu().float(), sc.gather_rows(slc).float(),
                               rtol=1e-2, atol=1e-3)
    torch.testing.assert_close(sg.acc[slg].cpu(), sc.acc[slc], rtol=1e-5, atol=1e-7)
    sg.update_rows(slg, grad16=g.cuda().to(torch.bfloat16), lr=0.1)  # bf16 push path runs


def test_expand_and_grad_reduce():
    B, S, D = 777, 39, 128
    keys, _ = criteo_batch(B, seed=1, row0=0, num_features=1 << 20, cards=[50] * 26)
    kg = keys.cuda()
    loc = Localizer(B * S, 20, "cuda")(kg)
    U = loc.num_unique()
    src = torch.randn(U, D, device="cuda").to(torch.bfloat16)
    X0 = E.expand(loc.local_col, B * S, src)
    assert torch.equal(X0, src[loc.local_col.long()])
    dX0 = torch.randn(B * S, D, device="cuda").to(torch.bfloat16)
    dE = E.grad_reduce(loc, dX0, D, B * S)
    ref = torch.zeros(U, D, device="cuda").index_add_(0, loc.local_col.long(), dX0.float())
    torch.testing.assert_close(dE[:U], ref, rtol=1e-5, atol=1e-4)
    lc = localize_torch(keys, 20)
    torch.testing.assert_close(E.grad_reduce(lc, dX0.cpu(), D, U).sum(), ref.sum().cpu(),
                               rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("D,n,hot", [(128, 64 * 300, 0), (128, 100003, 40000), (256, 5000, 4999),
                                     (128, 65, 64), (256, 1, 0), (64, 7777, 3000),
                                     (16, 100003, 40000), (8, 4097, 100), (32, 640, 639),
                                     (24, 3000, 500)])
def test_grad_reduce_segments_cross_runs(D, n, hot):
    """Segmented wavefront reduction (64-entry runs): segments inside a run, crossing
    one boundary, spanning hundreds of runs, ending exactly at a run end, ragged tail."""
    g = torch.Generator().manual_seed(n + D)
    k = torch.randint(0, 1 << 20, (n,), generator=g, dtype=torch.int64)
    if hot:
        k[torch.randperm(n, generator=g)[:hot]] = 4242
    loc = Localizer(n, 20, "cuda")(k.cuda())
    U = loc.num_unique()
    dX0 = torch.randn(n, D, generator=g).to(torch.bfloat16)
    ref = torch.zeros(U, D, dtype=torch.float64).index_add_(0, loc.local_col.long().cpu(),
                                                            dX0.double())
    dE = E.grad_reduce(loc, dX0.cuda(), D, n)
    torch.testing.assert_close(dE[:U].double().cpu(), ref, rtol=1e-4, atol=1e-3)
    again = E.grad_reduce(loc, dX0.cuda(), D, n)
    assert torch.equal(again[:U], dE[:U]) or D == 24  # deterministic (no atomics)


@pytest.mark.parametrize("D,B,S,hot", [(128, 3000, 39, 0), (128, 4000, 39, 60000), (256, 777, 13, 5000),
                                       (128, 2, 39, 0), (128, 1, 1, 0)])
def test_grad_reduce_fused_wide_gradient(D, B, S, hot):
    """The wide gradient riding along the segmented reduction: g_wide[u] = sum of
    coef[row] over u's occurrences (row = position // S), against an fp64 index_add;
    dE unchanged by it; deterministic."""
    n = B * S
    g = torch.Generator().manual_seed(n + D)
    k = torch.randint(0, 1 << 20, (n,), generator=g, dtype=torch.int64)
    if hot:
        k[torch.randperm(n, generator=g)[:min(hot, n)]] = 4242
    loc = Localizer(n, 20, "cuda")(k.cuda())
    U = loc.num_unique()
    dX0 = torch.randn(n, D, generator=g).to(torch.bfloat16)
    coef = torch.randn(B, generator=g)
    col = loc.local_col.long().cpu()
    ref = torch.zeros(U, dtype=torch.float64).index_add_(
        0, col, coef.double().repeat_interleave(S))
    gw = torch.full((n,), float("nan"), device="cuda")
    assert E.grad_wide_fused(D, True)
    dE = E.grad_reduce(loc, dX0.cuda(), D, n, coef=coef.cuda(), width=S, g_wide=gw)
    torch.testing.assert_close(gw[:U].double().cpu(), ref, rtol=1e-5, atol=1e-4)
    plain = E.grad_reduce(loc, dX0.cuda(), D, n)
    assert torch.equal(plain[:U], dE[:U])
    gw2 = torch.zeros_like(gw)
    E.grad_reduce(loc, dX0.cuda(), D, n, coef=coef.cuda(), width=S, g_wide=gw2)
    assert torch.equal(gw2[:U], gw[:U])


@pytest.mark.parametrize("algo", ["ftrl", "adagrad", "sgd"])
def test_fused_row_and_wide_update_is_the_two_pass_update(algo):
    """emb_update with the wide slots (one pass) = emb_update then kv_update: rows,
    AdaGrad accumulators and slots bitwise, stats to fp64 rounding; NaN-marked wide
    gradients skip only the slot."""
    from parameter_server_amd.ops.kv_table import UpdateRule
    from parameter_server_amd.ops.native import hipops

    H = hipops()
    D, cap, n = 128, 1 << 14, 5000
    g = torch.Generator().manual_seed(7)
    keys = torch.randperm(1 << 30, generator=g)[:n].to(torch.int64)
    dE = torch.randn(n, D, generator=g).cuda()
    gw = torch.randn(n, generator=g).cuda()
    gw[::97] = float("nan")
    sh = E.EmbeddingShard(cap, D, "cuda", seed=3)
    slot, _ = sh.resolve(keys.cuda())  # (one placement for both variants)
    sh.table.slots.view(torch.float32).view(-1, 8)[:, 2:6] = 0.25  # (w, z, n, acc)
    start = (sh.rows.clone(), sh.acc.clone(), sh.table.slots.clone())
    runs = []
    for fused in (False, True):
        sh.rows.copy_(start[0])
        sh.acc.copy_(start[1])
        sh.table.slots.copy_(start[2])
        rule = UpdateRule(algo=algo, alpha=0.05, beta=1.0, l1=0.01, l2=0.1)
        stats = torch.zeros(8, dtype=torch.float64, device="cuda")
        nd = torch.tensor([n - 3], dtype=torch.int32, device="cuda")
        if fused:
            H.emb_update(slot, nd, dE, None, sh.rows, sh.acc, 0.05, 1e-8, sh.table.slots, gw,
                         list(rule.args()), stats)
        else:
            H.emb_update(slot, nd, dE, None, sh.rows, sh.acc, 0.05, 1e-8)
            H.kv_update(sh.table.slots, slot, gw, nd, *rule.args(), stats)
        torch.cuda.synchronize()
        runs.append((sh.rows.clone(), sh.acc.clone(), sh.table.slots.clone(), stats.clone()))
    (r0, a0, s0, st0), (r1, a1, s1, st1) = runs
    assert torch.equal(r0, r1) and torch.equal(a0, a1) and torch.equal(s0, s1)
    torch.testing.assert_close(st1[:3], st0[:3], rtol=1e-9, atol=1e-9)


def test_head_colsum_adam_match_cpu():
    B, H, S = 1000, 256, 39
    torch.manual_seed(0)
    h = torch.relu(torch.randn(B, H)).to(torch.bfloat16)
    w, b = torch.randn(H) * 0.1, torch.tensor([0.2])
    U = 500
    wide = torch.randn(U) * 0.1
    lc = torch.randint(0, U, (B * S,), dtype=torch.int32)
    y = torch.where(torch.rand(B) < 0.4, 1.0, -1.0)
    outs = {}
    for dev in ("cpu", "cuda"):
        coef = torch.zeros(B, device=dev)
        dh = torch.empty(B, H, dtype=torch.bfloat16, device=dev)
        dw, db = torch.zeros(H, device=dev), torch.zeros(1, device=dev)
        met = torch.zeros(8, dtype=torch.float64, device=dev)
        hist = torch.zeros(2 * 2048, dtype=torch.int32, device=dev)
        dbh = torch.full((H,), 0.5, device=dev)
        E.head(h.to(dev), w.to(dev), b.to(dev), wide.to(dev), lc.to(dev), S, y.to(dev), coef, dh,
               dw, db, met, hist, 2048, db_h=dbh)
        outs[dev] = [t.cpu() for t in (coef, dh, dw, db, met, hist, dbh)]
    c, g = outs["cpu"], outs["cuda"]
    torch.testing.assert_close(g[0], c[0], rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(g[1].float(), c[1].float(), rtol=1e-2, atol=1e-3)
    torch.testing.assert_close(g[2], c[2], rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(g[3], c[3], rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(g[4][:3], c[4][:3], rtol=1e-5, atol=1e-6)
    assert abs(int((g[5] - c[5]).abs().sum())) <= 4  # bin edges may differ by an ulp
    torch.testing.assert_close(g[6], c[6], rtol=1e-4, atol=1e-3)
    # db_h is the column sum of dh (up to dh's bf16 rounding)
    torch.testing.assert_close(g[6] - 0.5, g[1].float().sum(0), rtol=1e-2, atol=1e-2)
    x = torch.randn(300, 200).to(torch.bfloat16)
    torch.testing.assert_close(E.colsum(x.cuda(), torch.empty(200, device="cuda")).cpu(),
                               x.float().sum(0), rtol=1e-4, atol=1e-3)
    p, gr = torch.randn(1000), torch.randn(1000)
    st = [torch.zeros(1000) for _ in range(2)]
    pg, stg = p.cuda(), [t.cuda() for t in st]
    p16 = torch.empty(1000, dtype=torch.bfloat16, device="cuda")
    for step in (1, 2, 3):
        E.adam(p, gr, st[0], st[1], lr=1e-2, step=step, gscale=0.5)
        E.adam(pg, gr.cuda(), stg[0], stg[1], lr=1e-2, step=step, gscale=0.5, p16=p16)
    torch.testing.assert_close(pg.cpu(), p, rtol=1e-5, atol=1e-6)
    assert torch.equal(p16.cpu(), p.to(torch.bfloat16))


def test_wide_deep_gpu_matches_cpu_trainer():
    cfg = dict(num_features=1 << 20, embedding_dim=32, hidden=(128, 64), minibatch=512,
               table_capacity=1 << 15, emb_lr=0.05, mlp_lr=3e-3)
    tc = WideDeepTrainer(WideDeepConfig(**cfg), device="cpu")
    tg = WideDeepTrainer(WideDeepConfig(**cfg), device="cuda")
    lc, lg = [], []
    for s in range(8):
        k, l = criteo_batch(512, seed=9, row0=s * 512, num_features=1 << 20, cards=[200] * 26)
        tc.step(k, l)
        tg.step(k.cuda(), l.cuda())
        lc.append(tc.progress()["loss"])
        lg.append(tg.progress()["loss"])
    np.testing.assert_allclose(lg, lc, rtol=2e-2)
    assert lg[-1] < lg[0]


def test_wide_deep_gpu_full_width_learns():
    cfg = WideDeepConfig(num_features=10 ** 8, minibatch=4096, table_capacity=1 << 22)
    tr = WideDeepTrainer(cfg, device="cuda")
    for s in range(30):
        k, l = criteo_batch(4096, seed=2, row0=s * 4096, num_features=cfg.num_features,
                            device="cuda")
        tr.step(k, l)
        if s == 4:
            first = tr.progress()
    last = tr.progress()
    assert last["loss"] < first["loss"] and np.isfinite(last["loss"])


def _wd_rehearsal(rank, world, port, q, exchange="padded", model="wd", steps=6):
    import os

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), PSAMD_DIST_BACKEND="gloo")
    import torch.distributed as dist

    from parameter_server_amd.parallel.comm import init_from_env

    comm, dev = init_from_env("cuda")
    if model == "wd":
        cfg = WideDeepConfig(num_features=1 << 22, embedding_dim=64, hidden=(256, 128),
                             minibatch=1024, table_capacity=1 << 16, exchange=exchange)
        tr = WideDeepTrainer(cfg, comm, dev)
    else:
        from parameter_server_amd.models.fm import FMConfig, FMTrainer

        tr = FMTrainer(FMConfig(num_features=1 << 22, embedding_dim=16, minibatch=1024,
                                table_capacity=1 << 16, emb_lr=0.05, lambda_v=0.5,
                                exchange=exchange), comm, dev)
    for s in range(steps):
        k, l = criteo_batch(1024, seed=50 + rank, row0=s * 1024, num_features=1 << 22,
                            cards=[1000] * 26, device=dev)
        tr.step(k, l)
    p = tr.progress()
    occ, _ = tr.shard.table.census()
    from parameter_server_amd.ops.kv_table import EMPTY_KEY

    idx = torch.nonzero(tr.shard.table.slots[:, 0] != EMPTY_KEY).flatten()
    keys, w, _, _ = tr.shard.table.occupied()
    o = torch.argsort(keys)
    rows = tr.shard.rows[idx[o]].float().cpu()
    # numpy by value: a torch tensor goes through a shared-memory fd that the parent
    # may fetch only after this process exited (FileNotFoundError in resource_sharer)
    q.put((rank, p, tr.param.cpu().numpy() if model == "wd" else None, occ,
           keys[o].cpu().numpy(), w[o].cpu().numpy(), rows.numpy()))
    dist.barrier()
    dist.destroy_process_group()


def _run_rehearsal(exchange, model="wd", steps=6):
    import socket

    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_wd_rehearsal, args=(r, 2, port, q, exchange, model, steps))
          for r in range(2)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=120) for _ in ps], key=lambda r: r[0])
    for p in ps:
        p.join(timeout=60)
    t = lambda a: None if a is None else torch.from_numpy(a)  # noqa: E731
    return [(r, p, t(a), occ, t(k), t(w), t(rows)) for r, p, a, occ, k, w, rows in res]


@pytest.mark.parametrize("exchange", ["padded", "exact"])
def test_wide_deep_two_rank_gpu_rehearsal(exchange):
    res = _run_rehearsal(exchange)
    assert torch.equal(res[0][2], res[1][2])
    assert res[0][1]["examples"] == 2 * 6 * 1024 and np.isfinite(res[0][1]["loss"])
    assert res[0][3] > 0 and res[1][3] > 0


@pytest.mark.parametrize("model", ["wd", "fm"])
def test_padded_exchange_matches_exact(model):
    """Sync-free padded pull/push (fixed rows, device-side counts) trains what the
    count-sized all-to-all-v exchange trains: same shard keys, wide weights, loss."""
    # 2 steps: the second pulls rows the first pushed. (Over 6 steps the two runs drift
    # apart chaotically from the order of fp32 atomics in the wide / bias gradients: at
    # steps 1-2 the embedding rows are bitwise equal, at step 6 ~8 % of them differ by up
    # to one AdaGrad step, benchmarks/archive/wd_exchange_debug.py.)
    pad, ex = _run_rehearsal("padded", model, 2), _run_rehearsal("exact", model, 2)
    for rp, re_ in zip(pad, ex):
        assert rp[3] == re_[3]
        assert torch.equal(rp[4], re_[4])
        # wide gradients of hot keys combine per-wave pieces atomically (any order)
        torch.testing.assert_close(rp[5], re_[5], rtol=1e-3, atol=2e-5)
        torch.testing.assert_close(rp[6], re_[6], rtol=1e-2, atol=1e-3)
        assert abs(rp[1]["loss"] - re_[1]["loss"]) < 1e-4
        if model == "wd":
            torch.testing.assert_close(rp[2], re_[2], rtol=1e-3, atol=1e-5)


@pytest.mark.parametrize("model", ["wd", "fm"])
def test_part_localisation_matches_sort(model):
    """localize='part' (partition + per-bucket LDS dedup) trains what the radix sort
    trains: same unique keys, the order inside a key's segment only changes the
    order of the fp32 gradient sums."""
    from parameter_server_amd.models import FMConfig, FMTrainer

    losses = {}
    for mode in ("sort", "part"):
        if model == "wd":
            tr = WideDeepTrainer(WideDeepConfig(num_features=10 ** 8, minibatch=4096,
                                                table_capacity=1 << 20, localize=mode),
                                 device="cuda")
        else:
            tr = FMTrainer(FMConfig(num_features=10 ** 8, minibatch=4096,
                                    table_capacity=1 << 20, localize=mode), device="cuda")
        assert tr.localizer.mode == mode
        ls = []
        for s in range(6):
            k, l = criteo_batch(4096, seed=4, row0=s * 4096, num_features=10 ** 8,
                                device="cuda")
            tr.step(k, l)
            ls.append(tr.progress()["loss"])
        losses[mode] = ls
    np.testing.assert_allclose(losses["part"], losses["sort"], rtol=2e-3)
