"""Darlin BCD HIP kernels (csrc/hip/bcd.hip) vs the fp64 PyTorch reference, and the
GPU trainer vs the CPU trainer."""
import numpy as np
import pytest
import torch

from parameter_server_amd.data.synthetic import criteo_slots, sparse_classification
from parameter_server_amd.models.darlin import DarlinConfig, DarlinTrainer
from parameter_server_amd.ops import bcd

pytestmark = pytest.mark.gpu


def _csc(ncols, rows, seed, valued, head=5000):
    rng = np.random.default_rng(seed)
    cols, rws = [], []
    for c in range(ncols):
        n = int(rng.integers(0, 12))
        if c % 97 == 0:
            n = min(head, rows)  # head columns span many wave64 chunks (atomic path)
        r = np.sort(rng.choice(rows, size=n, replace=False))
        cols.append(np.full(r.size, c))
        rws.append(r)
    col = np.concatenate(cols).astype(np.int32)
    row = np.concatenate(rws).astype(np.int32)
    val = rng.uniform(0.1, 2.0, col.size).astype(np.float32) if valued else None
    colptr = np.zeros(ncols + 1, np.int64)
    np.cumsum(np.bincount(col, minlength=ncols), out=colptr[1:])
    return col, row, val, colptr


@pytest.mark.parametrize("valued", [False, True])
def test_bcd_kernels_match_torch(valued):
    ncols, rows = 3000, 20000
    col, row, val, colptr = _csc(ncols, rows, 0, valued)
    rng = np.random.default_rng(1)
    y = np.where(rng.random(rows) < 0.5, 1.0, -1.0).astype(np.float32)
    ym = rng.normal(0, 2, rows)
    delta = rng.uniform(0.1, 2, ncols)
    active = (rng.random(ncols) < 0.9).astype(np.uint8)
    w = np.where(rng.random(ncols) < 0.6, 0.0, rng.normal(0, 1, ncols))
    T = lambda a: None if a is None else torch.from_numpy(a)  # noqa: E731
    D = lambda a: None if a is None else torch.from_numpy(a).cuda()  # noqa: E731
    for c0, c1 in [(0, ncols), (97, 1234), (1500, 1501), (2000, 2000)]:
        p0, p1 = int(colptr[c0]), int(colptr[c1])
        Gc, Uc = bcd.grad(T(col), T(row), T(val), p0, p1, c0, c1 - c0, T(ym), T(y), T(delta),
                          T(active))
        Gg, Ug = bcd.grad(D(col), D(row), D(val), p0, p1, c0, c1 - c0, D(ym), D(y), D(delta),
                          D(active))
        torch.testing.assert_close(Gg.cpu(), Gc, rtol=1e-10, atol=1e-10)
        torch.testing.assert_close(Ug.cpu(), Uc, rtol=1e-10, atol=1e-10)
        for small, hot in ((64, 4096), (64, 1000), (16, 64)):  # load-balanced chunk kernel
            ch = D(bcd.build_chunks(colptr, c0, c1, small=small, hot=hot))
            Gk, Uk = bcd.grad(D(col), D(row), D(val), p0, p1, c0, c1 - c0, D(ym), D(y),
                              D(delta), D(active), chunks=ch)
            torch.testing.assert_close(Gk.cpu(), Gc, rtol=1e-10, atol=1e-10)
            torch.testing.assert_close(Uk.cpu(), Uc, rtol=1e-10, atol=1e-10)
        # per-example factors packed for the block's own examples only (urows): the
        # other rows of rowq stay NaN and are never read
        if p1 > p0:
            ch = D(bcd.build_chunks(colptr, c0, c1, hot=256))
            rq = torch.full((2 * rows,), float("nan"), dtype=torch.float64, device="cuda")
            ur = torch.unique(D(row[p0:p1]))
            Gq, Uq = bcd.grad(D(col), D(row), D(val), p0, p1, c0, c1 - c0, D(ym), D(y),
                              D(delta), D(active), chunks=ch, rowq=rq, urows=ur)
            torch.testing.assert_close(Gq.cpu(), Gc, rtol=1e-10, atol=1e-10)
            torch.testing.assert_close(Uq.cpu(), Uc, rtol=1e-10, atol=1e-10)
        for thr in (1e20, 0.05):
            wc, dc, ac = T(w.copy()), T(delta.copy()), T(active.copy())
            wg, dg, ag = D(w.copy()), D(delta.copy()), D(active.copy())
            dwc, vc = bcd.update(c0, c1 - c0, Gc, Uc, wc, dc, ac, 1.0, 0.5, 5.0, thr)
            dwg, vg = bcd.update(c0, c1 - c0, Gg, Ug, wg, dg, ag, 1.0, 0.5, 5.0, thr)
            torch.testing.assert_close(wg.cpu(), wc, rtol=1e-9, atol=1e-12)
            torch.testing.assert_close(dg.cpu(), dc, rtol=1e-9, atol=1e-12)
            assert torch.equal(ag.cpu(), ac)
            torch.testing.assert_close(dwg.cpu(), dwc, rtol=1e-9, atol=1e-12)
            assert abs(bcd.violation(vg) - bcd.violation(vc)) <= 1e-9 * max(1, bcd.violation(vc))
        ymc, ymg = T(ym.copy()), D(ym.copy())
        bcd.dual(T(col), T(row), T(val), p0, p1, c0, c1 - c0, dwc, T(y), ymc)
        bcd.dual(D(col), D(row), D(val), p0, p1, c0, c1 - c0, dwg, D(y), ymg)
        torch.testing.assert_close(ymg.cpu(), ymc, rtol=1e-10, atol=1e-10)
        oc, og = bcd.objective(ymc), bcd.objective(ymg)
        torch.testing.assert_close(og.cpu(), oc, rtol=1e-11, atol=0)
        sc, sg = bcd.server_stats(wc, ac, 10, ncols - 10), bcd.server_stats(wg, ag, 10, ncols - 10)
        torch.testing.assert_close(sg.cpu(), sc, rtol=1e-11, atol=0)


def test_darlin_gpu_trainer_matches_cpu():
    sd = sparse_classification(6000, groups=(1, 2, 3, 4), keys_per_group=2000,
                               nnz_per_row=(1, 3, 5, 2), binary=False, seed=7)
    cfg = DarlinConfig(l1=1.0, max_pass=8, epsilon=1e-12, tail_freq=1, seed=1)
    pc = DarlinTrainer(sd, cfg, device="cpu").train()
    tg = DarlinTrainer(sd, cfg, device="cuda")
    pg = tg.train()
    np.testing.assert_allclose([p.objective for p in pg], [p.objective for p in pc], rtol=1e-8)
    assert [p.nnz_w for p in pg] == [p.nnz_w for p in pc]
    assert pg[-1].objective < pg[0].objective


@pytest.mark.parametrize("tau", [0, 2])
def test_darlin_gpu_groups_layout_matches_cpu(tau):
    """CTR-log-shaped groups (2 keys per example and group, each group in 1/3 of the
    examples): wide blocks without a dense layout gather ym / y per entry (Block.few_rows,
    no rowq packing pass), small narrow blocks run gradient + coordinate update in one launch
    (the last workgroup updates), hot columns in pieces sized from the block; the
    GPU trainer follows the CPU trainer's objectives and sparsity."""
    from parameter_server_amd.data.synthetic import sparse_groups

    sd = sparse_groups(60_000, groups=6, present=2, keys_per_group=100_000, seed=9, alpha=0.8)
    cfg = DarlinConfig(l1=2.0, max_pass=4, epsilon=1e-12, tail_freq=1, tau=tau, seed=3)
    tg = DarlinTrainer(sd, cfg, device="cuda")
    assert any(b.few_rows for b in tg.blocks)
    assert any(b.row_mode and b.dcol is None and tg._fused_update(b, True) for b in tg.blocks)
    pg = tg.train()
    pc = DarlinTrainer(sd, cfg, device="cpu").train()
    np.testing.assert_allclose([p.objective for p in pg], [p.objective for p in pc], rtol=1e-8)
    assert [p.nnz_w for p in pg] == [p.nnz_w for p in pc]
    assert pg[-1].objective < pg[0].objective


def test_hot_piece_sizes():
    from parameter_server_amd.models.darlin import _hot_piece

    assert _hot_piece(10) == 256 and _hot_piece(400_000) == 256
    assert _hot_piece(4_000_000) == 2048 and _hot_piece(10 ** 9) == 4096


def test_darlin_gpu_criteo_shaped_with_delay():
    sd = criteo_slots(200_000, seed=3, num_features=10 ** 6, device="cuda")
    # 39 one-block groups: a delay of 1 block is still stable (large tau needs many blocks)
    tr = DarlinTrainer(sd, DarlinConfig(l1=4.0, max_pass=3, tail_freq=2, tau=1, seed=0),
                       device="cuda")
    assert len(tr.blocks) == 39 and tr.nnz > 0
    prog = tr.train()
    assert prog[-1].objective < prog[0].objective
    assert prog[-1].objective < sd.rows * np.log(2)  # better than the zero model


def _rehearsal_worker(rank, world, port, q, shard="auto"):
    import os

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), PSAMD_DIST_BACKEND="gloo")
    import torch.distributed as dist

    from parameter_server_amd.data.slot_reader import SlotData
    from parameter_server_amd.parallel.comm import init_from_env

    comm, dev = init_from_env("cuda")
    sd = sparse_classification(4000, groups=(1, 2, 3), keys_per_group=800, nnz_per_row=(1, 3, 4),
                               seed=21)
    n = sd.rows // world
    a, b = rank * n, (rank + 1) * n
    part = SlotData(labels=sd.labels[a:b], groups={
        g: (off[a:b + 1] - off[a], k[off[a]:off[b]], None) for g, (off, k, v) in sd.groups.items()})
    tr = DarlinTrainer(part, DarlinConfig(l1=1.0, max_pass=5, tail_freq=1, tau=1, seed=2,
                                          shard_server=shard), comm=comm, device=dev)
    prog = tr.train()
    q.put((rank, [p.objective for p in prog], tr.w.cpu().numpy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("shard", ["auto", "on"])
def test_darlin_two_rank_gpu_rehearsal_matches_single(shard):
    """2 ranks on one GPU (gloo-staged all-reduce, or the sharded server: reduce-scatter,
    owner update with NaN marks, all-gather of dw, bcd_replica): same objectives as 1
    rank, bitwise-equal replicas."""
    import socket

    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_rehearsal_worker, args=(r, 2, port, q, shard)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=300) for _ in ps], key=lambda r: r[0])
    for p in ps:
        p.join(timeout=60)
    sd = sparse_classification(4000, groups=(1, 2, 3), keys_per_group=800, nnz_per_row=(1, 3, 4),
                               seed=21)
    ref = DarlinTrainer(sd, DarlinConfig(l1=1.0, max_pass=5, tail_freq=1, tau=1, seed=2),
                        device="cuda").train()
    for _, objs, w in res:
        np.testing.assert_allclose(objs, [p.objective for p in ref], rtol=1e-8)
    np.testing.assert_array_equal(res[0][2], res[1][2])


def _same_csc(a, b):
    assert a.num_cols == b.num_cols and a.nnz == b.nnz and a.num_ex == b.num_ex
    np.testing.assert_array_equal(a.colptr, b.colptr)
    assert torch.equal(a.col.cpu(), b.col.cpu()) and torch.equal(a.row.cpu(), b.row.cpu())
    assert (a.val is None) == (b.val is None)
    if a.val is not None:
        assert torch.equal(a.val.cpu(), b.val.cpu())
    assert sorted(a.group_keys) == sorted(b.group_keys)
    for g in a.group_keys:
        np.testing.assert_array_equal(a.group_keys[g], b.group_keys[g])
    assert [(k.c0, k.c1, k.p0, k.p1) for k in a.blocks] == [(k.c0, k.c1, k.p0, k.p1) for k in b.blocks]
    assert a.info == b.info


@pytest.mark.parametrize("valued,freq", [(False, 0), (True, 2)])
def test_darlin_gpu_preprocess_bit_identical_to_host(valued, freq):
    """Device CSC build (own radix sort + RLE, device tail filter / column map) ==
    the numpy reference path, array for array."""
    sd = sparse_classification(5000, groups=(1, 2, 3, 5), keys_per_group=3000,
                               nnz_per_row=(1, 3, 5, 2), binary=not valued, seed=11)
    cfg = DarlinConfig(l1=1.0, tail_freq=freq, seed=0)
    g = DarlinTrainer(sd, cfg, device="cuda")
    h = DarlinTrainer(sd, DarlinConfig(l1=1.0, tail_freq=freq, seed=0, host_preprocess=True),
                      device="cuda")
    _same_csc(g, h)


def test_darlin_gpu_preprocess_criteo_and_device_data():
    """Criteo-shaped slots: host numpy groups and device-resident groups give the same
    CSC as the numpy path."""
    sd = criteo_slots(50_000, seed=5, num_features=10 ** 7, device="cuda")
    cfg = DarlinConfig(l1=1.0, tail_freq=3, seed=0)
    h = DarlinTrainer(sd, DarlinConfig(l1=1.0, tail_freq=3, seed=0, host_preprocess=True),
                      device="cuda")
    g = DarlinTrainer(sd, cfg, device="cuda")
    _same_csc(g, h)
    dev_sd = criteo_slots(50_000, seed=5, num_features=10 ** 7, device="cuda", on_device=True)
    d = DarlinTrainer(dev_sd, cfg, device="cuda")
    _same_csc(d, h)


@pytest.mark.parametrize("ncols,valued", [(35, False), (1500, False), (300, True)])
def test_grad_rows_matches_column_kernel(ncols, valued):
    """Row-order narrow-block gradient (LDS fixed point, W partials) == the column-order
    kernel and the fp64 PyTorch reference, on a block with hot and cold columns."""
    import torch

    from parameter_server_amd.ops import bcd

    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(ncols)
    nrows, n = 50000, 200000
    # power-law columns, sorted CSC (col, row) for the column kernel
    col = (torch.rand(n, generator=g) ** 3 * ncols).long().clamp(max=ncols - 1)
    row = torch.randint(0, nrows, (n,), generator=g)
    key = col * nrows + row
    key = torch.unique(key)
    col, row = (key // nrows).int(), (key % nrows).int()
    n = col.numel()
    val = (torch.rand(n, generator=g) * 3 - 1).float() if valued else None
    ym = (torch.randn(nrows, generator=g, dtype=torch.float64) * 2)
    y = torch.where(torch.rand(nrows, generator=g) > 0.5, 1.0, -1.0).float()
    c0 = 7
    base = c0 + ncols + 5
    delta = torch.rand(base, generator=g, dtype=torch.float64)
    active = (torch.rand(base, generator=g) > 0.1).to(torch.uint8)
    colg = col + c0
    G0, U0 = bcd.grad(colg, row, val, 0, n, c0, ncols, ym, y, delta, active)
    d = lambda t: None if t is None else t.to(dev)  # noqa: E731
    perm = torch.argsort(row.long() * base + colg.long())
    W = 768
    k2 = bcd.fixed_point_shift(n, 1.0 if val is None else float(val.abs().max()))
    part = torch.empty(W * 2 * 2048, dtype=torch.int64, device=dev)
    G1 = torch.empty(ncols, dtype=torch.float64, device=dev)
    U1 = torch.empty(ncols, dtype=torch.float64, device=dev)
    bcd.grad_rows(d(colg[perm].contiguous()), d(row[perm].contiguous()),
                  None if val is None else d(val[perm].contiguous()), 0, n, c0, ncols, d(ym), d(y),
                  d(delta), d(active), G1, U1, part, W, k2)
    torch.testing.assert_close(G1.cpu(), G0, rtol=1e-10, atol=1e-9)
    torch.testing.assert_close(U1.cpu(), U0, rtol=1e-10, atol=1e-9)
    # deterministic: a second run is bitwise equal
    G2 = torch.empty_like(G1)
    U2 = torch.empty_like(U1)
    bcd.grad_rows(d(colg[perm].contiguous()), d(row[perm].contiguous()),
                  None if val is None else d(val[perm].contiguous()), 0, n, c0, ncols, d(ym), d(y),
                  d(delta), d(active), G2, U2, part, W, k2)
    assert torch.equal(G1, G2) and torch.equal(U1, U2)


@pytest.mark.parametrize("tau,valued", [(1, False), (0, False), (2, True)])
def test_fused_row_pass_bitwise_equal_to_separate_kernels(monkeypatch, tau, valued):
    """The row pass (a block's dual update fused into the next block's gradient over dense
    per-example layouts, bcd.rowpass) gives the same margins, weights and objectives as
    the separate dual / gradient / rowq kernels (PSAMD_DARLIN_FUSE=0), to fp64 rounding."""
    if valued:  # one valued entry per example and group (dense layouts with values)
        sd = sparse_classification(30_000, groups=(1, 2, 3), keys_per_group=3000,
                                   nnz_per_row=(1, 1, 1), binary=False, seed=5)
    else:
        sd = criteo_slots(120_000, seed=4, num_features=10 ** 6, device="cuda")
    cfg = dict(l1=2.0, max_pass=3, tail_freq=2, tau=tau, seed=0, epsilon=1e-12)
    out = {}
    for fuse in ("1", "0"):
        monkeypatch.setenv("PSAMD_DARLIN_FUSE", fuse)
        tr = DarlinTrainer(sd, DarlinConfig(**cfg), device="cuda")
        if fuse == "1":
            assert any(b.dcol is not None for b in tr.blocks)
            assert any(b.dcol is not None and b.row_mode for b in tr.blocks)
            if not valued:  # wide slots: hot columns in LDS, cold ones column-wise
                assert any(b.hcols is not None for b in tr.blocks)
        else:
            assert all(b.dcol is None for b in tr.blocks)
        prog = tr.train()
        out[fuse] = ([p.objective for p in prog], tr.ym.cpu(), tr.w.cpu(), tr.active.cpu())
    # (not bitwise: the wide blocks' hot columns and the objective add fp64 partial sums
    # atomically, in a run-dependent order, on both paths)
    np.testing.assert_allclose(out["1"][0], out["0"][0], rtol=1e-11)
    torch.testing.assert_close(out["1"][1], out["0"][1], rtol=1e-9, atol=1e-9)
    torch.testing.assert_close(out["1"][2], out["0"][2], rtol=1e-9, atol=1e-12)
    assert (out["1"][3] != out["0"][3]).sum().item() <= 2


@pytest.mark.parametrize("data,tau", [("criteo", 1), ("groups", 8)])
def test_fp32_tau_row_pass_keeps_the_objective_trajectory(data, tau):
    """tau32 (the benchmark's fast row pass: tau_i = 1 / (1 + exp(ym_i)) in fp32, G / U
    sums still fp64 fixed point) follows the fp64 trainer's per-pass objective to 1e-5
    relative, on the Criteo-shaped slots at tau = 1 and the converging groups data at
    tau = 8."""
    if data == "criteo":
        sd = criteo_slots(200_000, seed=3, num_features=10 ** 6, device="cuda")
    else:
        from parameter_server_amd.data.synthetic import sparse_groups

        sd = sparse_groups(60_000, seed=5)
    objs = {}
    for t32 in (False, True):
        cfg = DarlinConfig(l1=4.0, max_pass=4, tail_freq=2, tau=tau, seed=0, epsilon=0.0,
                           tau32=t32)
        tr = DarlinTrainer(sd, cfg, device="cuda")
        if data == "criteo":  # (the groups blocks are too sparse for the dense row layouts)
            assert any(b.dcol is not None for b in tr.blocks)
        objs[t32] = [p.objective for p in tr.train()]
    np.testing.assert_allclose(objs[True], objs[False], rtol=1e-5)
    assert objs[True][-1] < objs[True][0]
