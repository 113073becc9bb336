"""Darlin BCD (L1 logistic regression): ops vs a literal transcription of the
reference loops, trainer vs liblinear, multi-rank (gloo) vs single rank, and the
1 scheduler + 2 servers + 2 workers runtime app vs the trainer."""
import math
import os
import re
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from parameter_server_amd.data.slot_reader import SlotData, SlotReader
from parameter_server_amd.data.synthetic import sparse_classification, write_text
from parameter_server_amd.models.darlin import DarlinConfig, DarlinTrainer
from parameter_server_amd.ops import bcd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _random_csc(ncols=40, rows=200, seed=0, valued=True, heavy=True):
    rng = np.random.default_rng(seed)
    cols, rws = [], []
    for c in range(ncols):
        n = int(rng.integers(0, 8))
        if heavy and c % 13 == 0:
            n = 150  # a head column spanning several wave64 chunks
        r = np.sort(rng.choice(rows, size=min(n, rows), replace=False))
        cols.append(np.full(r.size, c))
        rws.append(r)
    col = np.concatenate(cols).astype(np.int32)
    row = np.concatenate(rws).astype(np.int32)
    val = rng.uniform(0.1, 2.0, col.size).astype(np.float32) if valued else None
    colptr = np.zeros(ncols + 1, np.int64)
    np.cumsum(np.bincount(col, minlength=ncols), out=colptr[1:])
    return col, row, val, colptr


def _naive_grad(col, row, val, c0, c1, colptr, dual, y, delta, active):
    """darlin.h:381-427 transcribed (dual = exp(y Xw))."""
    G = np.zeros(c1 - c0)
    U = np.zeros(c1 - c0)
    for j in range(c0, c1):
        if not active[j]:
            continue
        g = u = 0.0
        d = math.exp(delta[j]) if val is None else delta[j]
        for o in range(colptr[j], colptr[j + 1]):
            i = row[o]
            tau = 1 / (1 + dual[i])
            if val is None:
                g -= float(y[i]) * tau
                u += min(tau * (1 - tau) * d, .25)
            else:
                v = float(val[o])
                g -= float(y[i]) * tau * v
                u += min(tau * (1 - tau) * math.exp(abs(v) * d), .25) * v * v
        G[j - c0], U[j - c0] = g, u
    return G, U


def _naive_update(c0, G, U, w, delta, active, eta, lam, dmax, thr):
    """darlin.h:206-246 transcribed (filtered -> inactive, w stays 0)."""
    vio_max = 0.0
    dw = np.zeros(G.size)
    for i in range(G.size):
        k = c0 + i
        if not active[k]:
            continue
        g, u = G[i], U[i] / eta + 1e-10
        gp, gn = g + lam, g - lam
        d, vio = -w[k], 0.0
        if w[k] == 0:
            if gp < 0:
                vio = -gp
            elif gn > 0:
                vio = gn
            elif gp > thr and gn < -thr:
                active[k] = 0
                continue
        vio_max = max(vio_max, vio)
        if gp <= u * w[k]:
            d = -gp / u
        elif gn >= u * w[k]:
            d = -gn / u
        d = min(delta[k], max(-delta[k], d))
        delta[k] = min(dmax, 2 * abs(d) + .1)
        w[k] += d
        dw[i] = d
    return dw, vio_max


@pytest.mark.parametrize("valued", [True, False])
def test_bcd_ops_match_reference_loops(valued):
    col, row, val, colptr = _random_csc(valued=valued)
    rows, ncols = 200, 40
    rng = np.random.default_rng(1)
    y = np.where(rng.random(rows) < 0.5, 1.0, -1.0).astype(np.float32)
    ym = rng.normal(0, 1, rows)
    delta = rng.uniform(0.1, 2, ncols)
    active = (rng.random(ncols) < 0.85).astype(np.uint8)
    c0, c1 = 5, 33
    Gt, Ut = bcd.grad(torch.from_numpy(col), torch.from_numpy(row),
                      None if val is None else torch.from_numpy(val), int(colptr[c0]),
                      int(colptr[c1]), c0, c1 - c0, torch.from_numpy(ym), torch.from_numpy(y),
                      torch.from_numpy(delta), torch.from_numpy(active))
    Gn, Un = _naive_grad(col, row, val, c0, c1, colptr, np.exp(ym), y, delta, active)
    np.testing.assert_allclose(Gt.numpy(), Gn, rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(Ut.numpy(), Un, rtol=1e-12, atol=1e-12)
    # update: a mix of zero / non-zero weights and a finite KKT threshold
    w = np.where(rng.random(ncols) < 0.5, 0.0, rng.normal(0, 1, ncols))
    for thr in (1e20, 0.3):
        wt, dt, at = torch.from_numpy(w.copy()), torch.from_numpy(delta.copy()), \
            torch.from_numpy(active.copy())
        wn, dn, an = w.copy(), delta.copy(), active.copy()
        dwt, vio = bcd.update(c0, c1 - c0, Gt, Ut, wt, dt, at, 1.0, 0.7, 5.0, thr)
        dwn, vn = _naive_update(c0, Gn, Un, wn, dn, an, 1.0, 0.7, 5.0, thr)
        np.testing.assert_allclose(wt.numpy(), wn, rtol=1e-12, atol=1e-14)
        np.testing.assert_allclose(dt.numpy(), dn, rtol=1e-12)
        np.testing.assert_array_equal(at.numpy(), an)
        np.testing.assert_allclose(dwt.numpy(), dwn, atol=1e-14)
        assert abs(bcd.violation(vio) - vn) < 1e-12
    # dual update == multiplicative dual of the reference (darlin.h:472-502)
    ymt = torch.from_numpy(ym.copy())
    bcd.dual(torch.from_numpy(col), torch.from_numpy(row),
             None if val is None else torch.from_numpy(val), int(colptr[c0]), int(colptr[c1]), c0,
             c1 - c0, dwt, torch.from_numpy(y), ymt)
    dual = np.exp(ym)
    for j in range(c0, c1):
        for o in range(colptr[j], colptr[j + 1]):
            i = row[o]
            x = 1.0 if val is None else float(val[o])
            dual[i] *= math.exp(float(y[i]) * dwt[j - c0].item() * x)
    np.testing.assert_allclose(np.exp(ymt.numpy()), dual, rtol=1e-10)
    obj = float(bcd.objective(ymt)[0])
    assert abs(obj - np.log1p(1 / dual).sum()) < 1e-8 * obj


def _design_matrix(sd: SlotData, tr: DarlinTrainer):
    import scipy.sparse as sp

    keys, _ = tr.model()
    rows, cols, vals = [], [], []
    for g in sorted(sd.groups):
        off, k, v = sd.groups[g]
        base = tr.group_base[g]
        gk = keys[base:base + tr.group_keys[g].size]
        pos = np.searchsorted(gk, k)
        rows.append(np.repeat(np.arange(sd.rows), np.diff(off)))
        cols.append(base + pos)
        vals.append(np.ones(k.size) if v is None else v)
    return sp.csr_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))),
                         shape=(sd.rows, keys.size))


def test_trainer_reaches_liblinear_optimum():
    from sklearn.linear_model import LogisticRegression

    sd = sparse_classification(2000, groups=(1, 2, 3), keys_per_group=300,
                               nnz_per_row=(1, 3, 5), binary=False, seed=1)
    cfg = DarlinConfig(l1=1.0, max_pass=60, epsilon=1e-8, seed=0)
    tr = DarlinTrainer(sd, cfg)
    prog = tr.train()
    X = _design_matrix(sd, tr)
    y = sd.labels
    lr = LogisticRegression(penalty="l1", C=1.0, solver="liblinear", fit_intercept=False,
                            tol=1e-8, max_iter=5000).fit(X, y)
    f = lambda w: np.log1p(np.exp(-y * (X @ w))).sum() + np.abs(w).sum()  # noqa: E731
    _, w = tr.model()
    assert abs(prog[-1].objective - f(w)) < 1e-6 * f(w)
    assert f(w) <= f(lr.coef_[0]) * (1 + 2e-4), (f(w), f(lr.coef_[0]))
    assert prog[-1].objective < prog[0].objective


def test_trainer_tau_and_prior_groups_converge():
    sd = sparse_classification(1500, groups=(1, 2, 3), keys_per_group=200,
                               nnz_per_row=(1, 3, 5), seed=2)
    base = DarlinTrainer(sd, DarlinConfig(l1=1.0, max_pass=25, epsilon=1e-9)).train()
    # bounded delay: stale margins for tau blocks slow convergence but it still converges
    tr = DarlinTrainer(sd, DarlinConfig(l1=1.0, max_pass=25, epsilon=1e-9, tau=1,
                                        prior_groups=(2,), prior_iters=2))
    prog = tr.train()
    assert len(tr.prior_order) == 2 * sum(b.group == 2 for b in tr.blocks)
    assert abs(prog[-1].objective - base[-1].objective) < 1e-2 * base[-1].objective


def test_tail_filter_drops_rare_keys():
    sd = sparse_classification(800, groups=(1, 2), keys_per_group=400, nnz_per_row=(2, 3),
                               seed=4)
    tr = DarlinTrainer(sd, DarlinConfig(tail_freq=3, max_pass=2))
    for g, (off, k, _) in sd.groups.items():
        u, c = np.unique(k, return_counts=True)
        assert tr.group_keys[g].size == int((c > 3).sum())


def test_slot_reader_cache_roundtrip(tmp_path):
    sd = sparse_classification(300, groups=(1, 5), keys_per_group=50, nnz_per_row=(2, 1),
                               binary=False, seed=0)
    f = tmp_path / "part-0"
    write_text(sd, str(f), "SPARSE")
    r1 = SlotReader([str(f)], "SPARSE", cache_prefix=str(tmp_path / "cache" / "c_"))
    a = r1.read()
    assert r1.hit_cache == 0
    r2 = SlotReader([str(f)], "SPARSE", cache_prefix=str(tmp_path / "cache" / "c_"))
    b = r2.read()
    assert r2.hit_cache == 1
    assert np.array_equal(a.labels, b.labels) and sorted(a.groups) == [1, 5]
    for g in a.groups:
        for x, z in zip(a.groups[g], b.groups[g]):
            assert np.array_equal(x, z)
    assert np.array_equal(a.groups[1][1], sd.groups[1][1])
    np.testing.assert_allclose(a.groups[5][2], sd.groups[5][2], rtol=1e-5)
    info = a.info()
    assert info["slots"][5]["max_key"] == int(sd.groups[5][1].max()) + 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dist_worker(rank, world, port, q, shard="auto"):
    import torch.distributed as dist

    from parameter_server_amd.parallel.comm import DistComm

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    sd = sparse_classification(1200, groups=(1, 2, 3), keys_per_group=250,
                               nnz_per_row=(1, 3, 4), seed=5)
    n = sd.rows // world
    a, b = rank * n, (rank + 1) * n
    part = SlotData(labels=sd.labels[a:b], groups={
        g: (off[a:b + 1] - off[a], k[off[a]:off[b]], None) for g, (off, k, v) in sd.groups.items()})
    tr = DarlinTrainer(part, DarlinConfig(l1=1.0, max_pass=6, tail_freq=1, seed=3,
                                          shard_server=shard), comm=DistComm("cpu"))
    prog = tr.train()
    q.put((rank, [p.objective for p in prog], [p.nnz_w for p in prog], tr.w.numpy().copy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,shard", [(2, "auto"), (2, "on"), (3, "on")])
def test_trainer_two_ranks_gloo_equals_single_rank(world, shard):
    """All-reduce path (auto: these blocks are small) and sharded server (reduce-scatter of [G | U] to the owners, owner update with NaN
    marks, all-gather of dw, replica replay): every rank's replica equals the
    single-rank trainer and the replicas stay bitwise identical (world 3: blocks whose
    width is not a multiple of 3, padded slices)."""
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_dist_worker, args=(r, world, port, q, shard))
          for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=240) for _ in ps])
    for p in ps:
        p.join(timeout=60)
    sd = sparse_classification(1200, groups=(1, 2, 3), keys_per_group=250,
                               nnz_per_row=(1, 3, 4), seed=5)
    tr = DarlinTrainer(sd, DarlinConfig(l1=1.0, max_pass=6, tail_freq=1, seed=3))
    prog = tr.train()
    for _, objs, nnz, w in res:
        np.testing.assert_allclose(objs, [p.objective for p in prog], rtol=1e-9)
        assert nnz == [p.nnz_w for p in prog]
        np.testing.assert_allclose(w, tr.w.numpy(), atol=1e-9)
    for r in range(1, world):  # replicas stay bitwise identical
        np.testing.assert_array_equal(res[0][3], res[r][3])


def test_darlin_plumbing_1_2_2_matches_trainer(tmp_path):
    sd = sparse_classification(1800, groups=(1, 2, 3), keys_per_group=300,
                               nnz_per_row=(1, 3, 5), seed=3)
    data = tmp_path / "data"
    data.mkdir()
    n = sd.rows // 3
    for p in range(3):
        a, b = p * n, (p + 1) * n
        part = SlotData(labels=sd.labels[a:b], groups={
            g: (off[a:b + 1] - off[a], k[off[a]:off[b]], None)
            for g, (off, k, v) in sd.groups.items()})
        write_text(part, str(data / f"part-{p}"), "SPARSE_BINARY")
    model = tmp_path / "model" / "m"
    conf = tmp_path / "batch.conf"
    conf.write_text(f"""linear_method {{
training_data {{ format: TEXT text: SPARSE_BINARY file: "{data}/part.*" }}
model_output {{ format: TEXT file: "{model}" }}
loss {{ type: LOGIT }}
penalty {{ type: L1 lambda: 1 }}
learning_rate {{ type: CONSTANT alpha: 1 }}
darlin {{ max_pass_of_data: 6 epsilon: 1e-9 feature_block_ratio: 2
  random_feature_block_order: false max_block_delay: 0
  local_cache {{ format: BIN file: "{tmp_path}/cache/c_" }} }}
}}""")
    cmd = [sys.executable, "-m", "parameter_server_amd.launch", "local", "2", "2", "--timeout",
           "150", "--", sys.executable, "-u", "-m", "parameter_server_amd.app.main", "-app_file",
           str(conf), "-timeout", "140"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=170)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out
    objs = [float(m.group(1)) for m in re.finditer(r"^\s+\d+ \| (\S+)\s", out, re.M)]
    assert len(objs) == 6, out
    # same data through the GPU-style trainer (single rank, same block order)
    full = SlotReader(sorted(str(p) for p in data.iterdir()), "SPARSE_BINARY").read()
    tr = DarlinTrainer(full, DarlinConfig(l1=1.0, max_pass=6, epsilon=1e-9, block_ratio=2,
                                          random_order=False))
    prog = tr.train()
    np.testing.assert_allclose(objs, [p.objective for p in prog], rtol=2e-5)
    files = sorted(os.listdir(model.parent))
    assert files == ["m_S0", "m_S1"]
    saved = {}
    for fn in files:
        for line in open(model.parent / fn):
            k, v = line.split("\t")
            saved[int(k)] = float(v)
    keys, w = tr.model()
    ref = {int(k): float(v) for k, v in zip(keys, w) if v != 0}
    assert set(saved) == set(ref)
    for k in ref:
        assert abs(saved[k] - ref[k]) < 1e-4 * max(1.0, abs(ref[k]))


def test_build_chunks_partitions_columns():
    """Chunked-gradient work list: chunks tile [colptr[c0], colptr[c1]) exactly, small
    chunks hold whole columns (<= small entries), hot chunks one column's piece."""
    import numpy as np

    from parameter_server_amd.ops.bcd import HOT_BIT, build_chunks

    rng = np.random.default_rng(3)
    n = rng.integers(0, 20, 500)
    n[::37] = rng.integers(65, 9000, n[::37].size)
    cp = np.zeros(n.size + 1, np.int64)
    np.cumsum(n, out=cp[1:])
    for c0, c1, small, hot in [(0, 500, 64, 4096), (37, 38, 64, 4096), (5, 300, 16, 100),
                               (200, 200, 64, 4096)]:
        ch = build_chunks(cp, c0, c1, small=small, hot=hot)
        pos, isHot = ch & ~HOT_BIT, (ch & HOT_BIT) != 0
        assert pos[0] == cp[c0] or c0 == c1 and pos[0] == cp[c1]
        assert pos[-1] == cp[c1]
        col_of = np.repeat(np.arange(n.size), n)
        for a, b, h in zip(pos[:-1], pos[1:], isHot[:-1]):
            cols = np.unique(col_of[a:b])
            if h:
                assert cols.size == 1 and n[cols[0]] > small and b - a <= hot
            else:
                assert b - a <= small and cp[cols[0]] == a and cp[cols[-1] + 1] == b


def test_hot_layout_splits_wide_block():
    """Wide-block hot / cold split of the row pass (ops/bcd.py hot_layout): the nhot most
    frequent columns get LDS slots (kenc = -2 - slot), every other entry keeps its column,
    and the cold chunk list skips exactly the hot columns, each as one SKIP_BIT chunk."""
    import numpy as np
    import torch

    from parameter_server_amd.ops.bcd import HOT_BIT, SKIP_BIT, hot_layout

    rng = np.random.default_rng(5)
    ncols, rows, nhot = 600, 5000, 64
    p = 1.0 / np.arange(1, ncols + 1) ** 1.3
    col = rng.choice(ncols, size=rows, p=p / p.sum())
    keep = rng.random(rows) < 0.9  # some examples without an entry in the block
    dcol = torch.from_numpy(np.where(keep, col, -1).astype(np.int32))
    c0 = 100  # block columns [c0, c0 + ncols) of a larger model
    cnt = np.bincount(col[keep], minlength=ncols)
    cp = np.zeros(c0 + ncols + 1, np.int64)
    cp[c0 + 1:] = np.cumsum(cnt)
    out = hot_layout(dcol, cp, c0, c0 + ncols, nhot=nhot)
    assert out is not None
    kenc, hcols, chunks, nh = out
    hc = hcols.numpy()
    assert hc.size == nhot and np.all(np.diff(hc) > 0)
    assert nh == cnt[hc].sum() and cnt[hc].min() >= np.sort(cnt)[-nhot]
    k = kenc.numpy()
    d = dcol.numpy()
    hot = k <= -2
    assert np.array_equal(hc[-2 - k[hot]], d[hot])        # slot -> its column
    assert np.array_equal(k[~hot], d[~hot])                # cold entries / no entry kept
    assert not np.isin(d[~hot & (d >= 0)], hc).any()
    skip = (chunks & SKIP_BIT) != 0
    pos = chunks & ~(HOT_BIT | SKIP_BIT)
    col_start = {int(cp[c0 + j]): j for j in range(ncols) if cnt[j]}
    assert sorted(col_start[int(a)] for a in pos[:-1][skip[:-1]]) == sorted(
        j for j in hc if cnt[j])
    assert pos[-1] == cp[c0 + ncols] and np.all(np.diff(pos) > 0)
    # no split when the hot columns hold too little of the block
    assert hot_layout(dcol, cp, c0, c0 + ncols, nhot=nhot, min_share=0.999) is None


def _max_delay_reference(X, y, blocks, order, cfg, passes):
    """Independent transcription of the reference's bounded-delay BCD at its MAXIMAL
    delay: DarlinScheduler::run (darlin.h:58-122: block i may start once block i-tau-1
    has finished; KKT threshold and reset per pass), the worker's gradient (darlin.h:381-427,
    _naive_grad), the server's coordinate update (darlin.h:206-246, _naive_update) and the
    worker's multiplicative dual update dual_i *= exp(y_i dw_j x_ij) (darlin.h:480-500).
    Every in-flight block computes its gradient against the margins of the blocks that
    had finished when it started. Returns the per-pass objective."""
    from collections import deque

    Xc = X.tocsc()
    col, row = Xc.indices.astype(np.int32), None
    colptr = Xc.indptr.astype(np.int64)
    rowidx = Xc.indices
    ncols = X.shape[1]
    w = np.zeros(ncols)
    delta = np.full(ncols, cfg.delta_init)
    active = np.ones(ncols, np.uint8)
    dual = np.ones(X.shape[0])
    kkt_thr, reset, objs, prev = 1e20, False, [], None
    for it in range(passes):
        if reset:
            active[:] = 1
        vio = [0.0]
        inflight = deque()

        def finish(item):
            c0, c1, G, U = item
            dw, v = _naive_update(c0, G, U, w, delta, active, cfg.eta, cfg.l1, cfg.delta_max,
                                  kkt_thr)
            vio[0] = max(vio[0], v)
            for j in range(c0, c1):
                if dw[j - c0] != 0:
                    r = rowidx[colptr[j]:colptr[j + 1]]
                    dual[r] *= np.exp(y[r] * dw[j - c0])

        for i, k in enumerate(order):
            while inflight and inflight[0][0] <= i - cfg.tau - 1:
                finish(inflight.popleft()[1])
            c0, c1 = blocks[k]
            G, U = _naive_grad(col, rowidx, None, c0, c1, colptr, dual, y, delta, active)
            inflight.append((i, (c0, c1, G, U)))
        while inflight:
            finish(inflight.popleft()[1])
        obj = float(np.log1p(1 / dual).sum() + cfg.l1 * np.abs(w).sum())
        objs.append(obj)
        rel = 1.0 if prev is None else prev / obj - 1
        prev = obj
        kkt_thr = vio[0] / X.shape[0] * cfg.kkt_ratio
        if 0 < rel <= cfg.epsilon:
            if reset:
                break
            reset = True
        else:
            reset = False
    return objs


@pytest.mark.parametrize("data,tau", [("one_hot", 1), ("one_hot", 8), ("groups", 8)])
def test_trainer_matches_max_delay_reference(data, tau):
    """The trainer's bounded block delay IS the reference algorithm at its maximal delay:
    its per-pass objective equals an independent transcription of darlin.h:58-122 /
    206-246 / 381-427 / 480-500 to 1e-6 relative.
    * one_hot: Criteo-shaped slots (39 groups, one key per example each: one block per
      group). At the reference batch config's tau = 8, nine such blocks take their
      Newton steps against the same stale margins (every example is in all of them) and
      the objective of BOTH grows: the divergence is the algorithm's, not the port's.
    * groups: CTR-log-shaped data (120 groups, 8 present per example; the reference's
      batch CTR workload has group ids into the hundreds): blocks in flight share few
      examples and tau = 8 converges."""
    from parameter_server_amd.data.synthetic import criteo_slots, sparse_groups

    if data == "one_hot":
        sd = criteo_slots(3000, seed=7, num_features=10 ** 5)
    else:
        sd = sparse_groups(3000, groups=60, present=6, keys_per_group=2000, seed=2)
    cfg = DarlinConfig(l1=1.0, tau=tau, random_order=False, max_pass=5, epsilon=1e-12, seed=0)
    tr = DarlinTrainer(sd, cfg)
    prog = tr.train()
    X = _design_matrix(sd, tr)
    y = sd.labels.astype(np.float64)
    blocks = [(b.c0, b.c0 + b.ncols) for b in tr.blocks]
    ref = _max_delay_reference(X, y, blocks, list(tr.blk_order), cfg, 5)
    np.testing.assert_allclose([p.objective for p in prog], ref, rtol=1e-6)
    if data == "one_hot" and tau == 8:
        assert ref[-1] > ref[0]  # diverges at the reference's delay on one-hot blocks
    else:
        assert all(b <= a * (1 + 1e-9) for a, b in zip(ref, ref[1:])), ref  # converges
