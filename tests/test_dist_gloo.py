"""Multi-process (gloo, world_size 2) data-plane tests on CPU: the same all-to-all
code path RCCL runs on the GPU node."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir, cfg_kw, steps):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from parameter_server_amd.models import SparseLRConfig, SparseLRTrainer
    from parameter_server_amd.ops.synthetic import criteo_batch
    from parameter_server_amd.parallel.comm import init_from_env

    comm, dev = init_from_env("cpu")
    cfg = SparseLRConfig(**cfg_kw)
    tr = SparseLRTrainer(cfg, comm, dev)
    B = cfg.minibatch
    for s in range(steps):
        k, l = criteo_batch(B, seed=100 + rank, row0=s * B, num_features=cfg.num_features,
                            cards=[200] * 26)
        tr.step(k, l)
    p = tr.progress()
    sd = tr.state_dict()
    torch.save({"progress": p, "state": sd}, os.path.join(out_dir, f"r{rank}.pt"))
    dist.destroy_process_group()


def _run(tmp_path, cfg_kw, steps=4, world=2):
    tmp_path.mkdir(parents=True, exist_ok=True)
    port = _free_port()
    mp.spawn(_worker, args=(world, port, str(tmp_path), cfg_kw, steps), nprocs=world, join=True)
    return [torch.load(tmp_path / f"r{r}.pt", weights_only=False) for r in range(world)]


def _reference(cfg_kw, steps, world, lag=0):
    """Single-process simulation of the protocol: every worker pulls from the same
    model state, then pushes are applied per worker in rank order. ``lag`` = 1: the
    pushes of step s are applied only after the pulls of step s + 1 (SSP, one step
    of staleness: the padded exchange's pipelined mode)."""
    from parameter_server_amd.models import SparseLRConfig
    from parameter_server_amd.ops import KVTable, linear_backward, linear_forward, localize_torch
    from parameter_server_amd.ops.synthetic import criteo_batch

    cfg = SparseLRConfig(**cfg_kw)
    t = KVTable(1 << 16)
    bits = 20
    rule = cfg.update_rule()
    pending = []
    for s in range(steps):
        pushes = []
        for r in range(world):
            k, l = criteo_batch(cfg.minibatch, seed=100 + r, row0=s * cfg.minibatch,
                                num_features=cfg.num_features, cards=[200] * 26)
            loc = localize_torch(k, bits)
            slot, w = t.resolve(loc.uniq)
            _, coef, _ = linear_forward(loc.local_col, w, l, B=cfg.minibatch, width=39)
            g, _ = linear_backward(loc, coef, B=cfg.minibatch, width=39)
            pushes.append((slot, g.clone()))
        pending.append(pushes)
        while len(pending) > lag:
            for slot, g in pending.pop(0):
                t.update(slot, g, rule)
    for pushes in pending:
        for slot, g in pushes:
            t.update(slot, g, rule)
    k, w, _, _ = t.occupied()
    from parameter_server_amd.ops.keymix import unmix

    return dict(zip(unmix(k, bits).tolist(), w.tolist()))


@pytest.mark.parametrize("ff_bytes,exchange,world", [(0, "padded", 2), (0, "exact", 2),
                                                    (3, "padded", 2), (3, "exact", 2),
                                                    (0, "padded", 3), (2, "padded", 3)])
def test_two_rank_training_matches_protocol_reference(tmp_path, ff_bytes, exchange, world):
    cfg_kw = dict(num_features=1 << 20, minibatch=128, table_capacity=1 << 15, l1=0.5,
                  fixing_float_bytes=ff_bytes, exchange=exchange)
    res = _run(tmp_path, cfg_kw, world=world)
    merged = {}
    for r in res:
        st = r["state"]
        for k, w in zip(st["keys"].tolist(), st["w"].tolist()):
            assert k not in merged, "a key lives on exactly one shard"
            merged[k] = w
    assert all(r["progress"]["examples"] == world * 4 * 128 for r in res)
    ref = _reference(cfg_kw, 4, world)
    assert merged.keys() == ref.keys()
    tol = 1e-5 if ff_bytes == 0 else 2e-3
    worst = max(abs(merged[k] - ref[k]) for k in ref)
    assert worst < tol, worst


def _reference_aggregate(cfg_kw, steps, world):
    """Protocol simulation of push_mode="aggregate": every worker pulls the same model,
    the owner sums the workers' gradients per key and applies one update."""
    from parameter_server_amd.models import SparseLRConfig
    from parameter_server_amd.ops import KVTable, linear_backward, linear_forward, localize_torch
    from parameter_server_amd.ops.keymix import unmix
    from parameter_server_amd.ops.synthetic import criteo_batch

    cfg = SparseLRConfig(**cfg_kw)
    t = KVTable(1 << 16)
    rule = cfg.update_rule()
    for s in range(steps):
        slots, grads = [], []
        for r in range(world):
            k, l = criteo_batch(cfg.minibatch, seed=100 + r, row0=s * cfg.minibatch,
                                num_features=cfg.num_features, cards=[200] * 26)
            loc = localize_torch(k, 20)
            slot, w = t.resolve(loc.uniq)
            _, coef, _ = linear_forward(loc.local_col, w, l, B=cfg.minibatch, width=39)
            g, _ = linear_backward(loc, coef, B=cfg.minibatch, width=39)
            slots.append(slot)
            grads.append(g.clone())
        su, inv = torch.unique(torch.cat(slots), return_inverse=True)
        g = torch.zeros(su.numel()).index_add_(0, inv, torch.cat(grads))
        t.update(su, g, rule)
    k, w, _, _ = t.occupied()
    return dict(zip(unmix(k, 20).tolist(), w.tolist()))


@pytest.mark.parametrize("exchange,world,ff", [("padded", 2, 0), ("exact", 2, 0), ("padded", 3, 0),
                                               ("padded", 2, 3)])
def test_aggregate_mode_matches_protocol_reference(tmp_path, exchange, world, ff):
    cfg_kw = dict(num_features=1 << 20, minibatch=128, table_capacity=1 << 15, l1=0.5,
                  push_mode="aggregate", exchange=exchange, fixing_float_bytes=ff)
    res = _run(tmp_path, cfg_kw, world=world)
    merged = {}
    for r in res:
        for k, w in zip(r["state"]["keys"].tolist(), r["state"]["w"].tolist()):
            merged[k] = w
    ref = _reference_aggregate(cfg_kw, 4, world)
    assert merged.keys() == ref.keys()
    tol = 1e-5 if ff == 0 else 2e-3
    assert max(abs(merged[k] - ref[k]) for k in ref) < tol


def test_padded_exchange_overflow_is_loud(tmp_path):
    """A per-peer capacity below the live key count must fail, not silently drop."""
    cfg_kw = dict(num_features=1 << 20, minibatch=128, table_capacity=1 << 15,
                  exchange="padded", exchange_capacity=64)
    with pytest.raises(Exception, match="overflow"):
        _run(tmp_path, cfg_kw, steps=2)


@pytest.mark.parametrize("tau,world,ff,apply,merge", [
    (1, 2, 0, "post", "off"), (2, 2, 0, "post", "off"), (4, 2, 0, "post", "off"),
    (1, 3, 0, "post", "off"), (2, 3, 0, "post", "off"), (4, 3, 0, "post", "off"),
    (4, 2, 3, "post", "off"), (2, 2, 0, "pre", "off"), (4, 3, 0, "pre", "off"),
    # one all-to-all per step (MergedSchedule): lag 1 / 2 apply before the resolve,
    # lag >= 3 after it
    (1, 2, 0, "post", "on"), (2, 2, 0, "post", "on"), (4, 2, 0, "post", "on"),
    (1, 3, 0, "post", "on"), (2, 3, 0, "post", "on"), (3, 3, 0, "post", "on"),
    (4, 3, 0, "post", "on"), (4, 2, 3, "post", "on"), (4, 3, 2, "post", "on")])
def test_ssp_exchange_matches_stale_reference(tmp_path, tau, world, ff, apply, merge):
    """consistency ssp:tau -> the pull of step s sees exactly the pushes of steps
    <= s-1-tau (ring of tau+1 exchange buffers), with the owner applying the carried
    pushes after (post: exchange t carries step t-tau) or before (pre: step t-1-tau)
    resolving the pulls; merge="on": the one-collective schedule, same bound."""
    steps = 7
    cfg_kw = dict(num_features=1 << 20, minibatch=128, table_capacity=1 << 15, l1=0.5,
                  consistency=f"ssp:{tau}", fixing_float_bytes=ff, ssp_apply=apply,
                  exchange_merge=merge)
    res = _run(tmp_path, cfg_kw, steps=steps, world=world)
    merged = {}
    for r in res:
        for k, w in zip(r["state"]["keys"].tolist(), r["state"]["w"].tolist()):
            merged[k] = w
    ref = _reference(cfg_kw, steps, world, lag=tau)
    assert merged.keys() == ref.keys()
    tol = 1e-5 if ff == 0 else 2e-3
    assert max(abs(merged[k] - ref[k]) for k in ref) < tol
    if ff == 0:  # and it differs from the neighbouring staleness (the lag is real)
        other = _reference(cfg_kw, steps, world, lag=tau - 1)
        assert max(abs(merged[k] - other[k]) for k in ref) > 1e-4


def test_explicit_smaller_lag_within_bound(tmp_path):
    """exchange_lag < tau is a legal SSP(tau) schedule with staleness exactly lag."""
    cfg_kw = dict(num_features=1 << 20, minibatch=128, table_capacity=1 << 15, l1=0.5,
                  consistency="ssp:4", exchange_lag=1)
    res = _run(tmp_path, cfg_kw, steps=5, world=2)
    merged = {k: w for r in res for k, w in zip(r["state"]["keys"].tolist(),
                                                 r["state"]["w"].tolist())}
    ref = _reference(cfg_kw, 5, 2, lag=1)
    assert max(abs(merged[k] - ref[k]) for k in ref) < 1e-5
    # (lag 1 is served by the two-collective schedule unless exchange_merge="on")


@pytest.mark.parametrize("merge,lag,algo", [("off", 2, "ftrl"), ("auto", 3, "ftrl"),
                                            ("auto", 2, "sgd"), ("on", 3, "ftrl"),
                                            ("on", 3, "sgd")])
def test_asp_differs_from_ssp1(tmp_path, merge, lag, algo):
    """asp, two collectives: the owner applies the pushes an exchange carries AFTER
    resolving its pulls (on the GPU on its own stream, which pulls never wait for). Run
    in program order (CPU) that is one more step of staleness than ssp:1. On the merged
    one-collective schedule asp is served with staleness exactly 3 (an admissible asp
    schedule); "auto" takes it for FTRL / AdaGrad, plain SGD keeps two collectives."""
    cfg_kw = dict(num_features=1 << 20, minibatch=128, table_capacity=1 << 15, l1=0.5,
                  consistency="asp", exchange_merge=merge, algo=algo)
    if algo == "sgd":
        cfg_kw.update(alpha=0.05)
    res = _run(tmp_path, cfg_kw, steps=6, world=2)
    merged = {k: w for r in res for k, w in zip(r["state"]["keys"].tolist(),
                                                 r["state"]["w"].tolist())}
    ref = _reference(cfg_kw, 6, 2, lag=lag)
    assert max(abs(merged[k] - ref[k]) for k in ref) < 1e-5
    ssp1 = _reference(cfg_kw, 6, 2, lag=1)
    assert max(abs(merged[k] - ssp1[k]) for k in ref) > 1e-4


def test_merged_schedule_rings():
    from parameter_server_amd.parallel.consistency import MergedSchedule

    m = MergedSchedule(4)  # post apply, d = 3
    assert (m.lag, m.post, m.d, m.R) == (4, True, 3, 5)
    assert m.grads_in(10) == 7 and m.grad_ring(7) == 10 % 5 and m.visible_through(10) == 5
    m2 = MergedSchedule(2)  # pre apply, d = 2
    assert (m2.lag, m2.post, m2.d, m2.R) == (2, False, 2, 4)
    a = MergedSchedule(float("inf"))
    assert a.asp and (a.lag, a.d, a.post) == (3, 2, True)
    assert MergedSchedule(4, lag=1).d == 1
    with pytest.raises(ValueError):
        MergedSchedule(0)
    with pytest.raises(ValueError):
        MergedSchedule(2, lag=3)


def test_exchange_schedule_rings():
    from parameter_server_amd.parallel.consistency import ExchangeSchedule

    s = ExchangeSchedule(4, post=False)
    assert (s.lag, s.R, s.asp, s.post) == (4, 5, False, False)
    for t in range(20):  # the send buffer of exchange t holds grads(t-5), written by step t-5
        assert s.grad_ring(t) == (t - 5) % 5 and s.visible_through(t) == t - 5
    assert list(s.pending(exchanged=10, computed=10)) == [5, 6, 7, 8, 9]
    # post apply (ssp default): exchange t carries grads(t-4), applied after its pulls
    p = ExchangeSchedule(4)
    assert (p.lag, p.R, p.post) == (4, 5, True)
    for t in range(20):
        assert p.grad_ring(t) == (t - 4) % 5 and p.visible_through(t) == t - 5
    assert list(p.pending(exchanged=10, computed=10)) == [6, 7, 8, 9]
    assert not ExchangeSchedule(0).post and not ExchangeSchedule(float("inf")).post
    b = ExchangeSchedule(0)
    assert (b.lag, b.R) == (0, 2) and b.visible_through(3) == 2
    a = ExchangeSchedule(float("inf"), asp_depth=3)
    assert a.asp and a.lag == 1 and a.R == 5 and a.apply_gate(7) == 4 and a.apply_gate(1) is None
    assert list(a.pending(exchanged=10, computed=10)) == [8, 9]
    with pytest.raises(ValueError):
        ExchangeSchedule(2, lag=3)


@pytest.mark.parametrize("world,ff", [(2, 0), (3, 0), (2, 2)])
def test_tail_filter_padded_matches_exact(tmp_path, world, ff):
    """tail_feature_freq on the sync-free padded exchange (device CountMin insert /
    query + keep-mask compaction) trains the same weights as the host-synchronous
    exact path (reference MinibatchReader::read, sgd.h:131-150)."""
    base = dict(num_features=1 << 20, minibatch=128, table_capacity=1 << 15, l1=0.5,
                tail_feature_freq=1, countmin_n=1 << 16, fixing_float_bytes=ff)
    res_p = _run(tmp_path / "p", dict(base, exchange="padded"), steps=5, world=world)
    res_e = _run(tmp_path / "e", dict(base, exchange="exact"), steps=5, world=world)
    wp = {k: w for r in res_p for k, w in zip(r["state"]["keys"].tolist(), r["state"]["w"].tolist())}
    we = {k: w for r in res_e for k, w in zip(r["state"]["keys"].tolist(), r["state"]["w"].tolist())}
    assert wp.keys() == we.keys()
    tol = 1e-5 if ff == 0 else 2e-3
    assert max(abs(wp[k] - we[k]) for k in we) < tol
    # the filter is live: fewer keys than without it
    res_n = _run(tmp_path / "n", dict(base, tail_feature_freq=0), steps=5, world=world)
    assert sum(r["state"]["keys"].numel() for r in res_n) > len(wp)


@pytest.mark.parametrize("tau,xd", [(4, 2), (2, 1), (3, 2), (4, 1)])
def test_merged_pipeline_order_matches_two_collective(tau, xd):
    """bench.py's merged pipeline issue order, in program order on the CPU (loopback
    exchange, 2 emulated peers): exchanges -1 .. xd-1 first, then per iteration the
    worker half of step t and exchange t+xd; mx_drain at the end. Leaves the table of
    the two-collective sequential trainer (same staleness bound) on every trained key."""
    from parameter_server_amd.models import SparseLRConfig, SparseLRTrainer
    from parameter_server_amd.ops.synthetic import criteo_batch
    from parameter_server_amd.parallel.comm import LoopbackComm

    B, N, T = 256, 1 << 20, 9
    batches = [criteo_batch(B, seed=9, row0=m * B, num_features=N, cards=[200] * 26)
               for m in range(T + xd + 2)]

    def trainer(merge):
        cfg = SparseLRConfig(num_features=N, minibatch=B, consistency=f"ssp:{tau}",
                             table_capacity=1 << 16, l1=0.5, exchange_merge=merge)
        return SparseLRTrainer(cfg, LoopbackComm(2), "cpu")

    tr = trainer("on")
    assert tr.merged and xd <= tr.msched.d
    locs = {}

    def loc(m):
        if m not in locs:
            locs[m] = tr.localize(batches[m][0], buf=m % 4)
        return locs[m]

    def issue(s):
        parts = tr.mx_exchange(s, loc(s + 1))
        parts["pack"]()
        parts["comm"]()
        if parts["post"]:
            parts["resolve"]()
            parts["apply"]()
        else:
            parts["apply"]()
            parts["resolve"]()
        tr._mx_next = s + 1

    for s in range(-1, xd):
        issue(s)
    for t in range(T):
        tr.mx_worker(t, loc(t), batches[t][1], width=39)()
        tr.mx_done(B)
        issue(t + xd)
    tr.mx_drain()
    ref = trainer("off")
    for m in range(T):
        ref.step(batches[m][0], batches[m][1], width=39)
    ref.flush()
    k1, w1, _, _ = tr.table.occupied()
    k2, w2, _, _ = ref.table.occupied()
    a = dict(zip(k1.tolist(), w1.tolist()))
    b = dict(zip(k2.tolist(), w2.tolist()))
    assert set(b) <= set(a)  # (the pipeline also pulled the minibatches issued ahead)
    assert max(abs(a[k] - b[k]) for k in b) < 1e-6
    assert all(a[k] == 0 for k in set(a) - set(b))
