"""Fused per-tile forward + backward on a "tp" localisation (tploc.hip tp_fwd_bwd)
against the plain PyTorch fp32 reference of the same step (margins, dL/dm, loss /
accuracy / AUC histogram, gradient per unique key)."""
import pytest
import torch

from parameter_server_amd.ops.linear import (AUC_BINS, linear_fwd_bwd, loss_terms_torch,
                                             new_accum, accum_total)
from parameter_server_amd.ops.localize import Localizer, ensure_local_col
from parameter_server_amd.ops.synthetic import criteo_batch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _reference(keys_cols, w, labels, B, width, vals):
    """Plain torch: margins from local columns, logistic terms, scatter-add grads."""
    col = keys_cols.long()
    x = vals if vals is not None else torch.ones_like(w[col])
    m = (w[col] * x).reshape(B, width).double().sum(1).float()
    lo, c, _ = loss_terms_torch(m, labels, 2)
    g = torch.zeros_like(w).index_add_(0, col, (c.repeat_interleave(width) * x))
    return m, c, lo, g


@pytest.mark.parametrize("B,width,with_vals", [(65536, 39, False), (20011, 39, True),
                                               (5000, 16, False), (3001, 60, True), (7001, 9, False)])
def test_tp_fused_matches_reference(B, width, with_vals):
    if width == 39:
        keys, labels = criteo_batch(B, seed=3, row0=0, num_features=10 ** 9, device=DEV)
    else:
        g = torch.Generator(device="cpu").manual_seed(width)
        keys = (torch.randint(0, 1 << 20, (B * width,), generator=g) ** 2 % 1000003).to(DEV)
        labels = torch.where(torch.rand(B, generator=g) < 0.3, 1.0, -1.0).to(DEV)
    n = keys.numel()
    loc = Localizer(n, 30, DEV, mode="tp", lazy_cols=True)
    assert loc.mode == "tp"
    L = loc(keys)
    U = int(L.n_uniq.item())
    w = (torch.randn(U, device=DEV) * 0.05)
    vals = torch.rand(n, device=DEV) + 0.5 if with_vals else None
    coef = torch.empty(B, device=DEV)
    metrics = new_accum(DEV)
    hist = torch.zeros(8 * 2 * AUC_BINS, dtype=torch.int32, device=DEV)
    c_f, g_f = linear_fwd_bwd(L, w, labels, B=B, width=width, vals=vals, coef=coef,
                              metrics=metrics, hist=hist)
    torch.cuda.synchronize()
    assert not L.tile.cols_ready  # the fused path never materialised local columns
    cols = ensure_local_col(L)[:n]
    m, c, lo, g = _reference(cols, w, labels, B, width, vals)
    torch.testing.assert_close(c_f[:B], c, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(g_f[:U], g, rtol=1e-3, atol=1e-4)
    tot = accum_total(metrics).cpu()
    assert abs(float(tot[0]) - float(lo.double().sum())) < 1e-3 * B
    y = labels > 0
    assert int(tot[1]) == pytest.approx(int(((m > 0) == y).sum()), abs=3)
    assert int(tot[2]) == B
    h = hist.view(-1, 2 * AUC_BINS).sum(0).cpu()
    assert int(h.sum()) == B and int(h[AUC_BINS:].sum()) == int(y.sum())


def test_tp_fused_falls_back_for_variable_rows():
    """A CSR minibatch (row_ptr) on a lazy tp localisation takes the unfused path,
    which materialises the local columns first."""
    B, width = 4096, 39
    keys, labels = criteo_batch(B, seed=5, row0=0, num_features=10 ** 9, device=DEV)
    loc = Localizer(keys.numel(), 30, DEV, mode="tp", lazy_cols=True)
    L = loc(keys)
    U = int(L.n_uniq.item())
    w = torch.randn(U, device=DEV) * 0.05
    row_ptr = torch.arange(0, B + 1, device=DEV, dtype=torch.int64) * width
    rows = torch.arange(B, device=DEV, dtype=torch.int32).repeat_interleave(width)
    c_f, g_f = linear_fwd_bwd(L, w, labels, B=B, row_ptr=row_ptr, rows=rows)
    assert L.tile.cols_ready
    m, c, lo, g = _reference(L.local_col[:B * width], w, labels, B, width, None)
    torch.testing.assert_close(c_f[:B], c, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(g_f[:U], g, rtol=1e-3, atol=1e-4)


def test_tp_fused_fixed_point_partials_are_deterministic_and_exact():
    """The per-tile entry partials accumulate in 64-bit fixed point with integer LDS
    atomics: repeated runs give bitwise identical partials whatever the atomic order,
    and the gradient matches an fp64 scatter-add to ~1 ulp. (The entry scan combines
    runs cut by a wave boundary with float atomics into the gradient the localiser
    zeroed, so the gradient is compared from the first run only.)"""
    B, width = 65536, 39
    keys, labels = criteo_batch(B, seed=9, row0=0, num_features=10 ** 9, device=DEV)
    n = keys.numel()
    L = Localizer(n, 30, DEV, mode="tp", lazy_cols=True)(keys)
    U = int(L.n_uniq.item())
    w = torch.randn(U, device=DEV) * 0.05
    outs, parts = [], []
    for _ in range(3):
        c_f, g_f = linear_fwd_bwd(L, w, labels, B=B, width=width, coef=torch.empty(B, device=DEV))
        outs.append(g_f[:U].clone())
        parts.append(L.tile.psum.clone())
    # bitwise (as int32: entries past a tile's count are never written, and uninitialised
    # memory may hold NaN patterns, which torch.equal on floats reports as unequal)
    assert all(torch.equal(parts[0].view(torch.int32), p.view(torch.int32)) for p in parts[1:])
    cols = ensure_local_col(L)[:n].long()
    m = w[cols].reshape(B, width).double().sum(1).float()
    _, c, _ = loss_terms_torch(m, labels, 2)
    g64 = torch.zeros(U, dtype=torch.float64, device=DEV).index_add_(
        0, cols, c.double().repeat_interleave(width))
    # exactly rounded tile partials, then an fp32 scan over <= 312 tiles per key
    torch.testing.assert_close(outs[0].double(), g64, rtol=1e-5, atol=1e-6)


def test_kv_update_folds_the_auc_epilogue():
    """kv_update(..., hist=, metrics=, step_counter=) computes the step's bucketed AUC in
    its block 0 exactly like auc_from_hist, zeroes the histogram and ticks the clock."""
    from parameter_server_amd.ops.kv_table import KVTable, UpdateRule
    from parameter_server_amd.ops.linear import HIST_STRIPES, auc_from_hist
    from parameter_server_amd.ops.native import hipops

    g = torch.Generator(device="cpu").manual_seed(4)
    hist = torch.randint(0, 50, (HIST_STRIPES * 2 * AUC_BINS,), generator=g,
                         dtype=torch.int32).to(DEV)
    h2 = hist.clone()
    m_ref, m_new = new_accum(DEV), new_accum(DEV)
    s_ref = torch.zeros(1, dtype=torch.int64, device=DEV)
    s_new = torch.zeros(1, dtype=torch.int64, device=DEV)
    auc_from_hist(h2, m_ref, s_ref)
    t = KVTable(1 << 12, DEV)
    keys = torch.arange(1, 1001, dtype=torch.int64, device=DEV)
    slot, _ = t.resolve(keys)
    grad = torch.randn(1000, device=DEV)
    stats = new_accum(DEV)
    rule = UpdateRule("ftrl", "decay", 0.01, 10.0, 1.0, 1.0)
    hipops().kv_update(t.slots, slot, grad, None, *rule.args(), stats, hist=hist,
                       metrics=m_new, step_counter=s_new)
    torch.cuda.synchronize()
    assert int(hist.abs().sum()) == 0 and int(s_new.item()) == 1
    torch.testing.assert_close(accum_total(m_new)[3:5], accum_total(m_ref)[3:5], rtol=0, atol=0)
    # the update itself is unchanged
    t2 = KVTable(1 << 12, DEV)
    slot2, _ = t2.resolve(keys)
    hipops().kv_update(t2.slots, slot2, grad, None, *rule.args(), new_accum(DEV))
    # (concurrent inserts may place colliding keys differently: compare by key)
    a, b = t.occupied(), t2.occupied()
    oa, ob = torch.argsort(a[0]), torch.argsort(b[0])
    for x, y in zip(a, b):
        assert torch.equal(x[oa], y[ob])


@pytest.mark.parametrize("algo", ["ftrl", "adagrad", "sgd"])
def test_fused_seg_update_matches_scan_then_update(algo, monkeypatch):
    """1 GPU: the entry scan that applies the optimizer update itself (tp_seg_update,
    hot keys combined by piece counting) trains the same table as tp_seg_reduce +
    kv_update: same keys, weights and state to float rounding, same metrics."""
    from parameter_server_amd.models import SparseLRConfig, SparseLRTrainer
    from parameter_server_amd.models.sparse_lr import algo_defaults

    B = 16384
    outs = []
    monkeypatch.setenv("PSAMD_FLAT", "0")  # the compact tp path (the flat one: test_tpf_gpu.py)
    for fused in ("1", "0"):
        monkeypatch.setenv("PSAMD_FUSED_UPDATE", fused)
        cfg = SparseLRConfig(num_features=10 ** 8, minibatch=B, table_capacity=1 << 22, algo=algo,
                             **algo_defaults(algo))
        tr = SparseLRTrainer(cfg, device=DEV)
        assert tr.localize_mode == "tp"
        for t in range(6):
            k, lab = criteo_batch(B, seed=21, row0=t * B, num_features=cfg.num_features,
                                  device=DEV)
            tr.step(k, lab, width=39)
        p = tr.progress()
        keys, w, z, n = tr.table.occupied()
        o = torch.argsort(keys)
        outs.append((p, keys[o].cpu(), w[o].cpu(), z[o].cpu(), n[o].cpu()))
    (pa, ka, wa, za, na), (pb, kb, wb, zb, nb) = outs
    assert torch.equal(ka, kb)
    torch.testing.assert_close(wa, wb, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(za, zb, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(na, nb, rtol=1e-4, atol=1e-4)
    assert pa["examples"] == pb["examples"] == 6 * B
    assert pa["loss"] == pytest.approx(pb["loss"], rel=1e-4)
    assert pa["auc"] == pytest.approx(pb["auc"], abs=1e-3)
    assert pa["nnz_w"] == pytest.approx(pb["nnz_w"], abs=3)


def test_native_step_plan_matches_op_by_op(monkeypatch):
    """1 GPU: the step issued from the validate-once native LaunchList (_step_plan) runs
    the launches the op-by-op path issues: the same keys, and weights / state / metrics
    equal to float rounding (hot keys combine their chunk pieces through atomics, whose
    order varies from run to run)."""
    from parameter_server_amd.models import SparseLRConfig, SparseLRTrainer

    B = 16384
    outs = []
    monkeypatch.setenv("PSAMD_FLAT", "0")  # the compact tp path's launch list
    for native in (True, False):
        cfg = SparseLRConfig(num_features=10 ** 8, minibatch=B, table_capacity=1 << 22)
        tr = SparseLRTrainer(cfg, device=DEV)
        if not native:
            tr._step_plan = lambda *a, **k: None
        keys = torch.empty(B * 39, dtype=torch.int64, device=DEV)
        labels = torch.empty(B, dtype=torch.float32, device=DEV)
        for t in range(5):
            criteo_batch(B, seed=4, row0=t * B, num_features=cfg.num_features, device=DEV,
                         keys=keys, labels=labels)
            tr.step(keys, labels, width=39)
        if native:
            assert len(tr._plans) == 1  # one plan, replayed every step
        p = tr.progress()
        k, w, z, n = tr.table.occupied()
        o = torch.argsort(k)
        outs.append((p, k[o].cpu(), w[o].cpu(), z[o].cpu(), n[o].cpu()))
    (pa, ka, wa, za, na), (pb, kb, wb, zb, nb) = outs
    assert torch.equal(ka, kb)
    torch.testing.assert_close(wa, wb, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(za, zb, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(na, nb, rtol=1e-4, atol=1e-4)
    assert pa["examples"] == pb["examples"] == 5 * B
    assert pa["loss"] == pytest.approx(pb["loss"], rel=1e-4)
    assert pa["auc"] == pytest.approx(pb["auc"], abs=1e-3)
