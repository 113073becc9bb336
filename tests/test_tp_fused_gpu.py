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
