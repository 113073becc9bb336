"""Tile-deduplicating localisation (csrc/hip/tileloc.hip + sort32.hip device-count
sort) against the plain-PyTorch localiser: unique keys and local columns must
match exactly; the backward (per-tile LDS partial sums + segmented reduction over
the sorted entries) must match the fp32 index_add reference."""
import pytest
import torch

from parameter_server_amd.ops.linear import linear_backward
from parameter_server_amd.ops.localize import Localizer, localize_torch
from parameter_server_amd.ops.synthetic import criteo_batch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ref_grad(ref, coef, width, rows=None, vals=None):
    n = ref.local_col.numel()
    r = rows.long() if rows is not None else torch.arange(n) // width
    x = vals if vals is not None else torch.ones(n)
    g = torch.zeros(ref.uniq.numel(), dtype=torch.float64)
    g.index_add_(0, ref.local_col.long(), (coef.double()[r] * x.double()))
    return g


def _check(k, bits, width, cap=None, rows=None, vals=None):
    n = k.numel()
    ref = localize_torch(k, bits)
    lz = Localizer(cap or n, bits, DEV, mode="tile")
    assert lz.mode == "tile"
    loc = lz(k.to(DEV))
    U = loc.num_unique()
    assert U == ref.uniq.numel()
    assert torch.equal(loc.uniq[:U].cpu(), ref.uniq)
    assert torch.equal(loc.local_col.cpu(), ref.local_col)
    B = (n + width - 1) // width if rows is None else int(rows.max()) + 1
    g = torch.Generator().manual_seed(n)
    coef = torch.randn(B, generator=g)
    grad, _ = linear_backward(loc, coef.to(DEV), B=B, width=width,
                              rows=None if rows is None else rows.to(DEV),
                              vals=None if vals is None else vals.to(DEV))
    want = _ref_grad(ref, coef, width, rows, vals)
    got = grad[:U].double().cpu()
    assert torch.allclose(got, want, rtol=1e-4, atol=1e-3), (got - want).abs().max()
    return loc


@pytest.mark.parametrize("bits,n", [(30, 200000), (12, 30000), (30, 2555904), (7, 5000),
                                    (20, 1), (31, 300000), (16, 70001), (24, 9999)])
def test_tile_localize_matches_torch(bits, n):
    g = torch.Generator().manual_seed(n + bits)
    k = torch.randint(0, 1 << bits, (n,), generator=g, dtype=torch.int64)
    if n > 3:
        k[::3] = k[0]  # heavy hitter
    _check(k, bits, width=1)


def test_tile_localize_criteo_batch():
    k, _ = criteo_batch(65536, seed=3, row0=0, num_features=10**9)
    _check(k, 30, width=39)


def test_tile_localize_csr_rows_and_values():
    k, _ = criteo_batch(3000, seed=5, row0=0, num_features=10**6)
    n = k.numel()
    rows = (torch.arange(n) // 39).to(torch.int32)
    vals = torch.rand(n, generator=torch.Generator().manual_seed(1))
    _check(k, 20, width=0, rows=rows, vals=vals)


def test_tile_localize_workspace_reuse_and_smaller_batches():
    lz = Localizer(39 * 5000, 30, DEV, mode="tile")
    for s, B in enumerate([5000, 1234, 4096, 77]):
        k, _ = criteo_batch(B, seed=s, row0=s * B, num_features=10**9)
        ref = localize_torch(k, 30)
        loc = lz(k.to(DEV))
        U = loc.num_unique()
        assert U == ref.uniq.numel()
        assert torch.equal(loc.uniq[:U].cpu(), ref.uniq)
        assert torch.equal(loc.local_col.cpu(), ref.local_col)


def test_trainer_tile_mode_matches_sort_mode():
    from parameter_server_amd.models import SparseLRConfig, SparseLRTrainer

    res = {}
    for mode in ("sort", "tile"):
        cfg = SparseLRConfig(num_features=10**8, minibatch=8192, table_capacity=1 << 22,
                             localize=mode)
        tr = SparseLRTrainer(cfg, device=DEV)
        for s in range(4):
            k, lab = criteo_batch(8192, seed=9, row0=s * 8192, num_features=10**8, device=DEV)
            tr.step(k, lab, width=39)
        torch.cuda.synchronize()
        keys, w, _, _ = tr.table.occupied()
        order = torch.argsort(keys)
        res[mode] = (keys[order].cpu(), w[order].cpu(), tr.progress())
    assert torch.equal(res["sort"][0], res["tile"][0])
    assert torch.allclose(res["sort"][1], res["tile"][1], rtol=1e-4, atol=1e-6)
    assert abs(res["sort"][2]["loss"] - res["tile"][2]["loss"]) < 1e-5


@pytest.mark.parametrize("hot", [0, 1500, 50000])
def test_sort_backward_hot_keys_matches_reference(hot):
    """CSC segmented backward with hot keys: segments spanning hundreds of
    wavefronts combine their per-wave pieces atomically."""
    g = torch.Generator().manual_seed(hot + 7)
    n = 200000
    k = torch.randint(0, 1 << 30, (n,), generator=g, dtype=torch.int64)
    if hot:
        idx = torch.randperm(n, generator=g)[:hot]
        k[idx] = 12345
        k[idx[: hot // 3]] = 777  # a second hot key
    ref = localize_torch(k, 30)
    loc = Localizer(n, 30, DEV, mode="sort")(k.to(DEV))
    width = 39
    B = (n + width - 1) // width
    coef = torch.randn(B, generator=g)
    grad, _ = linear_backward(loc, coef.to(DEV), B=B, width=width)
    U = loc.num_unique()
    want = _ref_grad(ref, coef, width)
    assert torch.allclose(grad[:U].double().cpu(), want, rtol=1e-4, atol=1e-3)
