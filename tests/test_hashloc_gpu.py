"""Sort-free localisation (csrc/hip/hashloc.hip) vs the sort-based localiser."""
import pytest
import torch

from parameter_server_amd.ops.keymix import mix
from parameter_server_amd.ops.linear import linear_backward
from parameter_server_amd.ops.localize import Localizer, localize_torch
from parameter_server_amd.ops.synthetic import criteo_batch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B", [1, 1000, 65536])
def test_hash_localize_matches_sort(B):
    bits = 30
    hl = Localizer(B * 39, bits, "cuda", mode="hash")
    sl = Localizer(B * 39, bits, "cuda", mode="sort")
    for step in range(3):  # epochs: stale entries of earlier steps must be ignored
        keys, _ = criteo_batch(B, seed=step, row0=step * B, num_features=10 ** 9, device="cuda")
        a = hl(keys)
        b = sl(keys)
        U = a.num_unique()
        assert U == b.num_unique()
        ua = a.uniq[:U]
        assert torch.equal(torch.sort(ua).values, b.uniq[:U])
        assert torch.equal(ua[a.local_col.long()], mix(keys, bits))
        assert int(hl.err.item()) == 0
        # backward: identical per-key gradients (fp32 sums in different orders)
        coef = torch.randn(B, device="cuda")
        ga = linear_backward(a, coef, B=B, width=39)[0][:U].clone()
        gb = linear_backward(b, coef, B=B, width=39)[0][:U].clone()
        order = torch.argsort(ua)
        torch.testing.assert_close(ga[order], gb, rtol=1e-5, atol=1e-4)


def test_hash_backward_csr_rows_and_values():
    B, n = 300, 300 * 7
    keys = torch.randint(0, 50, (n,), device="cuda")
    rows = torch.arange(B, device="cuda", dtype=torch.int32).repeat_interleave(7)
    vals = torch.rand(n, device="cuda")
    a = Localizer(n, 20, "cuda", mode="hash")(keys)
    U = a.num_unique()
    coef = torch.randn(B, device="cuda")
    g = linear_backward(a, coef, B=B, rows=rows, vals=vals)[0][:U]
    ref = torch.zeros(U, device="cuda").index_add_(0, a.local_col.long(), coef[rows.long()] * vals)
    torch.testing.assert_close(g, ref, rtol=1e-5, atol=1e-4)


def test_trainer_hash_vs_sort_localize():
    from parameter_server_amd.models import SparseLRConfig, SparseLRTrainer

    res = {}
    for mode in ("hash", "sort"):
        cfg = SparseLRConfig(num_features=10 ** 8, minibatch=4096, table_capacity=1 << 22,
                             localize=mode)
        tr = SparseLRTrainer(cfg, device="cuda")
        assert tr.localize_mode == mode
        for s in range(10):
            k, l = criteo_batch(4096, seed=4, row0=s * 4096, num_features=10 ** 8, device="cuda")
            tr.step(k, l, width=39)
        res[mode] = tr.progress()
    for key in ("loss", "auc", "nnz_w"):
        assert res["hash"][key] == pytest.approx(res["sort"][key], rel=1e-3)
