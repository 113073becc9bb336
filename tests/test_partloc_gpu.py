"""Partition + per-bucket LDS dedup localisation (csrc/hip/partloc.hip) against the
plain-PyTorch localisation: identical unique keys, segment starts, local columns and
segment ids; the CSC order may permute positions inside a key's segment only."""
import pytest
import torch

from parameter_server_amd.ops.localize import Localizer, localize_torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _check(k, bits, with_hess=False):
    n = k.numel()
    ref = localize_torch(k, bits)
    lz = Localizer(n + 5, bits, DEV, with_hess=with_hess, mode="part")
    assert lz.mode == "part"
    loc = lz(k.to(DEV))
    lz.check()
    U = loc.num_unique()
    assert U == ref.uniq.numel()
    assert torch.equal(loc.uniq[:U].cpu(), ref.uniq)
    assert torch.equal(loc.seg_start[:U + 1].cpu(), ref.seg_start)
    assert torch.equal(loc.local_col.cpu(), ref.local_col)
    assert torch.equal(loc.segid.cpu(), ref.segid)
    pos = loc.pos_s.cpu().long()
    assert torch.equal(torch.sort(pos).values, torch.arange(n))  # a permutation
    assert torch.equal(ref.local_col[pos].long() + 1, ref.segid.long())  # grouped by key
    assert torch.all(loc.grad[:U].cpu() == 0)
    if with_hess:
        assert torch.all(loc.hess[:U].cpu() == 0)


@pytest.mark.parametrize("bits,n", [(30, 1), (30, 1000), (30, 100003), (20, 300000), (8, 5000),
                                    (32, 2000000), (27, 65536 * 39), (30, 65536 * 39)])
def test_partloc_matches_torch(bits, n):
    g = torch.Generator().manual_seed(n + bits)
    k = torch.randint(0, 1 << min(bits + 4, 62), (n,), generator=g, dtype=torch.int64)
    if n > 10:
        k[::3] = k[0]       # a heavy hitter: one bucket holds a third of the batch
        k[1::7] = k[1]
    _check(k, bits, with_hess=(n == 100003))


def test_partloc_criteo_batch():
    from parameter_server_amd.ops.synthetic import criteo_batch

    keys, _ = criteo_batch(65536, seed=3, row0=0, num_features=10 ** 9, device=DEV)
    _check(keys.cpu(), 30)


def test_partloc_all_distinct():
    n = 65536 * 39
    k = torch.randperm(1 << 22)[:n].to(torch.int64) * 97 + 11
    _check(k, 30)
