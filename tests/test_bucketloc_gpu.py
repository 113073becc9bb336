"""Bucketed localisation (csrc/hip/bucketloc.hip) against the plain-PyTorch
localiser: unique keys, local columns, segment starts and segment ids must match
exactly; positions must match as a set within every key's segment (their order
inside a segment is not deterministic)."""
import pytest
import torch

from parameter_server_amd.ops.keymix import unmix
from parameter_server_amd.ops.localize import Localizer, localize_torch
from parameter_server_amd.ops.synthetic import criteo_batch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _check(k, bits, with_hess=False):
    n = k.numel()
    ref = localize_torch(k, bits)
    lz = Localizer(n + 5, bits, DEV, mode="bucket", with_hess=with_hess)
    assert lz.mode == "bucket"
    loc = lz(k.to(DEV))
    U = loc.num_unique()
    assert U == ref.uniq.numel()
    assert torch.equal(loc.uniq[:U].cpu(), ref.uniq)
    assert torch.equal(loc.seg_start[:U + 1].cpu(), ref.seg_start)
    assert torch.equal(loc.local_col.cpu(), ref.local_col)
    assert torch.equal(loc.segid.cpu(), ref.segid)
    # positions: same multiset inside each segment
    seg = ref.segid.long()
    canon = lambda p: torch.sort(seg * (n + 1) + p.long())[0]  # noqa: E731
    assert torch.equal(canon(loc.pos_s.cpu()), canon(ref.pos_s))
    assert float(loc.grad[:U].abs().sum()) == 0.0
    if with_hess:
        assert float(loc.hess[:U].abs().sum()) == 0.0
    return loc


@pytest.mark.parametrize("bits,n", [(30, 200000), (12, 30000), (30, 2600000), (7, 5000),
                                    (20, 1), (32, 300000), (16, 70000), (24, 9999)])
def test_bucket_localize_matches_torch(bits, n):
    g = torch.Generator().manual_seed(n + bits)
    k = torch.randint(0, 1 << bits, (n,), generator=g, dtype=torch.int64)
    if n > 3:
        k[::3] = k[0]  # heavy hitter: one bucket holds a third of the keys
    _check(k, bits)


def test_bucket_localize_criteo_batch_and_hess():
    k, _ = criteo_batch(65536, seed=3, row0=0, num_features=10**9)
    _check(k, 30, with_hess=True)


def test_bucket_localize_many_uniques_in_one_subrange():
    """> kCntCap (3584) distinct keys inside one bucket sub-range (chunked counts)
    and several sub-ranges per bucket (bits = 32 -> 4 sub-ranges of 2^18)."""
    bits = 32
    g = torch.Generator().manual_seed(0)
    low = torch.randperm(1 << 18, generator=g)[:9000].to(torch.int64)
    mixed = (7 << 20) | (1 << 18) | low               # bucket 7, sub-range 1
    other = (7 << 20) | (3 << 18) | low[:500]          # same bucket, sub-range 3
    rnd = torch.randint(0, 1 << 32, (20000,), generator=g, dtype=torch.int64)
    raw_mixed = torch.cat([mixed, mixed[:100], other, rnd])
    k = unmix(raw_mixed, bits)
    _check(k[torch.randperm(k.numel(), generator=g)], bits)


def test_bucket_localize_workspace_reuse():
    lz = Localizer(100000, 30, DEV, mode="bucket")
    for s in range(3):
        k, _ = criteo_batch(2000, seed=s, row0=s * 2000, num_features=10**9)
        ref = localize_torch(k, 30)
        loc = lz(k.to(DEV))
        U = loc.num_unique()
        assert torch.equal(loc.uniq[:U].cpu(), ref.uniq)
        assert torch.equal(loc.local_col.cpu(), ref.local_col)


def test_trainer_bucket_mode_matches_sort_mode():
    from parameter_server_amd.models import SparseLRConfig, SparseLRTrainer

    res = {}
    for mode in ("sort", "bucket"):
        cfg = SparseLRConfig(num_features=10**9, minibatch=4096, algo="ftrl", lr_type="decay",
                             alpha=0.01, beta=10.0, l1=1.0, l2=1.0, localize=mode,
                             table_capacity=1 << 20)
        tr = SparseLRTrainer(cfg, device=DEV)
        for s in range(5):
            k, l = criteo_batch(4096, seed=1, row0=s * 4096, num_features=10**9, device=DEV)
            tr.step(k, l)
        res[mode] = tr.progress()
    a, b = res["sort"], res["bucket"]
    assert abs(a["loss"] - b["loss"]) < 1e-4 * max(1.0, abs(a["loss"]))
    assert a["nnz_w"] == b["nnz_w"]
