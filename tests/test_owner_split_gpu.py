"""owner_split (csrc/hip/localize.hip, 256-ary search per bound) against
torch.searchsorted: offsets[g] = lower_bound(uniq[:U], bounds[g]), offsets[G] = U."""
import pytest
import torch

from parameter_server_amd.ops.native import hipops

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("U", [0, 1, 200, 256, 257, 65_537, 233_866, 1_000_003])
@pytest.mark.parametrize("G", [1, 2, 3, 8])
def test_owner_split_matches_searchsorted(U, G):
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(U * 31 + G)
    cap = max(U, 1) + 17  # buffer longer than the device count
    keys = torch.randint(0, 1 << 30, (cap,), generator=g, dtype=torch.int64)
    keys[:U] = torch.sort(torch.unique(keys[:U]))[0].repeat(2)[:U].sort()[0]  # duplicates ok
    bounds = torch.tensor([(i << 30) // G for i in range(G)] + [1 << 30], dtype=torch.int64)
    if G > 2:  # a bound below every key and one above every key
        bounds[1] = 0
        bounds[G - 1] = 1 << 30
    n = torch.tensor([U], dtype=torch.int32, device=dev)
    off = torch.empty(G + 1, dtype=torch.int64, device=dev)
    hipops().owner_split(keys.to(dev), n, bounds.to(dev), off)
    torch.cuda.synchronize()
    want = torch.searchsorted(keys[:U], bounds[:G], right=False).tolist() + [U]
    want[0] = 0
    assert off.cpu().tolist() == want
