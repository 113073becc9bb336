"""HIP kernels vs plain-PyTorch fp32 (or exact C++ host) references of the same op."""
import pytest
import torch

from parameter_server_amd.ops import (CountMinSketch, KVTable, Localizer, UpdateRule,
                                      exact_auc, linear_backward, linear_forward, localize_torch)
from parameter_server_amd.ops import fixing_float as ff
from parameter_server_amd.ops.keymix import mix, unmix
from parameter_server_amd.ops.linear import AUC_BINS, auc_from_hist
from parameter_server_amd.ops.native import hipops
from parameter_server_amd.ops.synthetic import criteo_batch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_extension_is_native():
    h = hipops()
    assert h.__file__.endswith(".so")


@pytest.mark.parametrize("bits", [20, 30, 64])
def test_mix_roundtrip_gpu_vs_cpu(bits):
    g = torch.Generator().manual_seed(bits)
    hi = (1 << bits) if bits < 63 else (1 << 62)
    k = torch.randint(0, hi, (100000,), generator=g, dtype=torch.int64)
    if bits == 64:
        k[:10] = torch.tensor([-2, -1 - (1 << 40), 0, 1, 2, 3, 4, 5, 6, 7])
    hc = mix(k, bits)
    hg = mix(k.to(DEV), bits).cpu()
    assert torch.equal(hc, hg)
    assert torch.equal(unmix(hg.to(DEV), bits).cpu(), k)


@pytest.mark.parametrize("bits,n", [(30, 200000), (64, 50000), (12, 30000), (30, 2600000),
                                    (64, 1500000), (7, 5000),
                                    # 33..40 bits: 4 x 10-bit passes (sort40), then >= 2^22
                                    # keys on the generic u64 sort
                                    (34, 200000), (33, 5001), (40, 1000003), (34, 1),
                                    (36, 2555904), (34, 4200000)])
def test_localize_matches_torch(bits, n):
    g = torch.Generator().manual_seed(n)
    hi = min(1 << bits, 1 << 62)
    k = torch.randint(0, hi, (n,), generator=g, dtype=torch.int64)
    k[::3] = k[0]  # heavy hitter
    ref = localize_torch(k, bits)
    loc = Localizer(n + 17, bits, DEV)(k.to(DEV))
    U = loc.num_unique()
    assert U == ref.uniq.numel()
    assert torch.equal(loc.uniq[:U].cpu(), ref.uniq)
    assert torch.equal(loc.seg_start[:U + 1].cpu(), ref.seg_start)
    assert torch.equal(loc.local_col.cpu(), ref.local_col)
    assert torch.equal(loc.pos_s.cpu(), ref.pos_s)  # LSD radix sort is stable
    assert torch.equal(loc.segid.cpu(), ref.segid)


@pytest.mark.parametrize("n,end_bit", [(1, 30), (2047, 30), (2048, 12), (2049, 64),
                                       (100003, 30), (3000000, 30), (777777, 64)])
def test_radix_sort_pairs_matches_stable_torch_sort(n, end_bit):
    g = torch.Generator().manual_seed(n)
    hi = (1 << end_bit) if end_bit < 63 else (1 << 62)
    k = torch.randint(0, hi, (n,), generator=g, dtype=torch.int64)
    if end_bit == 64 and n > 10:
        k[:5] = torch.tensor([-1, -2, -(1 << 62), 0, 5])  # top bit set: unsigned order
        k[5:10] = -1  # duplicates of the max key
    v = torch.arange(n, dtype=torch.int32)
    kd, vd = k.to(DEV), v.to(DEV)
    ko = torch.empty_like(kd)
    vo = torch.empty_like(vd)
    H = hipops()
    temp = torch.empty(H.sort_pairs_temp_bytes(n, end_bit), dtype=torch.uint8, device=DEV)
    H.sort_pairs(temp, kd, ko, vd, vo, n, end_bit)
    order_key = k ^ torch.tensor(-(1 << 63)) if end_bit == 64 else k
    _, perm = torch.sort(order_key, stable=True)
    assert torch.equal(ko.cpu(), k[perm])
    assert torch.equal(vo.cpu(), v[perm])


@pytest.mark.parametrize("n", [1, 5, 2048, 2049, 1000003])
def test_device_scan_i32(n):
    x = torch.randint(0, 3, (n,), dtype=torch.int32)
    H = hipops()
    temp = torch.empty(H.scan_temp_bytes(n), dtype=torch.uint8, device=DEV)
    out = torch.empty(n, dtype=torch.int32, device=DEV)
    H.inclusive_scan_i32(temp, x.to(DEV), out, n)
    assert torch.equal(out.cpu(), torch.cumsum(x, 0).to(torch.int32))


def _ref_update(w, z, n, cnt, g, rule):
    import math

    a, b, l1, l2 = rule.alpha, rule.beta, rule.l1, rule.l2

    def prox(zz, eta):
        leta = l1 * eta
        out = torch.where(zz.abs() <= leta, torch.zeros_like(zz),
                          (zz - torch.sign(zz) * leta) / (1 + l2 * eta))
        return out

    if rule.algo == "ftrl":
        n_new = torch.sqrt(n * n + g * g)
        sigma = (n_new - n) / a
        z = z + g - sigma * w
        eta = torch.full_like(n_new, a) if rule.lr_type == "constant" else a / (n_new + b)
        return prox(-z * eta, eta), z, n_new, cnt
    if rule.algo == "adagrad":
        n = n + g * g
        eta = a / (b + torch.sqrt(n))
        return prox(w - eta * g, eta), z, n, cnt
    cnt = cnt + 1
    eta = torch.full_like(w, a) if rule.lr_type == "constant" else a / (b + torch.sqrt(cnt))
    return prox(w - eta * g, eta), z, n, cnt


@pytest.mark.parametrize("algo,lr", [("ftrl", "decay"), ("ftrl", "constant"),
                                     ("adagrad", "decay"), ("sgd", "decay"), ("sgd", "constant")])
def test_kv_update_matches_torch(algo, lr):
    torch.manual_seed(0)
    n = 5000
    rule = UpdateRule(algo, lr, alpha=0.1, beta=1.0, l1=0.05, l2=0.5)
    t = KVTable(1 << 14, DEV)
    keys = torch.unique(torch.randint(0, 1 << 40, (2 * n,), dtype=torch.int64))[:n]
    keys = keys[torch.randperm(n)].to(DEV)
    slot, w0 = t.resolve(keys, insert=True)
    assert (slot >= 0).all() and torch.unique(slot).numel() == n
    assert (w0 == 0).all()
    w = torch.zeros(n); z = torch.zeros(n); nn = torch.zeros(n); c = torch.zeros(n)
    stats = torch.zeros(3, dtype=torch.float64, device=DEV)
    for it in range(5):
        g = torch.randn(n) * 0.3
        t.update(slot, g.to(DEV), rule, stats)
        w, z, nn, c = _ref_update(w, z, nn, c, g, rule)
    got = t.gather(slot, 0).cpu()
    torch.testing.assert_close(got, w, rtol=2e-5, atol=2e-6)
    if algo == "ftrl":
        torch.testing.assert_close(t.gather(slot, 1).cpu(), z, rtol=2e-5, atol=2e-6)
    slot2, w2 = t.resolve(keys, insert=False)
    assert torch.equal(slot2, slot)
    torch.testing.assert_close(w2.cpu(), w, rtol=2e-5, atol=2e-6)
    occ, nnz = t.census()
    assert occ == n and nnz == int((w != 0).sum())
    assert abs(float(stats[0].item()) - nnz) < 0.5


def test_kv_resolve_concurrent_duplicates_and_missing():
    t = KVTable(1 << 12, DEV)
    keys = torch.arange(1000, dtype=torch.int64).repeat(7)[torch.randperm(7000)].to(DEV)
    slot, _ = t.resolve(keys, insert=True)
    # every occurrence of a key got the same slot; distinct keys distinct slots
    pairs = torch.unique(torch.stack([keys, slot]).T.cpu(), dim=0)
    assert pairs.shape[0] == 1000
    assert torch.unique(pairs[:, 1]).numel() == 1000
    miss, _ = t.resolve(torch.tensor([123456789], device=DEV), insert=False)
    assert int(miss.item()) == -1
    assert t.census()[0] == 1000


def test_kv_table_matches_cpu_table_values():
    rule = UpdateRule("ftrl", "decay", alpha=0.05, beta=1.0, l1=0.01, l2=0.1)
    keys = torch.randint(0, 1 << 30, (3000,), dtype=torch.int64).unique()
    g = torch.randn(keys.numel())
    out = []
    for dev in ("cpu", DEV):
        t = KVTable(1 << 13, dev)
        s, _ = t.resolve(keys.to(dev))
        t.update(s, g.to(dev), rule)
        t.update(s, (g * 0.5).to(dev), rule)
        out.append(t.gather(s).cpu())
    torch.testing.assert_close(out[0], out[1], rtol=1e-5, atol=1e-6)


def test_aggregate_mode_sums_duplicates():
    rule = UpdateRule("sgd", "constant", alpha=1.0, beta=0.0)
    t = KVTable(1 << 10, DEV)
    keys = torch.tensor([5, 6, 7], device=DEV)
    s, _ = t.resolve(keys)
    slot = torch.cat([s, s[:2]])
    g = torch.tensor([1.0, 2.0, 3.0, 10.0, 20.0], device=DEV)
    touched = torch.empty(16, dtype=torch.int64, device=DEV)
    nt = torch.zeros(1, dtype=torch.int32, device=DEV)
    H = hipops()
    H.kv_accumulate(t.slots, slot, g, None, touched, nt)
    assert int(nt.item()) == 3
    H.kv_apply_accumulated(t.slots, touched[:5], nt, *rule.args(), None)
    torch.testing.assert_close(t.gather(s).cpu(), torch.tensor([-11.0, -22.0, -3.0]))


@pytest.mark.parametrize("loss", ["logit", "square", "hinge", "square_hinge"])
@pytest.mark.parametrize("valued", [False, True])
def test_linear_fwd_bwd_matches_torch(loss, valued):
    torch.manual_seed(1)
    B, W = 3000, 39
    keys = torch.randint(0, 5000, (B * W,), dtype=torch.int64)
    labels = torch.where(torch.rand(B) < 0.3, 1.0, -1.0)
    vals = torch.rand(B * W) if valued else None
    ref = localize_torch(keys, 30, with_hess=True)
    U = ref.uniq.numel()
    w_local = torch.randn(U) * 0.1
    m_ref = torch.zeros(8, dtype=torch.float64)
    h_ref = torch.zeros(2 * AUC_BINS, dtype=torch.int32)
    xw_r, c_r, c2_r = linear_forward(ref.local_col, w_local, labels, B=B, width=W, vals=vals,
                                     loss=loss, metrics=m_ref, hist=h_ref)
    linear_backward(ref, c_r, B=B, width=W, vals=vals, coef2=c2_r)
    loc = Localizer(B * W, 30, DEV, with_hess=True)(keys.to(DEV))
    m = torch.zeros(8, dtype=torch.float64, device=DEV)
    h = torch.zeros(2 * AUC_BINS, dtype=torch.int32, device=DEV)
    xw = torch.empty(B, device=DEV)
    c = torch.empty(B, device=DEV)
    c2 = torch.empty(B, device=DEV)
    vd = vals.to(DEV) if valued else None
    linear_forward(loc.local_col, w_local.to(DEV), labels.to(DEV), B=B, width=W, vals=vd,
                   loss=loss, xw=xw, coef=c, coef2=c2, metrics=m, hist=h)
    torch.testing.assert_close(xw.cpu(), xw_r, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(c.cpu(), c_r, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(c2.cpu(), c2_r, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(m.cpu()[:3], m_ref[:3], rtol=1e-6, atol=1e-3)
    assert torch.equal(h.cpu(), h_ref) or (h.cpu() - h_ref).abs().sum() <= 4
    linear_backward(loc, c, B=B, width=W, vals=vd, coef2=c2)
    torch.testing.assert_close(loc.grad[:U].cpu(), ref.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(loc.hess[:U].cpu(), ref.hess, rtol=1e-4, atol=1e-4)


def test_linear_bwd_with_row_ptr():
    torch.manual_seed(2)
    B = 500
    lens = torch.randint(1, 80, (B,))
    row_ptr = torch.zeros(B + 1, dtype=torch.int64)
    row_ptr[1:] = torch.cumsum(lens, 0)
    nnz = int(row_ptr[-1])
    keys = torch.randint(0, 300, (nnz,), dtype=torch.int64)
    labels = torch.where(torch.rand(B) < 0.5, 1.0, -1.0)
    vals = torch.rand(nnz)
    ref = localize_torch(keys, 20)
    U = ref.uniq.numel()
    w = torch.randn(U)
    _, c_r, _ = linear_forward(ref.local_col, w, labels, B=B, row_ptr=row_ptr, vals=vals)
    rows = torch.repeat_interleave(torch.arange(B), lens).to(torch.int32)
    linear_backward(ref, c_r, B=B, rows=rows, vals=vals)
    loc = Localizer(nnz, 20, DEV)(keys.to(DEV))
    c = torch.empty(B, device=DEV)
    linear_forward(loc.local_col, w.to(DEV), labels.to(DEV), B=B, row_ptr=row_ptr.to(DEV),
                   vals=vals.to(DEV), coef=c)
    rows_d = torch.empty(nnz, dtype=torch.int32, device=DEV)
    hipops().csr_rows(row_ptr.to(DEV), rows_d)
    assert torch.equal(rows_d.cpu(), rows)
    linear_backward(loc, c, B=B, rows=rows_d, vals=vals.to(DEV))
    torch.testing.assert_close(loc.grad[:U].cpu(), ref.grad, rtol=1e-4, atol=1e-4)


def test_bucketed_auc_close_to_exact():
    torch.manual_seed(3)
    n = 20000
    y = torch.where(torch.rand(n) < 0.3, 1.0, -1.0)
    s = torch.randn(n) + 0.8 * (y > 0)
    hist = torch.zeros(2 * AUC_BINS, dtype=torch.int32, device=DEV)
    p = torch.sigmoid(s)
    b = torch.clamp((p * AUC_BINS).long(), 0, AUC_BINS - 1) + torch.where(y > 0, AUC_BINS, 0)
    hist += torch.bincount(b, minlength=2 * AUC_BINS).to(torch.int32).to(DEV)
    m = torch.zeros(8, dtype=torch.float64, device=DEV)
    auc_from_hist(hist, m)
    assert abs(float(m[3]) - exact_auc(s, y)) < 2e-3
    assert int(hist.sum().item()) == 0


def test_countmin_gpu_equals_cpu():
    torch.manual_seed(4)
    keys = torch.randint(0, 1 << 40, (20000,), dtype=torch.int64)
    counts = torch.randint(1, 200, (20000,), dtype=torch.int64).to(torch.uint8)
    cms = [CountMinSketch(4096, 3, d) for d in ("cpu", DEV)]
    for cm in cms:
        cm.insert(keys.to(cm.device), counts.to(cm.device))
        cm.insert(keys[:5000].to(cm.device))
    assert torch.equal(cms[0].cells, cms[1].cells.cpu())
    k0, c0 = cms[0].query(keys, 3)
    k1, c1 = cms[1].query(keys.to(DEV), 3)
    assert torch.equal(k0, k1.cpu()) and torch.equal(c0, c1.cpu())


def test_countmin_partitioned_gpu_equals_cpu():
    """The trainers' partitioned sketch (regions by mixed-key range): GPU kernels = the
    CPU reference, cell for cell."""
    torch.manual_seed(6)
    bits = 30
    keys = torch.randint(0, 1 << bits, (30000,), dtype=torch.int64)
    counts = torch.randint(1, 200, (30000,), dtype=torch.int64).to(torch.uint8)
    cms = [CountMinSketch(1 << 18, 2, d, key_bits=bits) for d in ("cpu", DEV)]
    for cm in cms:
        cm.insert(keys.to(cm.device), counts.to(cm.device))
        cm.insert(keys[:7000].to(cm.device))
    assert torch.equal(cms[0].cells, cms[1].cells.cpu())
    k0, c0 = cms[0].query(keys, 3)
    k1, c1 = cms[1].query(keys.to(DEV), 3)
    assert torch.equal(k0, k1.cpu()) and torch.equal(c0, c1.cpu())


@pytest.mark.parametrize("nbytes", [1, 2, 3])
def test_fixing_float_roundtrip(nbytes):
    torch.manual_seed(5)
    x = torch.randn(100000, device=DEV)
    code, mm = ff.encode(x, nbytes, seed=7)
    y = ff.decode(code, nbytes, mm)
    step = float(mm[1] - mm[0]) / ((1 << (8 * nbytes)) - 2)
    ulp = 2.4e-7 * float(x.abs().max())  # fp32 rounding of the decoded value
    assert float((y - x).abs().max()) <= step * 1.0001 + ulp
    assert abs(float((y - x).mean())) < step * 0.02 + ulp  # unbiased stochastic rounding
    code_c, _ = ff.encode(x.cpu(), nbytes, mm=mm.cpu(), seed=7)
    yc = ff.decode(code_c, nbytes, mm.cpu())
    assert float((yc - x.cpu()).abs().max()) <= step * 1.0001 + ulp


def test_key_signature_cpu_gpu():
    k = torch.randint(0, 1 << 62, (777,), dtype=torch.int64)
    assert ff.key_signature(k) == ff.key_signature(k.to(DEV))
    k2 = k.clone()
    k2[[3, 4]] = k2[[4, 3]]
    assert ff.key_signature(k2.to(DEV)) != ff.key_signature(k.to(DEV))


def test_criteo_gen_gpu_matches_cpu():
    kg, lg = criteo_batch(64, seed=11, row0=100, num_features=10 ** 9, device=DEV)
    kc, lc = criteo_batch(64, seed=11, row0=100, num_features=10 ** 9)
    assert float((kg.cpu() == kc).float().mean()) > 0.97
    assert float((lg.cpu() == lc).float().mean()) > 0.9
    assert int(kg.min()) >= 0 and int(kg.max()) < 10 ** 9


@pytest.mark.gpu
def test_criteo_gen_advances_its_device_cursor():
    """criteo_batch(row0_dev=A, row0_out=B): the kernel generates rows row0 + A * scale
    and writes A + 1 into B; alternating the two words (A -> B, B -> A: a captured graph
    pair) generates rows row0 + k * scale for k = c, c + 1, c + 2, ..."""
    from parameter_server_amd.ops.synthetic import criteo_batch

    dev = torch.device("cuda")
    B = 3000
    ctr = torch.tensor([5, -1], dtype=torch.int64, device=dev)
    for i, k in enumerate((5, 6, 7)):
        a = i % 2
        keys, labels = criteo_batch(B, seed=3, row0=11, num_features=10 ** 9, device=dev,
                                    row0_dev=ctr[a:a + 1], row_scale=B,
                                    row0_out=ctr[1 - a:2 - a])
        rk, rl = criteo_batch(B, seed=3, row0=11 + k * B, num_features=10 ** 9, device=dev)
        assert torch.equal(keys, rk) and torch.equal(labels, rl)
    assert ctr.tolist() == [7, 8]
    # the same through graph replays: two captured launches alternating the words
    ctr = torch.tensor([2, -1], dtype=torch.int64, device=dev)
    kb = [torch.empty(B * 39, dtype=torch.int64, device=dev) for _ in range(2)]
    lb = [torch.empty(B, dtype=torch.float32, device=dev) for _ in range(2)]
    gs = []
    for a in range(2):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            criteo_batch(B, seed=3, row0=11, num_features=10 ** 9, device=dev, keys=kb[a],
                         labels=lb[a], row0_dev=ctr[a:a + 1], row_scale=B,
                         row0_out=ctr[1 - a:2 - a])
        gs.append(g)
    for i, k in enumerate((2, 3, 4, 5)):
        gs[i % 2].replay()
        rk, rl = criteo_batch(B, seed=3, row0=11 + k * B, num_features=10 ** 9, device=dev)
        assert torch.equal(kb[i % 2], rk) and torch.equal(lb[i % 2], rl)
