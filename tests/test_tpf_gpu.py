"""Flat 1-GPU layout (Localizer mode "tpf", csrc/hip/tploc.hip tpf_*): the localisation
covers every occurrence exactly, and the fused 1-GPU step built on it (pull issued in the
previous step's update launch, fused forward + tile backward, per-bucket fixed-point
gradient sums + optimizer update) trains the table a plain-PyTorch fp32 FTRL / AdaGrad /
SGD loop trains (torch.unique, index_add, the reference's per-key update,
src/app/linear_method/async_sgd.h:107-119)."""
import math

import pytest
import torch

from parameter_server_amd.models import SparseLRConfig, SparseLRTrainer
from parameter_server_amd.models.sparse_lr import algo_defaults
from parameter_server_amd.ops.keymix import key_bits_for, mix, unmix
from parameter_server_amd.ops.localize import TP_TILE, Localizer
from parameter_server_amd.ops.native import hipops
from parameter_server_amd.ops.synthetic import criteo_batch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _skewed_batch(step: int, bits: int = 20, B: int = 2048, width: int = 16):
    """A minibatch whose first bucket pair overflows the bucket kernel's LDS capacity:
    1500 distinct keys in each of the pair's two fine buckets, every one of them in the
    first two 8192-occurrence tiles (6000 entries > 4064), so the pair falls back to its
    two fine buckets as separate units. Raw keys (the trainer mixes them)."""
    g = torch.Generator().manual_seed(100 + step)
    n = B * width
    shift = bits - 5  # n = 32768 -> 32 fine buckets
    k0 = torch.randperm(1 << shift, generator=g)[:1500]
    k1 = (1 << shift) + torch.randperm(1 << shift, generator=g)[:1500]
    hot = torch.cat([k0, k1])
    mixed = torch.randint(1 << (shift + 1), 1 << bits, (n,), generator=g)
    for t in range(2):
        pos = t * TP_TILE + torch.randperm(TP_TILE, generator=g)[:hot.numel()]
        mixed[pos] = hot
    keys = unmix(mixed.to(DEV), bits)
    labels = torch.where(torch.rand(B, generator=g) < 0.3, 1.0, -1.0).to(DEV)
    return keys, labels


def _overflow_batch(B: int = 2048, width: int = 16, bits: int = 20):
    """A minibatch that no flat bucket unit can hold: 2500 distinct keys of the first
    fine bucket (> the 2048-key unit hash) in each of the 4 tiles (10,000 entries > the
    8192-entry region)."""
    g = torch.Generator().manual_seed(5)
    n = B * width
    shift = bits - 5
    hot = torch.randperm(1 << shift, generator=g)[:2500]
    mixed = torch.randint(1 << (shift + 1), 1 << bits, (n,), generator=g)
    for t in range(n // TP_TILE):
        pos = t * TP_TILE + torch.randperm(TP_TILE, generator=g)[:hot.numel()]
        mixed[pos] = hot
    keys = unmix(mixed.to(DEV), bits)
    labels = torch.where(torch.rand(B, generator=g) < 0.3, 1.0, -1.0).to(DEV)
    return keys, labels


def _tile(n: int) -> int:
    """Occurrences per tile of the flat layout for an n-key minibatch (tp_flat_lts)."""
    from parameter_server_amd.ops.native import hipops

    return 1 << hipops().tpf_tile_log2(n)


def test_flat_localizer_overflow_fails_loudly(monkeypatch):
    """A localisation overflow (entries dropped from the flat regions) must not train
    silently: progress() and check_ok() raise."""
    monkeypatch.setenv("PSAMD_FLAT", "1")
    monkeypatch.setenv("PSAMD_TILE_LTS", "13")  # (the batch is built for 8192-key tiles)
    keys, labels = _overflow_batch()
    B = labels.numel()
    cfg = SparseLRConfig(num_features=1 << 20, minibatch=B, max_nnz_per_example=16,
                         table_capacity=1 << 22)
    tr = SparseLRTrainer(cfg, device=DEV)
    assert tr.localize_mode == "tpf"
    tr.step(keys, labels, width=16)
    torch.cuda.synchronize()
    assert int(tr.localizer.err.item()) != 0
    with pytest.raises(RuntimeError, match="localize_tpf overflow"):
        tr.progress()
    with pytest.raises(RuntimeError, match="overflow"):
        tr.check_ok()


def _flat_entry_keys(f, n):
    """tile entry id -> mixed key, from the flat regions (host side)."""
    H = hipops()
    G = H.tpf_groups(n, f.bits)
    kr, er = H.tpf_key_region(), H.tpf_entry_region()
    cnt = f.cnt[:4 * G].view(G, 4).cpu()
    uq = f.uniqf[:G * kr].view(G, 2, kr // 2).cpu()
    pos = f.ent_pos[:G * er].view(G, er).cpu()
    jj = f.ent_j[:G * er].view(G, er).cpu().to(torch.int64) & 0xFFFF
    ent_key = {}
    for b in range(G):
        e0 = int(cnt[b, 1])
        for s in range(2):
            D, E = int(cnt[b, 2 * s]), int(cnt[b, 2 * s + 1])
            base = 0 if s == 0 else e0
            p = pos[b, base:base + E]
            j = jj[b, base:base + E]
            assert E == 0 or int(j.max()) < D
            ks = uq[b, s, j]
            ent_key.update(zip(p.tolist(), ks.tolist()))
    return ent_key, cnt


@pytest.mark.parametrize("case", ["criteo", "uniform", "few"])
def test_tpf_sorted_units_are_key_ordered(case):
    """sorted_keys=True (the multi-GPU exchange rows): every unit's keys strictly
    increase (binned rank order for units of > 64 keys, the O(D^2) scan below), the
    entry map still gives every occurrence its own key, and the key set equals the
    unsorted localisation's."""
    if case == "criteo":
        keys, _ = criteo_batch(65536, seed=21, row0=0, num_features=10 ** 9, device=DEV)
        bits = 30
    elif case == "uniform":  # ~2000 distinct keys per unit: the densest bins
        keys, bits = torch.randint(0, 1 << 34, (400_000,), device=DEV), 34
    else:  # <= 64 keys in the one unit: the O(D^2) path
        keys, bits = torch.randint(0, 1 << 30, (60,), device=DEV), 30
    n = keys.numel()
    fs = Localizer(n, bits, DEV, mode="tpf", sorted_keys=True)(keys)
    torch.cuda.synchronize()
    assert int(fs.err.item()) == 0
    H = hipops()
    G, kr = H.tpf_groups(n, bits), H.tpf_key_region()
    cnt = fs.cnt[:4 * G].view(G, 4).cpu()
    uq = fs.uniqf[:G * kr].view(G, 2, kr // 2).cpu()
    big = 0
    for b in range(G):
        for s in range(2):
            D = int(cnt[b, 2 * s])
            u = uq[b, s, :D]
            assert D < 2 or bool((u[1:] > u[:-1]).all()), (b, s)
            big += D > 64
    assert (big > 0) == (case != "few")
    mk = mix(keys, bits).cpu()
    ent_key, _ = _flat_entry_keys(fs, n)
    rep = fs.rep[:n].cpu().to(torch.int64) & 0xFFFF
    eid = ((torch.arange(n) // _tile(n)) * TP_TILE + rep).tolist()
    assert torch.equal(torch.tensor([ent_key[e] for e in eid]), mk)
    fu = Localizer(n, bits, DEV, mode="tpf")(keys)
    assert torch.equal(fs.unique_keys().sort().values, fu.unique_keys().sort().values)


@pytest.mark.parametrize("case", ["criteo", "criteo_small", "uniform", "skewed", "small_in_big"])
def test_tpf_localisation_covers_every_occurrence(case, monkeypatch):
    """Every occurrence's tile entry maps (ent_pos / ent_j / uniqf) to its own mixed key,
    every distinct key appears once, and each tile's entry count is its distinct-key
    count (tiles of 2^tpf_tile_log2(n) occurrences: 8192 at the driver's B, 1024 for
    criteo_small, 2048 for the 400 k uniform keys)."""
    if case == "criteo":
        B, bits = 65536, 30
        keys, _ = criteo_batch(B, seed=11, row0=0, num_features=10 ** 9, device=DEV)
    elif case == "criteo_small":
        B, bits = 3000, 30
        keys, _ = criteo_batch(B, seed=12, row0=0, num_features=10 ** 9, device=DEV)
    elif case == "small_in_big":  # a workspace sized for the driver's B takes B = 10,000,
        B, bits = 10000, 30       # whose 2048-key tiles are 191 (vs 313 tiles of 8192)
        keys, _ = criteo_batch(B, seed=13, row0=0, num_features=10 ** 9, device=DEV)
    elif case == "uniform":  # nearly all distinct: the densest buckets
        bits = 34
        keys = torch.randint(0, 1 << 34, (400_000,), device=DEV)
    else:
        bits = 20
        monkeypatch.setenv("PSAMD_TILE_LTS", "13")  # (built for 8192-key tiles)
        keys, _ = _skewed_batch(0, bits)
    n = keys.numel()
    ts = _tile(n)
    assert ts == {"criteo": 8192, "criteo_small": 1024, "uniform": 2048, "skewed": 8192,
                  "small_in_big": 2048}[case]
    lz = Localizer(65536 * 39 if case == "small_in_big" else n, bits, DEV, mode="tpf")
    assert lz.mode == "tpf"
    f = lz(keys)
    torch.cuda.synchronize()
    assert int(f.err.item()) == 0
    mk = mix(keys, bits).cpu()
    ent_key, cnt = _flat_entry_keys(f, n)
    rep = f.rep[:n].cpu().to(torch.int64) & 0xFFFF
    tile = torch.arange(n) // ts
    eid = (tile * TP_TILE + rep).tolist()
    got = torch.tensor([ent_key[e] for e in eid])
    assert torch.equal(got, mk)
    uq = f.unique_keys()
    assert uq.numel() == torch.unique(mk).numel() == torch.unique(uq).numel()
    T = (n + ts - 1) // ts
    dc = f.dcnt[:T].cpu()
    for t in range(T):
        assert int(dc[t]) == torch.unique(mk[t * ts:(t + 1) * ts]).numel()
    if case == "skewed":  # the overflowing pair ran as two fine units
        assert cnt[0].tolist() == [1500, 3000, 1500, 3000]


def _reference_train(batches, rule, bits):
    """Plain PyTorch fp32 FTRL / AdaGrad / SGD over raw keys, one update per minibatch
    (the per-key rules of kv_slot.cuh apply_update)."""
    allk = torch.unique(torch.cat([k.cpu() for k, _ in batches]))
    K = allk.numel()
    W, Z, Nn, C = (torch.zeros(K) for _ in range(4))
    for keys, labels in batches:
        k, y = keys.cpu(), labels.cpu()
        B = y.numel()
        width = k.numel() // B
        idx = torch.searchsorted(allk, k)
        m = W[idx].view(B, width).double().sum(1).float()
        yy = torch.where(y > 0, 1.0, -1.0)
        coef = -yy * torch.sigmoid(-yy * m)
        g = torch.zeros(K, dtype=torch.float64).index_add_(
            0, idx, coef.double().repeat_interleave(width)).float() * rule.grad_scale
        u = torch.unique(idx)
        gu, w_old = g[u], W[u]
        if rule.algo == "ftrl":
            n_new = torch.sqrt(Nn[u] * Nn[u] + gu * gu)
            sigma = (n_new - Nn[u]) / rule.alpha
            Z[u] = Z[u] + gu - sigma * w_old
            Nn[u] = n_new
            eta = rule.alpha / (n_new + rule.beta)
            zz = -Z[u] * eta
        elif rule.algo == "adagrad":
            Nn[u] = Nn[u] + gu * gu
            eta = rule.alpha / (rule.beta + torch.sqrt(Nn[u]))
            zz = w_old - eta * gu
        else:
            C[u] += 1
            eta = rule.alpha / (rule.beta + torch.sqrt(C[u]))
            zz = w_old - eta * gu
        leta = rule.l1 * eta
        W[u] = torch.where(zz.abs() <= leta, torch.zeros_like(zz),
                           (zz - torch.sign(zz) * leta) / (1 + rule.l2 * eta))
    return allk, W, Z, Nn


def _table_by_raw_key(tr, allk):
    keys, w, z, n = tr.table.occupied()
    raw = unmix(keys, tr.bits).cpu()
    o = torch.argsort(raw)
    raw, w, z, n = raw[o], w.cpu()[o], z.cpu()[o], n.cpu()[o]
    assert torch.equal(raw, allk)  # exactly the keys seen
    return w, z, n


@pytest.mark.parametrize("mode,algo,B,cap", [
    ("tpf", "ftrl", 16384, 1 << 22), ("tpf", "adagrad", 16384, 1 << 22),
    ("tpf", "sgd", 16384, 1 << 22), ("tp", "ftrl", 16384, 1 << 22),
    # the reference operating point (online_l1lr.conf minibatch: 10,000): 2048-key tiles
    ("tpf", "ftrl", 10000, 1 << 22),
    # the driver's shape: B = 65,536 on the 2^31-slot (64 GiB) table of 10^9 features
    ("tpf", "ftrl", 65536, 1 << 31)])
def test_fused_1gpu_step_matches_fp32_reference(mode, algo, B, cap, monkeypatch):
    """5 fused 1-GPU steps (flat: pulls issued ahead via next_loc; tp: resolve + fused
    forward/backward + fused scan/update) against the fp32 PyTorch loop on the same
    keys: weights, z and n to rtol 1e-4."""
    monkeypatch.setenv("PSAMD_FLAT", "1" if mode == "tpf" else "0")
    steps = 5
    cfg = SparseLRConfig(num_features=10 ** 8 if cap < (1 << 31) else 10 ** 9, minibatch=B,
                         table_capacity=cap, algo=algo, **algo_defaults(algo))
    tr = SparseLRTrainer(cfg, device=DEV)
    assert tr.localize_mode == mode
    batches = [criteo_batch(B, seed=31, row0=t * B, num_features=cfg.num_features, device=DEV)
               for t in range(steps)]
    if mode == "tpf":
        loc = tr.localize(batches[0][0], buf=0)
        for t in range(steps):
            nxt = tr.localize(batches[t + 1][0], buf=(t + 1) % 2) if t + 1 < steps else None
            tr.step(batches[t][0], batches[t][1], width=39, loc=loc, next_loc=nxt)
            loc = nxt
    else:
        for k, lab in batches:
            tr.step(k, lab, width=39)
    torch.cuda.synchronize()
    p = tr.progress()
    assert p["examples"] == steps * B
    allk, W, Z, Nn = _reference_train(batches, cfg.update_rule(), tr.bits)
    w, z, n = _table_by_raw_key(tr, allk)
    torch.testing.assert_close(w, W, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(z, Z, rtol=1e-4, atol=1e-4)
    if algo != "sgd":
        torch.testing.assert_close(n, Nn, rtol=1e-4, atol=1e-4)
    assert (w != 0).sum() > 100  # the comparison covers trained weights, not only zeros


def test_flat_step_overflow_units_match_reference(monkeypatch):
    """Minibatches whose first bucket pair overflows (two fine units per workgroup, the
    tpf_unit_light path) train like the fp32 reference."""
    monkeypatch.setenv("PSAMD_FLAT", "1")
    monkeypatch.setenv("PSAMD_TILE_LTS", "13")  # (the batches are built for 8192-key tiles)
    bits = 20
    batches = [_skewed_batch(s, bits) for s in range(3)]
    B = batches[0][1].numel()
    cfg = SparseLRConfig(num_features=1 << bits, minibatch=B, max_nnz_per_example=16,
                         table_capacity=1 << 22, l1=0.1, l2=0.1, alpha=0.1)
    tr = SparseLRTrainer(cfg, device=DEV)
    assert tr.localize_mode == "tpf" and tr.bits == bits
    for k, lab in batches:
        tr.step(k, lab, width=16)
    torch.cuda.synchronize()
    assert int(tr.localizer.err.item()) == 0
    allk, W, Z, Nn = _reference_train(batches, cfg.update_rule(), bits)
    w, z, n = _table_by_raw_key(tr, allk)
    torch.testing.assert_close(w, W, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(z, Z, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(n, Nn, rtol=1e-4, atol=1e-4)


def test_flat_near_distinct_pairs_match_reference(monkeypatch):
    """Near-distinct keys (uniform over 10^8, ~1024 occurrences per fine bucket): the bucket
    pairs overflow their 2048-key hash, and each runs as two fine units (the LDS build per
    fine bucket); 3 steps train like the fp32 reference."""
    monkeypatch.setenv("PSAMD_FLAT", "1")
    B = (1 << 20) // 39  # n just under 2^20: 1024 buckets of ~1024 occurrences
    N = 10 ** 8
    g = torch.Generator(device=DEV)
    g.manual_seed(5)
    batches = [(torch.randint(0, N, (B * 39,), device=DEV, generator=g),
                torch.where(torch.rand(B, device=DEV, generator=g) < 0.3, 1.0, -1.0))
               for _ in range(3)]
    cfg = SparseLRConfig(num_features=N, minibatch=B, table_capacity=1 << 23)
    tr = SparseLRTrainer(cfg, device=DEV)
    assert tr.localize_mode == "tpf"
    f = tr.localizer(batches[0][0])
    torch.cuda.synchronize()
    assert int(f.err.item()) == 0
    H = hipops()
    G = H.tpf_groups(f.nnz, f.bits)
    c = f.cnt[:4 * G].view(G, 4).cpu()
    assert int((c[:, 2] > 0).sum()) > G // 2  # most pairs ran as two units
    uq = f.unique_keys()
    assert uq.numel() == torch.unique(mix(batches[0][0], tr.bits)).numel()
    for k, lab in batches:
        tr.step(k, lab, width=39)
    torch.cuda.synchronize()
    tr.check_ok()
    allk, W, Z, Nn = _reference_train(batches, cfg.update_rule(), tr.bits)
    w, z, n = _table_by_raw_key(tr, allk)
    torch.testing.assert_close(w, W, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(z, Z, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(n, Nn, rtol=1e-4, atol=1e-4)


def test_flat_pull_ahead_is_bitwise_the_plain_step(monkeypatch):
    """A pull issued ahead inside the previous step's update launch (next_loc) gives the
    same table, bitwise, as pulling at the step; a pull issued for a minibatch that is
    then NOT the next step (or whose buffer was refilled) is not used."""
    monkeypatch.setenv("PSAMD_FLAT", "1")
    B = 8192
    outs = []
    batches = [criteo_batch(B, seed=41, row0=t * B, num_features=10 ** 9, device=DEV)
               for t in range(6)]
    for variant in ("ahead", "plain", "stale"):
        cfg = SparseLRConfig(num_features=10 ** 9, minibatch=B, table_capacity=1 << 22)
        tr = SparseLRTrainer(cfg, device=DEV)
        if variant == "ahead":
            loc = tr.localize(batches[0][0], buf=0)
            for t in range(6):
                nxt = tr.localize(batches[t + 1][0], buf=(t + 1) % 2) if t < 5 else None
                tr.step(batches[t][0], batches[t][1], width=39, loc=loc, next_loc=nxt)
                loc = nxt
        elif variant == "plain":
            for k, lab in batches:
                tr.step(k, lab, width=39)
        else:  # pulls issued ahead for a buffer that is refilled before its step
            for t in range(6):
                loc = tr.localize(batches[t][0], buf=0)
                other = tr.localize(batches[(t + 3) % 6][0], buf=1)
                tr.step(batches[t][0], batches[t][1], width=39, loc=loc, next_loc=other)
        p = tr.progress()
        k, w, z, n = tr.table.occupied()
        o = torch.argsort(k)
        outs.append((p, k[o].cpu(), w[o].cpu(), z[o].cpu(), n[o].cpu()))
    for other in outs[1:]:
        for a, b in zip(outs[0][1:], other[1:]):
            assert torch.equal(a, b)
        # (the loss sum takes float LDS atomics in any order: equal to rounding)
        assert outs[0][0]["loss"] == pytest.approx(other[0]["loss"], rel=1e-6)


def test_flat_gaussian_init_matches_compact(monkeypatch):
    """Non-zero initial weights (inserted in the flat pull) train like the compact path."""
    outs = []
    B = 8192
    from parameter_server_amd.ops.kv_table import InitRule

    for flat in ("1", "0"):
        monkeypatch.setenv("PSAMD_FLAT", flat)
        cfg = SparseLRConfig(num_features=10 ** 8, minibatch=B, table_capacity=1 << 22,
                             init=InitRule("gaussian", 0.0, 0.01, 7))
        tr = SparseLRTrainer(cfg, device=DEV)
        for t in range(4):
            k, lab = criteo_batch(B, seed=51, row0=t * B, num_features=cfg.num_features, device=DEV)
            tr.step(k, lab, width=39)
        k, w, z, n = tr.table.occupied()
        o = torch.argsort(k)
        outs.append((k[o].cpu(), w[o].cpu(), z[o].cpu(), n[o].cpu()))
    assert torch.equal(outs[0][0], outs[1][0])
    for a, b in zip(outs[0][1:], outs[1][1:]):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)


def test_prep_plan_generates_and_localises_like_the_ops():
    """The native preparation launch list (generator with a row cursor + tile + flat
    bucket) yields the rows and localisation of criteo_batch + Localizer."""
    B = 4096
    cfg = SparseLRConfig(num_features=10 ** 9, minibatch=B, table_capacity=1 << 20)
    tr = SparseLRTrainer(cfg, device=DEV)
    keys = torch.empty(B * 39, dtype=torch.int64, device=DEV)
    labels = torch.empty(B, dtype=torch.float32, device=DEV)
    run = tr.prep_plan(1, keys, labels, seed=77, row0=3 * B, row_step=5 * B,
                       num_features=cfg.num_features)
    for r in range(3):
        f = run()
        k2, l2 = criteo_batch(B, seed=77, row0=(3 + 5 * r) * B, num_features=cfg.num_features,
                              device=DEV)
        assert torch.equal(keys, k2) and torch.equal(labels, l2)
        assert f.gen == r + 1 and f.nnz == B * 39
        ref = Localizer(B * 39, tr.bits, DEV, mode="tpf")(k2)
        # (tile entry numbers depend on the LDS-hash insert order: compare what they
        # mean, every occurrence's key, and the per-bucket counts)
        n = B * 39
        ek, _ = _flat_entry_keys(f, n)
        rep = f.rep[:n].cpu().to(torch.int64) & 0xFFFF
        eid = ((torch.arange(n) // _tile(n)) * TP_TILE + rep).tolist()
        assert torch.equal(torch.tensor([ek[e] for e in eid]), mix(k2, tr.bits).cpu())
        assert torch.equal(f.cnt[0::2], ref.cnt[0::2])  # distinct keys per unit
        assert torch.equal(f.unique_keys().sort().values, ref.unique_keys().sort().values)


def test_launch_list_control_ops_order_two_streams():
    """A native launch list switching streams and ordering them with event waits /
    records (bench.py's one-call iteration): the generator on stream 1, then, ordered
    behind its event, a second generator run on stream 2; both rows as criteo_batch.
    A failing op is named in the error."""
    B = 2048
    H = hipops()
    s1, s2 = torch.cuda.Stream(DEV), torch.cuda.Stream(DEV)
    ev = torch.cuda.Event()
    ev.record(s1)  # (created)
    k1 = torch.empty(B * 39, dtype=torch.int64, device=DEV)
    l1 = torch.empty(B, dtype=torch.float32, device=DEV)
    k2, l2 = torch.empty_like(k1), torch.empty_like(l1)
    from parameter_server_amd.ops.synthetic import CRITEO_1TB_CARDS, _set_cards

    _set_cards(torch.device(DEV), CRITEO_1TB_CARDS)
    g1, g2 = H.LaunchList(), H.LaunchList()
    g1.add_criteo_gen(5, 0, 2 * B, B, 10 ** 9, 1.1, k1, l1)
    g2.add_criteo_gen(5, B, 2 * B, B, 10 ** 9, 1.1, k2, l2)
    L = H.LaunchList()
    L.add_stream(s1)
    L.extend(g1)
    L.add_record(ev)
    L.add_stream(s2)
    L.add_wait(ev)
    L.extend(g2)
    L.add_record(ev)
    L.add_stream(torch.cuda.current_stream(DEV).cuda_stream)  # (raw handle)
    L.add_wait(ev)
    assert len(L) == 9
    del ev, s1, s2  # the list keeps the torch event and streams alive
    for r in range(2):
        L.run()
        torch.cuda.current_stream(DEV).synchronize()
        for row0, k, lab in ((2 * r * B, k1, l1), ((2 * r + 1) * B, k2, l2)):
            kr, lr = criteo_batch(B, seed=5, row0=row0, num_features=10 ** 9, device=DEV)
            assert torch.equal(k, kr) and torch.equal(lab, lr)


@pytest.mark.parametrize("data,init", [("criteo", "zero"), ("uniform", "zero"),
                                       ("uniform", "gaussian")])
def test_overlapped_step_kernel_is_bitwise_the_sequential_one(monkeypatch, data, init):
    """tpf_step2 (both units' load chains issued together, B's probes before A's update,
    weights of existing B keys re-read after it) leaves the same table, bitwise, as the
    sequential tpf_step kernel: Criteo-shaped batches, and uniform keys whose workgroups
    hold > 1024 keys and > 2048 entries (the register batches' fallback loops), with
    zero and gaussian initial weights."""
    from parameter_server_amd.ops.kv_table import InitRule

    monkeypatch.setenv("PSAMD_FLAT", "1")
    # (uniform: the driver's B, where the unit geometry is capped at 1024 pairs of fine
    # buckets, ~2,500 nearly distinct occurrences each; at smaller B the geometry keeps
    # every unit <= 2,048 entries and the fallback loops never run)
    B = 8192 if data == "criteo" else 65536
    g = torch.Generator(device=DEV).manual_seed(3)
    if data == "criteo":
        batches = [criteo_batch(B, seed=43, row0=t * B, num_features=10 ** 9, device=DEV)
                   for t in range(5)]
    else:  # every key of a batch drawn uniformly: mostly distinct, a quarter seen again
        pool = torch.randint(0, 10 ** 9, (B * 39 * 3,), device=DEV, generator=g)
        batches = [(pool[torch.randint(0, pool.numel(), (B * 39,), device=DEV, generator=g)],
                    torch.where(torch.rand(B, device=DEV, generator=g) < 0.5, 1.0, -1.0))
                   for _ in range(5)]
    outs = []
    for v1 in ("1", "0"):
        monkeypatch.setenv("PSAMD_TPF_STEP2", "0" if v1 == "1" else "1")
        cfg = SparseLRConfig(num_features=10 ** 9, minibatch=B, table_capacity=1 << 25,
                             init=InitRule(init, 0.0, 0.01 if init == "gaussian" else 0.0, 5))
        tr = SparseLRTrainer(cfg, device=DEV)
        assert tr.localize_mode == "tpf"
        loc = tr.localize(batches[0][0], buf=0)
        for t in range(5):
            nxt = tr.localize(batches[t + 1][0], buf=(t + 1) % 2) if t < 4 else None
            tr.step(batches[t][0], batches[t][1], width=39, loc=loc, next_loc=nxt)
            loc = nxt
        if data == "uniform":  # the fallback loops ran
            c = tr._localizers[0].flat.cnt.view(-1, 4)
            assert int((c[:, 0] + c[:, 2]).max()) > 1024 and int((c[:, 1] + c[:, 3]).max()) > 2048
        p = tr.progress()
        k, w, z, n = tr.table.occupied()
        o = torch.argsort(k)
        outs.append((p, k[o].cpu(), w[o].cpu(), z[o].cpu(), n[o].cpu()))
    for a, b in zip(outs[0][1:], outs[1][1:]):
        assert torch.equal(a, b)
    assert outs[0][0]["nnz_w"] == outs[1][0]["nnz_w"]


# ---------------------------------------------- valued / variable-width rows (CSR)
def _csr_batch(B: int, seed: int, lo: int = 5, hi: int = 145, valued: bool = True,
               long_row: int = 0, N: int = 10 ** 8):
    """rcv1-like minibatch: widths uniform in [lo, hi) (~75 on average), power-law keys
    (a hot head shared across rows), tf-idf-like values in (0, 1]; optionally one row of
    ``long_row`` features (longer than a tile: spans >= 2 tiles)."""
    g = torch.Generator().manual_seed(seed)
    w = torch.randint(lo, hi, (B,), generator=g)
    if long_row:
        w[B // 2] = long_row
    row_ptr = torch.zeros(B + 1, dtype=torch.int64)
    row_ptr[1:] = torch.cumsum(w, 0)
    n = int(row_ptr[-1])
    u = torch.rand(n, generator=g, dtype=torch.float64)
    keys = (N * u ** 4).long().clamp(max=N - 1)  # power law: many repeats of small ids
    vals = (torch.rand(n, generator=g) * 0.9 + 0.1) if valued else None
    labels = torch.where(torch.rand(B, generator=g) < 0.35, 1.0, -1.0)
    return (keys.to(DEV), labels.to(DEV), row_ptr.to(DEV),
            None if vals is None else vals.to(DEV))


def _reference_train_csr(batches, rule, losses=None):
    """Plain fp32 PyTorch loop over CSR minibatches (valued), one update per minibatch.
    ``losses``: a list that gets each minibatch's summed logistic loss."""
    allk = torch.unique(torch.cat([b[0].cpu() for b in batches]))
    K = allk.numel()
    W, Z, Nn = torch.zeros(K), torch.zeros(K), torch.zeros(K)
    for keys, labels, row_ptr, vals in batches:
        k, y, rp = keys.cpu(), labels.cpu(), row_ptr.cpu()
        B = y.numel()
        x = vals.cpu() if vals is not None else torch.ones(k.numel())
        row = torch.repeat_interleave(torch.arange(B), rp[1:] - rp[:-1])
        idx = torch.searchsorted(allk, k)
        m = torch.zeros(B, dtype=torch.float64).index_add_(0, row, (W[idx] * x).double()).float()
        yy = torch.where(y > 0, 1.0, -1.0)
        coef = -yy * torch.sigmoid(-yy * m)
        if losses is not None:
            losses.append(float(torch.nn.functional.softplus(-yy * m).sum()))
        g = torch.zeros(K, dtype=torch.float64).index_add_(0, idx, (coef[row] * x).double()).float()
        u = torch.unique(idx)
        gu, w_old = g[u] * rule.grad_scale, W[u]
        n_new = torch.sqrt(Nn[u] * Nn[u] + gu * gu)
        sigma = (n_new - Nn[u]) / rule.alpha
        Z[u] = Z[u] + gu - sigma * w_old
        Nn[u] = n_new
        eta = rule.alpha / (n_new + rule.beta)
        zz = -Z[u] * eta
        leta = rule.l1 * eta
        W[u] = torch.where(zz.abs() <= leta, torch.zeros_like(zz),
                           (zz - torch.sign(zz) * leta) / (1 + rule.l2 * eta))
    return allk, W, Z, Nn


@pytest.mark.parametrize("B,valued,long_row", [(1000, True, 0), (10000, True, 0),
                                                (3000, False, 0), (2000, True, 20000)])
def test_flat_csr_step_matches_fp32_reference(monkeypatch, B, valued, long_row):
    """5 steps of valued / variable-width rows on the flat 1-GPU path (CSR fused forward +
    tile backward, tpf_step) against the fp32 PyTorch loop: weights, z, n to rtol 1e-4.
    Covers rows straddling tiles and a row longer than a tile."""
    monkeypatch.setenv("PSAMD_FLAT", "1")
    batches = [_csr_batch(B, 200 + s, valued=valued, long_row=long_row) for s in range(5)]
    maxn = max(int(b[2][-1]) for b in batches)
    cfg = SparseLRConfig(num_features=10 ** 8, minibatch=B,
                         max_nnz_per_example=(maxn + B - 1) // B, table_capacity=1 << 22,
                         alpha=0.05, l1=1.0, l2=0.1)
    tr = SparseLRTrainer(cfg, device=DEV)
    assert tr.localize_mode == "tpf"
    for k, lab, rp, v in batches:
        tr.step(k, lab, row_ptr=rp, vals=v)
    torch.cuda.synchronize()
    assert tr._compact is None  # the flat path ran every step
    p = tr.progress()
    assert p["examples"] == 5 * B
    allk, W, Z, Nn = _reference_train_csr(batches, cfg.update_rule())
    w, z, n = _table_by_raw_key(tr, allk)
    torch.testing.assert_close(w, W, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(z, Z, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(n, Nn, rtol=1e-4, atol=1e-4)
    assert (w != 0).sum() > 50


def test_flat_csr_empty_rows_are_counted(monkeypatch):
    """rows with no features (label-only lines) before the first non-empty
    row, after the last one, in long runs and at tile cuts are still examples: margin 0,
    counted once in loss / examples. Weights still match the fp32 loop."""
    monkeypatch.setenv("PSAMD_FLAT", "1")
    B = 6000
    batches = []
    for s in range(4):
        k, lab, rp, v = _csr_batch(B, 400 + s)
        w = (rp[1:] - rp[:-1]).cpu()
        g = torch.Generator().manual_seed(s)
        w[torch.rand(B, generator=g) < 0.15] = 0  # scattered empties (some at tile cuts)
        w[:7] = 0                                  # leading
        w[-11:] = 0                                # trailing
        w[2000:2900] = 0                           # a long run
        rp2 = torch.zeros(B + 1, dtype=torch.int64)
        rp2[1:] = torch.cumsum(w, 0)
        # keep each row's first w[r] keys of the original row
        old = rp.cpu()
        idx = torch.cat([torch.arange(int(old[r]), int(old[r]) + int(w[r])) for r in range(B)])
        batches.append((k[idx.to(DEV)].contiguous(), lab, rp2.to(DEV),
                        v[idx.to(DEV)].contiguous()))
    maxn = max(int(b[2][-1]) for b in batches)
    cfg = SparseLRConfig(num_features=10 ** 8, minibatch=B,
                         max_nnz_per_example=(maxn + B - 1) // B + 1, table_capacity=1 << 22,
                         alpha=0.05, l1=1.0, l2=0.1)
    tr = SparseLRTrainer(cfg, device=DEV)
    assert tr.localize_mode == "tpf"
    for k, lab, rp, v in batches:
        tr.step(k, lab, row_ptr=rp, vals=v)
    torch.cuda.synchronize()
    assert tr._compact is None
    p = tr.progress()
    assert p["examples"] == 4 * B, p
    losses = []
    allk, W, Z, Nn = _reference_train_csr(batches, cfg.update_rule(), losses)
    assert abs(p["loss"] - sum(losses) / (4 * B)) < 1e-4, (p, sum(losses) / (4 * B))
    w, z, n = _table_by_raw_key(tr, allk)
    torch.testing.assert_close(w, W, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(n, Nn, rtol=1e-4, atol=1e-4)


def _reference_train_filtered(batches, rule, bits, freq, cm):
    """The fp32 FTRL loop with the reference's tail filter (MinibatchReader::read,
    sgd.h:131-150): per minibatch, CountMin insert of every distinct key's occurrence count
    (a byte), then query; keys whose estimate <= freq are dropped from the minibatch (no
    margin contribution, no update, never stored). ``cm``: a CPU CountMinSketch with the
    trainer's hashes (partitioned by mixed-key range). Returns (ever-kept raw keys, W, Z, N,
    filtered-occurrence count)."""
    allk = torch.unique(torch.cat([b[0].cpu() for b in batches]))
    K = allk.numel()
    W, Z, Nn = torch.zeros(K), torch.zeros(K), torch.zeros(K)
    ever = torch.zeros(K, dtype=torch.bool)
    dropped = 0
    for keys, labels, row_ptr, vals in batches:
        k, y = keys.cpu(), labels.cpu()
        B = y.numel()
        rp = row_ptr.cpu() if row_ptr is not None else torch.arange(0, k.numel() + 1,
                                                                    k.numel() // B)
        x = vals.cpu() if vals is not None else torch.ones(k.numel())
        mk = mix(k, bits)
        um, inv, cnt = torch.unique(mk, return_inverse=True, return_counts=True)
        cm.insert(um, cnt.clamp(max=255).to(torch.uint8))
        keep, _ = cm.query(um, freq)
        kocc = keep.bool()[inv]
        dropped += int((~kocc).sum())
        x = torch.where(kocc, x, torch.zeros_like(x))
        row = torch.repeat_interleave(torch.arange(B), rp[1:] - rp[:-1])
        idx = torch.searchsorted(allk, k)
        m = torch.zeros(B, dtype=torch.float64).index_add_(0, row, (W[idx] * x).double()).float()
        yy = torch.where(y > 0, 1.0, -1.0)
        coef = -yy * torch.sigmoid(-yy * m)
        g = torch.zeros(K, dtype=torch.float64).index_add_(0, idx, (coef[row] * x).double()).float()
        u = torch.unique(idx[kocc])
        ever[u] = True
        gu, w_old = g[u] * rule.grad_scale, W[u]
        n_new = torch.sqrt(Nn[u] * Nn[u] + gu * gu)
        sigma = (n_new - Nn[u]) / rule.alpha
        Z[u] = Z[u] + gu - sigma * w_old
        Nn[u] = n_new
        eta = rule.alpha / (n_new + rule.beta)
        zz = -Z[u] * eta
        leta = rule.l1 * eta
        W[u] = torch.where(zz.abs() <= leta, torch.zeros_like(zz),
                           (zz - torch.sign(zz) * leta) / (1 + rule.l2 * eta))
    return allk[ever], W[ever], Z[ever], Nn[ever], dropped


@pytest.mark.parametrize("kind", ["fixed", "fixed_pre", "csr", "skewed"])
def test_flat_tail_filter_matches_fp32_reference(monkeypatch, kind):
    """the tail filter on the flat fast path (CountMin insert + query fused into
    the bucket kernel, filtered keys removed from the minibatch) against the fp32 loop with
    a CPU CountMin of the same hashes, 5 steps, rtol 1e-4. tail_feature_freq 1 (the
    reference CTR conf) and a small sketch, so collisions happen too."""
    from parameter_server_amd.ops.countmin import CountMinSketch

    monkeypatch.setenv("PSAMD_FLAT", "1")
    steps, freq = 5, 1
    if kind == "skewed":  # overflowing bucket pairs: the register-light units, filtered
        monkeypatch.setenv("PSAMD_TILE_LTS", "13")
        bits = 20
        batches = [(k, lab, None, None) for k, lab in (_skewed_batch(s, bits) for s in range(3))]
        B, width, N = batches[0][1].numel(), 16, 1 << bits
        steps = 3
    elif kind == "csr":
        B, N = 3000, 10 ** 6
        batches = [_csr_batch(B, 500 + s, N=N) for s in range(steps)]
        width = None
    else:
        B, N, width = 8192, 10 ** 6, 39
        batches = [(*criteo_batch(B, seed=77, row0=t * B, num_features=N, device=DEV), None, None)
                   for t in range(steps)]
    maxn = max(b[0].numel() for b in batches)
    cfg = SparseLRConfig(num_features=N, minibatch=B, max_nnz_per_example=(maxn + B - 1) // B,
                         table_capacity=1 << 22, alpha=0.05, l1=1.0, l2=0.1,
                         tail_feature_freq=freq, countmin_n=1 << 16)
    tr = SparseLRTrainer(cfg, device=DEV)
    assert tr.localize_mode == "tpf" and tr.filter is not None
    if kind == "fixed_pre":  # pulls issued ahead (the pipelined form), localised in order
        loc = tr.localize(batches[0][0], buf=0)
        for t in range(steps):
            nxt = tr.localize(batches[t + 1][0], buf=(t + 1) % 2) if t + 1 < steps else None
            tr.step(batches[t][0], batches[t][1], width=width, loc=loc, next_loc=nxt)
            loc = nxt
    else:
        for k, lab, rp, v in batches:
            tr.step(k, lab, width=width, row_ptr=rp, vals=v)
    torch.cuda.synchronize()
    assert tr._compact is None  # every step ran the flat path
    tr.check_ok()
    p = tr.progress()
    assert p["examples"] == steps * B
    cm = CountMinSketch(cfg.countmin_n, cfg.countmin_k, "cpu", key_bits=tr.bits)
    allk, W, Z, Nn, dropped = _reference_train_filtered(batches, cfg.update_rule(), tr.bits,
                                                        freq, cm)
    assert dropped > 0  # the filter removed something
    assert torch.equal(tr.filter.cells.cpu(), cm.cells)  # same sketch, cell for cell
    w, z, n = _table_by_raw_key(tr, allk)  # only ever-kept keys were stored
    torch.testing.assert_close(w, W, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(z, Z, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(n, Nn, rtol=1e-4, atol=1e-4)
    assert (w != 0).sum() > 20


def test_flat_fixed_width_valued_rows_take_the_csr_kernel(monkeypatch):
    """Fixed-width rows WITH values (no row_ptr): the flat step synthesises row_ptr."""
    monkeypatch.setenv("PSAMD_FLAT", "1")
    B = 4096
    batches = []
    for s in range(4):
        k, lab = criteo_batch(B, seed=61, row0=s * B, num_features=10 ** 8, device=DEV)
        v = torch.rand(k.numel(), device=DEV, generator=torch.Generator(device=DEV).manual_seed(s))
        batches.append((k, lab, torch.arange(0, (B + 1) * 39, 39, device=DEV), v))
    cfg = SparseLRConfig(num_features=10 ** 8, minibatch=B, table_capacity=1 << 22)
    tr = SparseLRTrainer(cfg, device=DEV)
    for k, lab, _, v in batches:
        tr.step(k, lab, width=39, vals=v)
    torch.cuda.synchronize()
    allk, W, Z, Nn = _reference_train_csr(batches, cfg.update_rule())
    w, z, n = _table_by_raw_key(tr, allk)
    torch.testing.assert_close(w, W, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(n, Nn, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("merge", ["on", "off"])
def test_flat_csr_multi_peer_matches_compact(monkeypatch, merge):
    """2 emulated peers, ssp:2: the flat exchange with the CSR fused kernel leaves the
    same table as the compact layout with the generic kernels (PSAMD_FLAT=0)."""
    from parameter_server_amd.parallel.comm import LoopbackComm

    B = 3000
    batches = [_csr_batch(B, 300 + s) for s in range(6)]
    maxn = max(int(b[2][-1]) for b in batches)
    outs = []
    for flat in ("1", "0"):
        monkeypatch.setenv("PSAMD_FLAT", flat)
        cfg = SparseLRConfig(num_features=10 ** 8, minibatch=B, consistency="ssp:2",
                             max_nnz_per_example=(maxn + B - 1) // B, table_capacity=1 << 22,
                             alpha=0.05, l1=1.0, l2=0.1, exchange_merge=merge)
        tr = SparseLRTrainer(cfg, LoopbackComm(2, "cuda"), DEV)
        assert (tr.localize_mode == "tpf") == (flat == "1")
        for k, lab, rp, v in batches:
            tr.step(k, lab, row_ptr=rp, vals=v)
        p = tr.progress()
        kk, w, z, n = tr.table.occupied()
        o = torch.argsort(kk)
        outs.append((kk[o].cpu(), w[o].cpu(), n[o].cpu(), p))
    assert torch.equal(outs[0][0], outs[1][0])
    torch.testing.assert_close(outs[0][1], outs[1][1], rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(outs[0][2], outs[1][2], rtol=1e-4, atol=1e-4)
    assert abs(outs[0][3]["loss"] - outs[1][3]["loss"]) < 1e-4
