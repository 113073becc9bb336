import numpy as np
import pytest
import torch

from parameter_server_amd.ops import (CountMinSketch, KVTable, UpdateRule, exact_auc,
                                      localize_torch)
from parameter_server_amd.ops import fixing_float as ff
from parameter_server_amd.ops.keymix import key_bits_for, mix, unmix
from parameter_server_amd.ops.native import core
from parameter_server_amd.parallel.partition import KeyPartition, even_divide


@pytest.mark.parametrize("bits", [2, 7, 30, 33, 64])
def test_keymix_bijection(bits):
    n = min(1 << bits, 5000)
    if bits <= 12:
        k = torch.arange(1 << bits, dtype=torch.int64)
    else:
        k = torch.randint(0, min(1 << bits, 1 << 62), (n,), dtype=torch.int64)
    h = mix(k, bits)
    assert torch.equal(unmix(h, bits), k)
    if bits < 63:
        assert int(h.min()) >= 0 and int(h.max()) < (1 << bits)
    if bits <= 12:
        assert torch.unique(h).numel() == (1 << bits)


def test_key_bits_for():
    assert key_bits_for(10 ** 9) == 30
    assert key_bits_for(1 << 20) == 20
    assert key_bits_for(0) == 64


def test_localize_torch_semantics():
    k = torch.tensor([5, 3, 5, 9, 3, 5], dtype=torch.int64)
    loc = localize_torch(k, 8)
    U = loc.uniq.numel()
    assert U == 3
    h = mix(k, 8)
    assert torch.equal(loc.uniq[loc.local_col.long()], h)
    assert (loc.uniq[1:] > loc.uniq[:-1]).all()
    counts = loc.seg_start[1:] - loc.seg_start[:-1]
    assert sorted(counts.tolist()) == [1, 2, 3]


def test_kv_table_cpu_ftrl_matches_formula():
    rule = UpdateRule("ftrl", "decay", alpha=0.1, beta=1.0, l1=0.5, l2=0.2)
    t = KVTable(1 << 8)
    keys = torch.tensor([1, 2, 3], dtype=torch.int64)
    s, w = t.resolve(keys)
    assert (w == 0).all() and torch.unique(s).numel() == 3
    g = torch.tensor([2.0, -0.1, -3.0])
    t.update(s, g, rule)
    # one FTRL step from zero state: n=|g|, z=g, eta=a/(n+b), w=prox(-z eta)
    n = g.abs()
    eta = 0.1 / (n + 1.0)
    zz = -g * eta
    exp = torch.where(zz.abs() <= 0.5 * eta, torch.zeros(3), (zz - torch.sign(zz) * 0.5 * eta) / (1 + 0.2 * eta))
    torch.testing.assert_close(t.gather(s), exp)
    assert t.census() == (3, int((exp != 0).sum()))


def test_kv_table_full_raises():
    t = KVTable(64)
    with pytest.raises(RuntimeError):
        t.resolve(torch.arange(100, dtype=torch.int64))


def test_kv_table_load_and_occupied():
    t = KVTable(1 << 10)
    keys = torch.tensor([10, 20, 30], dtype=torch.int64)
    t.load(keys, torch.tensor([1.0, 0.0, -2.0]), torch.tensor([0.1, 0.2, 0.3]), torch.ones(3))
    k, w, z, n = t.occupied()
    d = dict(zip(k.tolist(), w.tolist()))
    assert d == {10: 1.0, 20: 0.0, 30: -2.0}


def test_countmin_saturates_and_filters():
    cm = CountMinSketch(1024, 2)
    keys = torch.tensor([1, 2, 3], dtype=torch.int64)
    cm.insert(keys, torch.tensor([200, 1, 3], dtype=torch.uint8))
    cm.insert(keys, torch.tensor([200, 1, 0], dtype=torch.uint8))
    keep, cnt = cm.query(keys, freq=2)
    assert cnt.tolist()[0] == 254  # saturated at v_max
    assert cnt.tolist()[1] >= 2 and cnt.tolist()[2] >= 3
    assert keep.tolist() == [1, int(cnt[1]) > 2, 1]


def test_countmin_partitioned_regions_and_saturation():
    """Partitioned sketch (the trainers'): a key's cells stay inside its mixed-key region;
    repeated inserts saturate at v_max exactly like the chain of saturating adds; the hash
    is the C++ one."""
    from parameter_server_amd.ops.countmin import sketch_hash_torch
    from parameter_server_amd.ops.native import core

    bits = 24
    cm = CountMinSketch(1 << 16, 3, key_bits=bits)
    assert cm.rsize % 64 == 0 and cm.rsize << cm.lgR == cm.n and cm.rshift == bits - 11
    g = torch.Generator().manual_seed(3)
    keys = torch.randint(0, 1 << bits, (5000,), dtype=torch.int64, generator=g)
    cells = cm._cells_of(keys)
    region = keys >> cm.rshift
    assert bool(((cells // cm.rsize) == region[:, None]).all())
    # blocked: a key's k cells are distinct and share one 64-cell block (one cache line)
    assert bool((cells // 64 == cells[:, :1] // 64).all())
    assert bool((cells[:, 0] != cells[:, 1]).all() & (cells[:, 1] != cells[:, 2]).all())
    h = sketch_hash_torch(keys[:50])
    assert h.tolist() == [core().sketch_hash(int(k)) for k in keys[:50]]
    for _ in range(3):
        cm.insert(keys[:10], torch.full((10,), 100, dtype=torch.uint8))
    keep, cnt = cm.query(keys[:10], freq=253)
    assert cnt.tolist() == [254] * 10 and keep.tolist() == [1] * 10
    keep, cnt = cm.query(keys[10:20], freq=0)
    assert bool((cnt < 254).all())


def test_fixing_float_cpu_roundtrip():
    x = torch.randn(1000)
    code, mm = ff.encode(x, 2)
    y = ff.decode(code, 2, mm)
    step = float(mm[1] - mm[0]) / (65536 - 2)
    assert float((x - y).abs().max()) <= step * 1.0001


def test_hash_vectors():
    c = core()
    assert c.crc32c(b"123456789") == 0xE3069283
    assert c.crc32c(b"") == 0
    assert c.crc32c(bytes(32)) == 0x8A9136AA  # RFC 3720 B.4: 32 bytes of zeros
    assert c.crc32c(b"\xff" * 32) == 0x62A8AB43
    assert c.murmur3_32(b"hello", 0) == 0x248BFA47
    assert c.murmur3_32(b"", 1) == 0x514E28B7
    assert c.murmur3_x64_128(b"hello", 0)[0] == 0xCBD8A7B341BD9B02


def test_partition_even_divide_and_split():
    assert even_divide(0, 10, 3, 0) == (0, 3)
    assert even_divide(0, 10, 3, 2) == (6, 10)
    p = KeyPartition(30, 4)
    h = mix(torch.randint(0, 10 ** 9, (10000,), dtype=torch.int64), 30)
    own = p.owner_of(h)
    counts = torch.bincount(own.long(), minlength=4)
    assert counts.min() > 2200  # balanced
    s = torch.unique(h)
    off = p.split_sorted(s)
    for g in range(4):
        seg = s[off[g]:off[g + 1]]
        assert (p.owner_of(seg) == g).all()
    p64 = KeyPartition(64, 3)
    h64 = mix(torch.randint(-(1 << 62), 1 << 62, (3000,), dtype=torch.int64), 64)
    o = p64.owner_of(h64)
    assert set(o.tolist()) == {0, 1, 2}


def test_exact_auc():
    s = torch.tensor([0.1, 0.4, 0.35, 0.8])
    y = torch.tensor([-1.0, -1.0, 1.0, 1.0])
    assert abs(exact_auc(s, y) - 0.75) < 1e-9


def test_staged_localisation_needs_the_flat_tail_filter():
    """Localizer(keys, stage): the tile + bucket / filter split exists only for the flat
    layout with a tail filter; anything else is refused loudly."""
    from parameter_server_amd.ops.localize import Localizer

    lz = Localizer(1000, 20, "cpu", mode="sort")
    keys = torch.randint(0, 1 << 20, (500,), dtype=torch.int64)
    lz(keys)  # (stage 0: fine)
    for stage in (3, 4):
        with pytest.raises(ValueError, match="staged localisation"):
            lz(keys, stage)
