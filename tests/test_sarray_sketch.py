"""Sorted-key algebra (utils/sarray.py -> csrc/core/setops.cc) and bit sketches
(utils/sketch.py), against numpy / pure-Python models of the reference semantics
(src/util/parallel_ordered_match.h, bloom_filter.h, block_bloom_filter.h, bitmap.h)."""
import numpy as np
import pytest

from parameter_server_amd.ops.native import core
from parameter_server_amd.utils import sarray
from parameter_server_amd.utils.sketch import Bitmap, BlockBloomFilter, BloomFilter


def _sorted_unique(rng, n, hi=1 << 62):
    return np.unique(rng.integers(0, hi, n, dtype=np.uint64))


@pytest.mark.parametrize("dtype", [np.float32, np.float64, np.int64])
@pytest.mark.parametrize("k", [1, 3])
@pytest.mark.parametrize("n", [10, 300_000])
def test_ordered_match_matches_model(dtype, k, n):
    rng = np.random.default_rng(n + k)
    dst = _sorted_unique(rng, n)
    src = np.unique(np.concatenate([rng.choice(dst, n // 2), _sorted_unique(rng, n // 3)]))
    sv = (rng.standard_normal(src.size * k) * 100).astype(dtype)
    # model: dict lookup
    pos = {int(x): i for i, x in enumerate(dst)}
    for op in ("ASSIGN", "PLUS", "MINUS"):
        base = (rng.standard_normal(dst.size * k) * 10).astype(dtype)
        want = base.copy().reshape(-1, k)
        hits = 0
        for i, key in enumerate(src):
            j = pos.get(int(key))
            if j is None:
                continue
            hits += 1
            s = sv.reshape(-1, k)[i]
            want[j] = s if op == "ASSIGN" else (want[j] + s if op == "PLUS" else want[j] - s)
        got, m = sarray.ordered_match(src, sv, dst, k, op, base.copy())
        assert m == hits
        np.testing.assert_allclose(got.reshape(-1, k), want, rtol=1e-6)


def test_ordered_match_or_and_threads_agree(monkeypatch):
    rng = np.random.default_rng(0)
    dst = _sorted_unique(rng, 500_000)
    src = dst[::3].copy()
    sv = rng.integers(0, 255, src.size).astype(np.uint8)
    out1, n1 = sarray.ordered_match(src, sv, dst, 1, "OR", np.zeros(dst.size, np.uint8))
    monkeypatch.setenv("PSAMD_NUM_THREADS", "1")
    out2, n2 = sarray.ordered_match(src, sv, dst, 1, "OR", np.zeros(dst.size, np.uint8))
    assert n1 == n2 == src.size and np.array_equal(out1, out2)
    assert np.array_equal(out1[::3], sv)


def test_union_intersection_find_range():
    rng = np.random.default_rng(1)
    a, b = _sorted_unique(rng, 5000, 10**6), _sorted_unique(rng, 7000, 10**6)
    assert np.array_equal(sarray.set_union(a, b), np.union1d(a, b))
    assert np.array_equal(sarray.set_intersection(a, b), np.intersect1d(a, b))
    lo, hi = sarray.find_range(a, 1000, 500_000)
    assert np.all(a[lo:hi] >= 1000) and np.all(a[lo:hi] < 500_000)
    assert (lo == 0 or a[lo - 1] < 1000) and (hi == a.size or a[hi] >= 500_000)
    va, vb = np.ones(a.size, np.float32), np.full(b.size, 2, np.float32)
    keys, vals = sarray.parallel_union(a, va, b, vb)
    both = np.isin(keys, np.intersect1d(a, b))
    assert np.all(vals[both] == 3) and np.all(np.isin(vals[~both], [1, 2]))
    # int keys of another dtype take the generic path
    ka = np.array([1, 5, 9], np.int64)
    got, n = sarray.ordered_match(ka, np.array([1., 2., 3.]), np.array([5, 9, 11], np.int64))
    assert n == 2 and list(got) == [2.0, 3.0, 0.0]


def _ref_hash(key):  # reference Sketch::hash (src/util/sketch.h:20-31)
    M = 0xFFFFFFFF
    m = 0xc6a4a793
    h = (0xbc9f1d34 ^ (8 * m)) & M
    for w in (key & M, key >> 32):
        h = (h + w) & M
        h = (h * m) & M
        h ^= h >> 16
    return h


def test_bloom_bit_layout_matches_reference_model():
    assert core().sketch_hash(123456789123) == _ref_hash(123456789123)
    bf = BloomFilter(1000, 4)
    keys = [3, 77, 2**40 + 5]
    bf.insert(keys)
    model = np.zeros(1000 // 8 + 1, np.uint8)
    for key in keys:
        h = _ref_hash(key)
        d = ((h >> 17) | (h << 15)) & 0xFFFFFFFF
        for _ in range(4):
            p = h % 1000
            model[p // 8] |= 1 << (p % 8)
            h = (h + d) & 0xFFFFFFFF
    assert np.array_equal(bf.bits, model)


@pytest.mark.parametrize("cls", [BloomFilter, BlockBloomFilter])
def test_bloom_no_false_negatives_and_fp_rate(cls):
    rng = np.random.default_rng(2)
    ins = rng.integers(0, 1 << 63, 20_000, dtype=np.uint64)
    other = rng.integers(0, 1 << 63, 20_000, dtype=np.uint64)
    bf = cls(20_000 * 10, 5)
    bf.insert(ins)
    assert bf.query(ins).all()
    fp = bf.query(np.setdiff1d(other, ins)).mean()
    assert fp < 0.05, fp
    assert int(ins[0]) in bf


def test_bitmap():
    bm = Bitmap(1000)
    assert bm.nnz() == 0 and bm.size() == 1000
    bm.set([1, 5, 64, 999])
    assert bm.test(5) and not bm.test(6) and bm[999]
    assert list(bm.test([1, 2, 64])) == [True, False, True]
    assert bm.nnz() == 4 and bm.nnz(2, 100) == 2
    bm.clear([5])
    assert not bm.test(5) and bm.nnz() == 3
    bm.fill(True)
    assert bm.nnz() == 1000 and bm.to_bool().all()
    bm.clear()
    assert bm.nnz() == 0
