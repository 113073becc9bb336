"""Host-side geometry of the flat localisation (tploc.hip tp_flat_lts / tpf_stride /
tpf_stride_max): tiles of 1024..8192 occurrences chosen from the minibatch size, and the
workspace bound that lets a Localizer sized for n keys take any smaller minibatch. Pure
host functions of the built extension: run on CPU (skipped when it is not built)."""
import pytest


def _H():
    try:
        from parameter_server_amd.ops.native import hipops

        return hipops()
    except Exception as e:  # pragma: no cover - extension not built here
        pytest.skip(f"_hipops not built: {e}")


def test_tile_size_follows_the_minibatch():
    H = _H()
    assert H.tpf_tile_log2(65536 * 39) == 13      # driver shape: 312 tiles of 8192
    assert H.tpf_tile_log2(10000 * 39) == 11      # reference operating point: 191 of 2048
    assert H.tpf_tile_log2(16384 * 39) == 12      # 157 of 4096
    assert H.tpf_tile_log2(1000 * 74) == 10       # rcv1-like B = 1,000: 73 of 1024
    for n in (1, 1000, 10 ** 5, 390000, 639000, 2555904, 5 * 10 ** 6):
        lts = H.tpf_tile_log2(n)
        assert 10 <= lts <= 13
        T = -(-n // (1 << lts))
        assert T <= 640                            # the bucket kernel's LDS tile runs
        assert H.tpf_stride(n) == T * 8192         # entry ids keep the 8192 stride
        if lts < 13:                               # a larger tile would give < 128 tiles
            assert -(-n // (1 << (lts + 1))) < 128


def test_workspace_bound_covers_every_smaller_minibatch():
    H = _H()
    for n in (32768, 390000, 2555904):
        cap = H.tpf_stride_max(n)
        for m in list(range(1, n + 1, max(1, n // 997))) + [n]:
            assert H.tpf_stride(m) <= cap, (n, m)


def test_tile_size_pin(monkeypatch):
    H = _H()
    monkeypatch.setenv("PSAMD_TILE_LTS", "13")
    assert H.tpf_tile_log2(390000) == 13
    monkeypatch.setenv("PSAMD_TILE_LTS", "10")
    assert H.tpf_tile_log2(390000) == 10
    assert H.tpf_tile_log2(2555904) == 12          # 2496 tiles of 1024 > 640: clamped up
    monkeypatch.delenv("PSAMD_TILE_LTS")
    monkeypatch.setenv("PSAMD_TILE_MIN", "32")
    assert H.tpf_tile_log2(390000) == 13           # 48 tiles >= 32
