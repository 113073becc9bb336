"""Binary example cache (data/bincache.py) and the feeder's cached streaming path
(data/feeder.py): a cached pass yields exactly the minibatches of the text pass, a stale
cache is rebuilt, and the GPU app agrees on its step count once when every file is
cached. CPU (the same code path as the GPU feeder up to the host->HBM copies)."""
import os
import sys

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.dirname(__file__))

from test_app_gpu import _conf, _flags, _mr_worker, _port, _write_libsvm  # noqa: E402


def _batches(feeder):
    out = []
    for b in feeder:
        rp = b.row_ptr
        if rp is None:
            rp = torch.arange(0, (b.rows + 1) * b.width, b.width, dtype=torch.int64)
        out.append((b.keys.clone(), b.labels.clone(), rp.clone(),
                    None if b.vals is None else b.vals.clone(), b.width))
        feeder.release(b)
    return out


@pytest.mark.parametrize("binary_width,num_features", [(0, 0), (0, 1 << 20), (16, 1 << 12)])
def test_cached_pass_equals_text_pass(tmp_path, binary_width, num_features):
    from parameter_server_amd.data.feeder import DeviceFeeder

    d = tmp_path / "data"
    _write_libsvm(str(d), nfiles=3, rows=500, binary_width=binary_width)
    files = sorted(str(d / f) for f in os.listdir(d))
    cache = str(tmp_path / "cache")
    # minibatch 300 over 500-row files: minibatches continue into the next file
    f = DeviceFeeder(files, "LIBSVM", 300, 300 * 40, "cpu", num_features=num_features,
                     passes=2, cache_dir=cache)
    got = _batches(f)
    assert f.text_passes == 1 and f.cached_passes == 1
    n = len(got) // 2
    assert len(got) == 2 * n and n == 5
    for a, b in zip(got[:n], got[n:]):
        assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1]) and torch.equal(a[2], b[2])
        if binary_width:
            assert a[3] is None and b[3] is None and b[4] == binary_width
        else:
            assert torch.equal(a[3], b[3])
    # a new run over the same files streams the cache from its first pass
    f2 = DeviceFeeder(files, "LIBSVM", 300, 300 * 40, "cpu", num_features=num_features,
                      passes=1, cache_dir=cache)
    assert f2.planned_batches() == n
    got2 = _batches(f2)
    assert f2.text_passes == 0 and f2.cached_passes == 1
    assert all(torch.equal(a[0], b[0]) for a, b in zip(got[:n], got2))
    if num_features and num_features <= (1 << 32):
        from parameter_server_amd.data.bincache import CacheFile

        cf = CacheFile(os.path.join(cache, sorted(os.listdir(cache))[0]))
        assert cf.key_bytes == 4 and cf.fixed == bool(binary_width)


def test_nnz_cap_cuts_like_the_text_reader(tmp_path):
    """minibatches also end at max_nnz features (the localisation workspace)."""
    from parameter_server_amd.data.feeder import DeviceFeeder

    d = tmp_path / "data"
    _write_libsvm(str(d), nfiles=2, rows=400)
    files = sorted(str(d / f) for f in os.listdir(d))
    f = DeviceFeeder(files, "LIBSVM", 1000, 2000, "cpu", passes=2, cache_dir=str(tmp_path / "c"))
    got = _batches(f)
    n = len(got) // 2
    assert n > 2
    for a, b in zip(got[:n], got[n:]):
        assert torch.equal(a[0], b[0]) and torch.equal(a[2], b[2])
        assert a[0].numel() <= 2000


def test_stale_cache_is_rebuilt(tmp_path):
    from parameter_server_amd.data.feeder import DeviceFeeder

    d = tmp_path / "data"
    _write_libsvm(str(d), nfiles=1, rows=300)
    files = [str(d / "part-0")]
    cache = str(tmp_path / "cache")
    _batches(DeviceFeeder(files, "LIBSVM", 100, 4000, "cpu", cache_dir=cache))
    _write_libsvm(str(d), nfiles=1, rows=200, seed=5)  # the source changed
    os.utime(files[0], ns=(1, 1))
    f = DeviceFeeder(files, "LIBSVM", 100, 4000, "cpu", cache_dir=cache)
    assert f.planned_batches() is None  # stale: text again (and rewritten)
    got = _batches(f)
    assert f.text_passes == 1 and sum(b[1].numel() for b in got) == 200
    f = DeviceFeeder(files, "LIBSVM", 100, 4000, "cpu", cache_dir=cache)
    assert f.planned_batches() == 2


def test_app_reruns_from_the_cache(tmp_path):
    """The GPU app (CPU tensors here) with -data_cache: the second run parses nothing and
    ends at the same weights."""
    from parameter_server_amd.app.gpu import run_async_sgd
    from parameter_server_amd.parallel.comm import LocalComm
    from parameter_server_amd.utils.config import load_app_config

    data = tmp_path / "data"
    _write_libsvm(str(data))
    ws = []
    for run in range(2):
        lm = load_app_config(str(_conf(tmp_path, data, tmp_path / f"m{run}" / "m",
                                       passes=2))).linear_method
        res = run_async_sgd(lm, LocalComm("cpu"), torch.device("cpu"),
                            _flags(data_cache=str(tmp_path / "cache")))
        assert res["examples"] == 2 * 3 * 600
        assert (res["text_passes"], res["cached_passes"]) == ((1, 1) if run == 0 else (0, 2))
        k, w, _, _ = res["trainer"].table.occupied()
        o = torch.argsort(k)
        ws.append((k[o], w[o]))
    assert torch.equal(ws[0][0], ws[1][0])
    torch.testing.assert_close(ws[0][1], ws[1][1], rtol=0, atol=0)


def _mr_cached_worker(rank, world, port, conf, out_dir, cache):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from parameter_server_amd.app.gpu import run_async_sgd
    from parameter_server_amd.parallel.comm import DistComm
    from parameter_server_amd.utils.config import load_app_config

    torch.set_num_threads(1)
    lm = load_app_config(conf).linear_method
    res = run_async_sgd(lm, DistComm("cpu"), torch.device("cpu"),
                        _flags(table_capacity=1 << 15, data_cache=cache))
    torch.save({"steps": res["steps"], "idle": res["idle_steps"], "agreed": res["agreed_steps"],
                "examples": res["examples"]}, os.path.join(out_dir, f"c{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_app_two_ranks_cached_agree_once(tmp_path):
    """Uneven files over 2 ranks with every file cached: the ranks agree on the step
    count up front (no per-step host gather); the rank with less data idles."""
    import torch.multiprocessing as mp

    data, model = tmp_path / "data", tmp_path / "model" / "m"
    _write_libsvm(str(data))
    conf = _conf(tmp_path, data, model, max_delay=2, passes=2)
    cache = str(tmp_path / "cache")
    # the first run parses pass 1 (agreement every step) and streams pass 2 from the
    # caches it wrote (agreed once); the second run streams both passes
    for run, want in ((0, [None, 6]), (1, [6, 6])):
        mp.spawn(_mr_cached_worker, args=(2, _port(), str(conf), str(tmp_path), cache),
                 nprocs=2, join=True)
        r = [torch.load(tmp_path / f"c{i}.pt") for i in range(2)]
        assert r[0]["agreed"] == r[1]["agreed"] == want
        assert r[0]["examples"] == 2400 and r[1]["examples"] == 1200
        assert r[0]["steps"] == 12 and r[1]["steps"] == 6 and r[1]["idle"] == 6
