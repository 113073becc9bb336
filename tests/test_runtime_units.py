import glob

import numpy as np
import pytest

from parameter_server_amd.data import ExampleBatch, StreamReader, divide_files, parse_text
from parameter_server_amd.data.recordio import decode_examples, encode_examples
from parameter_server_amd.filter import (CompressingFilter, FixingFloatFilter,
                                         KeyCachingFilter, SparseFilter)
from parameter_server_amd.ops.native import core
from parameter_server_amd.system.message import Message, new_task, slice_key_ordered
from parameter_server_amd.system.postoffice import Node, partition_key_space
from parameter_server_amd.utils.config import AppConfig, lm_to_sparse_lr
from parameter_server_amd.utils.flags import parse_flags

REF_CONFS = sorted(glob.glob("/root/reference/example/linear/*/*.conf"))


@pytest.mark.skipif(not REF_CONFS, reason="reference configs not mounted")
@pytest.mark.parametrize("path", REF_CONFS)
def test_reference_confs_parse_and_roundtrip(path):
    c = AppConfig.parse(open(path).read())
    assert c.has("linear_method")
    assert AppConfig.parse(c.to_text()) == c


def test_textproto_extensions_and_errors():
    c = AppConfig.parse("""linear_method { darlin { max_block_delay: 8
      [PS.LM.delta_init_value] : 2  # comment
      [PS.LM.kkt_filter_threshold_ratio]: 1e20 } }""")
    d = c.linear_method.darlin
    assert d.max_block_delay == 8 and d.ext("delta_init_value") == 2.0
    assert d.ext("delta_max_value") == 5.0 and d.ext("kkt_filter_threshold_ratio") == 1e20
    with pytest.raises(ValueError):
        AppConfig.parse("linear_method { loss { type: NOPE } }")
    with pytest.raises(ValueError):
        AppConfig.parse("linear_method { loss { type: LOGIT }")


def test_online_conf_maps_to_gpu_trainer():
    c = AppConfig.parse("""linear_method { loss { type: LOGIT } penalty { type: L1 lambda: 10 lambda: 1 }
      learning_rate { type: DECAY alpha: .01 beta: 10 }
      async_sgd { algo: FTRL minibatch: 10000 tail_feature_freq: 1 max_delay: 4 } }""")
    s = lm_to_sparse_lr(c.linear_method)
    assert (s.algo, s.l1, s.l2, s.alpha, s.beta, s.minibatch) == ("ftrl", 10, 1, .01, 10, 10000)
    assert s.tail_feature_freq == 1 and s.consistency == "ssp:4"


def test_flags():
    f = parse_flags(["-num_servers", "2", "--num_workers=3", "-print_van", "-nokey_cache",
                     "-my_node", "role:SERVER,hostname:'127.0.0.1',port:9600,id:'S0'", "file.txt"])
    assert (f.num_servers, f.num_workers, f.print_van, f.key_cache) == (2, 3, True, False)
    assert f.rest == ["file.txt"]
    n = Node.parse(f.my_node)
    assert (n.role, n.id, n.port) == ("SERVER", "S0", 9600)


def test_message_encode_decode_and_slice():
    m = Message(task=new_task(key_channel=3))
    m.set_key(np.array([1, 5, 9, 12, 20], dtype=np.uint64))
    m.add_value(np.arange(10, dtype=np.float32))  # 2 values per key
    m2 = Message.decode("W0", [f if isinstance(f, bytes) else f.tobytes() for f in m.encode()])
    assert np.array_equal(m2.key, m.key) and np.array_equal(m2.value[0], m.value[0])
    # reference sliceKeyOrderedMsg: pieces keep the message key_range; a piece is
    # invalid iff the receiver range misses the message range (message.h:120-159)
    m.task["key_range"] = [0, 13]
    parts = slice_key_ordered(m, [(0, 6), (6, 10), (10, 15), (15, 16)])
    assert [p.key.tolist() for p in parts] == [[1, 5], [9], [12], []]
    assert parts[0].value[0].tolist() == [0, 1, 2, 3]
    assert parts[2].value[0].tolist() == [6, 7]
    assert [p.valid for p in parts] == [True, True, True, False]
    assert all(p.task["key_range"] == [0, 13] for p in parts)


def test_partition_key_space():
    nodes = [Node("SERVER", f"S{i}") for i in range(3)]
    partition_key_space(nodes, 0, 99)
    assert [(n.key_begin, n.key_end) for n in nodes] == [(0, 33), (33, 66), (66, 99)]


def test_key_caching_filter_roundtrip():
    enc, dec = KeyCachingFilter(), KeyCachingFilter()
    for push in (False, True):
        m = Message(task=new_task(key_channel=1, request=True,
                                  shared_para={"cmd": "PUSH" if push else "PULL"}))
        m.set_key(np.arange(100, dtype=np.uint64))
        m.add_filter("KEY_CACHING", clear_cache_if_done=True)
        enc.encode(m)
        if push:
            assert m.key is None  # cache hit: key frame dropped
        dec.decode(m)
        assert np.array_equal(m.key, np.arange(100, dtype=np.uint64))
    assert not enc.cache and not dec.cache  # cleared after the PUSH


def test_compressing_and_fixing_float_filters():
    m = Message(task=new_task())
    m.set_key(np.arange(1000, dtype=np.uint64))
    v = np.random.default_rng(1).normal(size=1000).astype(np.float32)
    m.add_value(v.copy())
    m.add_filter("FIXING_FLOAT", fixed_point=[{"num_bytes": 2}])
    m.add_filter("COMPRESSING")
    f1, f2 = FixingFloatFilter(), CompressingFilter()
    f1.encode(m)
    f2.encode(m)
    assert m.value[0].dtype == np.uint8
    f2.decode(m)
    f1.decode(m)
    assert np.array_equal(m.key, np.arange(1000, dtype=np.uint64))
    assert np.abs(m.value[0] - v).max() < (v.max() - v.min()) / 65534 * 1.01 + 1e-6


def test_sparse_filter_nan_mark():
    v = np.ones(5, np.float32)
    SparseFilter.mark(v, np.array([0, 1, 0, 0, 1], bool))
    assert SparseFilter.marked(v).tolist() == [False, True, False, False, True]


@pytest.mark.parametrize("fmt,text,keys,labels", [
    ("LIBSVM", b"1 3:0.5 7:1\n-1 2:1\nbad\n", [3, 7, 2], [1, -1]),
    ("ADFEA", b"99 1 1 10:1 20:2\n7 1 0 30:1\n", [10, 20, 30], [1, -1]),
    ("TERAFEA", b"1 55 | 18014398509481985 5\n0 56 | 7\n", [18014398509481985, 5, 7], [1, -1]),
    ("SPARSE_BINARY", b"1; 3 10 11; 4 12\n0; 3 13\n", [10, 11, 12, 13], [1, -1]),
    ("SPARSE", b"1; 3 10:0.5 11:2\n", [10, 11], [1]),
    ("DENSE", b"1; 3 0.5 1.5 2.5\n", [0, 1, 2], [1]),
])
def test_text_parsers(fmt, text, keys, labels):
    b = parse_text(text, fmt, nthreads=1)
    assert b.keys.tolist() == keys
    assert b.labels.tolist() == labels


def test_terafea_groups_and_criteo():
    b = parse_text(b"1 55 | 18014398509481985 5\n", "TERAFEA")
    assert b.slots.tolist() == [1, 0]  # group id = key >> 54
    c = parse_text(b"1\t3\t\t5" + b"\t" * 11 + b"\ta1b2c3d4" + b"\t" * 25 + b"\n", "CRITEO",
                   hash_mod=10 ** 9)
    assert c.rows == 1 and c.nnz == 3 and int(c.keys.max()) < 10 ** 9


def test_parse_multithreaded_matches_single():
    lines = "".join(f"{1 if i % 3 else -1} {i % 50 + 1}:1 {i % 77 + 60}:0.5\n" for i in range(40000))
    a = parse_text(lines.encode(), "LIBSVM", nthreads=1)
    b = parse_text(lines.encode(), "LIBSVM", nthreads=4)
    assert np.array_equal(a.keys, b.keys) and np.array_equal(a.row_ptr, b.row_ptr)
    assert a.info == b.info or a.info["info"] == b.info["info"]


def test_recordio_roundtrip_and_stream_reader(tmp_path):
    b = parse_text(b"1 3:0.5 7:1\n-1 2:1\n1 9:2\n", "LIBSVM")
    raw = encode_examples(b)
    assert int.from_bytes(raw[:4], "little") == 0x3ED7230A
    back = decode_examples(raw)
    assert back.keys.tolist() == b.keys.tolist() and back.labels.tolist() == b.labels.tolist()
    for i in range(3):
        (tmp_path / f"f{i}.txt").write_text("".join(f"1 {j + 1}:1\n" for j in range(10)))
    r = StreamReader([str(tmp_path / f"f{i}.txt") for i in range(3)], "LIBSVM", 7)
    sizes = [x.rows for x in r]
    assert sum(sizes) == 30 and sizes[:4] == [7, 7, 7, 7]
    assert divide_files(list("abcde"), 2) == [["a", "c", "e"], ["b", "d"]]


def test_gzip_file_and_concat(tmp_path):
    p = str(tmp_path / "x.gz")
    core().write_file(p, b"1 1:1\n", True)
    assert core().read_file(p) == b"1 1:1\n"
    b1 = parse_text(b"1 1:1\n", "LIBSVM")
    b2 = parse_text(b"-1 2:1 3:1\n", "LIBSVM")
    c = ExampleBatch.concat([b1, b2])
    assert c.row_ptr.tolist() == [0, 1, 3]


def test_heartbeat_info_and_dashboard():
    import time

    from parameter_server_amd.system.heartbeat import Dashboard, HeartbeatInfo

    hb = HeartbeatInfo()
    x = 0
    for i in range(200000):  # burn a little CPU so the rates are non-trivial
        x += i * i
    rep = hb.get()
    for k in ("process_cpu_usage", "host_cpu_usage", "process_rss_mb", "host_in_use_mb",
              "host_net_in_mb_s", "host_net_out_mb_s"):
        assert k in rep and rep[k] >= 0
    assert rep["process_rss_mb"] > 10
    d = Dashboard()
    d.add_report("W10", rep)
    d.add_report("W2", rep)
    d.add_report("S0", rep)
    out = d.render().splitlines()
    assert "Dashboard" in out[0] and out[1].startswith("Node")
    assert [l.split()[0] for l in out[2:]] == ["S0", "W2", "W10"]
    assert d.stale(10.0) == []
    time.sleep(0.05)
    assert sorted(d.stale(0.01)) == ["S0", "W10", "W2"]
