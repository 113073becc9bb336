"""bench.py's multi-stream software pipeline must train exactly what the plain
sequential trainer trains: the same minibatches (per-stream row counters), the
exchange half of step t on the preparation stream of minibatch t (or on its own
stream) overlapping the worker half of step t-1, SSP lag 1. Any missing stream
dependency shows up here as different weights (an exchange reading a buffer
before its localisation, two owner updates racing, a push applied early/late).

Runs on one GPU over the loopback exchange (2 emulated ranks: the padded
exchange, owner updates and SSP split are the N-GPU code paths)."""
import argparse
import importlib.util
import os

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("psamd_bench", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _trainer(B, N, **kw):
    from parameter_server_amd.models import SparseLRConfig, SparseLRTrainer
    from parameter_server_amd.parallel.comm import LoopbackComm

    args = dict(num_features=N, minibatch=B, algo="ftrl", lr_type="decay", alpha=0.01,
                beta=10.0, l1=10.0, l2=1.0, consistency="ssp:4")
    args.update(kw)
    cfg = SparseLRConfig(**args)
    tr = SparseLRTrainer(cfg, LoopbackComm(2, "cuda"), "cuda")
    assert tr.padded
    return tr


def _weights(tr):
    keys, w, _, _ = tr.table.occupied()
    o = torch.argsort(keys)
    return keys[o].cpu(), w[o].float().cpu()


@pytest.mark.parametrize("xmode,nprep,graph,kw", [
    ("prep", 2, 1, {}), ("prep", 1, 1, {}), ("own", 2, 1, {}), ("prep", 3, 0, {}),
    ("prep", 3, 1, {}), ("prep", 3, 1, {"consistency": "ssp:2"}),
    ("prep", 2, 1, {"consistency": "ssp:1"}), ("prep", 2, 1, {"consistency": "ssp:2"}),
    ("prep", 3, 1, {"consistency": "bsp"}),
    ("prep", 2, 1, {"fixing_float_bytes": 2}), ("prep", 2, 1, {"push_mode": "aggregate"}),
    ("prep", 2, 1, {"algo": "adagrad"}),
    ("prep", 2, 1, {"ssp_apply": "pre"}), ("prep", 3, 1, {"ssp_apply": "pre", "consistency": "ssp:1"}),
    ("prep", 2, 1, {"_env": {"PSAMD_CAPTURE_COMM": "0"}}),
    ("prep", 3, 1, {"consistency": "bsp", "_env": {"PSAMD_CAPTURE_COMM": "0"}}),
    # the merged one-collective exchange (auto for ssp >= 2 / asp), against the
    # two-collective sequential trainer: same staleness, same table
    ("prep", 3, 1, {"exchange_merge": "on"}), ("prep", 3, 0, {"exchange_merge": "on"}),
    ("prep", 2, 1, {"exchange_merge": "on", "consistency": "ssp:2"}),
    ("prep", 3, 1, {"exchange_merge": "on", "consistency": "ssp:3"}),
    ("prep", 3, 1, {"exchange_merge": "on", "fixing_float_bytes": 2}),
    ("prep", 3, 1, {"exchange_merge": "on", "push_mode": "aggregate"}),
    ("prep", 3, 1, {"exchange_merge": "on", "_env": {"PSAMD_CAPTURE_COMM": "0"}}),
    # ... and its graphs replayed from one native launch list per iteration
    ("prep", 3, 1, {"exchange_merge": "on", "_env": {"PSAMD_MX_NATIVE": "1"}}),
    ("prep", 2, 1, {"exchange_merge": "on", "consistency": "ssp:2",
                    "_env": {"PSAMD_MX_NATIVE": "1"}}),
    # ... and from two graphs per iteration with the event waits / records as external
    # event nodes inside them
    ("prep", 3, 1, {"exchange_merge": "on", "_env": {"PSAMD_MX_NATIVE": "1", "PSAMD_MX_G2": "1"}}),
    ("prep", 2, 1, {"exchange_merge": "on", "consistency": "ssp:2",
                    "_env": {"PSAMD_MX_NATIVE": "1", "PSAMD_MX_G2": "1"}}),
    # the tail filter inside the flat localiser: preparations in minibatch order
    ("prep", 3, 1, {"exchange_merge": "on", "tail_feature_freq": 1}),
    ("prep", 3, 1, {"exchange_merge": "on", "tail_feature_freq": 1,
                    "_env": {"PSAMD_MX_NATIVE": "1", "PSAMD_MX_G2": "1"}}),
    ("prep", 2, 1, {"tail_feature_freq": 1})])
def test_pipeline_matches_sequential(monkeypatch, xmode, nprep, graph, kw):
    from parameter_server_amd.ops.synthetic import criteo_batch

    monkeypatch.setenv("PSAMD_XCHG_STREAM", xmode)
    kw = dict(kw)
    for k, v in kw.pop("_env", {}).items():  # (default: collectives captured in the graphs)
        monkeypatch.setenv(k, v)
    kw.setdefault("exchange_merge", "off")  # (the two-collective pipeline unless "on")
    bench = _bench()
    B, N, seed, extra = 4096, 10 ** 6, 77, 5
    dev = torch.device("cuda")
    tr = _trainer(B, N, **kw)
    assert tr.merged == (kw["exchange_merge"] == "on")
    keys = torch.empty(B * 39, dtype=torch.int64, device=dev)
    labels = torch.empty(B, dtype=torch.float32, device=dev)
    args = argparse.Namespace(warmup=0, graph=graph)
    it, _ = bench.pipeline(tr, B, N, seed, keys, labels, dev, args, nprep=nprep)
    for _ in range(extra):
        it()
    torch.cuda.synchronize()
    T = tr._xt  # worker steps the pipeline ran
    # pushes no issued exchange carried yet (none in prep mode, nprep >= 2)
    tr.mx_drain() if tr.merged else tr._x_flush()
    pk, pw = _weights(tr)
    loss_p = tr.progress()["loss"]

    kw_ref = dict(kw, exchange_merge="off")  # the two-collective schedule, same bound
    ref = _trainer(B, N, **kw_ref)
    for m in range(T):
        k, lab = criteo_batch(B, seed=seed, row0=m * B, num_features=N, device=dev)
        ref.step(k, lab, width=39)
    ref.flush()
    torch.cuda.synchronize()
    rk, rw = _weights(ref)
    # the pipeline also resolved (inserted) the keys of the minibatches prepared
    # ahead: those carry no update (w = 0); every trained key must agree
    pos = torch.searchsorted(pk, rk)
    assert torch.equal(pk[pos], rk)
    # FixingFloat: a 1-ulp difference of a gradient (hot-key sums combine per-wave
    # pieces atomically, in any order) can flip one stochastic-rounding step
    atol = 2e-5 if kw.get("fixing_float_bytes") else 1e-6
    assert torch.allclose(pw[pos], rw, rtol=1e-4, atol=atol), (pw[pos] - rw).abs().max()
    extra_mask = torch.ones(pk.numel(), dtype=torch.bool)
    extra_mask[pos] = False
    assert torch.all(pw[extra_mask] == 0)
    assert abs(loss_p - ref.progress()["loss"]) < 1e-4


def _g2_parity_main(env: str):
    """(run in a fresh process: a 1-rank RCCL group) the merged pipeline on the 2-peer
    RCCL loopback -- native launch lists, or PSAMD_MX_G2 two graph chains per iteration --
    against the two-collective sequential trainer; prints the max weight difference."""
    import json

    from parameter_server_amd.models import SparseLRConfig, SparseLRTrainer
    from parameter_server_amd.ops.synthetic import criteo_batch
    from parameter_server_amd.parallel.comm import LoopbackComm, nccl_loopback

    env = json.loads(env)
    tail = int(env.pop("TAIL", "0"))
    os.environ.update(env)
    bench = _bench()
    B, N, seed, extra = 4096, 10 ** 6, 77, 9
    dev = torch.device("cuda", 0)
    kw = dict(num_features=N, minibatch=B, consistency="ssp:4", exchange_merge="on",
              tail_feature_freq=tail)
    tr = SparseLRTrainer(SparseLRConfig(**kw), nccl_loopback(2, dev), dev)
    assert tr.merged
    keys = torch.empty(B * 39, dtype=torch.int64, device=dev)
    labels = torch.empty(B, dtype=torch.float32, device=dev)
    args = argparse.Namespace(warmup=0, graph=1)
    it, _ = bench.pipeline(tr, B, N, seed, keys, labels, dev, args, nprep=3)
    for _ in range(extra):
        it()
    torch.cuda.synchronize()
    T = tr._xt
    tr.mx_drain()
    pk, pw = _weights(tr)
    ref = SparseLRTrainer(SparseLRConfig(**dict(kw, exchange_merge="off")),
                          LoopbackComm(2, "cuda"), dev)
    for m in range(T):
        k, lab = criteo_batch(B, seed=seed, row0=m * B, num_features=N, device=dev)
        ref.step(k, lab, width=39)
    ref.flush()
    torch.cuda.synchronize()
    rk, rw = _weights(ref)
    pos = torch.searchsorted(pk, rk)
    assert torch.equal(pk[pos], rk)
    print(json.dumps({"native": getattr(args, "native_iter", None), "steps": T,
                      "maxdiff": float((pw[pos] - rw).abs().max())}), flush=True)


@pytest.mark.parametrize("g2,tail", [("0", "0"), ("1", "0"), ("0", "1"), ("1", "1")])
def test_merged_native_rccl_pipeline_matches_sequential(g2, tail):
    """The merged pipeline's native iteration on a real (1-rank RCCL) communicator, with
    the event ops as host calls (launch lists) or as event nodes inside two graph chains
    per iteration (PSAMD_MX_G2=1): same table as the sequential trainer."""
    import json
    import subprocess
    import sys

    env = json.dumps({"PSAMD_MX_G2": g2, "PSAMD_MX_NATIVE": "1", "TAIL": tail})
    code = ("import sys; sys.path.insert(0, 'tests'); import test_bench_pipeline_gpu as t; "
            f"t._g2_parity_main({env!r})")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True,
                       timeout=240, env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))
    assert r.returncode == 0, r.stdout + r.stderr
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["native"] == ("graph2" if g2 == "1" else True), out
    assert out["maxdiff"] < 1e-5, out


@pytest.mark.parametrize("apply", ["stream", "tail"])
def test_asp_pipeline_trains(monkeypatch, apply):
    """asp: the owner's push applies replay on their own stream (or at the tail of the
    exchange half) and pulls never wait for them, so the result is timing dependent;
    it must still train every key and stay within the ring (flush applies everything)."""
    monkeypatch.setenv("PSAMD_XCHG_STREAM", "prep")
    monkeypatch.setenv("PSAMD_ASP_APPLY", apply)
    bench = _bench()
    B, N, seed = 4096, 10 ** 6, 78
    dev = torch.device("cuda")
    tr = _trainer(B, N, consistency="asp", exchange_merge="off")
    assert tr.asp and tr.R == tr.lag + 1 + tr.async_depth
    keys = torch.empty(B * 39, dtype=torch.int64, device=dev)
    labels = torch.empty(B, dtype=torch.float32, device=dev)
    args = argparse.Namespace(warmup=0, graph=1)
    it, used = bench.pipeline(tr, B, N, seed, keys, labels, dev, args, nprep=2)
    assert used
    for _ in range(12):
        it()
    torch.cuda.synchronize()
    p = tr.progress()
    assert 0.0 < p["loss"] < 0.7 and p["nnz_w"] > 0
    tr.table.check_ok()


@pytest.mark.parametrize("consistency", ["asp", "bsp", "ssp:4"])
def test_bench_captured_collectives_exit_cleanly(consistency):
    """bench.py with emulated peers over the real 1-rank RCCL communicator: the
    all-to-alls replay inside the step graphs, and the process exits (graphs released
    before the process group is destroyed; round 2's capture attempt hung at exit)."""
    import json
    import subprocess
    import sys

    env = dict(os.environ, PSAMD_CAPTURE_COMM="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "20",
                        "--warmup", "6", "--emulate-peers", "4", "--minibatch", "16384",
                        "--consistency", consistency],
                       capture_output=True, text=True, timeout=100, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["config"]["hip_graph"] and out["config"]["emulated_peers"] == 4
    assert out["config"]["collectives_in_graphs"]
    assert out["comm"]["rccl_world"] == 1


@pytest.mark.parametrize("nprep,native,tail", [(1, "0", 0), (2, "0", 0), (2, "1", 0), (3, "1", 0),
                                               (3, "1", 1), (2, "0", 1)])
def test_flat_pipeline_matches_sequential(monkeypatch, nprep, native, tail):
    """1 GPU, flat layout: step t pulls minibatch t+1 inside its update launch, so every
    preparation must finish before the step that pulls it and must not refill a buffer a
    pending step still reads (nprep = 1 is run with 2 streams). The pipeline -- eager
    launch lists or the one-call native iteration -- must leave exactly the table that
    plain sequential ``step()`` calls leave."""
    from parameter_server_amd.models import SparseLRConfig, SparseLRTrainer
    from parameter_server_amd.ops.synthetic import criteo_batch

    monkeypatch.setenv("PSAMD_FLAT", "1")
    monkeypatch.setenv("PSAMD_NATIVE_ITER", native)
    bench = _bench()
    B, N, seed, extra = 4096, 10 ** 8, 91, 7
    dev = torch.device("cuda")

    def trainer():
        cfg = SparseLRConfig(num_features=N, minibatch=B, table_capacity=1 << 22,
                             tail_feature_freq=tail, countmin_n=1 << 20)
        tr = SparseLRTrainer(cfg, device=dev)
        assert tr.localize_mode == "tpf" and not tr.padded
        return tr

    tr = trainer()
    keys = torch.empty(B * 39, dtype=torch.int64, device=dev)
    labels = torch.empty(B, dtype=torch.float32, device=dev)
    args = argparse.Namespace(warmup=0, graph=0, prep_streams=nprep)
    it, _ = bench.pipeline(tr, B, N, seed, keys, labels, dev, args, nprep=nprep)
    assert args.prep_streams >= 2
    assert (getattr(args, "native_iter", False) is True) == (native == "1")
    for _ in range(extra):
        it()
    torch.cuda.synchronize()
    T = tr.step_count
    pk, pw = _weights(tr)
    loss_p = tr.progress()["loss"]
    ref = trainer()
    for m in range(T):
        k, lab = criteo_batch(B, seed=seed, row0=m * B, num_features=N, device=dev)
        ref.step(k, lab, width=39)
    torch.cuda.synchronize()
    rk, rw = _weights(ref)
    # the pipeline also pulled (inserted, w = 0) the minibatch after the last step
    pos = torch.searchsorted(pk, rk)
    assert torch.equal(pk[pos], rk)
    assert torch.equal(pw[pos], rw)
    extra_mask = torch.ones(pk.numel(), dtype=torch.bool)
    extra_mask[pos] = False
    assert torch.all(pw[extra_mask] == 0)
    assert abs(loss_p - ref.progress()["loss"]) < 1e-5


@pytest.mark.parametrize("kw", [{"consistency": "ssp:4"}, {"consistency": "ssp:2"},
                                {"consistency": "ssp:4", "fixing_float_bytes": 2}])
def test_merged_sequential_matches_two_collective(kw):
    """The sequential API on the merged exchange (step u trains minibatch u-1, flush the
    last) leaves exactly the table the two-collective schedule leaves (same staleness
    bound), on the GPU kernels (strided weight rows, in-place unpack)."""
    from parameter_server_amd.ops.synthetic import criteo_batch

    B, N = 4096, 10 ** 6
    dev = torch.device("cuda")
    outs = []
    for merge in ("on", "off"):
        tr = _trainer(B, N, exchange_merge=merge, **kw)
        assert tr.merged == (merge == "on")
        for m in range(7):
            k, lab = criteo_batch(B, seed=5, row0=m * B, num_features=N, device=dev)
            tr.step(k, lab, width=39)
        p = tr.progress()
        assert p["examples"] == 7 * B
        outs.append((_weights(tr), p))
    (k1, w1), p1 = outs[0]
    (k2, w2), p2 = outs[1]
    assert torch.equal(k1, k2)
    atol = 2e-5 if kw.get("fixing_float_bytes") else 1e-6
    assert torch.allclose(w1, w2, rtol=1e-4, atol=atol)
    assert abs(p1["loss"] - p2["loss"]) < 1e-4
