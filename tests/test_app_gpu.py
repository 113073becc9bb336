"""The GPU app path (app/gpu.py): a reference ``.conf`` + LIBSVM text files ->
DeviceFeeder (C++ parser, pinned staging, async host->HBM copies) -> SparseLRTrainer /
DarlinTrainer, progress lines and ``<file>_S<rank>`` text models.

Anchors:
* the app's table equals a plain-PyTorch fp32 FTRL loop over the same minibatches
  (same files, same order; valued, variable-width rows) to rtol 1e-4;
* the same conf through the CPU runtime app (1 scheduler + 1 server + 1 worker over
  TCP, reference script/local.sh) reaches the same loss / AUC and weights within
  tolerance (that app pipelines pulls ahead of pushes, as the reference does, so it is
  not bitwise the synchronous GPU run);
* multi-rank (gloo, world 2) with files that run out unevenly: the rank without data
  keeps joining the exchanges (idle steps) and both ranks finish."""
import os
import socket
import subprocess
import sys
import types

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _write_libsvm(d, nfiles=3, rows=600, seed=0, nkeys=3000, binary_width=0):
    rng = np.random.default_rng(seed)
    w = rng.normal(0, 1, nkeys) * (rng.random(nkeys) < 0.2)
    os.makedirs(d, exist_ok=True)
    for p in range(nfiles):
        with open(os.path.join(d, f"part-{p}"), "w") as f:
            for _ in range(rows):
                if binary_width:
                    k = np.sort(rng.choice(np.arange(1, nkeys), binary_width, replace=False))
                    v = np.ones(k.size)
                    y = 1 if w[k].sum() + 0.2 * rng.normal() > 0 else -1
                    f.write(f"{y} " + " ".join(f"{a}:1" for a in k) + "\n")
                    continue
                k = np.unique(rng.integers(1, nkeys, size=int(rng.integers(5, 40))))
                v = rng.random(k.size)
                y = 1 if (w[k] * v).sum() + 0.2 * rng.normal() > 0 else -1
                f.write(f"{y} " + " ".join(f"{a}:{b:.4f}" for a, b in zip(k, v)) + "\n")


def _conf(tmp_path, data, model, minibatch=200, passes=1, algo="FTRL", max_delay=0):
    c = tmp_path / "online.conf"
    c.write_text(f"""linear_method {{
training_data {{ format: TEXT text: LIBSVM file: "{data}/part.*" }}
model_output {{ format: TEXT file: "{model}" }}
loss {{ type: LOGIT }}
penalty {{ type: L1 lambda: 0.05 lambda: 0.01 }}
learning_rate {{ type: DECAY alpha: 0.5 beta: 1 }}
async_sgd {{ algo: {algo} minibatch: {minibatch} num_data_pass: {passes} max_delay: {max_delay}
             report_interval: 1 }}
}}""")
    return c


def _flags(**kw):
    d = dict(app_file=None, app_conf=None, num_features=0, max_nnz_per_example=128,
             num_threads=2, device="cpu", seed=0, table_capacity=1 << 16, quiet=True)
    d.update(kw)
    return types.SimpleNamespace(**d)


def _reference_ftrl(files, minibatch, rule):
    """Plain fp32 FTRL over the files' rows in order, one update per minibatch (the
    per-key rule of kv_slot.cuh; reference async_sgd.h:107-119), valued features."""
    from parameter_server_amd.data import ExampleBatch, parse_text, read_file

    b = ExampleBatch.concat([parse_text(read_file(f), "LIBSVM", ignore_slot=True)
                             for f in files])
    keys = torch.from_numpy(b.keys.view(np.int64).copy())
    allk = torch.unique(keys)
    K = allk.numel()
    W, Z, Nn = torch.zeros(K), torch.zeros(K), torch.zeros(K)
    rp = b.row_ptr.astype(np.int64)
    for a in range(0, b.rows, minibatch):
        e = min(a + minibatch, b.rows)
        s0, s1 = int(rp[a]), int(rp[e])
        idx = torch.searchsorted(allk, keys[s0:s1])
        x = torch.from_numpy(b.vals[s0:s1].astype(np.float32))
        row = torch.repeat_interleave(torch.arange(e - a), torch.from_numpy(np.diff(rp[a:e + 1])))
        m = torch.zeros(e - a, dtype=torch.float64).index_add_(0, row, (W[idx] * x).double()).float()
        y = torch.from_numpy(b.labels[a:e].astype(np.float32))
        yy = torch.where(y > 0, 1.0, -1.0)
        coef = -yy * torch.sigmoid(-yy * m)
        g = torch.zeros(K, dtype=torch.float64).index_add_(0, idx, (coef[row] * x).double()).float()
        u = torch.unique(idx)
        gu, w_old = g[u], W[u]
        n_new = torch.sqrt(Nn[u] * Nn[u] + gu * gu)
        sigma = (n_new - Nn[u]) / rule.alpha
        Z[u] = Z[u] + gu - sigma * w_old
        Nn[u] = n_new
        eta = rule.alpha / (n_new + rule.beta)
        zz = -Z[u] * eta
        leta = rule.l1 * eta
        W[u] = torch.where(zz.abs() <= leta, torch.zeros_like(zz),
                           (zz - torch.sign(zz) * leta) / (1 + rule.l2 * eta))
    return allk, W


def _read_models(prefix_dir):
    keys, ws = [], []
    for name in sorted(os.listdir(prefix_dir)):
        with open(os.path.join(prefix_dir, name)) as f:
            for ln in f:
                k, w = ln.split("\t")
                keys.append(int(k))
                ws.append(float(w))
    return dict(zip(keys, ws))


def _app_vs_fp32(tmp_path, device, num_features):
    from parameter_server_amd.app.gpu import run_async_sgd
    from parameter_server_amd.parallel.comm import LocalComm
    from parameter_server_amd.utils.config import load_app_config, lm_to_sparse_lr

    data, model = tmp_path / "data", tmp_path / "model" / "m"
    _write_libsvm(str(data))
    conf = load_app_config(str(_conf(tmp_path, data, model)))
    lm = conf.linear_method
    dev = torch.device(device)
    res = run_async_sgd(lm, LocalComm(dev), dev, _flags(num_features=num_features,
                                                        device=device))
    assert res["examples"] == 3 * 600 and res["steps"] == 9
    assert os.path.basename(res["model"]) == "m_S0"
    files = [str(data / f"part-{p}") for p in range(3)]
    allk, W = _reference_ftrl(files, 200, lm_to_sparse_lr(lm).update_rule())
    tr = res["trainer"]
    from parameter_server_amd.ops.keymix import unmix

    k, w, _, _ = tr.table.occupied()
    raw = unmix(k, tr.bits).cpu()
    o = torch.argsort(raw)
    assert torch.equal(raw[o], allk)
    torch.testing.assert_close(w.cpu()[o], W, rtol=1e-4, atol=1e-5)
    assert (W != 0).sum() > 50
    saved = _read_models(model.parent)  # non-zero weights only
    assert set(saved) == set(allk[W != 0].tolist())
    return res


def test_app_async_sgd_cpu_matches_fp32_loop(tmp_path):
    res = _app_vs_fp32(tmp_path, "cpu", 0)
    p = res["progress"]
    assert 0 < p["loss"] < 0.69 and p["auc"] > 0.55


@pytest.mark.gpu
@pytest.mark.parametrize("num_features", [0, 1 << 12])
def test_app_async_sgd_gpu_matches_fp32_loop(tmp_path, num_features):
    """raw 64-bit keys (sort localisation) and 12-bit hashed keys (tile localisation)."""
    res = _app_vs_fp32(tmp_path, "cuda", num_features)
    assert res["h2d_bytes"] > 0


@pytest.mark.gpu
def test_app_fixed_width_binary_rows_take_the_flat_path(tmp_path):
    from parameter_server_amd.app.gpu import run_async_sgd
    from parameter_server_amd.parallel.comm import LocalComm
    from parameter_server_amd.utils.config import load_app_config

    data, model = tmp_path / "data", tmp_path / "model" / "m"
    _write_libsvm(str(data), binary_width=16)
    lm = load_app_config(str(_conf(tmp_path, data, model, minibatch=256))).linear_method
    dev = torch.device("cuda")
    res = run_async_sgd(lm, LocalComm(dev), dev, _flags(num_features=1 << 12, device="cuda"))
    tr = res["trainer"]
    assert tr.localize_mode == "tpf" and tr._compact is None  # never left the flat path
    assert res["progress"]["auc"] > 0.6


def _launch(S, W, args, timeout=150):
    cmd = [sys.executable, "-m", "parameter_server_amd.launch", "local", str(S), str(W),
           "--timeout", str(timeout - 10), "--", sys.executable, "-u", "-m"] + args
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout)
    return r.returncode, r.stdout + r.stderr


def test_app_matches_cpu_runtime_app(tmp_path):
    """Same conf, same files: the CPU runtime app (scheduler + server + worker over TCP)
    and the GPU app (here on CPU tensors) end at the same loss / AUC and weights within
    tolerance."""
    from parameter_server_amd.app.gpu import main

    data = tmp_path / "data"
    _write_libsvm(str(data))
    m_rt, m_app = tmp_path / "rt" / "m", tmp_path / "app" / "m"
    c_rt = _conf(tmp_path, data, m_rt, max_delay=1)
    rc, out = _launch(1, 1, ["parameter_server_amd.app.main", "-app_file", str(c_rt),
                             "-timeout", "120"])
    assert rc == 0, out
    rt_lines = [ln.split() for ln in out.splitlines() if ln.strip()[:1].isdigit()
                and len(ln.split()) == 7]
    # (a report interval in which no minibatch finished prints loss 0)
    rt_lines = [ln for ln in rt_lines if float(ln[2]) > 0]
    c_app = tmp_path / "app.conf"
    c_app.write_text(c_rt.read_text().replace(str(m_rt), str(m_app)))
    assert main(["-app_file", str(c_app), "-device", "cpu", "-quiet"]) == 0
    w_rt, w_app = _read_models(m_rt.parent), _read_models(m_app.parent)
    keys = sorted(set(w_rt) | set(w_app))
    a = np.array([w_rt.get(k, 0.0) for k in keys])
    b = np.array([w_app.get(k, 0.0) for k in keys])
    assert np.linalg.norm(a - b) <= 0.25 * np.linalg.norm(b), np.linalg.norm(a - b) / np.linalg.norm(b)
    assert np.corrcoef(a, b)[0, 1] > 0.95
    # the runtime app's last progress line (loss, auc) against the GPU app's run
    from parameter_server_amd.app.gpu import run_async_sgd
    from parameter_server_amd.parallel.comm import LocalComm
    from parameter_server_amd.utils.config import load_app_config

    # (one progress window over the whole run: the app's time-based windows would make
    # the comparison depend on how fast this host runs it)
    c_one = tmp_path / "app_one.conf"
    c_one.write_text(c_app.read_text().replace("report_interval: 1", "report_interval: 100000"))
    lm = load_app_config(str(c_one)).linear_method
    res = run_async_sgd(lm, LocalComm("cpu"), torch.device("cpu"), _flags())
    assert res["progress"]["examples"] == 3 * 600
    loss_rt, auc_rt = float(rt_lines[-1][2]), float(rt_lines[-1][3])
    assert abs(loss_rt - res["progress"]["loss"]) < 0.1, (loss_rt, res["progress"])
    assert abs(auc_rt - res["progress"]["auc"]) < 0.1, (auc_rt, res["progress"])


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _mr_worker(rank, world, port, conf, out_dir):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from parameter_server_amd.app.gpu import run_async_sgd
    from parameter_server_amd.parallel.comm import DistComm
    from parameter_server_amd.utils.config import load_app_config

    torch.set_num_threads(1)
    lm = load_app_config(conf).linear_method
    res = run_async_sgd(lm, DistComm("cpu"), torch.device("cpu"), _flags(table_capacity=1 << 15))
    torch.save({"steps": res["steps"], "idle": res["idle_steps"], "examples": res["examples"],
                "progress": res["progress"]}, os.path.join(out_dir, f"r{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_app_two_ranks_uneven_files(tmp_path):
    """3 files over 2 ranks (rank 0: 2 files, rank 1: 1): rank 1 runs out first and
    joins the remaining exchanges with idle steps; both write their shard's model."""
    import torch.multiprocessing as mp

    data, model = tmp_path / "data", tmp_path / "model" / "m"
    _write_libsvm(str(data))
    conf = _conf(tmp_path, data, model, max_delay=2)
    mp.spawn(_mr_worker, args=(2, _port(), str(conf), str(tmp_path)), nprocs=2, join=True)
    r = [torch.load(tmp_path / f"r{i}.pt") for i in range(2)]
    assert r[0]["examples"] == 1200 and r[1]["examples"] == 600
    assert r[0]["steps"] == 6 and r[1]["steps"] == 3 and r[1]["idle"] == 3
    assert r[0]["progress"]["loss"] < 0.69
    assert sorted(os.listdir(model.parent)) == ["m_S0", "m_S1"]


def _darlin_files(tmp_path):
    """3 SPARSE_BINARY files of grouped rows and a reference batch_l1lr-style conf."""
    from parameter_server_amd.data.slot_reader import SlotData
    from parameter_server_amd.data.synthetic import sparse_classification, write_text

    sd = sparse_classification(1800, groups=(1, 2, 3), keys_per_group=300,
                               nnz_per_row=(1, 3, 5), seed=3)
    data = tmp_path / "data"
    data.mkdir(parents=True)
    n = sd.rows // 3
    for p in range(3):
        a, b = p * n, (p + 1) * n
        part = SlotData(labels=sd.labels[a:b], groups={
            g: (off[a:b + 1] - off[a], k[off[a]:off[b]], None)
            for g, (off, k, v) in sd.groups.items()})
        write_text(part, str(data / f"part-{p}"), "SPARSE_BINARY")
    model = tmp_path / "model" / "m"
    conf = tmp_path / "batch.conf"
    conf.write_text(f"""linear_method {{
training_data {{ format: TEXT text: SPARSE_BINARY file: "{data}/part.*" }}
model_output {{ format: TEXT file: "{model}" }}
loss {{ type: LOGIT }}
penalty {{ type: L1 lambda: 1 }}
learning_rate {{ type: CONSTANT alpha: 1 }}
darlin {{ max_pass_of_data: 6 epsilon: 1e-9 feature_block_ratio: 2
  random_feature_block_order: false max_block_delay: 1 }}
}}""")
    return data, model, conf


def _app_darlin(tmp_path, device):
    """The app's darlin path (DarlinConfig.from_lm, files read by SlotReader, text model
    <file>_S0) against DarlinTrainer built directly on the same files and settings."""
    from parameter_server_amd.app.gpu import run_darlin
    from parameter_server_amd.data.slot_reader import SlotReader
    from parameter_server_amd.models.darlin import DarlinConfig, DarlinTrainer
    from parameter_server_amd.parallel.comm import LocalComm
    from parameter_server_amd.utils.config import load_app_config

    data, model, conf = _darlin_files(tmp_path)
    lm = load_app_config(str(conf)).linear_method
    dev = torch.device(device)
    res = run_darlin(lm, LocalComm(dev), dev, _flags(device=device))
    assert res["examples"] == 1800 and res["passes"] == 6
    assert os.path.basename(res["model"]) == "m_S0"
    cfg = DarlinConfig.from_lm(lm)
    assert (cfg.l1, cfg.eta, cfg.tau, cfg.max_pass, cfg.block_ratio, cfg.random_order) == \
        (1.0, 1.0, 1, 6, 2.0, False)
    full = SlotReader(sorted(str(p) for p in data.iterdir()), "SPARSE_BINARY").read()
    ref = DarlinTrainer(full, cfg, device=dev).train()
    objs = [p.objective for p in res["trainer"].progress]
    np.testing.assert_allclose(objs, [p.objective for p in ref], rtol=1e-6)
    assert objs[-1] < objs[0]
    keys, w = res["trainer"].model()
    want = {int(k): float(v) for k, v in zip(keys, w) if v != 0}
    saved = _read_models(model.parent)
    assert set(saved) == set(want) and len(want) > 10
    for k in want:
        assert abs(saved[k] - want[k]) < 1e-4 * max(1.0, abs(want[k]))
    return objs


def test_app_darlin_cpu_matches_trainer(tmp_path):
    _app_darlin(tmp_path, "cpu")


@pytest.mark.gpu
def test_app_darlin_gpu_matches_trainer_and_cpu(tmp_path):
    g = _app_darlin(tmp_path / "g", "cuda")
    c = _app_darlin(tmp_path / "c", "cpu")
    np.testing.assert_allclose(g, c, rtol=1e-5)
