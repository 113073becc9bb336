"""Control-plane runtime: multi-process localhost runs (reference script/local.sh
style: 1 scheduler + S servers + W workers over real sockets)."""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _launch(S, W, args, timeout=120):
    cmd = [sys.executable, "-m", "parameter_server_amd.launch", "local", str(S), str(W),
           "--timeout", str(timeout - 10), "--", sys.executable, "-u", "-m"] + args
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout)
    return r.returncode, r.stdout + r.stderr


def test_hello_world_matches_reference_output():
    rc, out = _launch(3, 2, ["parameter_server_amd.app.hello_world", "-timeout", "60"])
    assert rc == 0, out
    assert "W0: key: [4]: 0 2 4 5 ; value: [4]: 0 0.2 0.4 0.5" in out
    assert "W1: key: [4]: 0 1 3 4 ; value: [4]: 0 0.1 0.3 0.4" in out
    for s in ("S0, this is server 0", "S1, this is server 1", "S2, this is server 2"):
        assert s in out


def _write_libsvm(d, nfiles=3, rows=800, seed=0):
    rng = np.random.default_rng(seed)
    w = rng.normal(0, 1, 3000) * (rng.random(3000) < 0.2)
    os.makedirs(d, exist_ok=True)
    for p in range(nfiles):
        with open(os.path.join(d, f"part-{p}"), "w") as f:
            for _ in range(rows):
                k = np.unique(rng.integers(1, 3000, size=15))
                v = rng.random(k.size)
                y = 1 if (w[k] * v).sum() + 0.2 * rng.normal() > 0 else -1
                f.write(f"{y} " + " ".join(f"{a}:{b:.4f}" for a, b in zip(k, v)) + "\n")
    return w


@pytest.mark.parametrize("algo,extra", [("FTRL", ""), ("STANDARD", "ada_grad: true"),
                                        ("STANDARD", "ada_grad: false fixing_float_by_nbytes: 2")])
def test_async_sgd_plumbing_1_2_2_and_evaluation(tmp_path, algo, extra):
    data = tmp_path / "data"
    _write_libsvm(str(data))
    model = tmp_path / "model" / "m"
    conf = tmp_path / "online.conf"
    conf.write_text(f"""linear_method {{
training_data {{ format: TEXT text: LIBSVM file: "{data}/part.*" }}
model_output {{ format: TEXT file: "{model}" }}
loss {{ type: LOGIT }}
penalty {{ type: L1 lambda: 0.05 lambda: 0.01 }}
learning_rate {{ type: DECAY alpha: 0.5 beta: 1 }}
async_sgd {{ algo: {algo} minibatch: 200 num_data_pass: 2 {extra} }}
}}""")
    rc, out = _launch(2, 2, ["parameter_server_amd.app.main", "-app_file", str(conf),
                             "-timeout", "90"])
    assert rc == 0, out
    assert "sec  examples" in out
    files = sorted(os.listdir(model.parent))
    assert files == ["m_S0", "m_S1"], files
    assert os.path.getsize(model.parent / "m_S0") > 0
    ev = tmp_path / "eval.conf"
    ev.write_text(f"""linear_method {{
validation_data {{ format: TEXT text: LIBSVM file: "{data}/part-0" }}
model_input {{ format: TEXT file: "{model}_.*" }}
}}""")
    rc, out = _launch(0, 0, ["parameter_server_amd.app.main", "-app_file", str(ev),
                             "-timeout", "60"])
    assert rc == 0, out
    line = [l for l in out.splitlines() if l.startswith("evaluation:")][0]
    auc = float(line.split()[2])
    assert auc > 0.75, line


def test_heartbeat_detects_dead_worker_and_terminates_job():
    """Fault injection: W1 crashes; the scheduler's heartbeat watchdog fails the job and
    TERMINATEs the survivors well before the 60 s job timeout (reference: hangs)."""
    import time

    t0 = time.time()
    rc, out = _launch(1, 3, ["parameter_server_amd.app.fault_injection", "-timeout", "60",
                             "-heartbeat_interval", "0.2", "-kill_rank", "1"], timeout=90)
    assert rc != 0, out
    assert "W1: injected crash" in out
    assert "node W1 missed heartbeats" in out
    assert time.time() - t0 < 30, out


def test_heartbeat_dashboard_in_darlin_run(tmp_path):
    from parameter_server_amd.data.synthetic import sparse_classification, write_text

    sd = sparse_classification(600, groups=(1, 2), keys_per_group=100, nnz_per_row=(1, 3), seed=0)
    write_text(sd, str(tmp_path / "part-0"), "SPARSE_BINARY")
    conf = tmp_path / "b.conf"
    conf.write_text(f"""linear_method {{
training_data {{ format: TEXT text: SPARSE_BINARY file: "{tmp_path}/part-0" }}
loss {{ type: LOGIT }} penalty {{ type: L1 lambda: 1 }}
learning_rate {{ type: CONSTANT alpha: 1 }}
darlin {{ max_pass_of_data: 40 epsilon: 1e-12 }}
}}""")
    rc, out = _launch(1, 1, ["parameter_server_amd.app.main", "-app_file", str(conf),
                             "-timeout", "90", "-heartbeat_interval", "0.1", "-verbose"])
    assert rc == 0, out
    assert "Dashboard" in out and "MyRSS(M)" in out
    rows = [l.split()[0] for l in out.splitlines() if l.startswith(("S0 ", "W0 "))]
    assert "S0" in rows and "W0" in rows


def test_my_rank_auto_addressing_like_mpi():
    """Reference Van::assembleMyNode: -my_rank 0 = scheduler, 1..W workers, then servers;
    launched through scripts/mpi_node.sh with the rank in PMI_RANK."""
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, PS_SCHEDULER=f"role:SCHEDULER,hostname:'127.0.0.1',port:{port},id:'H'",
               PS_INTERFACE="lo", OMP_NUM_THREADS="1")
    procs = []
    for r in range(1 + 2 + 3):  # 2 workers (ranks 1-2), 3 servers (ranks 3-5)
        e = dict(env, PMI_RANK=str(r))
        procs.append(subprocess.Popen(
            ["bash", "scripts/mpi_node.sh", "3", "2", sys.executable, "-u", "-m",
             "parameter_server_amd.app.hello_world", "-timeout", "60"],
            cwd=ROOT, env=e, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        out, _ = p.communicate(timeout=90)
        assert p.returncode == 0, out
        outs.append(out)
    out = "".join(outs)
    assert "W0: key: [4]: 0 2 4 5 ; value: [4]: 0 0.2 0.4 0.5" in out
    assert "W1: key: [4]: 0 1 3 4 ; value: [4]: 0 0.1 0.3 0.4" in out
    assert "S2, this is server 2" in out
