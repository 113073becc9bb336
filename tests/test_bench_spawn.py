"""bench.py contract: ``python bench.py --gpus N`` fans out N ranks by itself
(no torchrun in front) and rank 0 prints one JSON line for the whole job."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--cpu", *args],
                         capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    return json.loads(lines[0])


def test_bench_self_spawns_ranks():
    B = 1024
    r = _run("--gpus", "3", "--steps", "2", "--warmup", "1", "--minibatch", str(B),
             "--num-features", "1e6")
    assert r["n_gpus"] == 3
    assert r["config"]["global_batch"] == 3 * B
    assert r["config"]["parallelism"] == "dp3+kvshard3"
    assert r["value"] > 0 and r["steps"] == 2


def test_bench_single_rank_unchanged():
    B = 1024
    r = _run("--gpus", "1", "--steps", "2", "--warmup", "1", "--minibatch", str(B),
             "--num-features", "1e6")
    assert r["n_gpus"] == 1 and r["config"]["global_batch"] == B
    for k in ("metric", "value", "unit", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data"):
        assert k in r


def test_bench_stalled_rank_fails_fast():
    """A rank that stops joining collectives (injected sleep at timed step 1) makes the
    job exit non-zero within the collective timeout, and the surviving ranks name
    their rank, phase, step and last collective (no silent hang)."""
    import time

    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(PSAMD_COMM_TIMEOUT="8", PSAMD_INJECT_STALL="1:1:600")
    t0 = time.time()
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--cpu", "--gpus", "3",
                          "--steps", "4", "--warmup", "1", "--minibatch", "1024",
                          "--num-features", "1e6"],
                         capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    dt = time.time() - t0
    assert out.returncode != 0
    assert dt < 120, dt
    assert "[psamd] FAILED rank 0: phase timed" in out.stderr or \
        "[psamd] FAILED rank 2: phase timed" in out.stderr, out.stderr[-3000:]
    assert not [ln for ln in out.stdout.splitlines() if ln.startswith("{")]


def test_bench_failed_captured_attempt_reruns_eagerly():
    """Multi-rank runs go through per-rank supervisors: when the first attempt (the
    collectives captured in the step graphs) fails on the ranks, every supervisor re-runs
    the job in fresh processes with eager collectives, and rank 0 still prints exactly
    one JSON line, which records the fallback."""
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(PSAMD_INJECT_CAPTURE_FAIL="1")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--cpu", "--gpus", "3",
                          "--steps", "2", "--warmup", "1", "--minibatch", "1024",
                          "--num-features", "1e6"],
                         capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    assert "re-running in fresh processes with eager collectives" in out.stderr
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    r = json.loads(lines[0])
    assert r["n_gpus"] == 3 and r["comm"]["fallback"] == 3 and r["comm"]["captured"] is False


def _spawn_env(**extra):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(extra)
    return env


def test_bench_post_timing_rank_failure_is_reported():
    """A rank that exits non-zero AFTER the timed region (rank 2, injected) does not void
    the measurement, but the JSON line records which rank failed with what code."""
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--cpu", "--gpus", "3",
                          "--steps", "2", "--warmup", "1", "--minibatch", "1024",
                          "--num-features", "1e6"],
                         capture_output=True, text=True, timeout=300, cwd=ROOT,
                         env=_spawn_env(PSAMD_INJECT_POST_EXIT="2:7"))
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    r = json.loads(lines[0])
    assert r["comm"]["post_timing_failures"] == [2]
    assert r["comm"]["rank_exit_codes"][2] == 7
    assert "re-running" not in out.stderr  # a complete measurement is not re-run


def test_bench_teardown_hang_is_capped():
    """A rank hanging after the timed region is killed PSAMD_TEARDOWN_TIMEOUT seconds
    after it passed the timed region, not at the attempt limit."""
    import time

    t0 = time.time()
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--cpu", "--gpus", "2",
                          "--steps", "2", "--warmup", "1", "--minibatch", "1024",
                          "--num-features", "1e6"],
                         capture_output=True, text=True, timeout=300, cwd=ROOT,
                         env=_spawn_env(PSAMD_INJECT_TEARDOWN_HANG="1:600",
                                        PSAMD_TEARDOWN_TIMEOUT="5"))
    assert out.returncode == 0, out.stderr[-3000:]
    assert time.time() - t0 < 150
    r = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][0])
    assert r["comm"]["post_timing_failures"] == [1]
    assert r["comm"]["rank_exit_codes"][1] == 125
