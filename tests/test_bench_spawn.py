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
