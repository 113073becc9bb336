#!/usr/bin/env python3
"""BASELINE.json config 1: the reference protocol on CPU — async SGD (FTRL) with
1 scheduler + 2 servers + 2 workers on localhost (script/local.sh layout), over
this framework's TCP control plane, on synthetic Criteo-shaped text data.

The reference publishes no throughput; its only throughput signal is the
scheduler's ``sec examples ...`` progress printer (src/learner/sgd.h:45-80).
This script runs the same protocol (pull keys -> gradient -> push with key
caching) and reports examples/sec from the wall clock of the UPDATE_MODEL phase,
as a CPU reference point for the GPU numbers.

    python benchmarks/bench_plumbing.py --rows 200000 --servers 2 --workers 2
"""
import argparse
import json
import os
import re
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def write_data(d, rows, files, num_features, seed=0):
    import numpy as np

    from parameter_server_amd.ops.synthetic import criteo_batch

    os.makedirs(d, exist_ok=True)
    per = rows // files
    for f in range(files):
        k, l = criteo_batch(per, seed=seed, row0=f * per, num_features=num_features)
        k = k.view(per, 39).numpy().view(np.uint64)
        with open(os.path.join(d, f"part-{f}"), "w") as out:
            for r in range(per):
                ks = np.unique(k[r])
                out.write(("1" if l[r] > 0 else "-1") + " " +
                          " ".join(f"{int(x)}:1" for x in ks) + "\n")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=200_000)
    ap.add_argument("--files", type=int, default=8)
    ap.add_argument("--servers", type=int, default=2)
    ap.add_argument("--workers", type=int, default=2)
    ap.add_argument("--minibatch", type=int, default=10000)
    ap.add_argument("--num-features", type=float, default=1e9)
    args = ap.parse_args()
    tmp = tempfile.mkdtemp(prefix="psamd_plumb_")
    data = os.path.join(tmp, "data")
    t0 = time.time()
    write_data(data, args.rows, args.files, int(args.num_features))
    conf = os.path.join(tmp, "online.conf")
    with open(conf, "w") as f:  # example/linear/ctr/online_l1lr.conf parameters
        f.write(f"""linear_method {{
training_data {{ format: TEXT text: LIBSVM file: "{data}/part.*" }}
model_output {{ format: TEXT file: "{tmp}/model/ctr_online" }}
loss {{ type: LOGIT }}
penalty {{ type: L1 lambda: 10 lambda: 1 }}
learning_rate {{ type: DECAY alpha: .01 beta: 10 }}
async_sgd {{ algo: FTRL minibatch: {args.minibatch} num_data_pass: 1 report_interval: 1 }}
}}""")
    gen = time.time() - t0
    cmd = [sys.executable, "-m", "parameter_server_amd.launch", "local", str(args.servers),
           str(args.workers), "--timeout", "3000", "--", sys.executable, "-u", "-m",
           "parameter_server_amd.app.main", "-app_file", conf, "-timeout", "2900"]
    t1 = time.time()
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=3100)
    wall = time.time() - t1
    out = r.stdout + r.stderr
    lines = re.findall(r"^\s*(\d+)\s+(\S+)\s+(\S+)\s+(\S+)\s+(\S+)", out, re.M)
    if r.returncode != 0 or not lines:
        print(out[-3000:], file=sys.stderr)
        raise SystemExit(f"plumbing run failed (rc={r.returncode})")
    sec, ex = float(lines[-1][0]), float(lines[-1][1])
    print(json.dumps({
        "metric": "examples/sec, async SGD FTRL, 1 scheduler + "
                  f"{args.servers} servers + {args.workers} workers on CPU localhost",
        "value": ex / wall, "unit": "examples/sec", "examples": ex, "wall_sec": wall,
        "printer_last_sec": sec, "data_gen_sec": gen,
        "config": {"rows": args.rows, "minibatch": args.minibatch,
                   "num_features": int(args.num_features), "nnz_per_example": "<=39"},
        "last_progress_line": " ".join(lines[-1]),
    }))


if __name__ == "__main__":
    main()
