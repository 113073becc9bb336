"""File-fed throughput of the GPU app (app/gpu.py): reference ``.conf`` + LIBSVM text
files -> C++ parser threads -> pinned staging -> async host->HBM copies -> the HBM
trainer. Generates the files first (not timed), then runs the app and reports
examples/s of the whole run (parse + copy + train), next to the trainer-only rate of
the same minibatches already in HBM.

    python benchmarks/bench_app.py --rows 2000000 --files 8 --minibatch 10000 --kind criteo

kind = criteo: 39 binary features per row (13 + 26 slots, power-law ids, "k:1" LIBSVM),
       rcv1:   5..145 features per row (~75), tf-idf-like values."""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def write_files(d, kind, rows, files, seed=0, N=10 ** 8):
    rng = np.random.default_rng(seed)
    per = rows // files
    for f in range(files):
        if kind == "criteo":
            w = np.full(per, 39)
        else:
            w = rng.integers(5, 145, per)
        n = int(w.sum())
        keys = (N * rng.random(n) ** 4).astype(np.int64)
        row = np.repeat(np.arange(per), w)
        order = np.lexsort((keys, row))  # LIBSVM wants non-decreasing ids per row
        keys = keys[order]
        y = np.where(rng.random(per) < 0.3, 1, -1)
        if kind == "criteo":
            toks = np.char.add(keys.astype(str), ":1")
        else:
            vals = rng.random(n) * 0.9 + 0.1
            toks = np.char.add(np.char.add(keys.astype(str), ":"),
                               np.char.mod("%.3f", vals))
        rp = np.zeros(per + 1, dtype=np.int64)
        rp[1:] = np.cumsum(w)
        with open(os.path.join(d, f"part-{f:03d}"), "w") as fh:
            for r in range(per):
                fh.write(f"{y[r]} " + " ".join(toks[rp[r]:rp[r + 1]]) + "\n")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=2_000_000)
    ap.add_argument("--files", type=int, default=8)
    ap.add_argument("--minibatch", type=int, default=10000)
    ap.add_argument("--kind", default="criteo", choices=["criteo", "rcv1"])
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--dir", default="")
    a = ap.parse_args()
    import torch

    from parameter_server_amd.app.gpu import run_async_sgd
    from parameter_server_amd.parallel.comm import LocalComm
    from parameter_server_amd.utils.config import load_app_config

    d = a.dir or tempfile.mkdtemp(prefix="psamd_app_")
    t0 = time.time()
    write_files(d, a.kind, a.rows, a.files)
    gen_s = time.time() - t0
    mb = sum(os.path.getsize(os.path.join(d, f)) for f in os.listdir(d)) / 1e6
    conf = os.path.join(d, "online.conf")
    with open(conf, "w") as f:
        f.write(f"""linear_method {{
training_data {{ format: TEXT text: LIBSVM file: "{d}/part.*" }}
loss {{ type: LOGIT }}
penalty {{ type: L1 lambda: 10 lambda: 1 }}
learning_rate {{ type: DECAY alpha: 0.01 beta: 10 }}
async_sgd {{ algo: FTRL minibatch: {a.minibatch} num_data_pass: 1 report_interval: 1000 }}
}}""")
    lm = load_app_config(conf).linear_method
    dev = torch.device("cuda")
    import types

    flags = types.SimpleNamespace(num_features=1e8, max_nnz_per_example=160 if a.kind == "rcv1" else 39,
                                  num_threads=a.threads, device="cuda", seed=0, table_capacity=1 << 26,
                                  quiet=True)
    res = run_async_sgd(lm, LocalComm(dev), dev, flags)
    tr = res["trainer"]
    out = {"bench": "app_file_fed", "kind": a.kind, "rows": res["examples"], "files": a.files,
           "text_mb": round(mb, 1), "minibatch": a.minibatch, "parser_threads": a.threads,
           "seconds": round(res["seconds"], 3),
           "examples_per_s": res["examples"] / res["seconds"],
           "text_mb_per_s": mb / res["seconds"], "steps": res["steps"],
           "localize": tr.localize_mode, "flat_csr": tr._compact is None,
           "loss": res["progress"]["loss"] if res["progress"] else None,
           "file_gen_s": round(gen_s, 1)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
