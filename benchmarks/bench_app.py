"""File-fed throughput of the GPU app (app/gpu.py): reference ``.conf`` + LIBSVM text
files -> C++ parser threads -> pinned staging -> async host->HBM copies -> the HBM
trainer. Generates the files first (not timed), then runs the app and reports
examples/s of the whole run (parse + copy + train), next to the trainer-only rate of
the same minibatches already in HBM.

    python benchmarks/bench_app.py --rows 2000000 --files 8 --minibatch 10000 --kind criteo

kind = criteo: 39 binary features per row (power-law ids, "k:1" LIBSVM, zero-padded ids),
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


def _write_criteo_fast(path, keys, y, N):
    """Fixed-width binary rows as fixed-length text built by digit arithmetic (no per-token
    Python): "+1 00001234:1 ...\n" (zero-padded ids parse as the same integers)."""
    per, width = keys.shape
    nd = len(str(N - 1))
    tok = nd + 3  # digits ":1 "
    L = 2 + width * tok  # "+1" then " ddd:1" per key, "\n" in the last token's space
    buf = np.empty((per, L), dtype=np.uint8)
    buf[:, 0] = np.where(y > 0, ord("+"), ord("-"))
    buf[:, 1] = ord("1")
    body = buf[:, 2:].reshape(per, width, tok)
    body[:, :, 0] = ord(" ")
    k = keys.copy()
    for p in range(nd - 1, -1, -1):
        body[:, :, 1 + p] = ord("0") + (k % 10)
        k //= 10
    body[:, :, 1 + nd] = ord(":")
    body[:, :, 2 + nd] = ord("1")
    out = np.empty((per, L + 1), dtype=np.uint8)
    out[:, :L] = buf
    out[:, L] = ord("\n")
    out.tofile(path)


def _breakdown(tr, d, a, steps, cache):
    """Where a cached run's time goes: the feeder alone (pread -> pinned -> HBM, no
    training) and the trainer alone (the same step count on one HBM-resident minibatch)."""
    import torch

    from parameter_server_amd.data.feeder import DeviceFeeder

    dev = torch.device("cuda")
    files = sorted(os.path.join(d, f) for f in os.listdir(d) if f.startswith("part-"))
    f = DeviceFeeder(files, "LIBSVM", a.minibatch, tr.max_nnz, dev, num_features=10 ** 8,
                     cache_dir=cache, io_threads=a.io_threads)
    torch.cuda.synchronize()
    t0 = time.time()
    n = ex = 0
    last = None
    for b in f:
        n += 1
        ex += b.rows
        last = (b.keys[:b.rows * 39].clone(), b.labels[:b.rows].clone()) if b.rows == a.minibatch \
            else last
        f.release(b)
    torch.cuda.synchronize()
    feed_s = time.time() - t0
    out = {"source": "breakdown", "feeder_only_examples_per_s": ex / feed_s,
           "feeder_only_h2d_gb_per_s": f.bytes_h2d / feed_s / 1e9, "feeder_batches": n}
    if last is not None and a.kind == "criteo":
        keys, labels = last
        for _ in range(3):
            tr.step(keys, labels, width=39)
        torch.cuda.synchronize()
        t0 = time.time()
        for _ in range(steps):
            tr.step(keys, labels, width=39)
        torch.cuda.synchronize()
        out["trainer_only_examples_per_s"] = steps * a.minibatch / (time.time() - t0)
    print(f"[bench_app] breakdown {out}", file=sys.stderr, flush=True)
    return out


def write_files(d, kind, rows, files, seed=0, N=10 ** 8):
    rng = np.random.default_rng(seed)
    per = rows // files
    for f in range(files):
        print(f"[bench_app] writing file {f + 1} / {files}", file=sys.stderr, flush=True)
        if kind == "criteo":
            keys = np.sort((N * rng.random((per, 39)) ** 4).astype(np.int64), axis=1)
            y = np.where(rng.random(per) < 0.3, 1, -1)
            _write_criteo_fast(os.path.join(d, f"part-{f:03d}"), keys, y, N)
            continue
        if kind == "criteo_slow":
            w = np.full(per, 39)
        else:
            w = rng.integers(5, 145, per)
        n = int(w.sum())
        keys = (N * rng.random(n) ** 4).astype(np.int64)
        row = np.repeat(np.arange(per), w)
        order = np.lexsort((keys, row))  # LIBSVM wants non-decreasing ids per row
        keys = keys[order]
        y = np.where(rng.random(per) < 0.3, 1, -1)
        if kind == "criteo_slow":
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
    ap.add_argument("--kind", default="criteo", choices=["criteo", "criteo_slow", "rcv1"])
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--dir", default="")
    ap.add_argument("--cache", type=int, default=1,
                    help="1: run twice with a binary example cache (the first run parses the "
                         "text and writes the cache, the second streams the cache)")
    ap.add_argument("--io-threads", type=int, default=16)
    ap.add_argument("--report-steps", type=int, default=0,
                    help="progress line every this many steps on cached passes (0: 10 per pass)")
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
async_sgd {{ algo: FTRL minibatch: {a.minibatch} num_data_pass: 1 report_interval: 10 }}
}}""")
    lm = load_app_config(conf).linear_method
    dev = torch.device("cuda")
    import types

    cache = os.path.join(d, "cache") if a.cache else "off"
    runs = []
    print(f"[bench_app] {a.rows} rows in {a.files} files ({mb:.0f} MB of text) in {gen_s:.1f} s",
          file=sys.stderr, flush=True)
    for r in range(2 if a.cache else 1):
        flags = types.SimpleNamespace(
            num_features=1e8, max_nnz_per_example=160 if a.kind == "rcv1" else 39,
            num_threads=a.threads, device="cuda", seed=0, table_capacity=1 << 27, quiet=False,
            data_cache=cache, io_threads=a.io_threads, report_steps=a.report_steps)
        res = run_async_sgd(lm, LocalComm(dev), dev, flags)
        tr = res["trainer"]
        print(f"[bench_app] run {r}: {res['examples'] / res['seconds'] / 1e6:.2f} M ex/s "
              f"({'cache' if res['cached_passes'] else 'text'})", file=sys.stderr, flush=True)
        runs.append({"source": "cache" if res["cached_passes"] else "text",
                     "rows": res["examples"], "steps": res["steps"],
                     "seconds": round(res["seconds"], 3),
                     "examples_per_s": res["examples"] / res["seconds"],
                     "h2d_gb_per_s": res["h2d_bytes"] / res["seconds"] / 1e9,
                     "loss": res["progress"]["loss"] if res["progress"] else None,
                     "localize": tr.localize_mode, "flat": tr._compact is None,
                     "host_feed_wait_s": round(res.get("host_feed_wait_s", 0.0), 4),
                     "host_step_issue_s": round(res.get("host_step_issue_s", 0.0), 4)})
        if a.cache and r == 1:
            runs.append(_breakdown(tr, d, a, res["steps"], cache))
        del tr, res
        torch.cuda.empty_cache()
    out = {"bench": "app_file_fed", "kind": a.kind, "files": a.files, "text_mb": round(mb, 1),
           "minibatch": a.minibatch, "parser_threads": a.threads, "io_threads": a.io_threads,
           "file_gen_s": round(gen_s, 1), "text_mb_per_s": mb / runs[0]["seconds"],
           "runs": runs}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
