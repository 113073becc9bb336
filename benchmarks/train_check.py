#!/usr/bin/env python3
"""Training-quality sweep on synthetic Criteo-shaped data: runs each named
configuration for --steps minibatches from zero/random init and prints the
progressive loss / AUC of the last --window steps (what bench.py reports as
``train``). Used to pick defaults that actually train (loss < ln 2).

    python benchmarks/train_check.py --steps 50 lr:ftrl lr:sgd lr:sgd:e8asp2 fm
    spec = lr:<algo>[:<mode>][:k=v,...] | fm[:k=v,...]
    mode = 1 (one GPU, bsp) | e8asp2 (8 emulated peers, asp + fixing-float 2 B)
"""
import argparse
import json
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def parse_kv(s):
    out = {}
    for kv in filter(None, s.split(",")):
        k, v = kv.split("=")
        out[k] = float(v) if any(c in v for c in ".e") or v.isdigit() else v
    return out


def run_lr(algo, mode, kv, steps, window, B, dev):
    from parameter_server_amd.models import SparseLRConfig, SparseLRTrainer
    from parameter_server_amd.models.sparse_lr import algo_defaults
    from parameter_server_amd.ops.synthetic import criteo_batch
    from parameter_server_amd.parallel.comm import LoopbackComm

    d = algo_defaults(algo)
    d.update(kv)
    cons = "bsp"
    ff = 0
    comm = None
    if mode.startswith("e"):
        peers = int(mode[1])
        comm = LoopbackComm(peers, dev)
        if "asp" in mode:
            cons = "asp"
        if mode.endswith("2"):
            ff = 2
    cfg = SparseLRConfig(num_features=10 ** 9, minibatch=B, algo=algo, consistency=cons,
                         fixing_float_bytes=ff, table_capacity=1 << 26, **d)
    tr = SparseLRTrainer(cfg, comm, dev)
    keys = torch.empty(B * 39, dtype=torch.int64, device=dev)
    labels = torch.empty(B, dtype=torch.float32, device=dev)
    hist = []
    for t in range(steps):
        criteo_batch(B, seed=1000003, row0=t * B, num_features=10 ** 9, device=dev, keys=keys,
                     labels=labels)
        tr.step(keys, labels, width=39)
        if t + 1 == steps - window:
            tr.progress(reset=True)
        if (t + 1) % 10 == 0:
            torch.cuda.synchronize()
    p = tr.progress(reset=True)
    return {"loss": p["loss"], "auc": p["auc"], "nnz_w": p["nnz_w"], "cfg": d}


def run_fm(kv, steps, window, B, dev):
    from parameter_server_amd.models.fm import FMConfig, FMTrainer
    from parameter_server_amd.ops.synthetic import criteo_batch

    cfg = FMConfig(num_features=10 ** 9, minibatch=B, table_capacity=1 << 24)
    for k, v in kv.items():
        if k.startswith("wide_"):
            setattr(cfg.wide, k[5:], v)
        else:
            setattr(cfg, k, type(getattr(cfg, k))(v))
    tr = FMTrainer(cfg, None, dev)
    keys = torch.empty(B * 39, dtype=torch.int64, device=dev)
    labels = torch.empty(B, dtype=torch.float32, device=dev)
    for t in range(steps):
        criteo_batch(B, seed=77, row0=t * B, num_features=10 ** 9, device=dev, keys=keys,
                     labels=labels)
        tr.step(keys, labels)
        if t + 1 == steps - window:
            tr.progress(reset=True)
    p = tr.progress(reset=True)
    return {"loss": p["loss"], "auc": p["auc"], "cfg": kv}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--window", type=int, default=10)
    ap.add_argument("--minibatch", type=int, default=65536)
    ap.add_argument("specs", nargs="+")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    for spec in a.specs:
        parts = spec.split(":")
        t0 = time.time()
        if parts[0] == "lr":
            algo = parts[1]
            mode = parts[2] if len(parts) > 2 and "=" not in parts[2] else "1"
            kv = parse_kv(parts[-1]) if "=" in parts[-1] else {}
            r = run_lr(algo, mode, kv, a.steps, a.window, a.minibatch, dev)
        else:
            kv = parse_kv(parts[-1]) if len(parts) > 1 else {}
            r = run_fm(kv, a.steps, a.window, a.minibatch, dev)
        r["spec"] = spec
        r["trains"] = r["loss"] < math.log(2)
        r["s"] = round(time.time() - t0, 1)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
