#!/usr/bin/env python3
"""Darlin BCD (L1 logistic regression) throughput on Criteo-shaped data.

Reference workload: example/linear/ctr/batch_l1lr.conf (lambda 10, tau 8, block
ratio 4, tail feature freq 4). Metric: examples x passes / second for the whole
node (every pass touches every nnz twice: block gradient + margin update).

    python benchmarks/bench_darlin.py --rows 4000000 --passes 5
    torchrun --nproc-per-node N benchmarks/bench_darlin.py ...   (N > 1, RCCL all-reduce)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=2_000_000, help="examples per GPU")
    ap.add_argument("--passes", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--num-features", type=float, default=1e9)
    ap.add_argument("--tau", type=int, default=1)
    ap.add_argument("--l1", type=float, default=10.0)
    ap.add_argument("--tail-freq", type=int, default=4)
    ap.add_argument("--data", default="criteo", choices=["criteo", "groups"],
                    help="criteo: 39 one-hot slots (one block per slot; tau = 8 diverges on "
                         "them, tests/test_darlin.py); groups: CTR-log-shaped, 120 groups with "
                         "8 present per example x 2 keys (tau = 8 converges)")
    ap.add_argument("--tau32", type=int, default=1,
                    help="1: row-pass tau_i in fp32 (G / U sums stay fp64 fixed point); 0: fp64 exp")
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--host-preprocess", action="store_true",
                    help="build the CSC with numpy (reference path) instead of on the GPU")
    ap.add_argument("--device-data", action="store_true",
                    help="keep the generated slots on the GPU (no host copy / upload)")
    args = ap.parse_args()

    from parameter_server_amd.data.synthetic import criteo_slots
    from parameter_server_amd.models.darlin import DarlinConfig, DarlinTrainer
    from parameter_server_amd.parallel.comm import init_from_env

    comm, device = init_from_env("cpu" if args.cpu else "cuda")
    G, rank = comm.world, comm.rank
    t0 = time.time()
    if args.data == "groups":
        from parameter_server_amd.data.synthetic import sparse_groups

        sd = sparse_groups(args.rows, seed=17 + rank)
    else:
        sd = criteo_slots(args.rows, seed=17, row0=rank * args.rows,
                          num_features=int(args.num_features), device=device,
                          on_device=args.device_data and not args.cpu)
    cfg = DarlinConfig(l1=args.l1, tau=args.tau, tail_freq=args.tail_freq,
                       max_pass=args.passes + args.warmup, epsilon=0.0, seed=0,
                       host_preprocess=args.host_preprocess, tau32=bool(args.tau32))
    tr = DarlinTrainer(sd, cfg, comm=comm, device=device)
    prep = time.time() - t0
    for it in range(args.warmup):
        tr.run_pass(it)
    comm.barrier()
    if device.type == "cuda":
        torch.cuda.synchronize()
    t1 = time.perf_counter()
    for it in range(args.warmup, args.warmup + args.passes):
        tr.run_pass(it)
    if device.type == "cuda":
        torch.cuda.synchronize()
    comm.barrier()
    dt = time.perf_counter() - t1
    t = torch.tensor([dt], dtype=torch.float64,
                     device=device if (G > 1 and device.type == "cuda") else "cpu")
    comm.all_reduce_(t, op="max")
    dt = float(t.item())
    if rank == 0:
        p = tr.progress[-1]
        print(json.dumps({
            "metric": "examples x passes / sec (whole node), Darlin L1-LR BCD, Criteo-shaped",
            "value": G * args.rows * args.passes / dt, "unit": "examples/sec",
            "n_gpus": G, "passes": args.passes, "warmup": args.warmup,
            "ms_per_pass": dt / args.passes * 1e3, "dtype": "fp64 (margins, G/U, w)",
            "config": {"rows_per_gpu": args.rows, "num_features": int(args.num_features),
                       "kept_features": tr.num_cols, "nnz_per_gpu": tr.nnz,
                       "blocks": len(tr.blocks), "tau": args.tau, "l1": args.l1,
                       "tail_freq": args.tail_freq, "data": args.data,
                       "tau_fp32": bool(args.tau32)},
            "preprocess_sec": prep,
            "trainer_preprocess_sec": tr.preprocess_time,
            "preprocess_breakdown_sec": tr.prep_times,
            "preprocess_path": "host numpy" if args.host_preprocess else "gpu",
            "train": {"objective": p.objective, "relative_obj": p.relative_obj,
                      "objectives": [q.objective for q in tr.progress],
                      "nnz_w": p.nnz_w, "active_set": p.nnz_active_set},
        }), flush=True)
    if G > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == "__main__":
    main()
