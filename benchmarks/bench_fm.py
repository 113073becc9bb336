#!/usr/bin/env python3
"""Factorization machine (reference src/app/factor_machine, fm.m): k-dim bf16 factor rows +
linear weights sharded over the ranks, packed [v | w] push/pull over RCCL.
Metric: examples/sec (whole node), weak scaling (fixed minibatch per GPU).

    python benchmarks/bench_fm.py --steps 20
    torchrun --nproc-per-node N benchmarks/bench_fm.py ...
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--localize", default="sort", choices=("sort", "part"))
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--minibatch", type=int, default=16384)
    ap.add_argument("--num-features", type=float, default=1e9)
    ap.add_argument("--dim", type=int, default=16)
    ap.add_argument("--compact-rows", type=int, default=1,
                    help="1 GPU: gather each unique key's row once per step (0: per occurrence "
                         "through the slot index)")
    ap.add_argument("--table-slots", type=int, default=1 << 28, help="slots per GPU")
    ap.add_argument("--prefetch", type=int, default=1,
                    help="generate + localise minibatch t+1 on a side stream during step t")
    args = ap.parse_args()
    from parameter_server_amd.models.fm import FMConfig, FMTrainer
    from parameter_server_amd.ops.synthetic import criteo_batch
    from parameter_server_amd.parallel.comm import init_from_env

    comm, dev = init_from_env("cuda")
    G, rank = comm.world, comm.rank
    B, N = args.minibatch, int(args.num_features)
    cfg = FMConfig(localize=args.localize, num_features=N, embedding_dim=args.dim, minibatch=B, compact_rows=bool(args.compact_rows),
                   table_capacity=args.table_slots, seed=0)
    tr = FMTrainer(cfg, comm, dev)
    bufs = [(torch.empty(B * 39, dtype=torch.int64, device=dev),
             torch.empty(B, dtype=torch.float32, device=dev)) for _ in range(2)]
    t = [0]
    locs = [None, None]
    side = torch.cuda.Stream(dev, priority=int(os.environ.get("PSAMD_PREP_PRIORITY", "-1")))  # own HW queues
    main_s = torch.cuda.current_stream(dev)
    ev_prep = [torch.cuda.Event() for _ in range(2)]
    ev_step = [torch.cuda.Event() for _ in range(2)]

    def prep(i):  # minibatch i into buffer i % 2, on the side stream
        b = i % 2
        side.wait_event(ev_step[b])  # the step that last read this buffer is done
        with torch.cuda.stream(side):
            k, lab = bufs[b]
            criteo_batch(B, seed=77 + rank, row0=i * B, num_features=N, device=dev, keys=k,
                         labels=lab)
            locs[b] = tr.localize(k, buf=b)
            ev_prep[b].record(side)

    def step():
        i = t[0]
        b = i % 2
        if args.prefetch:
            if i == 0:
                prep(0)
            prep(i + 1)
            main_s.wait_event(ev_prep[b])
            tr.step(bufs[b][0], bufs[b][1], loc=locs[b])
            ev_step[b].record(main_s)
        else:
            k, lab = bufs[0]
            criteo_batch(B, seed=77 + rank, row0=i * B, num_features=N, device=dev, keys=k,
                         labels=lab)
            tr.step(k, lab)
        t[0] += 1

    for _ in range(args.warmup):
        step()
    tr.progress()
    comm.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    comm.barrier()
    dt = time.perf_counter() - t0
    x = torch.tensor([dt], dtype=torch.float64, device=dev if G > 1 else "cpu")
    comm.all_reduce_(x, op="max")
    dt = float(x.item())
    p = tr.progress()
    occ, _ = tr.shard.table.census()
    if rank == 0:
        print(json.dumps({
            "metric": "examples/sec (whole node) factorization machine, 1e9 hashed features",
            "value": G * B * args.steps / dt, "unit": "examples/sec", "n_gpus": G,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "dtype": "bf16 rows (fp32 math)",
            "config": {"num_features": N, "embedding_dim": args.dim, "slots": 39,
                       "global_batch": G * B, "table_slots_per_gpu": tr.shard.capacity,
                       "shard_gb": tr.shard.nbytes() / 2 ** 30},
            "train": {**p, "rows_rank0": occ},
        }), flush=True)
    if G > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == "__main__":
    main()
