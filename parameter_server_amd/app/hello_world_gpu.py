"""GPU hello world on the KVWorker push/pull API (reference src/app/hello_world/main.cc,
src/ps.h): every rank is a worker + server shard on its own GPU.

Rank r pushes k = 4 values for its keys, waits on the timestamp, pulls every key
and prints what the servers hold (keys 0..5; rank 0 pushes keys {0, 2, 4, 5} with
values key / 10, rank 1 keys {0, 1, 3, 4}, so the values of 0 and 4 are summed):

    python -m parameter_server_amd.app.hello_world_gpu                      # 1 GPU
    torchrun --nproc-per-node 2 --master-addr 127.0.0.1 \\
        -m parameter_server_amd.app.hello_world_gpu                         # 2 GPUs, RCCL
    python -m parameter_server_amd.app.hello_world_gpu --cpu                # gloo / CPU
"""
from __future__ import annotations

import argparse
import sys

import torch


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--dim", type=int, default=4)
    ap.add_argument("--consistency", default="bsp")
    args = ap.parse_args(argv)
    from ..parallel.comm import init_from_env
    from ..parameter.sharded_kv import KVWorker

    comm, dev = init_from_env("cpu" if args.cpu or not torch.cuda.is_available() else "cuda")
    kv = KVWorker(comm, dev, capacity=1 << 10, dim=args.dim, key_bits=32, max_keys=64,
                  consistency=args.consistency)
    mine = [0, 2, 4, 5] if comm.rank % 2 == 0 else [0, 1, 3, 4]
    keys = torch.tensor(mine, dtype=torch.int64, device=dev)
    vals = (keys.float() / 10).reshape(-1, 1).expand(-1, args.dim).contiguous()
    kv.wait(kv.push(keys, vals))
    kv.flush()
    allk = torch.arange(6, dtype=torch.int64, device=dev)
    got = kv.wait(kv.pull(allk)).reshape(6, -1).cpu()
    kv.barrier()
    # one write per rank: lines of two ranks sharing a pipe must not interleave
    sys.stdout.write("".join(f"rank {comm.rank}: key {i}: {' '.join(f'{x:g}' for x in got[i].tolist())}\n"
                             for i in range(6)))
    sys.stdout.flush()
    if comm.world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
