"""Probe: can several RCCL ranks share one GPU on this pool? (2-rank NCCL path
rehearsal on a 1-GPU box). Prints one line per rank and exits."""
import os
import sys

import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
world = int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
dist.init_process_group("nccl", device_id=dev)
x = torch.arange(world * 4, dtype=torch.int32, device=dev) + 100 * rank
y = torch.empty_like(x)
dist.all_to_all_single(y, x)
torch.cuda.synchronize()
print(f"rank {rank}: a2a ok {y.tolist()}", flush=True)
t = torch.ones(1, device=dev) * (rank + 1)
dist.all_reduce(t)
print(f"rank {rank}: allreduce {t.item()}", flush=True)
dist.barrier(device_ids=[0])
dist.destroy_process_group()
sys.exit(0)
