#!/usr/bin/env python3
"""Standalone time of the Criteo-shaped synthetic minibatch kernel (criteo_gen):
B rows x 39 keys + labels, on the device, per call (us)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from parameter_server_amd.ops.synthetic import criteo_batch  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    reps = 50
    dev = torch.device("cuda")
    k = torch.empty(B * 39, dtype=torch.int64, device=dev)
    lab = torch.empty(B, dtype=torch.float32, device=dev)
    criteo_batch(B, seed=1, row0=0, num_features=10 ** 9, device=dev, keys=k, labels=lab)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for i in range(reps):
        criteo_batch(B, seed=1, row0=i * B, num_features=10 ** 9, device=dev, keys=k, labels=lab)
    b.record()
    torch.cuda.synchronize()
    us = a.elapsed_time(b) * 1e3 / reps
    print(json.dumps({"B": B, "criteo_gen_us": us, "keys_per_us": B * 39 / us,
                      "positive_rate": float((lab > 0).float().mean())}))


if __name__ == "__main__":
    main()
