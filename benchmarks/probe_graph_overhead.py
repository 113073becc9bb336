#!/usr/bin/env python3
"""Probe: GPU time per HIP-graph replay vs eager launches of the same small kernels on
one stream (does a graph replay add device-side time per launch on this ROCm?).
Prints one JSON line: us per iteration for eager / graph with 1 and 5 kernels per
iteration, on one stream and with a second stream joined by events."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    x = torch.zeros(1 << 20, device=dev)

    def body(k):
        for _ in range(k):
            x.add_(1.0)  # ~1M-element elementwise kernel, a few us

    def timed(fn, n=400):
        for _ in range(20):
            fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(n):
            fn()
        e.record()
        torch.cuda.synchronize()
        return round(s.elapsed_time(e) / n * 1e3, 2)

    out = {}
    for k in (1, 5):
        out[f"eager_{k}"] = timed(lambda: body(k))
        g = torch.cuda.CUDAGraph()
        torch.cuda.synchronize()
        with torch.cuda.graph(g):
            body(k)
        out[f"graph_{k}"] = timed(g.replay)
        # k graphs of one kernel each (the pipeline's many small graphs)
        gs = []
        for _ in range(k):
            gi = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gi):
                body(1)
            gs.append(gi)
        out[f"graphs_{k}x1"] = timed(lambda: [gi.replay() for gi in gs])
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
