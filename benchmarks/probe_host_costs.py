#!/usr/bin/env python3
"""Host cost (us per call) of the per-step HIP API calls of the pipeline: event record,
stream wait, both, and a 1-rank RCCL equal-split all-to-all with and without the
device chain. Prints one JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def per_call(fn, n=2000):
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    dt = (time.perf_counter() - t) / n * 1e6
    torch.cuda.synchronize()
    return round(dt, 2)


def main():
    from parameter_server_amd.parallel.comm import nccl_loopback

    dev = torch.device("cuda", 0)
    s1, s2 = torch.cuda.Stream(dev, priority=-1), torch.cuda.Stream(dev, priority=-1)
    ev = torch.cuda.Event()
    out = {}
    out["event_record"] = per_call(lambda: ev.record(s1))
    out["stream_wait_event"] = per_call(lambda: s2.wait_event(ev))
    comm = nccl_loopback(8, dev)
    send = torch.zeros(8 * 90000, dtype=torch.int32, device=dev)
    recv = torch.empty_like(send)
    with torch.cuda.stream(s1):
        out["a2a_chained"] = per_call(lambda: comm.all_to_all_fixed(send, recv), 500)
    comm.chain.on = False
    with torch.cuda.stream(s1):
        out["a2a_plain"] = per_call(lambda: comm.all_to_all_fixed(send, recv), 500)
    print(json.dumps(out), flush=True)
    import torch.distributed as dist

    dist.destroy_process_group()


if __name__ == "__main__":
    main()
