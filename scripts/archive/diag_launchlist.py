"""Which raw event / stream ops of a native LaunchList fail with torch's HIP runtime
(bench.py native iteration: 'std::get: wrong index for variant' on a record)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from parameter_server_amd.ops.native import hipops  # noqa: E402

H = hipops()
dev = torch.device("cuda", 0)
main = torch.cuda.current_stream(dev)
side = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
print("main handle", main.cuda_stream, "side handles", [s.cuda_stream for s in side], flush=True)


def run_seq(name, handles, main_h, side_h, rounds=3, torch_first=None):
    """bench-like phases: [main: wait P[cur], wait P[nxt], record Bf[cur]] [side: wait Bf[nb],
    record P[nb]], NB = 4 buffers, 2 side streams."""
    NB = 4
    P, Bf = handles
    Ls = []
    for j in range(NB):
        cur, nxt, nb = j, (j + 1) % NB, (j + 2) % NB
        L = H.LaunchList()
        L.add_stream(main_h)
        L.add_wait(P[cur])
        L.add_wait(P[nxt])
        L.add_record(Bf[cur])
        L.add_stream(side_h[nb % 2])
        L.add_wait(Bf[nb])
        L.add_record(P[nb])
        Ls.append(L)
    t = 0
    try:
        for r in range(rounds):
            for j in range(NB):
                Ls[j].run()
                t += 1
            torch.cuda.synchronize()
        print(f"{name}: ok", flush=True)
    except Exception as e:
        print(f"{name}: FAILED at iteration {t}: {e}", flush=True)
        torch.cuda.synchronize()


def torch_events(record_streams):
    P = [torch.cuda.Event() for _ in range(4)]
    Bf = [torch.cuda.Event() for _ in range(4)]
    for e in P + Bf:
        e.record(record_streams)
    torch.cuda.synchronize()
    return P, Bf


own = torch.cuda.Stream(dev)
for label, mh in (("null main", main.cuda_stream), ("own main", own.cuda_stream)):
    P, Bf = torch_events(main)
    run_seq(f"torch events, {label}", ([e.cuda_event for e in P], [e.cuda_event for e in Bf]),
            mh, [s.cuda_stream for s in side])
    raw = [H.event_create() for _ in range(8)]
    run_seq(f"raw events, {label}", (raw[:4], raw[4:]), mh, [s.cuda_stream for s in side])
    for e in raw:
        H.event_destroy(e)
# single-op cases
for label, h in (("null", main.cuda_stream), ("side", side[0].cuda_stream)):
    ev = torch.cuda.Event()
    ev.record(side[0])
    torch.cuda.synchronize()
    L = H.LaunchList()
    L.add_stream(h)
    L.add_record(ev.cuda_event)
    try:
        for r in range(4):
            L.run()
        torch.cuda.synchronize()
        print(f"repeat record on {label}: ok", flush=True)
    except Exception as e:
        print(f"repeat record on {label}: FAILED {e}", flush=True)
        torch.cuda.synchronize()
