"""Which raw event / stream ops of a native LaunchList fail with torch's HIP runtime
(bench.py native iteration: 'std::get: wrong index for variant' on a record)."""
import torch

from parameter_server_amd.ops.native import hipops

H = hipops()
dev = torch.device("cuda", 0)
main = torch.cuda.current_stream(dev)
side = torch.cuda.Stream(dev)
print("main handle", main.cuda_stream, "side handle", side.cuda_stream, flush=True)


def attempt(name, build, reps=3, sync_between=False):
    ev = torch.cuda.Event()
    ev.record(side)
    torch.cuda.synchronize()
    L = build(ev)
    for r in range(reps):
        try:
            L.run()
            if sync_between:
                torch.cuda.synchronize()
        except Exception as e:
            print(f"{name}: rep {r} FAILED {e}", flush=True)
            torch.cuda.synchronize()
            return
    torch.cuda.synchronize()
    print(f"{name}: ok", flush=True)


def rec_on(handle):
    def b(ev):
        L = H.LaunchList()
        L.add_stream(handle)
        L.add_record(ev.cuda_event)
        return L
    return b


def wait_rec(h1, h2):
    def b(ev):
        L = H.LaunchList()
        L.add_stream(h1)
        L.add_record(ev.cuda_event)
        L.add_stream(h2)
        L.add_wait(ev.cuda_event)
        return L
    return b


attempt("record on main (null) x3", rec_on(main.cuda_stream))
attempt("record on main (null) x3 sync", rec_on(main.cuda_stream), sync_between=True)
attempt("record on side x3", rec_on(side.cuda_stream))
attempt("record on side x3 sync", rec_on(side.cuda_stream), sync_between=True)
attempt("record main, wait side", wait_rec(main.cuda_stream, side.cuda_stream))
attempt("record side, wait main", wait_rec(side.cuda_stream, main.cuda_stream))
attempt("record side, wait main sync", wait_rec(side.cuda_stream, main.cuda_stream), sync_between=True)
# torch records in between
ev = torch.cuda.Event()
ev.record(main)
L = rec_on(main.cuda_stream)(ev)
for r in range(3):
    try:
        L.run()
        ev.record(main)
        torch.cuda.synchronize()
        ev.query()
    except Exception as e:
        print("mixed torch/native records: FAILED", r, e, flush=True)
        break
else:
    print("mixed torch/native records: ok", flush=True)
# timing events created in between (bench PSAMD_STEP_EVENTS)
ev = torch.cuda.Event()
ev.record(main)
L = rec_on(main.cuda_stream)(ev)
sev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
try:
    for r in range(3):
        sev[r].record()
        L.run()
    sev[3].record()
    torch.cuda.synchronize()
    print("with timing events: ok", sev[0].elapsed_time(sev[3]), flush=True)
except Exception as e:
    print("with timing events: FAILED", e, flush=True)
