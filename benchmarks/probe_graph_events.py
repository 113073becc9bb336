#!/usr/bin/env python3
"""Probe: the merged-exchange iteration's host issue cost with its cross-stream event ops
as host calls (a native LaunchList of 6 graph launches + 11 event ops, bench.py today)
against 2 graph launches per iteration whose event waits / records are event nodes inside
the graphs (a native GraphChain: the captured pieces as child graphs, chained with
hipGraphAddEventWaitNode / hipGraphAddEventRecordNode). Same dependency pattern as bench.py pipeline_merged (main stream
worker, 3 preparation streams, exchange issued 2 iterations ahead), small kernels, plus
an ordering check: the worker of step t must see exchange t done (a device counter).

Prints one JSON line per variant: host us / iteration (issue loop, no sync), device us /
iteration (wall incl. drain / n), ordering violations."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    from parameter_server_amd.ops.native import hipops

    H = hipops()
    dev = torch.device("cuda", 0)
    nprep, xd = 3, 2
    NB = 2 * nprep
    P = NB * 5  # lcm(6 buffers, ring 5) as in the ssp:4 bench
    size = int(os.environ.get("PROBE_SIZE", str(1 << 16)))
    main_s = torch.cuda.current_stream(dev)
    sides = [torch.cuda.Stream(dev, priority=-1) for _ in range(nprep)]
    work = [torch.zeros(size, device=dev) for _ in range(8)]
    cM = torch.zeros(1, dtype=torch.int64, device=dev)   # exchanges done
    cW = torch.zeros(1, dtype=torch.int64, device=dev)   # workers done
    bad = torch.zeros(1, dtype=torch.int64, device=dev)
    k_side = int(os.environ.get("PROBE_SIDE_K", "3"))

    def kern(i, k=1):
        for _ in range(k):
            work[i].mul_(0.999).add_(1e-3)

    def worker():
        kern(0, 3)
        bad.add_((cM < cW + 1).to(torch.int64))  # exchange t done before worker t
        cW.add_(1)

    def prep():
        kern(1, 3)

    def pack():
        kern(2)

    def comm():
        kern(3, k_side)
        cM.add_(1)

    def resolve():
        kern(4)

    def apply():
        kern(5)

    results = {}
    for variant in ("list6", "graph2"):
        cM.zero_(), cW.zero_(), bad.zero_()
        E = P * -(-8 // P)
        ev = {k: [torch.cuda.Event() for _ in range(E)] for k in ("w", "M", "res", "app")}
        cev = torch.cuda.Event()
        for e in [x for v in ev.values() for x in v] + [cev]:
            e.record(main_s)
        torch.cuda.synchronize()
        # bootstrap: exchanges -1 .. xd-1 eagerly (M recorded), counters consistent
        for s in range(0, xd):
            with torch.cuda.stream(sides[(s + 1) % nprep]):
                comm()
                ev["M"][s % E].record()
                ev["res"][s % E].record()
                ev["app"][s % E].record()
        torch.cuda.synchronize()
        plans = []
        held = []
        for k in range(E):
            t = k
            s = t + xd
            xs = sides[((s + 1) % NB) % nprep]
            if variant == "list6":
                gs = {}
                for name, fn in (("w", worker), ("prep", prep), ("pack", pack), ("comm", comm),
                                 ("res", resolve), ("app", apply)):
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g):
                        fn()
                    gs[name] = g
                    held.append(g)
                L = H.LaunchList()
                L.add_stream(main_s)
                L.add_wait(ev["M"][t % E])
                L.add_graph(gs["w"])
                L.add_record(ev["w"][t % E])
                L.add_stream(xs)
                L.add_wait(ev["w"][(t + nprep - NB) % E])
                L.add_graph(gs["prep"])
                L.add_graph(gs["pack"])
                L.add_wait(ev["w"][(s - 3) % E])
                L.add_wait(ev["res"][(s - 1) % E])
                L.add_wait(cev)
                L.add_graph(gs["comm"])
                L.add_record(cev)
                L.add_record(ev["M"][s % E])
                L.add_wait(ev["app"][(s - 1) % E])
                L.add_graph(gs["res"])
                L.add_record(ev["res"][s % E])
                L.add_graph(gs["app"])
                L.add_record(ev["app"][s % E])
                L.add_stream(main_s)
            else:
                def cap(fn):
                    g = torch.cuda.CUDAGraph(keep_graph=True)
                    with torch.cuda.graph(g):
                        fn()
                    held.append(g)
                    return g

                gw, gpp = cap(worker), cap(lambda: (prep(), pack()))
                gc, gr, ga = cap(comm), cap(resolve), cap(apply)
                cm = H.GraphChain()
                cm.add_wait(ev["M"][t % E])
                cm.add_child(gw)
                cm.add_record(ev["w"][t % E])
                cm.instantiate()
                cs = H.GraphChain()
                cs.add_wait(ev["w"][(t + nprep - NB) % E])
                cs.add_child(gpp)
                cs.add_wait(ev["w"][(s - 3) % E])
                cs.add_wait(ev["res"][(s - 1) % E])
                cs.add_wait(cev)
                cs.add_child(gc)
                cs.add_record(cev)
                cs.add_record(ev["M"][s % E])
                cs.add_wait(ev["app"][(s - 1) % E])
                cs.add_child(gr)
                cs.add_record(ev["res"][s % E])
                cs.add_child(ga)
                cs.add_record(ev["app"][s % E])
                cs.instantiate()
                held += [cm, cs]
                L = H.LaunchList()
                L.add_stream(main_s)
                L.add_chain(cm)
                L.add_stream(xs)
                L.add_chain(cs)
                L.add_stream(main_s)
            plans.append(L)
        torch.cuda.synchronize()
        n = 30 * E
        for t in range(2 * E):  # warm
            plans[t % E].run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for t in range(n):
            plans[t % E].run()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        results[variant] = {"host_us": round((t1 - t0) / n * 1e6, 2),
                            "device_us": round((t2 - t0) / n * 1e6, 2),
                            "order_violations": int(bad.item()),
                            "exchanges": int(cM.item()), "workers": int(cW.item())}
        del plans, held
        torch.cuda.synchronize()
    print(json.dumps({"probe": "graph_events", "size": size, "side_k": k_side, **results}),
          flush=True)


if __name__ == "__main__":
    main()
