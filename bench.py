#!/usr/bin/env python3
"""Headline benchmark: sparse LR (FTRL-proximal, L1+L2) with 10^9 hashed features.

Metric (BASELINE.json): examples/sec for the whole node, 1/2/4/8 MI355X, synthetic
Criteo-shaped data (13 integer + 26 categorical slots, Criteo-1TB cardinalities,
power-law ids hashed into 10^9 features), random-init (zero) FTRL state.

Every rank is a colocated worker + server shard (weak scaling: the per-GPU
minibatch is fixed). A timed step is the full training step: on-device data
generation, key localisation, pull (RCCL all-to-all when N > 1), forward,
backward, push + server-side FTRL update, progress metrics (loss, accuracy,
bucketed AUC). Nothing is skipped or cached across steps.

    python bench.py --gpus N --steps K --warmup W
    torchrun --nproc-per-node N bench.py --gpus N ...   (N > 1)
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import torch

# thread-local capture: the RCCL watchdog thread of ProcessGroupNCCL keeps querying its
# events while a rank captures its compute segments; global mode would invalidate
# the capture on such a call from another thread
CAPTURE_MODE = "thread_local"
METRIC = "examples/sec (whole node) sparse LR 10^9 feats at 1/2/4/8 MI355X"
ALGO_NAMES = {"ftrl": "FTRL-proximal", "adagrad": "proximal AdaGrad", "sgd": "proximal SGD"}


def pipeline(tr, B, N, seed, keys, labels, device, args, nprep=1, watch=None):
    """Software pipeline over HIP streams (every piece replays from HIP graphs):

    * ``nprep`` preparation streams (high priority on 1 GPU): stream s generates and localises
      every nprep-th minibatch (t % nprep == s) into its own workspaces, issued nprep
      steps ahead; with 2 * nprep buffers a preparation waits only for the step that
      last used its buffer. The kernels of a localisation are latency bound, so
      several run concurrently with the step at little cost (1 GPU, 65,536 x 39 keys:
      1 stream 0.309 ms/step, 2 -> 0.241, 3 -> 0.230).
    * main stream: the worker half of the training step (``SparseLRTrainer.step_segments``,
      one linear graph per compute segment and ring position; a single multi-stream
      graph replays much slower on ROCm). N > 1: the padded exchange's two
      equal-split RCCL all-to-alls run between the graph replays, nothing reads back
      to the host.
    * N > 1 with exchange lag >= 1 (SSP / ASP): the exchange half of step t+xd (pack,
      all-to-all, owner push apply + pull resolve, all-to-all) is issued right after the
      worker half of step t, on the preparation stream of minibatch t+xd (behind its
      localisation), so it runs while the main stream trains; it waits only for the
      localisation of its minibatch, the worker step whose gradients it carries
      (t+xd-1-lag) and the previous exchange (owner updates in step order). Counting
      RCCL's own stream this keeps 4 busy streams; one more (a dedicated exchange
      stream, PSAMD_XCHG_STREAM=own) oversubscribes the hardware queues (8 emulated
      peers: 0.333 vs 0.308 ms/step).
    * ASP: the owner's push apply of each exchange replays at the tail of its exchange
      half, after the event the worker and the next exchange wait for; later exchanges
      wait for it only when they reuse its ring entry (the apply of exchange t - depth),
      never to see its pushes.

    Graphs are captured per phase t % P, P = lcm(2 * nprep buffers, exchange ring).
    tests/test_bench_pipeline_gpu.py checks the pipeline trains exactly what the
    sequential trainer trains. Each iteration = one full training step + one full
    data preparation; the first steps' data is prepared in warm-up and the last
    iterations' preparations are unused, so the timed region does exactly K
    generations, K localisations and K steps. Returns (run, graph_used)."""
    import math

    from parameter_server_amd.ops.synthetic import criteo_batch
    from parameter_server_amd.parallel.consistency import EventClock

    if getattr(tr, "merged", False):  # one all-to-all per step (lag >= 1)
        return pipeline_merged(tr, B, N, seed, keys, labels, device, args, nprep=nprep,
                               watch=watch)
    # 1 GPU, flat layout: step t also pulls minibatch t+1 (in its update launch), and each
    # preparation (generator + tile + flat bucket kernels) is ONE native launch-list call:
    # buffer b holds minibatches b, b + NB, ... = rows (b + k * NB) * B
    flat = getattr(tr, "localize_mode", "") == "tpf" and not tr.padded
    if flat and nprep < 2:
        # step t pulls minibatch t+1, so t+1 must be prepared BEFORE step t is issued and
        # its buffer must not be refilled while step t+1 still reads it: with one
        # preparation stream (NB = 2) the preparation of t+1 is issued after step t and
        # overwrites the buffer step t pulls into. Two streams keep every pulled buffer
        # one full step ahead (tests/test_bench_pipeline_gpu.py::test_flat_pipeline_*).
        nprep = 2
        if hasattr(args, "prep_streams"):
            args.prep_streams = nprep
    NB = 2 * nprep
    R = tr.R if tr.padded else 1
    P = NB * R // math.gcd(NB, R)  # graph phases: (buffer, ring position) pairs
    main = torch.cuda.current_stream(device)
    set_stream = torch.cuda.set_stream
    # preparation streams at high priority, also with N > 1: ROCm maps streams of each
    # priority onto its own set of hardware queues, and normal-priority pool streams
    # share queues with the null stream and RCCL's streams, which serialises a
    # preparation stream behind the training step (rocprofv3 Queue_Id: 8 emulated peers
    # through a real RCCL communicator 0.304 -> 0.204 ms / step, loopback copy 0.227 ->
    # 0.208; profiles/r2_emulated8_priority.log)
    prio = int(os.environ.get("PSAMD_PREP_PRIORITY", "-1"))
    sides = [torch.cuda.Stream(device, priority=prio) for _ in range(nprep)]
    bufs = [(keys, labels)] + [(torch.empty_like(keys), torch.empty_like(labels))
                               for _ in range(NB - 1)]
    # row counter of each preparation stream: on the host while preparations are issued
    # eagerly (the rows go to the generator as a launch argument), on the device once
    # they replay from graphs (a captured preparation reads and advances it)
    hctr = [0] * nprep
    ctr = [torch.zeros(2, dtype=torch.int64, device=device) for _ in range(nprep)]
    locs = [None] * NB
    mode = {"capture": False}
    # 1 GPU, native iteration: the localisation (tile kernel) of the minibatch prepared in
    # iteration t waits for step t's fused forward/backward (PSAMD_TILE_GATE=0: off). The
    # two LDS-heavy 1024-thread kernels otherwise share the CUs whenever the pipeline's
    # phases line them up, and both run 1.3-1.7x longer: that was the 10^10-feature
    # slowdown (fwd/bwd 26 -> 46 us pipelined; 300 steps 0.1052 -> 0.0815 ms with the
    # gate, 10^9 0.0835 -> 0.0805, profiles/r6_1e10.log)
    tile_gate = flat and os.environ.get("PSAMD_TILE_GATE", "1") == "1"
    ev_fb = [torch.cuda.Event() for _ in range(NB)] if tile_gate else None
    if tile_gate:
        for e in ev_fb:
            e.record(torch.cuda.current_stream(device))
    # tail filter: the filter kernels (CountMin insert + query + compaction) in minibatch
    # order, the generators, tile and bucket kernels of the preparations still overlapping
    fchain = tr.filter is not None
    ev_bk = [torch.cuda.Event() for _ in range(NB)] if (flat and fchain) else None
    if ev_bk is not None:
        for e in ev_bk:
            e.record(torch.cuda.current_stream(device))
    fplans = ([tr.prep_plan(b, bufs[b][0], bufs[b][1], seed=seed, row0=b * B, row_step=NB * B,
                            num_features=N,
                            gate=ev_fb[(b - nprep) % NB] if tile_gate else None,
                            bucket_after=ev_bk[(b - 1) % NB] if ev_bk else None,
                            bucket_done=ev_bk[b] if ev_bk else None)
               for b in range(NB)] if flat else None)

    def prep(b):  # buffer b belongs to prep stream b % nprep (rows (nprep*k + s) * B)
        sidx = b % nprep
        k, lab = bufs[b]
        if fplans is not None:
            locs[b] = fplans[b]()
            return
        if mode["capture"]:
            # buffer b reads cursor word (b // nprep) % 2 of its stream and writes the
            # other: the stream's two buffers alternate, so each replay advances the cursor
            kk = (b // nprep) % 2
            criteo_batch(B, seed=seed, row0=sidx * B, num_features=N, device=device, keys=k,
                         labels=lab, row0_dev=ctr[sidx][kk:kk + 1], row_scale=nprep * B,
                         row0_out=ctr[sidx][1 - kk:2 - kk])
        else:
            criteo_batch(B, seed=seed, row0=(hctr[sidx] * nprep + sidx) * B, num_features=N,
                         device=device, keys=k, labels=lab)
            hctr[sidx] += 1
        locs[b] = tr.localize(k, buf=b)

    def segments(t):
        b = t % NB
        k, lab = bufs[b]
        return tr.step_segments(k, lab, width=39, loc=locs[b], step=t,
                                next_loc=locs[(t + 1) % NB] if flat else None)

    split = tr.padded and tr.lag >= 1
    asp = tr.padded and tr.asp
    ncut = tr.EXCHANGE_SEGMENTS if split else 0
    # where the exchange half runs: "prep" = on the preparation stream of its own
    # minibatch, right after the localisation (no extra stream: RCCL's own stream
    # is already one more, and past 4 busy streams the queues oversubscribe);
    # "own" = a dedicated high-priority exchange stream
    xmode = os.environ.get("PSAMD_XCHG_STREAM", "prep") if split else "none"
    comm_s = torch.cuda.Stream(device, priority=-1) if xmode == "own" else main
    # (normal priority: at high priority, like the preparation streams, 8 emulated peers
    # measured 0.369 vs 0.340 ms / step; PSAMD_APPLY_PRIORITY overrides)
    # ASP owner applies: "tail" (default) = at the end of the exchange half on its
    # (preparation) stream, after the weights went back and after the event that the
    # next exchange and the worker wait for, so neither waits for the apply (still
    # asynchronous) and no fifth busy stream oversubscribes the 4 hardware queues;
    # "stream" = on a stream of their own. 8 emulated peers: 0.355 -> 0.164 ms / step,
    # with fixing-float 1 B 0.392 -> 0.175 (profiles/r2_asp_tail.log)
    asp_apply = os.environ.get("PSAMD_ASP_APPLY", "tail") if asp else "none"
    apply_s = (torch.cuda.Stream(device, priority=int(os.environ.get("PSAMD_APPLY_PRIORITY", "0")))
               if asp_apply == "stream" else None)
    # exchange of step t + xd issued after worker t: needs the worker of the step it
    # carries (t + xd - 1 - lag, or t + xd - lag with post applies) issued and the
    # preparation of t + xd (xd <= nprep)
    post = tr.padded and tr.sched.post
    xd_cap = int(os.environ.get("PSAMD_XD", "2"))  # exchanges issued ahead (A/B knob)
    xd = min(nprep, xd_cap, tr.lag if post else tr.lag + 1) if split else 0
    # the key pack of exchange t runs before it waits for exchange t-1 (ssp post / asp
    # tail apply; not with the tail filter: its CountMin and keep-mask scratch are shared
    # by the key packs of consecutive exchanges). Otherwise the whole exchange half waits
    # first and replays as ONE captured graph (pack + all-to-all A + owner work + B).
    early = (post or asp_apply == "tail") and (tr.filter is None or tr._flat_x)
    # tail filter: the CountMin inserts and queries of consecutive minibatches run in
    # minibatch order (the reference's MinibatchReader::read sequence): a preparation
    # waits for the previous minibatch's (on another stream); the flat launch lists order
    # only their tail-filter kernels (ev_bk above)
    fchain = tr.filter is not None and fplans is None
    E = 64  # event rings, indexed by step (every look-back here is < 64 steps)
    ev_buf = [torch.cuda.Event() for _ in range(NB)]   # worker done with buffer b
    ev_w = [torch.cuda.Event() for _ in range(E)]      # worker half of step t done
    ev_prep = [torch.cuda.Event() for _ in range(NB)]
    ev_x = [torch.cuda.Event() for _ in range(E)]      # exchange half of step t done
    ev_post = [torch.cuda.Event() for _ in range(E)]   # ... and its post apply (ssp)
    aclock = EventClock(E)                             # asp: push apply of exchange t done

    def run_plan(plan, t, xs):
        """Run one half's segments; an "async" segment (ASP push apply) goes to its
        own stream behind what ``xs`` has issued so far."""
        for kind, fn in plan:
            if kind == "async":
                e = torch.cuda.Event()
                e.record(xs)
                apply_s.wait_event(e)
                with torch.cuda.stream(apply_s):
                    fn()
                aclock.record(t, apply_s)
            else:
                fn()

    def halves(t):
        segs = list(segments(t))
        return segs[:ncut], segs[ncut:]

    # eager plans until capture: phase j -> (exchange half, worker half)
    xplans = [None] * P
    wplans = [None] * P

    def xplan(t):
        j = t % P
        if xplans[j] is None or not graphs["on"]:
            return halves(t)[0]
        return xplans[j]

    def wplan(t):
        j = t % P
        if wplans[j] is None or not graphs["on"]:
            return halves(t)[1]
        return wplans[j]

    preps = [(lambda b=b: prep(b)) for b in range(NB)]
    graphs = {"on": False}
    state = {"t": 0}
    # 1 GPU, flat: the preparation of minibatch t + nprep also waits for step t-1
    # (implies the buffer wait: steps complete in order); PSAMD_PREP_GATE=0: buffer only
    # (measured slower at the driver shape, 0.0901-0.0906 vs 0.0870-0.0889 ms / step over
    # 20 steps, profiles/r5_prep_gate_and_merge.log: off unless PSAMD_PREP_GATE=1)
    prep_gate = flat and nprep >= 2 and os.environ.get("PSAMD_PREP_GATE", "0") == "1"

    def issue_exchange(t):
        xs = sides[(t % NB) % nprep] if xmode == "prep" else comm_s
        if xmode != "prep":
            xs.wait_event(ev_prep[t % NB])  # (on its prep stream it follows the prep)
        c = tr.sched.carried(t)
        if c >= 0:
            xs.wait_event(ev_w[c % E])      # the gradients it carries are packed
        # owner updates of consecutive steps in order: exchange t resolves after exchange
        # t-1 is done (ssp post: including its apply). With the apply at the tail only
        # the resolve needs that (it rewrites wsend and must see the apply), so the key
        # pack and all-to-all A of exchange t overlap the tail of exchange t-1
        chain = ev_post if post else ev_x
        if t >= 1 and not early:
            xs.wait_event(chain[(t - 1) % E])
        if asp:  # ring entry of exchange t is free again once that apply is done
            aclock.wait_for(tr.sched.apply_gate(t), xs)
        set_stream(xs)  # (main is current here; see iterate)
        try:
            if asp_apply == "tail" or post:
                # the apply after the event the worker waits for (ssp post apply: the
                # next exchange waits for it; asp: nothing waits for it)
                late = ("async", "post")
                plan = xplan(t)
                ncomm, waited = 0, t < 1 or not early
                for kind, fn in plan:
                    if kind in late:
                        continue
                    # the resolve (eager collectives: the compute after all-to-all A;
                    # captured: the graph of all-to-all A + resolve + all-to-all B)
                    if (kind == "cgraph" or (kind == "compute" and ncomm == 1)) and not waited:
                        xs.wait_event(chain[(t - 1) % E])
                        waited = True
                    fn()
                    ncomm += kind == "comm"
                ev_x[t % E].record(xs)
                if asp and t >= 1:
                    # push applies in exchange order: apply t-1 ran at the tail of its
                    # own (other) preparation stream; two applies at once would race on
                    # the hot keys' optimizer state (and on shared apply scratch)
                    aclock.wait_for(t - 1, xs)
                for kind, fn in plan:
                    if kind in late:
                        fn()
                if post:
                    ev_post[t % E].record(xs)
                else:
                    aclock.record(t, xs)
            else:
                run_plan(xplan(t), t, xs)
                ev_x[t % E].record(xs)
        finally:
            set_stream(main)

    def iterate():
        t = state["t"]
        if watch is not None and not graphs["on"]:
            watch.beat("pipeline-warmup", t)
        cur = t % NB
        if xmode == "own":
            issue_exchange(t + 1)
            main.wait_event(ev_x[t % E])      # exchange of step t done
        elif split:
            main.wait_event(ev_x[t % E])
        else:
            main.wait_event(ev_prep[cur])     # minibatch t is localised
            if flat:                          # ... and t+1 (its pull runs in step t)
                main.wait_event(ev_prep[(t + 1) % NB])
        # the training step is issued first: after an idle GPU (the first timed step)
        # its kernels start one graph launch earlier (short runs: step 0 took ~0.1 ms
        # longer than the steady state behind the preparation's launch)
        run_plan(wplan(t), t, main)
        ev_buf[cur].record(main)
        if split:  # (only the exchange halves wait for the worker half)
            ev_w[t % E].record(main)
        nb = (t + nprep) % NB                 # minibatch t + nprep
        s = sides[nb % nprep]
        # step(t + nprep - NB) done with bufs[nb]; with prep_gate the preparation also
        # waits for step t-1, so it runs beside step t and not in a burst with the other
        # streams' preparations (the first timed steps after an idle GPU)
        s.wait_event(ev_buf[(t - 1) % NB] if prep_gate else ev_buf[nb])
        if fchain:
            s.wait_event(ev_prep[(nb - 1) % NB])
        # a plain set_stream there and back (main is current here): the torch.cuda.stream
        # context re-queries the current stream and the lazy-init state on every use, ~10
        # us of host time per step (cProfile, profiles/r3_s3_host_issue.log)
        set_stream(s)
        try:
            preps[nb]()
            ev_prep[nb].record(s)
        finally:
            set_stream(main)
        if xmode == "prep":
            issue_exchange(t + xd)
        state["t"] = t + 1

    for e in ev_buf:
        e.record(main)
    for b in range(nprep):  # minibatches 0 .. nprep-1
        with torch.cuda.stream(sides[b]):
            if fchain and b:
                sides[b].wait_event(ev_prep[b - 1])
            prep(b)
            ev_prep[b].record(sides[b])
    if xmode == "own":
        issue_exchange(0)
    elif split:
        for t in range(xd):  # exchanges of minibatches 0 .. xd-1
            issue_exchange(t)
    warm = max(NB, args.warmup)
    warm += (-warm) % P  # capture at a multiple of P: phase j <-> buffer j % NB, ring j % R
    for _ in range(warm):
        iterate()
    # auto: on for large minibatches (B = 65,536: 0.0966-0.1007 -> 0.0949-0.0957 ms); at
    # B = 10,000 the GPU step took 0.050 vs 0.042 ms eagerly (profiles/r4_native_iter.log)
    native = os.environ.get("PSAMD_NATIVE_ITER", "auto")
    if flat and (native == "1" or (native == "auto" and B >= 32768)):
        # 1 GPU, flat: one iteration (both streams' event waits, the step's launches, the
        # next preparation's launches, the records) is ONE native launch-list call; phase
        # j = t % NB: step t on buffer j (its pull was issued by step t-1) pulling
        # buffer j+1, and the preparation of buffer j + nprep on its stream. The lists
        # share the launch objects of the eager path (the generators' row cursors).
        from parameter_server_amd.ops.native import hipops

        H = hipops()
        phases = []
        for j in range(NB):
            cur, nxt, nb = j, (j + 1) % NB, (j + nprep) % NB
            s = sides[nb % nprep]
            splan, _ = tr.flat_plan(locs[cur], bufs[cur][1], B, 39, locs[nxt], True,
                                    fb_record=ev_fb[j] if tile_gate else None)
            L = H.LaunchList()
            L.add_stream(main)
            L.add_wait(ev_prep[cur])
            L.add_wait(ev_prep[nxt])
            L.extend(splan)
            L.add_record(ev_buf[cur])
            L.add_stream(s)
            L.add_wait(ev_buf[(j - 1) % NB] if prep_gate else ev_buf[nb])
            if fchain:
                L.add_wait(ev_prep[(nb - 1) % NB])
            L.extend(fplans[nb].plan)
            L.add_record(ev_prep[nb])
            phases.append((L.run, locs[nxt], fplans[nb].done))

        def iterate_native():
            t = state["t"]
            run, nxt_loc, prep_done = phases[t % NB]
            run()
            tr.flat_done(B, nxt_loc)
            prep_done()
            state["t"] = t + 1

        try:  # (untimed: a failing launch list falls back to the eager iteration, loudly)
            for _ in range(NB):
                iterate_native()
            torch.cuda.synchronize()
        except Exception as e:
            print(f"[psamd] native iteration failed ({e}); eager launches", file=sys.stderr)
            torch.cuda.synchronize()
            args.native_iter = f"failed: {e}"
            return iterate, False
        args.native_iter = True
        return iterate_native, False
    if not args.graph or flat:  # (flat: eager launch lists; their row cursors live on the host)
        return iterate, False
    torch.cuda.synchronize()
    t0 = state["t"]
    held = []  # every captured graph

    def release():
        torch.cuda.synchronize()
        for g in held:
            g.reset()
        held.clear()

    iterate.release = release
    gp = []
    seed_cursors(ctr, hctr, state["t"], nprep, NB)  # the replays continue the eager rows
    mode["capture"] = True
    for b in range(NB):  # t0 % NB == 0: buffer b <-> minibatch t0 + b
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode=CAPTURE_MODE):
            prep(b)
        gp.append(g)
        held.append(g)
    if args.graph == 2:
        # preparations only: each replays as one graph on its side stream (one host
        # launch instead of ~5, its graph-launch latency off the training stream), the
        # training step is issued eagerly
        preps[:] = [g.replay for g in gp]
        torch.cuda.synchronize()
        for _ in range(P):
            iterate()
        torch.cuda.synchronize()
        return iterate, True

    # The all-to-alls are captured too (PSAMD_CAPTURE_COMM=0: eager between the graph
    # replays, as in round 2), so a step issues graph replays and event waits only.
    # Segments group into as few graphs as their waits allow: the compute before an
    # exchange's first collective (it need not wait for the previous exchange), then
    # everything up to the next late segment, whose collectives are ordered as a whole
    # on the communicator's device chain (wait before the replay, mark after it).
    # Every graph is released before the process group is destroyed: a live graph
    # holding RCCL work keeps the communicator's teardown waiting (the round-2 capture
    # experiment hung at exit that way, profiles/r2_capture_comm.log).
    # PSAMD_CAPTURE_COMM: 1 / auto (default) = capture, 0 = eager. Captured all-to-alls
    # are validated on the 1-rank RCCL loopback of emulated peers
    # (tests/test_bench_pipeline_gpu.py) but have not run between real ranks on this
    # project's hardware; a multi-rank job therefore runs under the rank supervisors of
    # ``supervise`` below, which re-run the whole job in fresh processes with eager
    # collectives if the captured attempt fails or stalls (its collective timeout is
    # short, PSAMD_COMM_TIMEOUT of the first attempt).
    cchain = getattr(tr.comm, "chain", None)
    cmode = os.environ.get("PSAMD_CAPTURE_COMM", "auto")
    ccomm = (tr.padded and cchain is not None and getattr(tr.comm, "backend", "") != "gloo"
             and cmode in ("1", "auto"))
    pipeline.captured_comm = ccomm

    def graph_of(fns):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode=CAPTURE_MODE):
            for fn in fns:
                fn()
        held.append(g)
        return g.replay

    def chained(rep, n):
        def f():
            s = torch.cuda.current_stream(device)
            cchain.wait(s)
            rep()
            cchain.mark(s, n)
        return f

    def capture(plan, split=True):
        out = []
        if not ccomm:
            for kind, fn in plan:  # in order: a segment may bake in buffers the previous
                if kind in ("compute", "async", "post"):  # one of the same ring entry selected
                    out.append((kind, graph_of([fn])))
                else:
                    out.append((kind, fn))
            return out
        grp, hosts = [], []

        def flush():
            if grp:
                nc = sum(k == "comm" for k, _ in grp)
                rep = graph_of([fn for _, fn in grp])
                out.append(("cgraph", chained(rep, nc)) if nc else ("compute", rep))
            out.extend(hosts)  # host bookkeeping right after the group it sat in
            grp.clear()
            hosts.clear()

        for kind, fn in plan:
            if kind == "host":
                hosts.append((kind, fn))
            elif kind in ("async", "post"):
                flush()
                out.append((kind, graph_of([fn])))
            else:
                if split and kind == "comm" and not any(k == "comm" for k, _ in grp):
                    flush()
                grp.append((kind, fn))
        flush()
        return out

    for j in range(P):
        if watch is not None:
            watch.beat("capture", j)
        xh, wh = halves(t0 + j)
        if ccomm and asp_apply == "tail":
            # the push apply replays at the tail of the exchange half anyway: move it
            # behind all-to-all B before grouping, so A + resolve + B stay ONE captured
            # graph (a graph replay costs ~6-8 us of GPU time and ~11 us of host time,
            # profiles/r3_s2_graph_ab.log; ASP issued 6 graphs per step, now 5)
            xh = [x for x in xh if x[0] != "async"] + [x for x in xh if x[0] == "async"]
        xplans[j] = capture(xh, split=early)
        wplans[j] = capture(wh)
    # capture ran nothing: the workspaces of the minibatches in flight still hold
    # their eager preparations (and the eager exchanges issued ahead), so the replays
    # continue from there
    preps[:] = [g.replay for g in gp]
    graphs["on"] = True
    torch.cuda.synchronize()
    for _ in range(P):
        iterate()
    torch.cuda.synchronize()
    return iterate, True


def seed_cursors(ctr, hctr, t, nprep, NB):
    """Before the first graph replay: each preparation stream's row cursor (host count of
    its eager preparations) into the word its first replayed buffer reads (prep of
    buffer b reads word (b // nprep) % 2; iteration t prepares buffer (t + nprep) % NB)."""
    for s in range(nprep):
        b = next((t + nprep + i) % NB for i in range(NB) if (t + nprep + i) % NB % nprep == s)
        ctr[s][(b // nprep) % 2].fill_(hctr[s])


def pipeline_merged(tr, B, N, seed, keys, labels, device, args, nprep=3, watch=None):
    """The multi-GPU pipeline on the merged exchange (one all-to-all per step,
    ``SparseLRTrainer.mx_exchange`` / ``mx_worker``, parallel/consistency.MergedSchedule).

    Exchange s carries keys(s+1), the pushes of step s-d and the weights of keys(s); it
    runs on the preparation stream of minibatch s+1 (right behind its localisation):

      pack keys(s+1) -> [wait: resolve after exchange s-1, worker s-d] -> all-to-all
      -> (event: worker s may start) -> [post: wait apply of exchange s-1]
      -> owner resolve keys(s+1) -> (event) -> owner apply of step s-d -> (event)

    and is issued ``xd`` iterations ahead of the worker half that needs it, so the
    chain all-to-all -> resolve -> all-to-all runs while the main stream trains. The
    worker half of step t waits only for the all-to-all of exchange t. Every piece
    replays from a HIP graph per phase (t % lcm(buffers, ring)), the all-to-all graphs
    ordered on the communicator's device chain. Returns (run, graph_used)."""
    import math

    from parameter_server_amd.ops.synthetic import criteo_batch

    ms = tr.msched
    R, d = ms.R, ms.d
    NB = 2 * nprep
    P = NB * R // math.gcd(NB, R)
    main = torch.cuda.current_stream(device)
    set_stream = torch.cuda.set_stream
    prio = int(os.environ.get("PSAMD_PREP_PRIORITY", "-1"))
    sides = [torch.cuda.Stream(device, priority=prio) for _ in range(nprep)]
    bufs = [(keys, labels)] + [(torch.empty_like(keys), torch.empty_like(labels))
                               for _ in range(NB - 1)]
    hctr = [0] * nprep
    ctr = [torch.zeros(2, dtype=torch.int64, device=device) for _ in range(nprep)]
    locs = [None] * NB
    mode = {"capture": False}
    tr._mx_external = True  # progress() must not drain: the exchanges below are in flight

    def prep(b, part=0):
        """part 0: generate + localise; (tail filter) 1: generate + tile + bucket, 2: the
        filter kernel (ordered across minibatches by the caller); 3: generate only, 4: the
        localisation only (tile + bucket with the tail filter, else all of it)"""
        sidx = b % nprep
        k, lab = bufs[b]
        if part == 2:
            locs[b] = tr.localize(k, buf=b, stage=3)
            return
        if part == 4:
            if fchain:
                tr.localize(k, buf=b, stage=4)
            else:
                locs[b] = tr.localize(k, buf=b)
            return
        if mode["capture"]:
            # buffer b reads cursor word (b // nprep) % 2 of its stream and writes the
            # other: the stream's two buffers alternate, so each replay advances the cursor
            kk = (b // nprep) % 2
            criteo_batch(B, seed=seed, row0=sidx * B, num_features=N, device=device, keys=k,
                         labels=lab, row0_dev=ctr[sidx][kk:kk + 1], row_scale=nprep * B,
                         row0_out=ctr[sidx][1 - kk:2 - kk])
        else:
            criteo_batch(B, seed=seed, row0=(hctr[sidx] * nprep + sidx) * B, num_features=N,
                         device=device, keys=k, labels=lab)
            hctr[sidx] += 1
        if part == 3:
            return
        if part == 1:
            tr.localize(k, buf=b, stage=4)
        else:
            locs[b] = tr.localize(k, buf=b)

    xd = max(1, min(d, nprep - 1, int(os.environ.get("PSAMD_XD", "2"))))
    E = P * -(-64 // P)  # (a multiple of the phase count: one native plan per t % E)
    ev = {k: [torch.cuda.Event() for _ in range(E)] for k in ("w", "M", "res", "app")}
    ev_buf = [torch.cuda.Event() for _ in range(NB)]
    ev_prep = [torch.cuda.Event() for _ in range(NB)]
    graphs = {"on": False}
    gx = {}   # phase -> dict of replays (pack, comm, resolve, apply)
    gw = {}   # phase -> worker replay
    cchain = getattr(tr.comm, "chain", None)

    def xparts(s):
        j = s % P
        if graphs["on"] and j in gx:
            return gx[j]
        return tr.mx_exchange(s, locs[(s + 1) % NB])

    def wpart(t):
        j = t % P
        if graphs["on"] and j in gw:
            return gw[j]
        b = t % NB
        return tr.mx_worker(t, locs[b], bufs[b][1], width=39)

    def issue_exchange(s):
        xs = sides[((s + 1) % NB) % nprep]  # the stream that localised minibatch s+1
        set_stream(xs)
        try:
            parts = xparts(s)
            parts["pack"]()
            if s - d >= 0:
                xs.wait_event(ev["w"][(s - d) % E])     # grads(s-d) packed
            if s >= 0:
                xs.wait_event(ev["res"][(s - 1) % E])   # weights(s) in the send rows
            parts["comm"]()
            ev["M"][s % E].record(xs)
            if s >= 0:
                # owner updates in exchange order: the resolve of keys(s+1) (post) or
                # this apply (pre) after the apply of exchange s-1, which so overlaps
                # this all-to-all instead of delaying it
                xs.wait_event(ev["app"][(s - 1) % E])
            if parts["post"]:
                parts["resolve"]()
                ev["res"][s % E].record(xs)
                parts["apply"]()
            else:
                parts["apply"]()
                parts["resolve"]()
                ev["res"][s % E].record(xs)
            ev["app"][s % E].record(xs)
            tr._mx_next = s + 1  # (mx_drain continues after the issued exchanges)
        finally:
            set_stream(main)

    state = {"t": 0}
    # (tail filter on the flat layout: the filter kernels of consecutive minibatches in
    # minibatch order. On the compact layout the sketch is updated by the key pack of
    # each exchange (sparse_lr._tail_filter, global CountMin atomics): those packs run on
    # the preparation streams unordered here, so a query may already see the next
    # minibatch's inserts -- the trainer's sequential step() keeps the exact order)
    fchain = tr.filter is not None and tr.localize_mode == "tpf"

    def iterate():
        t = state["t"]
        if watch is not None and not graphs["on"]:
            watch.beat("pipeline-warmup", t)
        cur = t % NB
        main.wait_event(ev["M"][t % E])
        wpart(t)()
        tr.mx_done(B)
        ev["w"][t % E].record(main)
        ev_buf[cur].record(main)
        nb = (t + nprep) % NB
        s_ = sides[nb % nprep]
        s_.wait_event(ev_buf[nb])
        set_stream(s_)
        try:
            if fchain:  # (tail filter: the CountMin filters in minibatch order)
                prep_fns[nb][0]()
                s_.wait_event(ev_prep[(nb - 1) % NB])
                prep_fns[nb][1]()
            else:
                prep_fns[nb]()
            ev_prep[nb].record(s_)
        finally:
            set_stream(main)
        issue_exchange(t + xd)
        state["t"] = t + 1

    prep_fns = [((lambda b=b: prep(b, 1)), (lambda b=b: prep(b, 2))) if fchain
                else (lambda b=b: prep(b)) for b in range(NB)]
    for e in ev_buf:
        e.record(main)
    for b in range(nprep):
        with torch.cuda.stream(sides[b]):
            if fchain:
                prep(b, 1)
                if b:
                    sides[b].wait_event(ev_prep[b - 1])
                prep(b, 2)
            else:
                prep(b)
            ev_prep[b].record(sides[b])
    if tr.xc is None:
        main.wait_event(ev_prep[0])
        tr._xc_setup(locs[0])  # (collective: the row capacity from minibatch 0)
    for s in range(-1, xd):  # exchanges -1 .. xd-1 carry keys(0) .. keys(xd)
        issue_exchange(s)
    warm = max(NB, args.warmup, d + 1)  # (captured exchanges all carry pushes: s - d >= 0)
    warm += (-warm) % P
    for _ in range(warm):
        iterate()
    if not args.graph:
        return iterate, False
    torch.cuda.synchronize()
    t0 = state["t"]
    held = []

    def release():
        torch.cuda.synchronize()
        for g in held:
            g.reset()
        held.clear()

    iterate.release = release
    cmode = os.environ.get("PSAMD_CAPTURE_COMM", "auto")
    ccomm = (cchain is not None and getattr(tr.comm, "backend", "") != "gloo"
             and cmode in ("1", "auto"))
    pipeline.captured_comm = ccomm

    gobj = {}  # replay -> its CUDAGraph (the native plans launch the graphs themselves)

    def graph_of(fn):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode=CAPTURE_MODE):
            fn()
        held.append(g)
        gobj[g.replay] = g
        return g.replay

    def chained(rep):
        def f():
            s_ = torch.cuda.current_stream(device)
            cchain.wait(s_)
            rep()
            cchain.mark(s_, 1)
        return f

    gp = []
    seed_cursors(ctr, hctr, state["t"], nprep, NB)
    mode["capture"] = True
    for b in range(NB):
        gp.append((graph_of(lambda b=b: prep(b, 1)), graph_of(lambda b=b: prep(b, 2)))
                  if fchain else graph_of(lambda b=b: prep(b)))
    for j in range(P):
        if watch is not None:
            watch.beat("capture", j)
        t = t0 + j
        b = t % NB
        gw[j] = graph_of(tr.mx_worker(t, locs[b], bufs[b][1], width=39))
        # exchange s = t + xd is issued at iteration t: its phase is (t + xd) % P
        s = t + xd
        parts = tr.mx_exchange(s, locs[(s + 1) % NB])
        gpack = graph_of(parts["pack"])  # (captured in issue order: pack, all-to-all, ...)
        gcomm = graph_of(parts["comm"]) if ccomm else None
        gx[s % P] = {"pack": gpack,
                     "comm": chained(gcomm) if ccomm else parts["comm"], "gcomm": gcomm,
                     "resolve": graph_of(parts["resolve"]), "apply": graph_of(parts["apply"]),
                     "post": parts["post"]}
    prep_fns[:] = gp
    graphs["on"] = True
    torch.cuda.synchronize()
    for _ in range(P):
        iterate()
    torch.cuda.synchronize()
    native = (os.environ.get("PSAMD_MX_NATIVE", "1") == "1" and ccomm and cchain.on
              and cchain.ev is not None)
    if not native:
        return iterate, True
    # one native LaunchList per t % E replays an iteration's graphs (worker, preparation,
    # pack, all-to-all, resolve, apply) with its event waits and records in ONE host call
    # instead of ~25 Python-level stream / event / replay calls (the HIP calls themselves
    # remain: ~8 us per graph launch, ~2.5 per event op, cProfile r5hostprof). 2 peers
    # 0.0963-0.0980 vs 0.0967-0.1123 ms, 8 peers 0.1004-0.1032 (one 0.133) vs 0.0989-0.1125
    # (profiles/r5_mx_native_ab.log; PSAMD_MX_NATIVE=0: the Python iteration)
    from parameter_server_amd.ops.native import hipops

    H = hipops()
    for e in [x for k in ev for x in ev[k]] + ev_buf + ev_prep:
        e.record(main)  # (create every event; each wait still follows its real record)
    torch.cuda.synchronize()
    plans = []
    for k in range(E):
        t = state["t"] + ((k - state["t"]) % E)  # the next t with t % E == k
        s = t + xd
        nb = (t + nprep) % NB
        L = H.LaunchList()
        L.add_stream(main)
        L.add_wait(ev["M"][t % E])
        L.add_graph(gobj[gw[t % P]])
        L.add_record(ev["w"][t % E])
        L.add_stream(sides[nb % nprep])
        # (buffer nb was last trained at t + nprep - NB: its worker-done event is the
        # buffer event; nothing waits for a preparation's own event after the setup)
        L.add_wait(ev["w"][(t + nprep - NB) % E])
        if fchain:  # (the filters in minibatch order)
            L.add_graph(gobj[gp[nb][0]])
            L.add_wait(ev_prep[(nb - 1) % NB])
            L.add_graph(gobj[gp[nb][1]])
            L.add_record(ev_prep[nb])
        else:
            L.add_graph(gobj[gp[nb]])
        xp = gx[s % P]
        L.add_stream(sides[((s + 1) % NB) % nprep])
        L.add_graph(gobj[xp["pack"]])
        L.add_wait(ev["w"][(s - d) % E])
        L.add_wait(ev["res"][(s - 1) % E])
        L.add_wait(cchain.ev)
        L.add_graph(gobj[xp["gcomm"]])
        L.add_record(cchain.ev)
        L.add_record(ev["M"][s % E])
        L.add_wait(ev["app"][(s - 1) % E])
        if xp["post"]:
            L.add_graph(gobj[xp["resolve"]])
            L.add_record(ev["res"][s % E])
            L.add_graph(gobj[xp["apply"]])
        else:
            L.add_graph(gobj[xp["apply"]])
            L.add_graph(gobj[xp["resolve"]])
            L.add_record(ev["res"][s % E])
        L.add_record(ev["app"][s % E])
        L.add_stream(main)
        plans.append(L)

    def iterate_native():
        t = state["t"]
        plans[t % E].run()
        tr.mx_done(B)
        cchain.n += 1
        tr._mx_next = t + xd + 1
        state["t"] = t + 1

    iterate_native.release = release
    for _ in range(P):
        iterate_native()
    torch.cuda.synchronize()
    args.native_iter = True  # (reported as config.native_iteration)
    if os.environ.get("PSAMD_MX_G2", "1") == "1":
        # TWO graph launches per iteration: the main stream's graph (wait for exchange t,
        # worker t, record) and the preparation stream's graph (preparation, pack,
        # all-to-all, owner resolve / apply), each a native GraphChain of the captured
        # pieces with every cross-stream event wait / record as an event node between
        # them, instead of 6 graph launches + 11 host event calls
        # (benchmarks/probe_graph_events.py)
        Eg = P * -(-8 // P)
        # (PSAMD_MX_TILE_GATE=1: the 1-GPU tile gate here too -- measured SLOWER at 8 emulated
        # peers, 0.1196 vs 0.1011-0.1021 ms, config 4 0.1245 vs 0.1020: the merged
        # iteration's preparation has no slack to wait for the worker, gpurun r6y)
        tgate = os.environ.get("PSAMD_MX_TILE_GATE", "0") == "1"
        evg = {k: [torch.cuda.Event() for _ in range(Eg)] for k in ("w", "M", "res", "app")}
        evp = [torch.cuda.Event() for _ in range(NB)]
        for e in [x for k in evg for x in evg[k]] + evp:
            e.record(main)
        torch.cuda.synchronize()
        g2 = []

        def piece(fn):  # a captured piece kept as a graph (cloned into the chains)
            g = torch.cuda.CUDAGraph(keep_graph=True)
            with torch.cuda.graph(g, capture_error_mode=CAPTURE_MODE):
                fn()
            held.append(g)
            return g

        for k in range(Eg):
            if watch is not None:
                watch.beat("capture2", k)
            t = state["t"] + ((k - state["t"]) % Eg)
            s = t + xd
            nb = (t + nprep) % NB
            b = t % NB
            cm = H.GraphChain()
            cm.add_wait(evg["M"][t % Eg])
            cm.add_child(piece(tr.mx_worker(t, locs[b], bufs[b][1], width=39)))
            cm.add_record(evg["w"][t % Eg])
            cm.instantiate()
            parts = tr.mx_exchange(s, locs[(s + 1) % NB])
            cs = H.GraphChain()
            cs.add_wait(evg["w"][(t + nprep - NB) % Eg])
            if tgate:
                # the localisation of minibatch t + nprep waits for worker t (its fused
                # forward / backward): the 1024-thread tile kernel and the forward /
                # backward then do not split the CUs (the 1-GPU pipeline's tile gate)
                cs.add_child(piece(lambda nb=nb: prep(nb, 3)))
                cs.add_wait(evg["w"][t % Eg])
                cs.add_child(piece(lambda nb=nb: prep(nb, 4)))
                if fchain:
                    cs.add_wait(evp[(nb - 1) % NB])
                    cs.add_child(piece(lambda nb=nb: prep(nb, 2)))
                    cs.add_record(evp[nb])
                cs.add_child(piece(parts["pack"]))
            elif fchain:  # (the filters in minibatch order)
                cs.add_child(piece(lambda nb=nb: prep(nb, 1)))
                cs.add_wait(evp[(nb - 1) % NB])
                cs.add_child(piece(lambda nb=nb: prep(nb, 2)))
                cs.add_record(evp[nb])
                cs.add_child(piece(parts["pack"]))
            else:
                cs.add_child(piece(lambda nb=nb, pk=parts["pack"]: (prep(nb), pk())))
            cs.add_wait(evg["w"][(s - d) % Eg])
            cs.add_wait(evg["res"][(s - 1) % Eg])
            cs.add_wait(cchain.ev)
            cs.add_child(piece(parts["comm"]))
            cs.add_record(cchain.ev)
            cs.add_record(evg["M"][s % Eg])
            cs.add_wait(evg["app"][(s - 1) % Eg])
            if parts["post"]:
                cs.add_child(piece(parts["resolve"]))
                cs.add_record(evg["res"][s % Eg])
                cs.add_child(piece(parts["apply"]))
            else:
                cs.add_child(piece(parts["apply"]))
                cs.add_child(piece(parts["resolve"]))
                cs.add_record(evg["res"][s % Eg])
            cs.add_record(evg["app"][s % Eg])
            cs.instantiate()
            held.extend([cm, cs])
            L = H.LaunchList()
            L.add_stream(main)
            L.add_chain(cm)
            L.add_stream(sides[nb % nprep])
            L.add_chain(cs)
            L.add_stream(main)
            g2.append(L)
        torch.cuda.synchronize()

        def iterate_g2():
            t = state["t"]
            g2[t % Eg].run()
            tr.mx_done(B)
            cchain.n += 1
            tr._mx_next = t + xd + 1
            state["t"] = t + 1

        iterate_g2.release = release
        for _ in range(P):
            iterate_g2()
        torch.cuda.synchronize()
        args.native_iter = "graph2"
        return iterate_g2, True
    return iterate_native, True


def spawn_ranks(n: int, argv: list[str] | None = None, script: str | None = None) -> int:
    """Re-launch this script as ``n`` ranks through torch.distributed.run (rendezvous on
    127.0.0.1, a free port) as a CHILD process, and return its exit code. Called
    before any GPU call, so the parent never initialises the device."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr=127.0.0.1", f"--master-port={port}",
           script or os.path.abspath(__file__)] + list(sys.argv[1:] if argv is None else argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


def supervise(argv: list[str]) -> int:
    """A torchrun rank of a multi-rank job, as a SUPERVISOR that never touches the GPU:
    it runs this script as a child process (the real rank, on a rendezvous of its own),
    and if the job's first attempt (collectives captured in the step graphs, short
    collective timeout) fails on any rank, every supervisor re-runs it in a fresh child
    with eager collectives (PSAMD_CAPTURE_COMM=0). The supervisors agree on ports,
    exit codes and the retry over a host-only gloo group of their own. Rank 0's child
    writes its JSON line to a file; rank 0's supervisor prints the one line, with
    ``comm.captured_attempt`` / ``comm.fallback`` saying what happened."""
    import datetime
    import signal
    import socket
    import subprocess
    import tempfile

    import torch.distributed as dist

    dist.init_process_group("gloo", timeout=datetime.timedelta(hours=2))
    rank, world = dist.get_rank(), dist.get_world_size()
    first_to = os.environ.get("PSAMD_FIRST_COMM_TIMEOUT", "60")
    attempt_limit = float(os.environ.get("PSAMD_ATTEMPT_TIMEOUT", "900"))
    teardown_limit = float(os.environ.get("PSAMD_TEARDOWN_TIMEOUT", "60"))
    attempts = [{"PSAMD_CAPTURE_COMM": os.environ.get("PSAMD_CAPTURE_COMM", "auto"),
                 "PSAMD_COMM_TIMEOUT": os.environ.get("PSAMD_COMM_TIMEOUT", first_to)},
                {"PSAMD_CAPTURE_COMM": "0"}]
    if attempts[0]["PSAMD_CAPTURE_COMM"] == "0":
        attempts = attempts[1:]
    result_dir = tempfile.mkdtemp(prefix="psamd_bench_")
    rc, first_rc, line = 1, None, None
    for i, extra in enumerate(attempts):
        port = [None]
        if rank == 0:
            with socket.socket() as sk:
                sk.bind(("127.0.0.1", 0))
                port[0] = sk.getsockname()[1]
        dist.broadcast_object_list(port, src=0)
        res = os.path.join(result_dir, f"attempt{i}.json")
        env = dict(os.environ, MASTER_PORT=str(port[0]), PSAMD_SUPERVISED="1",
                   PSAMD_RESULT_FILE=res, TORCHELASTIC_USE_AGENT_STORE="False", **extra)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if first_rc is not None:
            env["PSAMD_FALLBACK_FROM"] = str(first_rc)
        child = subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env,
                                 start_new_session=True)
        # wait for the child: at most the attempt limit, and once this rank has passed
        # the timed region (its ".timed" marker) at most PSAMD_TEARDOWN_TIMEOUT more --
        # a rank hanging in teardown (communicator destroy, graph release) must not
        # cost the whole attempt limit
        t_start, t_timed, rc = time.time(), None, None
        while rc is None:
            try:
                rc = child.wait(timeout=1.0)
            except subprocess.TimeoutExpired:
                now = time.time()
                if t_timed is None and os.path.exists(res + ".timed"):
                    t_timed = now
                if now - t_start > attempt_limit or (
                        t_timed is not None and now - t_timed > teardown_limit):
                    os.killpg(child.pid, signal.SIGKILL)
                    child.wait()
                    rc = 124 if t_timed is None else 125
        rcs = [None] * world
        dist.all_gather_object(rcs, rc)
        if rank == 0 and os.path.exists(res):
            with open(res) as f:
                line = f.read().strip() or None
        ok = [line is not None] if rank == 0 else [None]
        dist.broadcast_object_list(ok, src=0)
        if all(r == 0 for r in rcs):
            rc = 0
            break
        if ok[0]:
            # rank 0's result exists, so EVERY rank passed the timed region (it ends in a
            # barrier and a max all-reduce over ranks): the measurement is complete and
            # the failures came after it. Report them in the line instead of hiding them.
            if rank == 0:
                d = json.loads(line)
                d.setdefault("comm", {})["rank_exit_codes"] = rcs
                d["comm"]["post_timing_failures"] = [r for r, c in enumerate(rcs) if c != 0]
                line = json.dumps(d)
                print(f"[psamd] ranks {d['comm']['post_timing_failures']} exited non-zero "
                      f"after the timed region (exit codes {rcs}); result kept and the "
                      f"failures recorded in comm.post_timing_failures", file=sys.stderr,
                      flush=True)
            rc = 0
            break
        first_rc = max(r for r in rcs if r is not None)
        if rank == 0 and i + 1 < len(attempts):
            print(f"[psamd] attempt {i} ({extra}) failed on some rank (exit codes {rcs}); "
                  f"re-running in fresh processes with eager collectives", file=sys.stderr,
                  flush=True)
    if rank == 0 and line is not None:
        print(line, flush=True)
    dist.destroy_process_group()
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--minibatch", type=int, default=65536, help="examples per GPU per step")
    ap.add_argument("--num-features", type=float, default=1e9)
    ap.add_argument("--algo", default="ftrl")
    ap.add_argument("--consistency", default="ssp:4")
    ap.add_argument("--graph", type=int, default=-1,
                    help="replay the pipeline's pieces from HIP graphs: 1 / 0, 2 = the data "
                         "preparations only, -1 = auto (on with more than one rank or emulated "
                         "peers, off on one GPU)")
    ap.add_argument("--pipeline", type=int, default=1,
                    help="generate + localise minibatch t+1 on a high-priority side stream "
                         "while step t trains (HIP graphs per stream / step segment)")
    ap.add_argument("--prep-streams", type=int, default=0,
                    help="concurrent data-preparation streams (each generates + localises "
                         "every n-th minibatch ahead of the training step). Measured 1 GPU "
                         "ms/step: 1 -> 0.309, 2 -> 0.241, 3 -> 0.230, 4 -> 0.43; 8 emulated "
                         "peers with a communicator stream, exchange on the prep streams: "
                         "1 -> 0.46, 2 -> 0.308, 3 -> 0.334 in round 1; with the applies at the "
                         "tail of the exchange half (round 2): 2 -> 0.162, 3 -> 0.139). 0 = "
                         "auto: 3")
    ap.add_argument("--exchange", default="padded", choices=["padded", "exact", "p2p"],
                    help="N > 1: fixed-capacity sync-free exchange, count-sized all-to-all-v, "
                         "or one-sided peer-HBM pulls + inbox pushes (asp only, no collective "
                         "per step: parallel/p2p.py)")
    ap.add_argument("--fixing-float", type=int, default=0)
    ap.add_argument("--exchange-merge", default="auto", choices=["auto", "on", "off"],
                    help="N > 1, lag >= 1: one all-to-all per step carrying [keys(t+1) | "
                         "pushes | weights of keys(t)] (auto: ssp:tau >= 2) or the "
                         "two-collective exchange (off)")
    ap.add_argument("--exchange-lag", type=int, default=-1,
                    help="padded exchange lag (-1: from --consistency; asp on the merged "
                         "exchange: the staleness, default 3)")
    ap.add_argument("--ssp-apply", default="post", choices=["post", "pre"],
                    help="N > 1, ssp: the owner applies the carried pushes after sending the "
                         "pulled weights back (post) or before resolving the pulls (pre)")
    ap.add_argument("--push-mode", default="sequential", choices=["sequential", "aggregate"],
                    help="N > 1: one optimizer step per source row in rank order (per-push, "
                         "KVStore semantics), or the owner sums the G workers' gradients of a "
                         "key and applies one step (KVBufferedVector semantics; measured slower "
                         "on MI355X: device-scope atomics per entry, 0.437 vs 0.367 ms at 8 "
                         "emulated peers)")
    ap.add_argument("--localize", default="auto", choices=["sort", "tp", "part", "auto"])
    ap.add_argument("--emulate-peers", type=int, default=0,
                    help="1 process: run the N-GPU padded step with N emulated peers over a "
                         "loopback exchange (per-GPU device cost of the N-GPU step, no "
                         "collectives); reported as n_gpus 1 with 'emulated_peers'")
    ap.add_argument("--emulate-backend", default="auto", choices=["auto", "copy", "nccl"],
                    help="emulated peers: exchanges as stream copies, or through a real "
                         "1-rank RCCL communicator (RCCL kernels + ProcessGroupNCCL waits); "
                         "auto = nccl on the GPU (the stream structure of the real run: 8 "
                         "peers 0.137 ms/step, copy 0.268 with its extra copy stream), copy "
                         "on the CPU")
    ap.add_argument("--prefill", type=float, default=0,
                    help="insert this many random keys into each shard before timing (the "
                         "populated-table regime, e.g. 5e8 on 2^31 slots = 23%% load)")
    ap.add_argument("--tail-freq", type=int, default=0,
                    help="tail-feature filter: train only keys seen > this many times "
                         "(CountMin, the reference CTR conf's tail_feature_freq: 1); 0 = off")
    ap.add_argument("--countmin-n", type=float, default=1e8)
    ap.add_argument("--progress", action="store_true")
    ap.add_argument("--cpu", action="store_true", help="run on CPU (plumbing check)")
    ap.add_argument("--trace", default="",
                    help="write per-rank traffic/phase JSON here ({rank} substituted); "
                         "PSAMD_TRACE=1 adds roctx ranges + phase timers")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ and not args.emulate_peers:
        # `python bench.py --gpus N`: fan out N ranks (one per GPU) before anything
        # touches the GPU, like the reference's launcher owns process fan-out
        # (script/local.sh:1-43); this process only waits and forwards the exit code.
        return spawn_ranks(args.gpus)
    if (int(os.environ.get("WORLD_SIZE", "1")) > 1 and "PSAMD_SUPERVISED" not in os.environ
            and os.environ.get("PSAMD_SUPERVISE", "1") != "0"):
        return supervise(sys.argv[1:])  # (before anything touches the GPU)
    if os.environ.get("PSAMD_INJECT_CAPTURE_FAIL") == "1" and \
            os.environ.get("PSAMD_CAPTURE_COMM", "auto") != "0":
        # fault injection (tests/test_bench_spawn.py): the captured attempt dies like a
        # rank the stall watchdog ended
        from parameter_server_amd.utils.watchdog import EXIT_STALL

        print("[psamd] injected failure of the captured-collective attempt", file=sys.stderr)
        return EXIT_STALL

    from parameter_server_amd.models import SparseLRConfig, SparseLRTrainer
    from parameter_server_amd.ops.synthetic import criteo_batch
    from parameter_server_amd.parallel.comm import init_from_env

    from parameter_server_amd.utils.watchdog import (StallWatch, default_timeout, maybe_inject,
                                                     maybe_inject_post)

    watch = StallWatch(int(os.environ.get("RANK", "0")), default_timeout())
    comm, device = init_from_env("cpu" if args.cpu else "cuda")
    watch.comm = comm
    watch.beat("setup")
    if args.emulate_peers > 1 and comm.world == 1:
        from parameter_server_amd.parallel.comm import LoopbackComm, nccl_loopback

        eb = args.emulate_backend
        if eb == "auto":
            eb = "nccl" if device.type == "cuda" else "copy"
        comm = (nccl_loopback(args.emulate_peers, device) if eb == "nccl"
                else LoopbackComm(args.emulate_peers, device))
    G, rank = comm.world, comm.rank
    if args.graph < 0:
        # auto: one GPU issues its kernels eagerly -- the HIP-graph replays of the same
        # pipeline measured ~10 % slower there (0.119-0.120 vs 0.105-0.109 ms / step at
        # B = 65,536, 0.0645 vs 0.0575 at B = 10,000, same box; profiles/r3_s2_graph_ab.log)
        # while the host still issues a step in ~0.075 ms. With peers the step has many
        # more launches plus the collectives and the eager host issue becomes the bound
        # (8 emulated peers: 0.179 eager vs 0.147 graphs), so graphs stay on there.
        args.graph = 1 if G > 1 else 0
    if G != args.gpus and rank == 0 and not args.emulate_peers:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {G}", file=sys.stderr)
    B = args.minibatch
    N = int(args.num_features)
    # reference CTR online config (example/linear/ctr/online_l1lr.conf): FTRL, L1 10 / L2 1,
    # DECAY alpha .01 beta 10; AdaGrad / SGD with their own step sizes (sparse_lr.ALGO_DEFAULTS)
    from parameter_server_amd.models.sparse_lr import algo_defaults

    hyper = algo_defaults(args.algo)
    cfg = SparseLRConfig(num_features=N, minibatch=B, algo=args.algo, **hyper,
                         consistency=args.consistency,
                         fixing_float_bytes=args.fixing_float, exchange=args.exchange,
                         localize=args.localize, push_mode=args.push_mode,
                         ssp_apply=args.ssp_apply, exchange_merge=args.exchange_merge,
                         tail_feature_freq=args.tail_freq, countmin_n=args.countmin_n,
                         exchange_lag=args.exchange_lag,
                         seed=rank)
    tr = SparseLRTrainer(cfg, comm, device)
    prefill_occ = None
    if args.prefill > 0:
        t0 = time.time()
        prefill_occ = tr.prefill(int(args.prefill))
        if rank == 0:
            print(f"prefill: {prefill_occ} occupied slots of {tr.table.capacity} "
                  f"({prefill_occ / tr.table.capacity:.1%}) in {time.time() - t0:.1f} s",
                  file=sys.stderr, flush=True)
    keys = torch.empty(B * 39, dtype=torch.int64, device=device)
    labels = torch.empty(B, dtype=torch.float32, device=device)
    seed = 1000003 * (rank + 1)
    gpu = device.type == "cuda"

    def one_step():
        # fresh rows every step: row0 = device step clock * B (advanced by the
        # trainer's epilogue kernel, so graph replays generate new data)
        if gpu:
            criteo_batch(B, seed=seed, row0=0, num_features=N, device=device, keys=keys,
                         labels=labels, row0_dev=tr.step_dev, row_scale=B)
        else:
            criteo_batch(B, seed=seed, row0=tr.step_count * B, num_features=N, device=device,
                         keys=keys, labels=labels)
        tr.step(keys, labels, width=39)

    run = one_step
    graph_used = False
    one_graph = None
    if gpu and G > 1 and not tr.padded:
        # multi-GPU: double-buffered minibatches; minibatch t+1 is generated and
        # localised on a side stream while step t waits for its exchange counts
        side = torch.cuda.Stream(device)
        bufs = [(keys, labels), (torch.empty_like(keys), torch.empty_like(labels))]
        state = {"t": 0, "loc": None}

        def produce(t):
            k, lab = bufs[t % 2]
            side.wait_stream(torch.cuda.current_stream(device))
            with torch.cuda.stream(side):
                criteo_batch(B, seed=seed, row0=t * B, num_features=N, device=device, keys=k,
                             labels=lab)
                return tr.localize(k, buf=t % 2)

        def pipelined_step():
            t = state["t"]
            loc = state["loc"] if state["loc"] is not None else produce(t)
            torch.cuda.current_stream(device).wait_stream(side)
            nxt = {}
            k, lab = bufs[t % 2]
            tr.step(k, lab, width=39, loc=loc, prefetch=lambda: nxt.setdefault("loc", produce(t + 1)))
            state["loc"] = nxt.get("loc")
            state["t"] = t + 1

        run = pipelined_step
    import contextlib

    scope = contextlib.ExitStack()
    mprio = os.environ.get("PSAMD_MAIN_PRIORITY")
    if gpu and mprio is not None:
        # the training step on its own stream of this priority instead of the null stream
        scope.enter_context(torch.cuda.stream(torch.cuda.Stream(device, priority=int(mprio))))
    watch.beat("warmup")
    if gpu and args.pipeline and (G == 1 or tr.padded):
        # 3 preparation streams. 1 GPU at the driver's 20 timed steps: 0.0849-0.0869 ms
        # (mean 0.0860) with 3 vs 0.0852-0.0903 (mean 0.0873) with 2, 6 runs each on the
        # same boxes; over 300 steps 2 are ~1 % faster, 0.0813 vs 0.0823
        # (profiles/r5_prep_streams.log). Rounds 3-4 kept 2
        # on older kernels (0.109-0.110 vs 0.112-0.116 over 300 steps, r3_s2_graph_ab.log)
        nprep = args.prep_streams or 3
        args.prep_streams = nprep
        run, graph_used = pipeline(tr, B, N, seed, keys, labels, device, args, nprep=nprep,
                                   watch=watch)
    else:
        for i in range(max(1, args.warmup)):
            watch.beat("warmup", i)
            run()
    if gpu and G == 1 and args.graph and not args.pipeline:
        try:
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                one_step()  # warm the side stream
            torch.cuda.current_stream().wait_stream(s)
            torch.cuda.synchronize()
            with torch.cuda.graph(g, capture_error_mode=CAPTURE_MODE):
                one_step()
            run = g.replay
            run()
            torch.cuda.synchronize()
            graph_used = True
            one_graph = g
        except Exception as e:  # fall back to eager launches
            if rank == 0:
                print(f"graph capture unavailable ({e!r}); eager", file=sys.stderr)
            run = one_step
    watch.beat("pre-timing")
    tr.progress(reset=True)
    # two more untimed iterations after the metrics reset (its device reads idle the GPU
    # for a few ms): the timed region then starts right behind busy work, as in steady
    # state (PSAMD_PRE_TIMING_ITERS, default 2; the train block's loss / AUC include them)
    for _ in range(int(os.environ.get("PSAMD_PRE_TIMING_ITERS", "2"))):
        run()

    comm.barrier()
    if gpu:
        torch.cuda.synchronize()
    # PSAMD_STEP_EVENTS=1: a main-stream event after every timed step (diagnostic of the
    # pipeline's fill / drain in short runs; prints per-step GPU ms to stderr)
    sev = ([torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
           if gpu and os.environ.get("PSAMD_STEP_EVENTS") == "1" else None)
    t0 = time.perf_counter()
    if sev:
        sev[0].record()
    for i in range(args.steps):
        watch.beat("timed", i)
        maybe_inject(rank, i)
        run()
        if sev:
            sev[i + 1].record()
        if args.progress and rank == 0 and (i + 1) % 10 == 0:
            print(f"step {i + 1}", file=sys.stderr)
    t_issue = time.perf_counter() - t0  # host time to enqueue the K steps (CPU-bound check)
    watch.beat("timed-drain")
    if getattr(tr, "px", None) is not None:
        # p2p: apply every push every rank posted (collective, host channel) before the
        # device sync: a post still waiting for a peer's ring space completes only as the
        # peer drains (part of the timed work)
        tr.flush()
    if gpu:
        torch.cuda.synchronize()
    t_main = time.perf_counter() - t0
    if sev and rank == 0:
        print("step_events_ms", [round(sev[i].elapsed_time(sev[i + 1]), 4)
                                 for i in range(args.steps)],
              "wall_to_sync_ms", round(t_main * 1e3, 4), file=sys.stderr)
    comm.barrier()
    dt = time.perf_counter() - t0
    watch.beat("report")
    t = torch.tensor([dt, -dt], dtype=torch.float64,
                     device=device if comm.world > 1 and gpu else "cpu")
    comm.all_reduce_(t, op="max")
    dt, dt_min = float(t[0].item()), -float(t[1].item())
    prog = tr.progress(reset=True)
    tr.check_ok()  # table full, localisation or exchange overflow: fail, do not report
    occ, nnz = tr.table.census()
    emulated = comm.backend == "loopback" if hasattr(comm, "backend") else False
    n_ranks = 1 if emulated else G
    total_examples = n_ranks * B * args.steps
    value = total_examples / dt
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "examples/sec",
            "n_gpus": n_ranks,
            "steps": args.steps,
            "warmup": args.warmup,
            "host_issue_ms_per_step": t_issue / args.steps * 1e3,
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic (Criteo-1TB-shaped: 13 int + 26 categorical slots, power-law ids "
                    f"hashed into {N:.0e} features; zero-init optimizer state)",
            "config": {
                "model": f"sparse logistic regression, {ALGO_NAMES.get(args.algo, args.algo)} "
                         f"L1={hyper['l1']:g} L2={hyper['l2']:g} {hyper['lr_type'].upper()} "
                         f"alpha={hyper['alpha']:g} beta={hyper['beta']:g} (server-side), "
                         f"{N:.0e} hashed features",
                "global_batch": n_ranks * B,
                "seq_len": 39,
                "nnz_per_example": 39,
                "parallelism": f"dp{n_ranks}+kvshard{n_ranks}",
                "consistency": tr.consistency_desc(),
                "push": args.push_mode if G > 1 else None,
                "ssp_apply": ("merged" if getattr(tr, "merged", False) else
                              args.ssp_apply if G > 1 and tr.padded and tr.lag >= 1
                              and not tr.asp else None),
                "collectives_per_step": (1 if getattr(tr, "merged", False) else
                                         2 if G > 1 and tr.padded else None),
                "table_slots_per_gpu": tr.table.capacity,
                "hip_graph": graph_used,
                "collectives_in_graphs": bool(getattr(pipeline, "captured_comm", False)
                                              and graph_used),
                "prep_streams": args.prep_streams if (gpu and args.pipeline) else 1,
                "native_iteration": getattr(args, "native_iter", False),
                "localize": tr.localize_mode,
                "emulated_peers": G if emulated else None,
                "exchange": (f"{args.exchange} (capacity {tr.xc.C} keys/peer/step)"
                             if tr.xc is not None else (args.exchange if G > 1 else None)),
                "prefill_keys_per_gpu": int(args.prefill) if args.prefill > 0 else None,
                "tail_feature_freq": args.tail_freq or None,
            },
            "comm": {"backend": getattr(comm, "backend", "local"),
                     "world": comm.world,
                     "rccl_world": (torch.distributed.get_world_size()
                                    if torch.distributed.is_initialized()
                                    and torch.distributed.get_backend() == "nccl" else 0),
                     "per_rank_ms": [dt_min * 1e3, dt * 1e3],
                     "collectives_rank0": comm.chain.n if comm.chain is not None else 0,
                     "timeout_s": float(os.environ.get("PSAMD_COMM_TIMEOUT", "180")),
                     # multi-rank: the collectives rode the step graphs; fallback = the
                     # exit code of a failed captured attempt this eager run replaced
                     "captured": bool(getattr(pipeline, "captured_comm", False) and graph_used),
                     "fallback": (int(os.environ["PSAMD_FALLBACK_FROM"])
                                  if "PSAMD_FALLBACK_FROM" in os.environ else None)},
            "train": {"loss": prog["loss"], "auc": prog["auc"], "accuracy": prog["accuracy"],
                      "trains": bool(prog["loss"] < math.log(2)),
                      "table_occupied_rank0": occ, "nnz_w_rank0": nnz},
        }
        res = os.environ.get("PSAMD_RESULT_FILE")
        if res:  # (a supervised rank: the supervisor prints the one line)
            with open(res + ".tmp", "w") as f:
                f.write(json.dumps(out) + "\n")
            os.replace(res + ".tmp", res)
        else:
            print(json.dumps(out), flush=True)
    res = os.environ.get("PSAMD_RESULT_FILE")
    if res:  # this rank is past the timed region: its supervisor caps the teardown wait
        open(res + ".timed", "w").close()
    maybe_inject_post(rank)
    scope.close()
    if args.trace:
        from parameter_server_amd.utils import trace

        trace.dump(args.trace, rank)
    import torch.distributed as dist

    watch.beat("teardown")
    # graphs first (one holding RCCL work keeps the communicator's teardown waiting)
    if getattr(run, "release", None) is not None:
        run.release()
    if one_graph is not None:
        one_graph.reset()
    del run, one_graph
    if dist.is_initialized():
        dist.destroy_process_group()
    watch.stop()


if __name__ == "__main__":
    try:
        rc = main() or 0
    except BaseException as e:  # name the rank / phase / step / collective that failed
        from parameter_server_amd.utils import watchdog

        w = watchdog.CURRENT
        print(f"[psamd] FAILED {w.describe() if w is not None else ''}: {type(e).__name__}: "
              f"{str(e)[:300]}", file=sys.stderr, flush=True)
        raise
    sys.exit(rc)
