#!/usr/bin/env python3
"""Wide & deep (BASELINE.json config 5): 1e9 x 128 bf16 embedding table sharded over
the ranks, dense-block push/pull over RCCL, MLP on the bf16 MFMA GEMM.
Metric: examples/sec (whole node), weak scaling (fixed minibatch per GPU).

    python benchmarks/bench_wide_deep.py --steps 20
    torchrun --nproc-per-node N benchmarks/bench_wide_deep.py ...
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
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--table-slots", type=int, default=1 << 27, help="slots per GPU")
    ap.add_argument("--gemm", default="auto", choices=("auto", "mfma", "hipblaslt"))
    ap.add_argument("--prefetch", type=int, default=1,
                    help="generate + localise minibatch t+1 on a side stream during step t")
    ap.add_argument("--overlap-wgrad", type=int, default=1,
                    help="weight-gradient GEMMs on a side stream next to the dX chain")
    ap.add_argument("--emulate-peers", type=int, default=0,
                    help="1 process: the N-GPU step (key exchange + owner updates + dense "
                         "all-reduce) with N emulated peers over a loopback comm")
    ap.add_argument("--graph", type=int, default=0,
                    help="1 GPU: replay the preparation and the training step from HIP graphs "
                         "(one per buffer parity). Off by default: the step graph forks to the "
                         "weight-gradient stream, and that multi-stream graph replayed at "
                         "1.39 ms / step vs 0.97 eager (host issue 0.57 ms, so the eager step "
                         "is not host bound)")
    ap.add_argument("--prefill", type=float, default=0,
                    help="random keys (with rows) inserted per GPU before timing")
    args = ap.parse_args()
    from parameter_server_amd.models.wide_deep import WideDeepConfig, WideDeepTrainer
    from parameter_server_amd.ops.synthetic import criteo_batch
    from parameter_server_amd.parallel.comm import init_from_env

    comm, dev = init_from_env("cuda")
    if args.emulate_peers > 1 and comm.world == 1:
        from parameter_server_amd.parallel.comm import LoopbackComm

        comm = LoopbackComm(args.emulate_peers, dev)
    G, rank = comm.world, comm.rank
    emu = comm.backend == "loopback" if hasattr(comm, "backend") else False
    NG = 1 if emu else G  # GPUs actually running
    B, N = args.minibatch, int(args.num_features)
    cfg = WideDeepConfig(localize=args.localize, num_features=N, embedding_dim=args.dim, minibatch=B,
                         table_capacity=args.table_slots, gemm=args.gemm, seed=0,
                         overlap_wgrad=bool(args.overlap_wgrad))
    tr = WideDeepTrainer(cfg, comm, dev)
    if args.prefill > 0:
        import time as _t

        t0 = _t.time()
        occ = tr.prefill(int(args.prefill))
        print(f"prefill: {occ} occupied of {tr.shard.capacity} slots "
              f"({occ / tr.shard.capacity:.1%}) in {_t.time() - t0:.1f} s", flush=True)
    bufs = [(torch.empty(B * 39, dtype=torch.int64, device=dev),
             torch.empty(B, dtype=torch.float32, device=dev)) for _ in range(2)]
    t = [0]
    locs = [None, None]
    side = torch.cuda.Stream(dev, priority=int(os.environ.get("PSAMD_PREP_PRIORITY", "-1")))  # own HW queues
    main = torch.cuda.current_stream(dev)
    ev_prep = [torch.cuda.Event() for _ in range(2)]
    ev_step = [torch.cuda.Event() for _ in range(2)]
    # rows of minibatch i = (2 * ctr[i % 2] + i % 2) * B: a device counter per buffer, so a
    # captured preparation generates fresh rows on every replay
    ctr = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(2)]
    graphed = {"prep": None, "step": None}

    def prep_body(b):
        k, lab = bufs[b]
        criteo_batch(B, seed=77 + rank, row0=b * B, num_features=N, device=dev, keys=k,
                     labels=lab, row0_dev=ctr[b], row_scale=2 * B)
        ctr[b].add_(1)
        locs[b] = tr.localize(k, buf=b)

    def prep(i):  # minibatch i into buffer i % 2, on the side stream
        b = i % 2
        side.wait_event(ev_step[b])  # the step that last read this buffer is done
        with torch.cuda.stream(side):
            if graphed["prep"] is not None:
                graphed["prep"][b]()
            else:
                prep_body(b)
            ev_prep[b].record(side)

    def step():
        # generation + localisation of minibatch t+1 overlaps the training step of t
        i = t[0]
        b = i % 2
        if args.prefetch:
            if i == 0:
                prep(0)
            prep(i + 1)
            main.wait_event(ev_prep[b])
            if graphed["step"] is not None:
                graphed["step"][b]()
            else:
                tr.step(bufs[b][0], bufs[b][1], loc=locs[b])
            ev_step[b].record(main)
        else:
            k, lab = bufs[0]
            criteo_batch(B, seed=77 + rank, row0=i * B, num_features=N, device=dev, keys=k,
                         labels=lab)
            tr.step(k, lab)
        t[0] += 1

    for _ in range(max(args.warmup, 2)):
        step()
    use_graph = bool(args.graph and args.prefetch and G == 1 and not emu)
    if use_graph:
        # capture after the eager warm-up (the workspaces exist); each graph is one buffer
        # parity's preparation / training step. The minibatches in flight were prepared
        # eagerly, so the replays continue from there.
        torch.cuda.synchronize()
        gp, gs = [], []
        for b in range(2):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                prep_body(b)
            gp.append(g)
        for b in range(2):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                tr.step(bufs[b][0], bufs[b][1], loc=locs[b])
            gs.append(g)
        graphed["prep"] = [g.replay for g in gp]
        graphed["step"] = [g.replay for g in gs]
        torch.cuda.synchronize()
        for _ in range(2):
            step()
    tr.progress()
    comm.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    t_issue = time.perf_counter() - t0
    torch.cuda.synchronize()
    comm.barrier()
    dt = time.perf_counter() - t0
    x = torch.tensor([dt], dtype=torch.float64, device=dev if NG > 1 else "cpu")
    comm.all_reduce_(x, op="max")
    dt = float(x.item())
    p = tr.progress()
    occ, _ = tr.shard.table.census()
    if rank == 0:
        print(json.dumps({
            "metric": "examples/sec (whole node) wide&deep 1e9x128 bf16 embeddings + MLP",
            "value": NG * B * args.steps / dt, "unit": "examples/sec", "n_gpus": NG,
            "emulated_peers": G if emu else None,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3,
            "host_issue_ms_per_step": t_issue / args.steps * 1e3, "hip_graph": use_graph,
            "higher_is_better": True, "scaling": "weak", "dtype": "bf16 (fp32 accumulate)",
            "config": {"num_features": N, "embedding_dim": args.dim, "slots": 39,
                       "hidden": list(cfg.hidden), "global_batch": NG * B, "gemm": args.gemm,
                       "table_slots_per_gpu": tr.shard.capacity,
                       "table_slots_total": NG * tr.shard.capacity,
                       "table_note": ("ids hashed over num_features; rows are created on first "
                                      "touch, so a run needs slots only for the ids it touches. "
                                      "The default 2^27 slots per GPU is the per-GPU shard of "
                                      "the 8-GPU config: a 1e9-row table needs 8 GPUs at "
                                      "128 x bf16 (256 GB of rows alone)"),
                       "shard_gb": tr.shard.nbytes() / 2 ** 30, "mlp_params": tr.num_params},
            "train": {**p, "rows_rank0": occ},
        }), flush=True)
    if NG > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == "__main__":
    main()
