"""The reference's user entry point on the GPU engine: ``ps -app_file <conf>`` with text
data files, trained in HBM.

    python -m parameter_server_amd.app.gpu -app_file example/linear/ctr/online_l1lr.conf
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m parameter_server_amd.app.gpu \\
        -app_file batch_l1lr.conf

Reference path: ``main`` -> ``App::create`` -> ``LM::createApp`` (src/app/main/main.cc:15-39,
src/app/linear_method/linear.cc:8-33); async SGD workers stream their files through
``MinibatchReader`` (src/app/linear_method/async_sgd.h:197-239, src/learner/sgd.h:103-157),
Darlin workers load them through ``SlotReader`` (src/learner/bcd.h:316-322). Here every
torchrun rank is one GPU = a colocated worker + server shard:

* ``async_sgd`` -> ``SparseLRTrainer`` (models/sparse_lr.py) through ``lm_to_sparse_lr``:
  minibatch, loss, FTRL / AdaGrad / SGD, learning rate, L1 / L2, tail filter,
  fixing-float, ``max_delay`` -> ``ssp:max_delay`` (0: the reference's unbounded
  pipelining = ``asp`` with more than one rank). The rank's files (``divide_files``,
  round-robin as postmaster.cc:6-15) stream through ``DeviceFeeder``: C++ parser
  threads -> pinned double-buffered host slots -> async host->HBM copies on a side
  stream, overlapped with the step. Rows of one width without values take the fused
  fixed-width path; anything else the CSR (``row_ptr`` + ``vals``) path. With several
  ranks a rank whose files ran out keeps joining the exchanges with key-less steps
  (it still owns a shard) until every rank is done.
* ``darlin`` -> ``DarlinTrainer`` (models/darlin.py) through ``DarlinConfig.from_lm``.
* progress: the reference's ``sec examples loss auc accuracy |w|_0 updt ratio`` line
  (ISGDScheduler::showProgress, sgd.h:45-80) every ``report_interval`` seconds, and the
  Darlin tables (darlin.h:136-156).
* ``model_output`` -> text ``key\\tweight`` files ``<file>_S<rank>`` (async_sgd.h:160-175,
  bcd.h:251-272).

Flags: ``-app_file``, ``-app_conf`` (appended, reference semantics), ``-num_features N``
(hash keys mod N inside the parser: <= 34-bit keys take the tile localiser; 0 = raw
64-bit keys), ``-max_nnz_per_example`` (localisation workspace per row, default 128),
``-num_threads`` (parser threads), ``-device cpu|cuda``, ``-seed``."""
from __future__ import annotations

import os
import sys
import time


def _flags(argv):
    import argparse

    ap = argparse.ArgumentParser(prog="parameter_server_amd.app.gpu", prefix_chars="-")
    ap.add_argument("-app_file", "--app_file", default=None)
    ap.add_argument("-app_conf", "--app_conf", default=None)
    ap.add_argument("-num_features", "--num_features", type=float, default=0)
    ap.add_argument("-max_nnz_per_example", "--max_nnz_per_example", type=int, default=128)
    ap.add_argument("-num_threads", "--num_threads", type=int, default=4)
    ap.add_argument("-device", "--device", default="auto")
    ap.add_argument("-seed", "--seed", type=int, default=0)
    ap.add_argument("-table_capacity", "--table_capacity", type=int, default=0)
    # binary example cache (data/bincache.py): "" = $PSAMD_DATA_CACHE, else a private
    # temporary one when num_data_pass > 1; "off" = parse the text on every pass
    ap.add_argument("-data_cache", "--data_cache", default="")
    # cached-pass reader threads (pread -> pinned slots): the cached pass waits on them
    # (Criteo-shaped 8 M rows, B = 65,536: 8 threads 52-64 M ex/s, 16 threads 86 M,
    # profiles/r6_app_cache.log)
    ap.add_argument("-io_threads", "--io_threads", type=int, default=16)
    # progress lines every this many steps when the step count is agreed up front (a
    # fully cached multi-rank run); 0 = 20 lines per run
    ap.add_argument("-report_steps", "--report_steps", type=int, default=0)
    ap.add_argument("-quiet", "--quiet", action="store_true")
    return ap.parse_args(argv)


def rank_files(data_conf, G: int, rank: int) -> list[str]:
    from ..data import divide_files, search_files

    files = search_files(data_conf)
    if not files:
        raise FileNotFoundError(f"no training files match {list(data_conf.file)}")
    return divide_files(files, G, data_conf.max_num_files_per_worker)[rank]


class ProgressPrinter:
    """``sec examples loss auc accuracy |w|_0 updt ratio`` (reference sgd.h:45-80)."""

    def __init__(self, out=sys.stderr):
        self.out, self.t0, self.head, self.examples = out, time.time(), True, 0.0

    def __call__(self, p: dict):
        if self.head:
            print(" sec  examples    loss      auc   accuracy   |w|_0  updt ratio", file=self.out)
            self.head = False
        self.examples += p["examples"]
        print("%4d  %.2e  %.3e  %.4f  %.4f  %.2e  %.2e" % (
            int(time.time() - self.t0), self.examples, p["loss"], p["auc"], p["accuracy"],
            p["nnz_w"], p["updt_ratio"]), file=self.out, flush=True)


def run_async_sgd(lm, comm, device, flags, printer=None) -> dict:
    """Train ``lm.async_sgd`` on the GPU trainer from the conf's training files; returns
    a summary (examples, steps, seconds, last progress, model files)."""
    import torch

    from ..data.feeder import DeviceFeeder
    from ..models.sparse_lr import SparseLRTrainer
    from ..utils.config import lm_to_sparse_lr

    G, rank = comm.world, comm.rank
    sgd = lm.async_sgd
    N = int(flags.num_features)
    over = dict(num_features=N, max_nnz_per_example=flags.max_nnz_per_example,
                seed=flags.seed + rank)
    if flags.table_capacity:
        over["table_capacity"] = flags.table_capacity
    if G > 1 and sgd.max_delay <= 0:
        over["consistency"] = "asp"  # the reference's unbounded pipelining (async_sgd.h:219-238)
    cfg = lm_to_sparse_lr(lm, **over)
    tr = SparseLRTrainer(cfg, comm, device)
    td = lm.training_data
    cache_dir, tmp_cache = _cache_dir(flags, sgd.num_data_pass, rank)
    feeder = DeviceFeeder(rank_files(td, G, rank), td.text, cfg.minibatch, tr.max_nnz, device,
                          num_features=N, passes=sgd.num_data_pass, shuffle=sgd.num_data_pass > 1,
                          seed=flags.seed + rank, data_buf_mb=sgd.data_buf,
                          nthreads=flags.num_threads,
                          ignore_slot=True,
                          hadoop_home=td.hdfs.home if td.has("hdfs") else "",
                          max_lines_per_file=td.max_num_lines_per_file,
                          cache_dir=cache_dir, io_threads=getattr(flags, "io_threads", 16))
    interval = max(1, int(sgd.report_interval))
    printer = printer or (ProgressPrinter() if rank == 0 and not flags.quiet else None)
    t0 = last = time.time()
    steps = idle = 0
    t_feed = t_step = 0.0  # host seconds waiting for minibatches / issuing steps
    last_p = None
    agreed = []  # per pass: the agreed step count, or None (agreement every step)
    for ps in range(feeder.passes):
        # a pass that streams the binary cache knows its minibatch count: the ranks agree
        # on the pass's step count (and its report steps) ONCE; a text pass agrees every
        # step over the host channel
        planned = feeder.planned_pass(ps)
        total = None
        if G > 1:
            counts = comm.host_gather_obj(planned)
            if all(c is not None for c in counts):
                total = max(counts)
        elif planned is not None:
            total = planned
        agreed.append(total)
        every = getattr(flags, "report_steps", 0) or (max(1, -(-total // 10)) if total else 0)
        it = feeder.iter_pass(ps)
        t = 0
        while True:
            if total is not None:
                if t >= total:
                    break
                tf = time.perf_counter()
                b = next(it, None)
                t_feed += time.perf_counter() - tf
                report = (t + 1) % every == 0
            else:
                tf = time.perf_counter()
                b = next(it, None)
                t_feed += time.perf_counter() - tf
                report = time.time() - last >= interval
                if G > 1:  # (host channel: every rank steps, reports and stops together)
                    st = comm.host_gather_obj((b is not None, report))
                    if not any(s[0] for s in st):
                        break
                    report = st[0][1]
                elif b is None:
                    break
            t += 1
            if b is None:
                tr.idle_step()  # out of files: keep serving this shard and flushing pushes
                idle += 1
            else:
                ts = time.perf_counter()
                if b.vals is None and b.width:  # one width, binary: the fused fixed-width path
                    tr.step(b.keys, b.labels, width=b.width)
                else:
                    tr.step(b.keys, b.labels, width=b.width or None, row_ptr=b.row_ptr,
                            vals=b.vals)
                feeder.release(b)
                t_step += time.perf_counter() - ts
                steps += 1
            if report:
                last = time.time()
                last_p = tr.progress()
                if printer is not None:
                    printer(last_p)
        for _ in it:  # (a rank's pass ended early on the agreed count: none left)
            raise RuntimeError("feeder yielded more minibatches than planned")
    p = tr.progress()
    if printer is not None and p["examples"]:
        printer(p)
    tr.check_ok()
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    dt = time.time() - t0
    out = {"examples": feeder.num_examples, "steps": steps, "idle_steps": idle, "seconds": dt,
           "progress": p if p["examples"] else last_p, "trainer": tr, "h2d_bytes": feeder.bytes_h2d,
           "text_passes": feeder.text_passes, "cached_passes": feeder.cached_passes,
           "agreed_steps": agreed, "host_feed_wait_s": t_feed, "host_step_issue_s": t_step}
    if tmp_cache:
        import shutil

        shutil.rmtree(tmp_cache, ignore_errors=True)
    mo = lm.model_output
    if lm.has("model_output") and mo.has("file") and mo.format == "TEXT":
        d = os.path.dirname(mo.file[0])
        if d:
            os.makedirs(d, exist_ok=True)
        out["model"] = tr.save_model(mo.file[0])
    return out


def _cache_dir(flags, passes: int, rank: int):
    """(cache dir or None, temporary dir to delete at the end or None)."""
    d = getattr(flags, "data_cache", "") or os.environ.get("PSAMD_DATA_CACHE", "")
    if d == "off":
        return None, None
    if d:
        return d, None
    if passes > 1:  # later passes stream the binary cache of the first
        import tempfile

        t = tempfile.mkdtemp(prefix=f"psamd_cache_r{rank}_")
        return t, t
    return None, None


def run_darlin(lm, comm, device, flags, printer=None) -> dict:
    from ..data.slot_reader import SlotReader
    from ..models.darlin import DarlinConfig, DarlinTrainer, show_progress

    G, rank = comm.world, comm.rank
    td = lm.training_data
    cache = lm.darlin.local_cache if lm.darlin.has("local_cache") else None
    reader = SlotReader(rank_files(td, G, rank), td.text,
                        cache_prefix=(cache.file[0] if cache is not None and cache.has("file")
                                      else None), ignore_slot=td.ignore_feature_group,
                        hadoop_home=td.hdfs.home if td.has("hdfs") else "",
                        nthreads=flags.num_threads)
    data = reader.read()
    cfg = DarlinConfig.from_lm(lm, seed=flags.seed)
    t0 = time.time()
    tr = DarlinTrainer(data, cfg, comm, device)
    pr = printer if printer is not None else (show_progress if rank == 0 and not flags.quiet
                                              else None)
    prog = tr.train(printer=pr)
    out = {"examples": tr.num_ex, "passes": len(prog), "seconds": time.time() - t0,
           "progress": prog[-1] if prog else None, "trainer": tr}
    mo = lm.model_output
    if lm.has("model_output") and mo.has("file") and mo.format == "TEXT":
        d = os.path.dirname(mo.file[0])
        if d:
            os.makedirs(d, exist_ok=True)
        out["model"] = tr.save_model(mo.file[0])
    return out


def main(argv=None) -> int:
    flags = _flags(sys.argv[1:] if argv is None else argv)
    import torch

    from ..parallel.comm import init_from_env
    from ..utils.config import load_app_config

    conf = load_app_config(flags.app_file, flags.app_conf)
    if not conf.has("linear_method"):
        raise ValueError("the GPU app runs linear_method configs (async_sgd / darlin)")
    lm = conf.linear_method
    dev_type = flags.device if flags.device != "auto" else (
        "cuda" if torch.cuda.is_available() else "cpu")
    comm, device = init_from_env(dev_type)
    if lm.has("async_sgd"):
        res = run_async_sgd(lm, comm, device, flags)
    elif lm.has("darlin"):
        res = run_darlin(lm, comm, device, flags)
    else:
        raise ValueError("linear_method needs async_sgd or darlin")
    if comm.rank == 0 and not flags.quiet:
        rate = res["examples"] / max(res["seconds"], 1e-9)
        print(f"[psamd] {comm.world} rank(s), rank 0: {res['examples']} examples in "
              f"{res['seconds']:.2f} s ({rate:.3g} examples/s)"
              + (f", model {res['model']}" if "model" in res else ""), file=sys.stderr)
    import torch.distributed as dist

    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
