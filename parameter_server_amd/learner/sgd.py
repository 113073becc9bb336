"""Asynchronous-SGD learner framework (runtime / plumbing mode).

Reference src/learner/sgd.h:
* ``ISGDScheduler`` (:14-91): ``update_model`` installs the progress merger and
  printer, partitions the training files over workers and sends one
  ``SGDCall{UPDATE_MODEL}`` per worker; ``save_model`` sends ``SAVE_MODEL`` to all
  servers; ``show_progress`` prints ``sec examples loss auc accuracy |w|_0 updt ratio``.
* ``ISGDCompNode`` (:93-101): app base with a progress reporter to the scheduler.
* ``MinibatchReader`` (:103-157): producer thread + localisation + worker-local
  CountMin tail filter + remap to local column ids.
"""
from __future__ import annotations

import math
import sys

import numpy as np
import torch

from ..data import StreamReader, divide_files, search_files
from ..ops.countmin import CountMinSketch
from ..ops.localize import localize_torch
from ..system.customer import App
from ..system.message import SERVER_GROUP, WORKER_GROUP, Message, new_task
from ..system.monitor import MonitorMaster, MonitorSlaver


class ISGDScheduler(App):
    def __init__(self, name="app", conf=None):
        super().__init__(name, conf)
        self.monitor = MonitorMaster(name)
        self.num_ex_processed = 0
        self.show_head = True
        self.lines = []

    def save_model(self):
        m = Message(task=new_task(sgd={"cmd": "SAVE_MODEL"}))
        self.port(SERVER_GROUP).submit_and_wait(m)

    def update_model(self, data_conf, report_interval=1.0):
        self.monitor.set_merger(self.merge_progress)
        self.monitor.set_printer(report_interval, self.show_progress)
        files = search_files(data_conf)
        nw = self.po.yp.num_workers
        parts = divide_files(files, nw, data_conf.max_num_files_per_worker)
        tasks = []
        for p in parts:
            d = data_conf.copy()
            d._set["file"] = p
            tasks.append(new_task(sgd={"cmd": "UPDATE_MODEL", "data": d.to_text()}))
        msgs = [Message(task=t) for t in tasks]
        self.port(WORKER_GROUP).submit_and_wait(msgs)
        self.monitor.flush()

    def merge_progress(self, src: dict, dst: dict) -> dict:
        """Latest report replaces the old one, examples accumulate (sgd.h:82-87); the
        per-minibatch objective / auc / accuracy lists are appended (the reference's
        "TODO also append objv"), so the printed loss is over every example counted."""
        out = dict(src)
        out["num_examples_processed"] = src.get("num_examples_processed", 0) + \
            dst.get("num_examples_processed", 0)
        for k in ("objective", "auc", "accuracy"):
            if k in src or k in dst:
                out[k] = list(dst.get(k, [])) + list(src.get(k, []))
        return out

    def show_progress(self, t: float, progress: dict):
        num_ex = nnz_w = 0
        objv, auc, acc = [], [], []
        weight_sum, delta_sum = 0.0, 1e-20
        for p in progress.values():
            num_ex += p.get("num_examples_processed", 0)
            nnz_w += p.get("nnz", 0)
            objv += p.get("objective", [])
            auc += p.get("auc", [])
            acc += p.get("accuracy", [])
            weight_sum += p.get("weight_sum", 0.0)
            delta_sum += p.get("delta_sum", 0.0)
        progress.clear()
        self.num_ex_processed += num_ex
        if self.show_head:
            print(" sec  examples    loss      auc   accuracy   |w|_0  updt ratio", file=sys.stderr)
            self.show_head = False
        line = "%4d  %.2e  %.3e  %.4f  %.4f  %.2e  %.2e" % (
            int(t), float(self.num_ex_processed), sum(objv) / max(num_ex, 1),
            float(np.mean(auc)) if auc else float("nan"), float(np.mean(acc)) if acc else float("nan"),
            float(nnz_w), math.sqrt(delta_sum) / math.sqrt(max(weight_sum, 1e-20)))
        self.lines.append(line)
        print(line, file=sys.stderr)


class ISGDCompNode(App):
    def __init__(self, name="app", conf=None):
        super().__init__(name, conf)
        self.reporter = MonitorSlaver(self.scheduler_id(), name)


class MinibatchReader:
    """Stream minibatches, localise keys, apply the worker-local tail filter."""

    def __init__(self, files, fmt, minibatch, data_buf_mb=1000, ignore_slot=True, passes=1,
                 shuffle=True, seed=0):
        self.reader = StreamReader(files, fmt, minibatch, ignore_slot=ignore_slot,
                                   data_buf_mb=data_buf_mb, passes=passes, shuffle=shuffle,
                                   seed=seed)
        self.filter = None
        self.freq = 0

    def set_filter(self, n, k, freq):
        if freq > 0:
            self.filter = CountMinSketch(int(n), k)
            self.freq = freq

    def __iter__(self):
        for b in self.reader:
            # the wire carries raw keys sorted (key-ordered slicing over servers);
            # countUniqIndex + remapIndex (localizer.h:69-191) as one np.unique
            u, inv = np.unique(b.keys, return_inverse=True)
            uniq_raw = torch.from_numpy(u.view(np.int64).copy())
            counts = np.bincount(inv, minlength=uniq_raw.numel())
            keep = np.ones(uniq_raw.numel(), bool)
            if self.filter is not None:
                self.filter.insert(uniq_raw, torch.from_numpy(np.minimum(counts, 255).astype(np.uint8)))
                k, _ = self.filter.query(uniq_raw, self.freq)
                keep = k.numpy().astype(bool)
            remap = np.full(uniq_raw.numel(), -1, np.int64)
            remap[keep] = np.arange(int(keep.sum()))
            local_col = remap[inv].astype(np.int32)
            yield b, uniq_raw.numpy().view(np.uint64)[keep], local_col
