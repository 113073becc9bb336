"""Asynchronous SGD for sparse linear models over the runtime (plumbing mode).

Reference src/app/linear_method/async_sgd.h:
* scheduler (:18-28): ``update_model(training_data)`` then ``save_model``.
* worker (:180-301): streams minibatches; per minibatch ``pull(keys)`` on channel
  = minibatch id with ``fin_handle = compute_gradient(id)`` and does NOT wait
  between minibatches (ASP pipelining); ``compute_gradient`` evaluates Xw,
  objective / AUC / accuracy (reported to the scheduler), grad = X^T(-y tau),
  pushes it with KEY_CACHING(clear_cache_if_done) and optional FIXING_FLOAT.
* server (:128-178): KVStore whose entries are FTRL / SGD / AdaGrad; reports
  nnz, sum w^2, sum dw^2 per push; SAVE_MODEL writes ``<file>_<NodeID>``.

Differences: SGD and AdaGrad entries are implemented (the reference leaves them
as TODO stubs and picks them with an inverted ``ada_grad`` test), and
``max_delay`` bounds the number of in-flight minibatches (declared but unused
in the reference) — 0 keeps the reference's unbounded ASP pipelining.
"""
from __future__ import annotations

import threading

import numpy as np
import torch

from ...learner.sgd import ISGDCompNode, ISGDScheduler, MinibatchReader
from ...ops.kv_table import UpdateRule
from ...ops.linear import exact_auc, loss_id, loss_terms_torch
from ...parameter.kv import KVStore, KVVector
from ...system.message import SERVER_GROUP, Message, new_task
from ...utils.config import DataConfig


def update_rule_from(lm) -> UpdateRule:
    sgd = lm.async_sgd
    lam = list(lm.penalty.__getattr__("lambda")) or [0.0]
    l1, l2 = (lam[0], lam[1] if len(lam) > 1 else 0.0) if lm.penalty.type == "L1" else (0.0, lam[0])
    if sgd.algo == "FTRL":
        algo = "ftrl"
    elif sgd.algo == "ADAGRAD" or sgd.ada_grad:
        algo = "adagrad"
    else:
        algo = "sgd"
    return UpdateRule(algo, lm.learning_rate.type.lower(), lm.learning_rate.alpha,
                      lm.learning_rate.beta, l1, l2)


class AsyncSGDScheduler(ISGDScheduler):
    def __init__(self, lm, name="app"):
        super().__init__(name, lm)
        self.lm = lm

    def run(self):
        self.update_model(self.lm.training_data, self.lm.async_sgd.report_interval)
        self.save_model()


class AsyncSGDServer(ISGDCompNode):
    def __init__(self, lm, name="app"):
        super().__init__(name, lm)
        self.lm = lm
        cap = 1 << 22
        self.model = KVStore(name + "_model", update_rule_from(lm), capacity=cap, parent=name,
                             reporter=self._report)

    def _report(self, nnz, wsum, dsum):
        self.reporter.report({"nnz": int(nnz), "weight_sum": wsum, "delta_sum": dsum})

    def process(self, msg):
        if msg.task.get("sgd", {}).get("cmd") == "SAVE_MODEL":
            self.save_model()

    def save_model(self):
        out = self.lm.model_output
        if out.has("file") and out.format == "TEXT":
            path = f"{out.file[0]}_{self.my_node_id()}"
            self.model.write_to_file(path)
            return path


class AsyncSGDWorker(ISGDCompNode):
    def __init__(self, lm, name="app"):
        super().__init__(name, lm)
        self.lm = lm
        self.model = KVVector(name + "_model", parent=name)
        self.loss = loss_id(lm.loss.type.lower())
        self.data = {}
        self.mu = threading.Lock()
        self.processed = 0
        self.cv = threading.Condition()

    def process(self, msg):
        sgd = msg.task.get("sgd", {})
        if sgd.get("cmd") == "UPDATE_MODEL":
            self.update_model(DataConfig.parse(sgd["data"]))

    def update_model(self, data_conf):
        conf = self.lm.async_sgd
        reader = MinibatchReader(list(data_conf.file), data_conf.text, conf.minibatch,
                                 conf.data_buf, ignore_slot=True, passes=conf.num_data_pass,
                                 seed=self.my_rank())
        reader.set_filter(conf.countmin_n, conf.countmin_k, conf.tail_feature_freq)
        max_delay = conf.max_delay
        mid = 0
        for batch, keys, local_col in reader:
            with self.mu:
                self.data[mid] = (batch, local_col)
            if max_delay > 0:  # bounded staleness: at most max_delay minibatches in flight
                with self.cv:
                    self.cv.wait_for(lambda: self.processed >= mid - max_delay)
            m = Message(task=new_task(key_channel=mid))
            m.recver = SERVER_GROUP
            m.set_key(keys)
            m.fin_handle = (lambda i=mid: self.compute_gradient(i))
            self.model.set_key(mid, keys)
            self.model.pull(m)
            mid += 1
        with self.cv:
            self.cv.wait_for(lambda: self.processed >= mid)

    def compute_gradient(self, mid: int):
        with self.mu:
            batch, local_col = self.data.pop(mid)
        w = torch.from_numpy(self.model.value(mid).astype(np.float32))
        B = batch.rows
        rows = torch.repeat_interleave(torch.arange(B), torch.from_numpy(np.diff(batch.row_ptr)))
        col = torch.from_numpy(local_col.astype(np.int64))
        valid = col >= 0
        x = torch.from_numpy(batch.vals) if batch.vals is not None else torch.ones(col.numel())
        contrib = torch.where(valid, w[col.clamp(min=0)] if w.numel() else torch.zeros(col.numel()),
                              torch.zeros(())) * x
        xw = torch.zeros(B).index_add_(0, rows, contrib)
        y = torch.from_numpy(batch.labels)
        lo, coef, _ = loss_terms_torch(xw, y, self.loss)
        self.reporter.report({"objective": [float(lo.sum())], "auc": [exact_auc(xw, y)],
                              "accuracy": [float(((torch.where(y > 0, 1.0, -1.0) * xw) > 0).float().mean())],
                              "num_examples_processed": B})
        grad = torch.zeros(w.numel()).index_add_(0, col[valid], (coef[rows] * x)[valid])
        push = Message(task=new_task(key_channel=mid))
        push.recver = SERVER_GROUP
        push.set_key(self.model.key(mid))
        push.add_value(grad.numpy().astype(np.float32))
        push.add_filter("KEY_CACHING", clear_cache_if_done=True)
        nb = self.lm.async_sgd.fixing_float_by_nbytes
        if nb:
            push.add_filter("FIXING_FLOAT", fixed_point=[{"num_bytes": nb}])
        self.model.push(push)
        self.model.clear(mid)
        with self.cv:
            self.processed += 1
            self.cv.notify_all()
