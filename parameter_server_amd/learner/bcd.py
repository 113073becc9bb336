"""Block-coordinate-descent learner framework over the runtime (plumbing mode).

Reference src/learner/bcd.h:
* ``BCDScheduler`` (:26-191): ``load_training_data`` sends ``LOAD_DATA`` to each
  worker, merges the returned ExampleInfo, then ``PREPROCESS_DATA`` with the
  feature groups to all compute nodes; ``divide_feature_blocks`` splits each
  group into ``ceil(nnz_per_row * feature_block_ratio)`` key ranges and builds the
  prior-group block order; progress merge and the objective / time printers.
* ``BCDServer`` (:193-274): preprocess = per group wait for the workers' tail
  filter counts, then for their kept keys and initialise ``w``; ``SAVE_MODEL``
  writes ``key\\tw`` (skipping 0 and NaN).
* ``BCDWorker`` (:276-518): ``LOAD_DATA`` via SlotReader; preprocess per group =
  count unique keys -> push counts (tail-filter insert, time t) -> pull filtered
  keys (t+2, waits t+1) -> remap to local columns in CSC order -> push kept keys
  -> pull initial weights -> init the margins.

Task times of the model customer are ``app_time * TIME_RATIO`` (bcd.h:21, 201).
Payloads of protocol replies (LoadDataReturn, BCDProgress) are msgpack dicts in
``task["msg"]`` (the reference serialises protos there).
"""
from __future__ import annotations

import threading

import msgpack
import numpy as np
import torch

from ..data import divide_files, search_files
from ..data.slot_reader import SlotReader, merge_slot_info
from ..models.darlin import divide_feature_blocks
from ..parameter.kv import KVBufferedVector
from ..system.customer import App
from ..system.message import (COMP_GROUP, REPLY, SERVER_GROUP, WORKER_GROUP, Message, new_task)
from ..utils.checkpoint import write_text_model
from ..utils.config import DataConfig

TIME_RATIO = 10


def _pack(d: dict) -> bytes:
    return msgpack.packb(d, use_bin_type=True)


def _unpack(b) -> dict:
    return msgpack.unpackb(b, raw=False, strict_map_key=False)


def bcd_task(cmd: str, **kw) -> dict:
    return {"cmd": cmd, **kw}


class BCDCommon:
    def __init__(self, lm):
        self.lm = lm
        self.bcd_conf = lm.darlin
        self.fea_grp: list[int] = []


class BCDScheduler(App, BCDCommon):
    def __init__(self, lm, name="app"):
        App.__init__(self, name, lm)
        BCDCommon.__init__(self, lm)
        self.g_info = {"num_ex": 0, "slots": {}}
        self.g_progress: dict[int, dict] = {}
        self.fea_blk: list[tuple[int, int, int]] = []
        self.blk_order: list[int] = []
        self.prior_blk_order: list[int] = []
        self.busy: list[float] = []
        import time as _t

        self._t0 = _t.time()

    def load_training_data(self, data_conf):
        import sys
        import time as _t

        t0 = _t.time()
        files = search_files(data_conf)
        nw = self.po.yp.num_workers
        parts = divide_files(files, nw, data_conf.max_num_files_per_worker)
        msgs = []
        for p in parts:
            d = data_conf.copy()
            d._set["file"] = p
            m = Message(task=new_task(bcd=bcd_task("LOAD_DATA", data=d.to_text())))
            msgs.append(m)
        infos, hits = [], [0]

        def on_reply():
            r = _unpack(self.executor.last_reply().task["msg"])
            infos.append(r["example_info"])
            hits[0] += int(r.get("hit_cache", 0))

        for m in msgs:
            m.recv_handle = on_reply
        self.port(WORKER_GROUP).submit_and_wait(msgs)
        if hits[0] > 0 and hits[0] != len(msgs):
            raise RuntimeError("some workers hit their local cache and some did not: clear the caches")
        self.g_info = merge_slot_info(infos)
        print(f"Loaded {self.g_info['num_ex']} examples in {_t.time() - t0:.3f} sec",
              file=sys.stderr)
        self.fea_grp = [g for g in sorted(self.g_info["slots"]) if g != 0]
        t1 = _t.time()
        pre = Message(task=new_task(bcd=bcd_task("PREPROCESS_DATA", fea_grp=self.fea_grp,
                                                 hit_cache=hits[0] > 0)))
        self.port(COMP_GROUP).submit_and_wait(pre)
        print(f"Preprocessing is finished in {_t.time() - t1:.3f} sec", file=sys.stderr)
        if self.bcd_conf.tail_feature_freq:
            print(f"Features with frequency <= {self.bcd_conf.tail_feature_freq} are filtered",
                  file=sys.stderr)

    def divide_feature_blocks(self, rng):
        import sys

        c = self.bcd_conf
        self.fea_blk = divide_feature_blocks(self.g_info, c.feature_block_ratio)
        print(f"Features are partitioned into {len(self.fea_blk)} blocks", file=sys.stderr)
        self.blk_order = list(range(len(self.fea_blk)))
        hit = []
        for g in c.prior_fea_group:
            tmp = [k for k, b in enumerate(self.fea_blk) if b[0] == g]
            if not tmp:
                continue
            hit.append(str(g))
            for _ in range(c.num_iter_for_prior_fea_group):
                if c.random_feature_block_order:
                    rng.shuffle(tmp)
                self.prior_blk_order.extend(tmp)
        if hit:
            print("Prior feature groups: " + ", ".join(hit), file=sys.stderr)

    def save_model(self, data_conf):
        m = Message(task=new_task(bcd=bcd_task("SAVE_MODEL", data=data_conf.to_text())))
        self.port(SERVER_GROUP).submit_and_wait(m)

    def merge_progress(self, it: int):
        import time as _t

        r = _unpack(self.executor.last_reply().task["msg"])
        p = self.g_progress.setdefault(it, {"objective": 0.0, "nnz_w": 0, "violation": 0.0,
                                            "nnz_active_set": 0, "busy_time": []})
        p["objective"] += r.get("objective", 0.0)
        p["nnz_w"] += r.get("nnz_w", 0)
        if r.get("busy_time"):
            p["busy_time"].append(r["busy_time"][0])
        p["total_time"] = _t.time() - self._t0
        prev = self.g_progress.get(it - 1)
        p["relative_obj"] = 1.0 if it == 0 or not p["objective"] else \
            prev["objective"] / p["objective"] - 1
        p["violation"] = max(p["violation"], r.get("violation", 0.0))
        p["nnz_active_set"] += r.get("nnz_active_set", 0)

    # printers (bcd.h:146-178, darlin.h:136-156)
    def show_objective(self, it):
        if it == -3:
            return "     |        training        |  sparsity "
        if it == -2:
            return "iter |  objective    relative |     |w|_0 "
        if it == -1:
            return " ----+------------------------+-----------"
        p = self.g_progress[it]
        return f"{it:4d} | {p['objective']:.5e}  {p['relative_obj']:.3e} |{p['nnz_w']:10d} "

    def show_time(self, it):
        if it == -3:
            return "|    time (sec.)\n"
        if it == -2:
            return "|(app:min max) total\n"
        if it == -1:
            return "+-----------------\n"
        p = self.g_progress[it]
        ttl = p["total_time"] - (self.g_progress[it - 1]["total_time"] if it > 0 else 0)
        bt = p["busy_time"] or [0.0]
        return f"|{min(bt):6.1f}{max(bt):6.1f}{ttl:6.1f}\n"


class BCDServer(App, BCDCommon):
    def __init__(self, lm, name="app"):
        App.__init__(self, name, lm)
        BCDCommon.__init__(self, lm)
        self.model = KVBufferedVector(name + "_model", dtype=np.float64, parent=name)

    def process(self, msg: Message):
        call = msg.task.get("bcd")
        if not call:
            return
        t = msg.task["time"] * TIME_RATIO
        cmd = call["cmd"]
        if cmd == "PREPROCESS_DATA":
            self.preprocess_data(t, call)
        elif cmd == "UPDATE_MODEL":
            self.update_model(t, call)
        elif cmd in ("SAVE_MODEL", "EVALUATE_PROGRESS"):
            if cmd == "SAVE_MODEL":
                self.save_model(DataConfig.parse(call["data"]))
            prog = self.evaluate()
            self.po.reply(msg, Message(task=new_task(type=REPLY, msg=_pack(prog))))

    def init_value(self, n: int) -> np.ndarray:
        iw = self.bcd_conf.init_w if self.bcd_conf.has("init_w") else None
        if iw is None or iw.type == "ZERO":
            return np.zeros(n, np.float64)
        if iw.type == "CONSTANT":
            return np.full(n, iw.constant, np.float64)
        if iw.type == "GAUSSIAN":
            return np.random.default_rng(0).normal(iw.mean, iw.std, n)
        raise ValueError(f"init_w type {iw.type} is not supported")

    def preprocess_data(self, t: int, call: dict):
        self.fea_grp = list(call["fea_grp"])
        hit = call.get("hit_cache", False)
        for _ in self.fea_grp:  # tail filter: wait for all workers' counts
            if not hit:
                self.model.wait_in_msg(WORKER_GROUP, t)
                self.model.finish(WORKER_GROUP, t + 1)
            t += TIME_RATIO
        for g in self.fea_grp:  # kept keys arrived: initialise the weights
            self.model.wait_in_msg(WORKER_GROUP, t)
            self.model.clear_tail_filter(g)
            self.model.set_val(g, self.init_value(self.model.key(g).size))
            self.model.finish(WORKER_GROUP, t + 1)
            t += TIME_RATIO

    def update_model(self, t: int, call: dict):
        raise NotImplementedError

    def evaluate(self) -> dict:
        raise NotImplementedError

    def save_model(self, out):
        if out.format != "TEXT" or not out.file:
            return None
        path = f"{out.file[0]}_{self.my_node_id()}"
        keys, vals = [], []
        for g in self.fea_grp:
            k, v = self.model.key(g), self.model.value(g)
            m = (v != 0) & ~np.isnan(v)
            keys.append(k[m])
            vals.append(v[m])
        write_text_model(path, np.concatenate(keys) if keys else np.zeros(0, np.uint64),
                         np.concatenate(vals) if vals else np.zeros(0))
        import sys

        print(f"{self.my_node_id()} written the model to {path}", file=sys.stderr)
        return path


class CSC:
    """Column-major local training matrix of one feature group."""

    def __init__(self, col, row, val, ncols):
        order = np.argsort(col, kind="stable")
        self.col = torch.from_numpy(col[order].astype(np.int32))
        self.row = torch.from_numpy(row[order].astype(np.int32))
        self.val = None if val is None else torch.from_numpy(val[order].astype(np.float32))
        self.colptr = np.zeros(ncols + 1, np.int64)
        np.cumsum(np.bincount(col, minlength=ncols), out=self.colptr[1:])
        self.ncols = ncols


class BCDWorker(App, BCDCommon):
    def __init__(self, lm, name="app"):
        App.__init__(self, name, lm)
        BCDCommon.__init__(self, lm)
        self.model = KVBufferedVector(name + "_model", dtype=np.float64, parent=name)
        self.data = None
        self.X: dict[int, CSC] = {}
        self.y = None
        self.ym = None  # margins y * Xw (the reference's dual_ = exp(ym))
        self.mu = threading.Lock()

    def process(self, msg: Message):
        call = msg.task.get("bcd")
        if not call:
            return
        t = msg.task["time"] * TIME_RATIO
        cmd = call["cmd"]
        if cmd == "LOAD_DATA":
            ret = self.load_data(DataConfig.parse(call["data"]))
            self.po.reply(msg, Message(task=new_task(type=REPLY, msg=_pack(ret))))
        elif cmd == "PREPROCESS_DATA":
            self.preprocess_data(t, call)
        elif cmd == "UPDATE_MODEL":
            self.compute_gradient(t, call, msg)
            msg.finished = False  # finished by the weight pull's fin_handle
        elif cmd == "EVALUATE_PROGRESS":
            prog = self.evaluate()
            self.po.reply(msg, Message(task=new_task(type=REPLY, msg=_pack(prog))))

    def load_data(self, data_conf) -> dict:
        cache = self.bcd_conf.local_cache if self.bcd_conf.has("local_cache") else None
        reader = SlotReader.from_config(data_conf, cache)
        self.data = reader.read()
        info = self.data.info()
        return {"example_info": {"num_ex": info["num_ex"], "slots": info["slots"]},
                "hit_cache": 0}

    def preprocess_data(self, t: int, call: dict):
        self.fea_grp = list(call["fea_grp"])
        hit = call.get("hit_cache", False)
        c = self.bcd_conf
        sd = self.data
        rows = sd.rows
        self.y = torch.from_numpy(np.where(sd.labels > 0, 1.0, -1.0).astype(np.float32))
        # fin_handles run after the outgoing trackers finish: wait on explicit events
        localized = {g: threading.Event() for g in self.fea_grp}
        initialised = {g: threading.Event() for g in self.fea_grp}
        for g in self.fea_grp:
            if hit:
                t += TIME_RATIO
                continue
            off, keys, vals = sd.groups.get(g, (np.zeros(rows + 1, np.int64),
                                                np.zeros(0, np.uint64), None))
            uniq, cnt = np.unique(keys, return_counts=True)
            count = Message(task=new_task(key_channel=g, time=t,
                                          shared_para={"tail_filter": {
                                              "insert_count": True, "countmin_k": c.countmin_k,
                                              "countmin_n": int(uniq.size * c.countmin_n_ratio)}}))
            count.recver = SERVER_GROUP
            count.set_key(uniq)
            count.add_value(np.minimum(cnt, 255).astype(np.uint8))
            count.add_filter("KEY_CACHING")
            self.model.push(count)
            filt = Message(task=new_task(key_channel=g, time=t + 2, wait_time=[t + 1],
                                         shared_para={"tail_filter": {
                                             "query_key": int(c.tail_feature_freq)}}))
            filt.recver = SERVER_GROUP
            filt.set_key(uniq)
            filt.add_filter("KEY_CACHING")
            filt.fin_handle = (lambda g=g, off=off, keys=keys, vals=vals:
                               (self._localize(g, off, keys, vals), localized[g].set()))
            self.model.pull(filt)
            t += TIME_RATIO
        for g in self.fea_grp:
            if not hit:
                localized[g].wait()
            keys = self.model.key(g)
            push = Message(task=new_task(key_channel=g, time=t))
            push.recver = SERVER_GROUP
            push.set_key(keys)
            push.add_filter("KEY_CACHING")
            self.model.push(push)
            pv = Message(task=new_task(key_channel=g, time=t + 2, wait_time=[t + 1]))
            pv.recver = SERVER_GROUP
            pv.set_key(keys)
            pv.add_filter("KEY_CACHING", clear_cache_if_done=True)
            pv.fin_handle = (lambda g=g, tt=t + 2: (self._init_weights(g, tt),
                                                    initialised[g].set()))
            self.model.pull(pv)
            t += TIME_RATIO
        for g in self.fea_grp:
            initialised[g].wait()
        self.data = None

    def _localize(self, g, off, keys, vals):
        """remapIndex + toColMajor (bcd.h:399-413): local column = rank in the kept keys."""
        kept = self.model.key(g)
        rows = off.size - 1
        pos = np.searchsorted(kept, keys)
        hit = pos < kept.size
        hit[hit] = kept[pos[hit]] == keys[hit]
        r = np.repeat(np.arange(rows, dtype=np.int64), np.diff(off))
        with self.mu:
            self.X[g] = CSC(pos[hit], r[hit], None if vals is None else vals[hit], kept.size)

    def _init_weights(self, g, t):
        n = self.model.key(g).size
        X = self.X.get(g) or CSC(np.zeros(0, np.int64), np.zeros(0, np.int64), None, n)
        self.X[g] = X
        w = np.zeros(n, np.float64)
        if n:
            _, bufs = self.model.received(t)
            w = bufs[0].astype(np.float64)
        self.model.set_val(g, w)
        with self.mu:
            if self.ym is None:
                self.ym = torch.zeros(self.y.numel(), dtype=torch.float64)
            if n and np.any(w != 0):
                from ..ops import bcd

                bcd.dual(X.col, X.row, X.val, 0, int(X.colptr[-1]), 0, n, torch.from_numpy(w),
                         self.y, self.ym)

    def compute_gradient(self, t: int, call: dict, msg: Message):
        raise NotImplementedError

    def evaluate(self) -> dict:
        raise NotImplementedError
