"""Darlin (L1 logistic regression by block coordinate descent) over the runtime.

Reference src/app/linear_method/darlin.h:
* ``DarlinScheduler`` (:26-158): per pass, shuffled block order (prior blocks
  first in pass 0); each block is ``Task{bcd UPDATE_MODEL, key = block range,
  fea_grp}`` at time t+1 with ``wait_time = t - tau`` to all compute nodes
  (prior blocks of pass 0 wait for t); then ``EVALUATE_PROGRESS``; the KKT
  threshold becomes ``violation / num_ex * ratio``; stop when the relative
  objective <= epsilon twice with a KKT reset in between; finally save.
* ``DarlinWorker`` (:275-514): block gradient (G, U) pushed at t, weights pulled
  at t+2 (waits t+1), dual update in the pull's fin_handle, which then finishes
  the scheduler's task and replies.
* ``DarlinServer`` (:160-273): waits for all workers' (G, U) at t, coordinate
  update with trust region and KKT filter (filtered weights marked NaN), then
  finishes t+1 so the pulls proceed; ``evaluate`` reports l1 * |w|_1, nnz,
  violation and the active-set size.

The per-block math is ``ops.bcd`` (fp64 PyTorch on the host here; the same
functions run the HIP kernels for the GPU trainer ``models.darlin``). The worker
keeps margins ``ym = y * Xw`` instead of ``dual = exp(ym)``. Difference: a KKT
reset re-activates filtered weights from 0 (the reference's stay NaN).
"""
from __future__ import annotations

import random
import sys
import time

import numpy as np
import torch

from ...learner.bcd import (TIME_RATIO, BCDScheduler, BCDServer, BCDWorker,
                            bcd_task)
from ...ops import bcd
from ...system.message import (COMP_GROUP, INVALID_TIME, SERVER_GROUP, WORKER_GROUP, Message,
                               new_task)


def _new_delta(delta_max, dw):
    return np.minimum(delta_max, 2 * np.abs(dw) + .1)


class DarlinScheduler(BCDScheduler):
    def run(self):
        lm = self.lm
        if lm.loss.type != "LOGIT" or lm.penalty.type != "L1":
            raise ValueError("Darlin trains l1-regularised logistic regression (LOGIT + L1)")
        print("Train l_1 logistic regression by block coordinate descent", file=sys.stderr)
        self.load_training_data(lm.training_data)
        rng = random.Random(0)
        self.divide_feature_blocks(rng)
        d = self.bcd_conf
        tau = d.max_block_delay
        print(f"Maximal allowed delay: {tau}", file=sys.stderr)
        if not d.random_feature_block_order:
            print("Warning: Randomized block order often acclerates the convergence.",
                  file=sys.stderr)
        kkt_thr = 1e20
        reset_kkt = False
        pool = self.port(COMP_GROUP)
        t = max(10000, pool.time + len(self.fea_grp) * TIME_RATIO)
        first = t + 1
        for it in range(d.max_pass_of_data):
            order = list(self.blk_order)
            if d.random_feature_block_order:
                rng.shuffle(order)
            if it == 0:
                order = list(self.prior_blk_order) + order
            for i, k in enumerate(order):
                g, a, b = self.fea_blk[k]
                call = bcd_task("UPDATE_MODEL", key=[a, b], fea_grp=[g])
                if i == 0:
                    call["kkt_filter_threshold"] = kkt_thr
                    if reset_kkt:
                        call["reset_kkt_filter"] = True
                wait = t - tau
                if it == 0 and i < len(self.prior_blk_order):
                    wait = t  # force zero delay for important feature blocks
                if wait < first:
                    wait = INVALID_TIME
                m = Message(task=new_task(bcd=call, time=t + 1, wait_time=[wait]))
                t = pool.submit(m)
            ev = Message(task=new_task(bcd=bcd_task("EVALUATE_PROGRESS"),
                                       wait_time=[t - tau] if t - tau >= first else []))
            ev.recv_handle = (lambda it=it: self.merge_progress(it))
            t = pool.submit_and_wait(ev)
            self.show_progress(it, kkt_thr)
            p = self.g_progress[it]
            kkt_thr = p["violation"] / max(self.g_info["num_ex"], 1) * \
                d.ext("kkt_filter_threshold_ratio")
            rel = p["relative_obj"]
            if 0 < rel <= d.epsilon:
                if reset_kkt:
                    print(f"Stopped: relative objective <= {d.epsilon}", file=sys.stderr)
                    break
                reset_kkt = True
            else:
                reset_kkt = False
            if it == d.max_pass_of_data - 1:
                print(f"Reached maximal {d.max_pass_of_data} data passes", file=sys.stderr)
        if lm.has("model_output"):
            self.save_model(lm.model_output)

    def show_kkt(self, it, thr):
        if it == -3:
            return "|      KKT filter     "
        if it == -2:
            return "| threshold  #activet "
        if it == -1:
            return "+---------------------"
        return f"| {thr:.1e} {int(self.g_progress[it]['nnz_active_set']):11d} "

    def show_progress(self, it, thr):
        lines = []
        for i in range(-3 if it == 0 else it, it + 1):
            lines.append(self.show_objective(i) + self.show_kkt(i, thr) + self.show_time(i))
        sys.stderr.write("".join(lines))
        sys.stderr.flush()


class DarlinServer(BCDServer):
    def __init__(self, lm, name="app"):
        super().__init__(lm, name)
        self.active: dict[int, np.ndarray] = {}
        self.delta: dict[int, np.ndarray] = {}
        self.kkt_thr = 1e20
        self.violation = 0.0

    def preprocess_data(self, t, call):
        super().preprocess_data(t, call)
        for g in self.fea_grp:
            n = self.model.key(g).size
            self.active[g] = np.ones(n, np.uint8)
            self.delta[g] = np.full(n, self.bcd_conf.ext("delta_init_value"), np.float64)

    def update_model(self, t, call):
        if "kkt_filter_threshold" in call:
            self.kkt_thr = float(call["kkt_filter_threshold"])
            self.violation = 0.0
        if call.get("reset_kkt_filter"):
            for g in self.fea_grp:
                self.active[g][:] = 1
                w = self.model.value(g)
                w[np.isnan(w)] = 0.0
        g = call["fea_grp"][0]
        a, b = call["key"]
        lo, hi = self.my_node.key_begin, self.my_node.key_end
        if max(lo, a) >= min(hi, b):
            return  # none of my business
        keys = self.model.key(g)
        c0 = int(np.searchsorted(keys, np.uint64(a)))
        c1 = int(np.searchsorted(keys, np.uint64(b))) if b < (1 << 64) - 1 else keys.size
        self.model.wait_in_msg(WORKER_GROUP, t)
        if c1 > c0:
            (ra, rb), bufs = self.model.received(t)
            if (ra, rb) != (c0, c1) or len(bufs) != 2:
                raise RuntimeError(f"received block [{ra},{rb}) != [{c0},{c1})")
            self._update_weight(g, c0, c1, bufs[0], bufs[1])
        self.model.finish(WORKER_GROUP, t + 1)

    def _update_weight(self, g, c0, c1, G, U):
        lm, d = self.lm, self.bcd_conf
        w = torch.from_numpy(self.model.value(g))
        act = torch.from_numpy(self.active[g])
        before = act[c0:c1].clone()
        _, vio = bcd.update(c0, c1 - c0, torch.from_numpy(G).double(),
                            torch.from_numpy(U).double(), w, torch.from_numpy(self.delta[g]), act,
                            float(lm.learning_rate.alpha), float(list(lm.penalty.__getattr__("lambda"))[0]),
                            float(d.ext("delta_max_value")), self.kkt_thr)
        self.violation = max(self.violation, bcd.violation(vio))
        newly = (before == 1) & (act[c0:c1] == 0)
        w[c0:c1][newly] = float("nan")  # KKT mark travels to the workers (sparse_filter.h)

    def evaluate(self) -> dict:
        lam = float(list(self.lm.penalty.__getattr__("lambda"))[0])
        nnz, l1, nas = 0, 0.0, 0
        for g in self.fea_grp:
            v = self.model.value(g)
            m = (v != 0) & ~np.isnan(v)
            nnz += int(m.sum())
            l1 += float(np.abs(v[m]).sum())
            nas += int(self.active[g].sum())
        return {"objective": l1 * lam, "nnz_w": nnz, "violation": self.violation,
                "nnz_active_set": nas}


class DarlinWorker(BCDWorker):
    def __init__(self, lm, name="app"):
        super().__init__(lm, name)
        self.active: dict[int, torch.Tensor] = {}
        self.delta: dict[int, torch.Tensor] = {}
        self.busy = 0.0

    def preprocess_data(self, t, call):
        super().preprocess_data(t, call)
        for g in self.fea_grp:
            n = self.model.key(g).size
            self.active[g] = torch.ones(n, dtype=torch.uint8)
            self.delta[g] = torch.full((n,), float(self.bcd_conf.ext("delta_init_value")),
                                       dtype=torch.float64)

    def compute_gradient(self, t, call, msg):
        if call.get("reset_kkt_filter"):
            for g in self.fea_grp:
                self.active[g].fill_(1)
        g = call["fea_grp"][0]
        a, b = call["key"]
        keys = self.model.key(g)
        c0 = int(np.searchsorted(keys, np.uint64(a)))
        c1 = int(np.searchsorted(keys, np.uint64(b))) if b < (1 << 64) - 1 else keys.size
        X = self.X[g]
        t0 = time.time()
        with self.mu:
            G, U = bcd.grad(X.col, X.row, X.val, int(X.colptr[c0]), int(X.colptr[c1]), c0,
                            c1 - c0, self.ym, self.y, self.delta[g], self.active[g])
        inactive = self.active[g][c0:c1] == 0
        G[inactive] = float("nan")
        U[inactive] = float("nan")
        self.busy += time.time() - t0
        push = Message(task=new_task(key_channel=g, time=t, key_range=[a, b]))
        push.recver = SERVER_GROUP
        push.set_key(keys[c0:c1])
        push.add_value(G.numpy())
        push.add_value(U.numpy())
        push.add_filter("KEY_CACHING")
        self.model.push(push)
        pull = Message(task=new_task(key_channel=g, time=t + 2, wait_time=[t + 1],
                                     key_range=[a, b]))
        pull.recver = SERVER_GROUP
        pull.set_key(keys[c0:c1])
        pull.add_filter("KEY_CACHING")
        pull.fin_handle = lambda: self._pulled(g, c0, c1, t + 2, msg)
        self.model.pull(pull)

    def _pulled(self, g, c0, c1, t, msg):
        if c1 > c0:
            (ra, rb), bufs = self.model.received(t)
            if (ra, rb) != (c0, c1):
                raise RuntimeError(f"pulled block [{ra},{rb}) != [{c0},{c1})")
            self._update_dual(g, c0, c1, bufs[0].astype(np.float64))
        self.port(msg.sender).finish_incoming(msg.task["time"])
        self.po.reply(msg)

    def _update_dual(self, g, c0, c1, new_w):
        cur = self.model.value(g)
        marked = np.isnan(new_w)
        act = self.active[g]
        if marked.any():
            idx = torch.from_numpy(np.nonzero(marked)[0] + c0)
            act[idx] = 0
        cw = cur[c0:c1]
        dw = np.where(marked, 0.0, new_w - cw)
        dm = self.bcd_conf.ext("delta_max_value")
        dl = self.delta[g][c0:c1].numpy()
        dl[~marked] = _new_delta(dm, dw[~marked])
        cur[c0:c1] = np.where(marked, 0.0, new_w)
        X = self.X[g]
        t0 = time.time()
        with self.mu:
            bcd.dual(X.col, X.row, X.val, int(X.colptr[c0]), int(X.colptr[c1]), c0, c1 - c0,
                     torch.from_numpy(dw), self.y, self.ym)
        self.busy += time.time() - t0

    def evaluate(self) -> dict:
        with self.mu:
            obj = float(bcd.objective(self.ym)[0]) if self.ym is not None else 0.0
        busy, self.busy = self.busy, 0.0
        return {"objective": obj, "busy_time": [busy]}
