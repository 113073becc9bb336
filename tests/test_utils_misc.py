"""Host utilities: threads (ThreadPool / queues / ProducerConsumer), timers and
resource usage, evaluation metrics (reference src/util/*.h semantics)."""
import threading
import time

import numpy as np
import pytest
import torch

from parameter_server_amd.utils import evaluation
from parameter_server_amd.utils.resource import LocalMachine, ResUsage, ScopedTimer, Timer
from parameter_server_amd.utils.threads import (ProducerConsumer, ThreadPool, ThreadsafeLimitedQueue,
                                                ThreadsafeQueue)


def test_thread_pool_runs_all_and_propagates_errors():
    out = []
    lock = threading.Lock()
    pool = ThreadPool(4)
    for i in range(100):
        pool.add(lambda i=i: (lock.acquire(), out.append(i), lock.release()))
    pool.start_workers()
    assert sorted(out) == list(range(100))
    bad = ThreadPool(2)
    bad.add(lambda: 1 / 0)
    with pytest.raises(ZeroDivisionError):
        bad.start_workers()


def test_limited_queue_blocks_on_byte_budget():
    q = ThreadsafeLimitedQueue(100)
    q.push("a", 60)
    t0 = time.time()

    def later():
        time.sleep(0.2)
        assert q.pop() == (True, "a")

    th = threading.Thread(target=later)
    th.start()
    q.push("b", 60)  # blocks until "a" is popped
    assert time.time() - t0 >= 0.15
    th.join()
    q.push("c", 10, finished=True)
    assert q.pop() == (True, "b") and q.pop() == (True, "c")
    assert q.pop() == (False, None) and q.pop() == (False, None)
    with pytest.raises(RuntimeError):
        q.push("d", 1)
    # oversize item admitted into an empty queue instead of deadlocking
    q2 = ThreadsafeLimitedQueue(10)
    q2.push("big", 50)
    assert q2.pop() == (True, "big")


def test_threadsafe_queue():
    q = ThreadsafeQueue()
    assert q.try_pop() == (False, None)
    q.push(1)
    assert q.wait_and_pop() == 1
    with pytest.raises(TimeoutError):
        q.wait_and_pop(timeout=0.05)


def test_producer_consumer():
    pc = ProducerConsumer(capacity_mb=0.001)  # 1000 bytes -> producer must wait
    it = iter(range(50))

    def produce():
        i = next(it, None)
        return (i, 300, i is not None)

    pc.start_producer(produce)
    got = []
    pc.start_consumer(got.append)
    pc.wait_consumer()
    assert got == list(range(50))
    bad = ProducerConsumer()
    bad.start_producer(lambda: 1 / 0)
    with pytest.raises(ZeroDivisionError):
        list(bad)


def test_timers_and_resources():
    t = Timer()
    with t:
        time.sleep(0.02)
    assert t.get() >= 0.015
    tm = Timer(milli=True).start()
    time.sleep(0.01)
    assert tm.stop() >= 8
    h = {}
    with ScopedTimer(h, "x"):
        pass
    assert h["x"] >= 0
    assert ResUsage.my_phy_mem() > 0 and ResUsage.host_total_mem() > 0
    assert ResUsage.my_cpu_seconds() > 0
    assert 1 <= LocalMachine.pickup_available_port() < 65536
    name, ip = LocalMachine.pickup_available_interface_and_ip()
    assert ip.count(".") == 3
    assert LocalMachine.num_cpus() >= 1


def _auc_pairs(y, p):  # O(n^2) definition with ties as 0 (matches a stable sort order)
    pos, neg = p[y > 0], p[y <= 0]
    return float((pos[:, None] > neg[None, :]).mean())


def test_evaluation_metrics():
    rng = np.random.default_rng(0)
    y = np.where(rng.random(2000) < 0.3, 1.0, -1.0)
    p = y * 0.5 + rng.standard_normal(2000)
    a = evaluation.auc(y, p)
    assert abs(a - _auc_pairs(y, p)) < 1e-9
    assert abs(evaluation.auc(y, -p) - a) < 1e-9  # reported as max(a, 1-a)
    assert abs(evaluation.auc(torch.tensor(y), torch.tensor(p)) - a) < 1e-9
    acc = evaluation.accuracy(y, p)
    assert abs(acc - max(np.mean((y > 0) == (p > 0)), 1 - np.mean((y > 0) == (p > 0)))) < 1e-12
    ll = evaluation.logloss(y, p)
    assert abs(ll - np.mean(np.log1p(np.exp(-y * p)))) < 1e-9
