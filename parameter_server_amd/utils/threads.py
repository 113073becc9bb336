"""Host threading helpers (reference src/util/threadpool.h, barrier.h,
threadsafe_queue.h, threadsafe_limited_queue.h, producer_consumer.h).

The data path uses these to overlap file reading / text parsing (C++ parser,
GIL released) with GPU training: ``ProducerConsumer`` runs a producer thread
that fills a queue bounded by a BYTE budget (``ThreadsafeLimitedQueue``, the
reference's capacity-in-MB semantics), so a fast reader cannot run host memory
out while the GPU consumes minibatches.
"""
from __future__ import annotations

import collections
import threading
from typing import Any, Callable


class ThreadPool:
    """Add tasks, then ``start_workers()`` runs them on ``n`` threads and joins
    (reference ThreadPool: add() before startWorkers(), which blocks until done).
    Exceptions from tasks are re-raised in the caller."""

    def __init__(self, num_workers: int):
        self.n = max(1, int(num_workers))
        self._tasks: collections.deque = collections.deque()
        self._lock = threading.Lock()
        self._errors: list[BaseException] = []

    def add(self, fn: Callable[[], Any]) -> None:
        self._tasks.append(fn)

    def _work(self):
        while True:
            with self._lock:
                if not self._tasks:
                    return
                fn = self._tasks.popleft()
            try:
                fn()
            except BaseException as e:  # noqa: BLE001
                with self._lock:
                    self._errors.append(e)

    def start_workers(self) -> None:
        ths = [threading.Thread(target=self._work, daemon=True) for _ in range(self.n)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        if self._errors:
            raise self._errors[0]


Barrier = threading.Barrier  # reference util/barrier.h: same semantics


class ThreadsafeQueue:
    """Unbounded blocking FIFO (reference threadsafe_queue.h)."""

    def __init__(self):
        self._q: collections.deque = collections.deque()
        self._cv = threading.Condition()

    def push(self, v) -> None:
        with self._cv:
            self._q.append(v)
            self._cv.notify()

    def wait_and_pop(self, timeout: float | None = None):
        with self._cv:
            if not self._cv.wait_for(lambda: bool(self._q), timeout):
                raise TimeoutError("queue empty")
            return self._q.popleft()

    def try_pop(self):
        with self._cv:
            return (True, self._q.popleft()) if self._q else (False, None)

    def __len__(self) -> int:
        with self._cv:
            return len(self._q)

    def empty(self) -> bool:
        return len(self) == 0


class ThreadsafeLimitedQueue:
    """FIFO bounded by the summed ``capacity`` of its items (bytes). ``push(...,
    finished=True)`` marks the end; ``pop`` returns ``(False, None)`` after the last
    item (reference threadsafe_limited_queue.h)."""

    def __init__(self, max_capacity: int = 0):
        self.max_capacity = int(max_capacity)
        self._cur = 0
        self._done = False
        self._q: collections.deque = collections.deque()
        self._cv = threading.Condition()

    def set_max_capacity(self, c: int) -> None:
        with self._cv:
            self.max_capacity = int(c)
            self._cv.notify_all()

    def push(self, value, capacity: int, finished: bool = False) -> None:
        with self._cv:
            if self._done:
                raise RuntimeError("push after the queue was marked finished")
            if not finished and capacity == 0:
                return
            # an item larger than the whole budget is admitted when the queue is
            # empty (the reference would block forever here)
            self._cv.wait_for(lambda: self._cur + capacity <= self.max_capacity or not self._q)
            if capacity or not finished:
                self._q.append((value, capacity))
                self._cur += capacity
            if finished:
                self._q.append((None, 0))
                self._done = True
            self._cv.notify_all()

    def pop(self, timeout: float | None = None):
        with self._cv:
            if not self._cv.wait_for(lambda: bool(self._q), timeout):
                raise TimeoutError("queue empty")
            v, c = self._q[0]
            if c == 0 and self._done and len(self._q) == 1:
                return False, None  # end marker stays so later pops also see the end
            self._q.popleft()
            self._cur -= c
            self._cv.notify_all()
            return True, v

    def size(self) -> int:
        with self._cv:
            return sum(1 for _, c in self._q if c)

    def empty(self) -> bool:
        return self.size() == 0


class ProducerConsumer:
    """Producer thread -> byte-bounded queue -> consumer (reference
    producer_consumer.h). ``func(put)`` style: the producer function returns
    ``(item, nbytes, more)``; ``more=False`` ends the stream."""

    def __init__(self, capacity_mb: float = 1000):
        self.queue = ThreadsafeLimitedQueue(int(capacity_mb * 1_000_000))
        self._producer: threading.Thread | None = None
        self._consumer: threading.Thread | None = None
        self.error: BaseException | None = None

    def set_capacity(self, mb: float) -> None:
        self.queue.set_max_capacity(int(mb * 1_000_000))

    def start_producer(self, func: Callable[[], tuple]) -> None:
        def run():
            try:
                while True:
                    item, size, more = func()
                    if not more:
                        if item is not None and size:
                            self.queue.push(item, size)
                        self.queue.push(None, 0, finished=True)
                        return
                    self.queue.push(item, max(1, int(size)))
            except BaseException as e:  # noqa: BLE001
                self.error = e
                self.queue.push(None, 0, finished=True)

        self._producer = threading.Thread(target=run, daemon=True)
        self._producer.start()

    def start_consumer(self, func: Callable[[Any], None]) -> None:
        def run():
            while True:
                ok, v = self.pop()
                if not ok:
                    return
                func(v)

        self._consumer = threading.Thread(target=run, daemon=True)
        self._consumer.start()

    def wait_consumer(self) -> None:
        if self._consumer is not None:
            self._consumer.join()
        if self.error is not None:
            raise self.error

    def pop(self):
        ok, v = self.queue.pop()
        if not ok and self.error is not None:
            raise self.error
        return ok, v

    def push(self, item, size: int = 1, finished: bool = False) -> None:
        self.queue.push(item, size, finished)

    def set_finished(self) -> None:
        self.queue.push(None, 0, finished=True)

    def __iter__(self):
        while True:
            ok, v = self.pop()
            if not ok:
                return
            yield v
