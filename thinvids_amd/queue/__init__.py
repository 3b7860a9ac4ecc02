"""Task queues over the state store (replaces Huey on Redis DB0, reference common.py:49-64).

Two named queues as in the reference: ``<HUEY_NAME>:pipeline`` (transcode / split / stitch /
stamp orchestration) and ``<HUEY_NAME>:encode`` (per-segment encodes).  Messages are JSON in
a store list; consumers pop with ``blpop``.  Semantics kept from Huey as used by thinvids:

* calling a task enqueues it; ``.call_local`` runs it inline;
* per-task ``retries`` / ``retry_delay`` (e.g. transcode: 999999 x 5 s, worker/tasks.py:831);
* ``revoke_by_id`` (fixed: revokes the task id it is given);
* immediate mode (``TV_QUEUE_IMMEDIATE=1`` or ``TaskQueue.immediate = True``) for tests.

MI355X addition: :meth:`TaskQueue.pop_batch` lets a per-GPU consumer pull up to B compatible
encode tasks and run them as ONE batched engine call (GPU occupancy needs >> 1 segment).
"""
from __future__ import annotations

import json
import logging
import os
import threading
import time
import traceback
import uuid
from typing import Callable

from ..store import get_store

HUEY_NAME = os.environ.get("HUEY_NAME", "tasks")
log = logging.getLogger("thinvids.queue")


class TaskWrapper:
    def __init__(self, queue: "TaskQueue", fn: Callable, name: str, retries: int, retry_delay: float):
        self.queue, self.fn, self.name = queue, fn, name
        self.retries, self.retry_delay = retries, retry_delay
        self.__doc__ = fn.__doc__
        self.__name__ = fn.__name__

    def __call__(self, *args, **kwargs) -> str:
        return self.queue.enqueue(self.name, args, kwargs, retries=self.retries)

    def call_local(self, *args, **kwargs):
        return self.fn(*args, **kwargs)

    def schedule(self, args=(), kwargs=None, delay: float = 0.0) -> str:
        return self.queue.enqueue(self.name, args, kwargs or {}, retries=self.retries, delay=delay)


class TaskQueue:
    immediate = os.environ.get("TV_QUEUE_IMMEDIATE", "0") == "1"

    def __init__(self, name: str, store=None):
        self.name = name
        self.key = f"{HUEY_NAME}:{name}" if ":" not in name else name
        self._store = store
        self.registry: dict[str, TaskWrapper] = {}

    @property
    def store(self):
        return self._store or get_store()

    # ----------------------------------------------------------------- producer side
    def task(self, retries: int = 0, retry_delay: float = 0.0, name: str | None = None):
        def deco(fn):
            w = TaskWrapper(self, fn, name or fn.__name__, retries, retry_delay)
            self.registry[w.name] = w
            return w

        return deco

    def enqueue(self, task: str, args=(), kwargs=None, retries: int = 0, delay: float = 0.0,
                task_id: str | None = None) -> str:
        tid = task_id or str(uuid.uuid4())
        msg = {"id": tid, "task": task, "args": list(args), "kwargs": kwargs or {}, "retries": retries,
               "eta": time.time() + delay if delay else 0}
        if TaskQueue.immediate:
            self._execute(msg)
            return tid
        self.store.rpush(self.key, json.dumps(msg))
        return tid

    def revoke_by_id(self, task_id: str) -> None:
        self.store.sadd(f"{self.key}:revoked", task_id)

    def pending(self) -> list[dict]:
        return [json.loads(m) for m in self.store.lrange(self.key, 0, -1)]

    def __len__(self) -> int:
        return self.store.llen(self.key)

    def flush(self) -> None:
        self.store.delete(self.key)

    # ----------------------------------------------------------------- consumer side
    def pop(self, timeout: float = 1.0) -> dict | None:
        r = self.store.blpop([self.key], timeout=timeout)
        if not r:
            return None
        msg = json.loads(r[1])
        if msg.get("eta") and msg["eta"] > time.time():  # not due yet: requeue at the tail
            self.store.rpush(self.key, r[1])
            time.sleep(min(0.2, msg["eta"] - time.time()))
            return None
        if self.store.sismember(f"{self.key}:revoked", msg["id"]):
            self.store.srem(f"{self.key}:revoked", msg["id"])
            return None
        return msg

    def pop_batch(self, max_n: int, compatible: Callable[[dict, dict], bool], timeout: float = 1.0) -> list[dict]:
        """Pop one due task, then up to max_n-1 more immediately available tasks that are
        `compatible` with it (others are pushed back to the head in order)."""
        first = self.pop(timeout)
        if first is None:
            return []
        batch, skipped = [first], []
        while len(batch) < max_n:
            raw = self.store.lpop(self.key)
            if raw is None:
                break
            msg = json.loads(raw)
            due = not msg.get("eta") or msg["eta"] <= time.time()
            if due and msg["task"] == first["task"] and compatible(first, msg):
                if not self.store.sismember(f"{self.key}:revoked", msg["id"]):
                    batch.append(msg)
            else:
                skipped.append(raw)
        for raw in reversed(skipped):
            self.store.lpush(self.key, raw)
        return batch

    def _execute(self, msg: dict):
        w = self.registry.get(msg["task"])
        if w is None:
            raise KeyError(f"unknown task {msg['task']!r} on queue {self.name}")
        try:
            return w.fn(*msg.get("args", []), **msg.get("kwargs", {}))
        except Exception:
            left = int(msg.get("retries", 0))
            log.error("task %s[%s] failed (%d retries left):\n%s", msg["task"], msg["id"], left,
                      traceback.format_exc())
            if left > 0 and not TaskQueue.immediate:
                self.enqueue(msg["task"], msg.get("args", []), msg.get("kwargs", {}), retries=left - 1,
                             delay=w.retry_delay, task_id=msg["id"])
            elif TaskQueue.immediate:
                raise
            return None

    def run_one(self, timeout: float = 1.0) -> bool:
        msg = self.pop(timeout)
        if msg is None:
            return False
        self._execute(msg)
        return True

    def drain(self, max_tasks: int = 10_000) -> int:
        """Run queued tasks inline until the queue is empty (tests / single-process mode)."""
        n = idle = 0
        while n < max_tasks and len(self) > 0 and idle <= len(self):
            if self.run_one(timeout=0.01):
                n, idle = n + 1, 0
            else:  # revoked (dropped) or not yet due (requeued)
                idle += 1
        return n


class Consumer:
    """Thread-pool consumer (`huey_consumer -k thread -w N`, ansible_workers.yml:351)."""

    def __init__(self, queue: TaskQueue, workers: int = 1, handler: Callable[[TaskQueue], bool] | None = None):
        self.queue, self.workers = queue, workers
        self.handler = handler or (lambda q: q.run_one(timeout=1.0))
        self._stop = threading.Event()
        self._threads: list[threading.Thread] = []

    def start(self) -> "Consumer":
        for i in range(self.workers):
            t = threading.Thread(target=self._loop, name=f"{self.queue.name}-consumer-{i}", daemon=True)
            t.start()
            self._threads.append(t)
        return self

    def _loop(self):
        while not self._stop.is_set():
            try:
                self.handler(self.queue)
            except Exception:
                log.error("consumer error:\n%s", traceback.format_exc())
                time.sleep(0.5)

    def stop(self, join: bool = True):
        self._stop.set()
        if join:
            for t in self._threads:
                t.join(timeout=5)


_queues: dict[str, TaskQueue] = {}


def get_queue(name: str) -> TaskQueue:
    if name not in _queues:
        _queues[name] = TaskQueue(name)
    return _queues[name]


def get_pipeline_queue() -> TaskQueue:
    return get_queue(os.environ.get("HUEY_PIPELINE_NAME", "pipeline"))


def get_encode_queue() -> TaskQueue:
    return get_queue(os.environ.get("HUEY_ENCODE_NAME", "encode"))
