"""Elastic node supervision: rank liveness, communicator abort + re-init, smaller-world
fallback (SURVEY.md §5.3 "New").

The reference's only elasticity is per-part: a failed encode re-enqueues itself for any
thin client (reference worker/tasks.py:1385-1464) and the manager watchdog fails stalled
jobs (manager/app.py:1420-1457).  On an 8-GPU node the encoders are RCCL ranks of one
process group, and a dead or hung rank takes the communicator down with it: every peer
blocks in the next collective.  The recovery therefore works on the rank group:

* every rank publishes a heartbeat ``node:rank:<host>:<rank>`` (generation, pid, physical
  GPU, current job, and a *progress* timestamp the main thread advances per segment — a
  beat thread keeps running while the main thread is stuck in a GPU wait, so liveness alone
  would not catch a hang);
* the :class:`Supervisor` (the node executor's parent process, which never touches the GPU)
  watches its ranks: a rank that exits non-zero, or — while a job runs — stops making
  progress for ``stall_sec`` (the culprit is the rank whose progress is oldest: its peers
  progressed until they reached the collective it never joined), triggers recovery;
* recovery = abort the communicator by killing the whole rank group (RCCL state dies with
  the processes; in-process ``ncclCommAbort`` cannot unblock a rank spinning in a hung
  kernel), quarantine the culprit's GPU (``node:gpu_quarantine:<host>``), requeue the
  in-flight job at the front of the node queue, and restart the ranks on the remaining GPUs
  (``HIP_VISIBLE_DEVICES``) — a smaller world with a fresh communicator and fresh
  rendezvous namespaces.  The requeued job resumes from its segment checkpoints;
* a rank whose collective fails without a culprit (a RCCL error surfaced as
  ``DistError``) exits with :data:`EXIT_COMM`: the group is re-initialised at the same
  world size.
"""
from __future__ import annotations

import json
import os
import signal
import subprocess
import sys
import threading
import time

EXIT_COMM = 77  # a rank saw its communicator fail: re-init the group, no GPU at fault
RANK_TTL = 30


def rank_key(host: str, rank: int) -> str:
    return f"node:rank:{host}:{rank}"


def quarantine_key(host: str) -> str:
    return f"node:gpu_quarantine:{host}"


class RankBeat:
    """Per-rank heartbeat thread.  The main thread calls :meth:`progress` whenever it
    completes work and :meth:`set_job` around a job."""

    def __init__(self, store, host: str, rank: int, gen: int, gpu: int, interval: float = 1.0):
        self.st, self.host, self.rank, self.gen, self.gpu = store, host, rank, gen, gpu
        self.interval = interval
        self.job: dict | None = None
        self.progress_ts = time.time()
        self.note = ""
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._loop, daemon=True, name=f"rank-beat-{rank}")

    def start(self) -> "RankBeat":
        self._publish()
        self._t.start()
        return self

    def progress(self, note: str = "") -> None:
        self.progress_ts = time.time()
        if note:
            self.note = note

    def set_job(self, job: dict | None) -> None:
        self.job = job
        self.progress("job start" if job else "idle")
        self._publish()

    def _publish(self) -> None:
        try:
            self.st.set(rank_key(self.host, self.rank), json.dumps(
                {"gen": self.gen, "pid": os.getpid(), "gpu": self.gpu, "ts": time.time(), "job": self.job,
                 "progress_ts": self.progress_ts, "note": self.note}), ex=RANK_TTL)
        except Exception:  # noqa: BLE001 - a store hiccup must not kill the rank
            pass

    def _loop(self) -> None:
        while not self._stop.wait(self.interval):
            self._publish()

    def stop(self) -> None:
        self._stop.set()
        try:
            self.st.delete(rank_key(self.host, self.rank))
        except Exception:  # noqa: BLE001
            pass


def is_comm_failure(e: BaseException) -> bool:
    """A collective / communicator failure (as opposed to a job-level error)."""
    try:
        import torch.distributed as dist

        kinds = tuple(k for k in (getattr(dist, "DistError", None), getattr(dist, "DistBackendError", None),
                                  getattr(dist, "DistNetworkError", None)) if k is not None)
    except ImportError:
        kinds = ()
    return bool(kinds) and isinstance(e, kinds)


def _killpg(p: subprocess.Popen, sig) -> None:
    try:
        os.killpg(p.pid, sig)
    except (ProcessLookupError, PermissionError):
        pass


class Supervisor:
    """Runs ``python *argv`` as one rank per healthy GPU and recovers from rank failures.

    gpus: physical GPU indices of this node.  ``requeue(job, reason)`` is called with the
    in-flight job of a failed generation (rank 0's heartbeat) and returns False when the
    job must not run again (its restart budget is spent)."""

    def __init__(self, argv: list[str], gpus: list[int], host: str, store, stall_sec: float = 600.0,
                 max_restarts: int = 8, extra_env: dict | None = None, requeue=None, log=None,
                 cpu_mode: bool = False):
        self.argv, self.gpus, self.host, self.st = argv, list(gpus), host, store
        self.stall_sec, self.max_restarts = stall_sec, max_restarts
        self.extra_env = dict(extra_env or {})
        self.requeue = requeue or (lambda job, reason: True)
        self.log = log or (lambda m: print(f"[supervisor] {m}", file=sys.stderr, flush=True))
        self.cpu_mode = cpu_mode
        self.quarantined: dict[int, str] = {}
        self.history: list[dict] = []

    def healthy(self) -> list[int]:
        return [g for g in self.gpus if g not in self.quarantined]

    def run(self) -> int:
        gen = int(self.extra_env.get("TORCHELASTIC_RESTART_COUNT", os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")))
        restarts = 0
        while True:
            world = self.healthy()
            if not world:
                self.log("no healthy GPU left on this node")
                return 1
            rc, culprit, reason, job = self._generation(world, gen)
            self.history.append({"gen": gen, "world": len(world), "rc": rc, "culprit": culprit, "reason": reason})
            if rc == 0:
                return 0
            if culprit is not None:
                self.quarantined[culprit] = reason
                try:
                    self.st.hset(quarantine_key(self.host), str(culprit), json.dumps({"reason": reason, "ts": time.time()}))
                except Exception:  # noqa: BLE001
                    pass
            if restarts >= self.max_restarts:
                self.log(f"giving up after {restarts} restarts: {reason}")
                return rc or 1
            if job:
                self.requeue(job, reason)
            restarts += 1
            gen += 1
            self.log(f"restarting on {len(self.healthy())} GPU(s) {self.healthy()} after: {reason}")

    def _generation(self, world: list[int], gen: int):
        from .launch import free_port

        port = free_port()
        n = len(world)
        procs = []
        for r, g in enumerate(world):
            env = dict(os.environ)
            env.update(self.extra_env)
            env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0",
                       MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), TORCHELASTIC_RESTART_COUNT=str(gen),
                       TV_PHYS_GPUS=",".join(map(str, world)), TV_PHYS_GPU=str(g))
            if not self.cpu_mode:
                env["HIP_VISIBLE_DEVICES"] = ",".join(map(str, world))
            procs.append(subprocess.Popen([sys.executable, *self.argv], env=env, start_new_session=True))
        last_job = None
        try:
            while True:
                codes = [p.poll() for p in procs]
                beats = self._beats(n, gen)
                if 0 in beats:  # rank 0 owns the job; None between jobs
                    last_job = beats[0].get("job")
                bad = [r for r, c in enumerate(codes) if c not in (None, 0)]
                if bad:
                    r = min(bad, key=lambda k: codes[k] == EXIT_COMM)  # a real death beats a comm error
                    c = codes[r]
                    culprit = None if c == EXIT_COMM else world[r]
                    why = f"rank {r} (GPU {world[r]}) exited with {c}" if culprit is not None else \
                        f"rank {r} reported a communicator failure"
                    return c, culprit, why, last_job
                if all(c == 0 for c in codes):
                    return 0, None, "", None
                stall = self._stalled(beats, n)
                if stall is not None:
                    return 75, world[stall], f"rank {stall} (GPU {world[stall]}) made no progress for " \
                                             f"{self.stall_sec:.0f} s", last_job
                time.sleep(0.2)
        finally:
            self._stop_all(procs)

    def _beats(self, n: int, gen: int) -> dict:
        out = {}
        for r in range(n):
            try:
                raw = self.st.get(rank_key(self.host, r))
                d = json.loads(raw) if raw else None
            except Exception:  # noqa: BLE001
                d = None
            if d and int(d.get("gen", -1)) == gen:
                out[r] = d
        return out

    def _stalled(self, beats: dict, n: int):
        busy = {r: b for r, b in beats.items() if b.get("job")}
        if not busy:
            return None
        now = time.time()
        r = min(busy, key=lambda k: float(busy[k].get("progress_ts") or 0))
        return r if now - float(busy[r].get("progress_ts") or now) > self.stall_sec else None

    def _stop_all(self, procs) -> None:
        for p in procs:
            if p.poll() is None:
                _killpg(p, signal.SIGTERM)
        t0 = time.monotonic()
        for p in procs:
            try:
                p.wait(timeout=max(0.1, 10 - (time.monotonic() - t0)))
            except subprocess.TimeoutExpired:
                _killpg(p, signal.SIGKILL)
                p.wait()
