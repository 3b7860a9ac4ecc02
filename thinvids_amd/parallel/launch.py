"""One-process-per-GPU launcher and per-rank host placement.

``python bench.py --gpus N`` (and ``node_job --gpus N``) must run N live RCCL ranks even
when started without ``torchrun``.  :func:`spawn_ranks` is called by the parent BEFORE
anything touches the GPU: it starts N child interpreters with the torchrun environment
contract (``RANK``, ``LOCAL_RANK``, ``WORLD_SIZE``, ``LOCAL_WORLD_SIZE``,
``MASTER_ADDR=127.0.0.1``, ``MASTER_PORT``), forwards their output and returns the first
non-zero exit status.  Children are plain subprocesses (no exec from a GPU-initialised
process, no fork of CUDA state).

:func:`pin_rank` gives every rank a disjoint CPU set on the NUMA node its GPU hangs off, so
the per-rank CABAC thread pools of eight ranks do not fight over the same cores (the
reference had one encode slot per host, ``ansible_workers.yml:30``; here one host drives
eight encoders).
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time
from pathlib import Path


def launched_by_torchrun() -> bool:
    return "WORLD_SIZE" in os.environ and "RANK" in os.environ


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int, argv: list[str], extra_env: dict | None = None, timeout: float | None = None) -> int:
    """Run ``sys.executable *argv`` as n ranks on this node; returns the job's exit code.
    Every child gets its own process group so a hung rank can be killed as a group."""
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ)
        env.update(extra_env or {})
        env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   TORCHELASTIC_RESTART_COUNT=env.get("TORCHELASTIC_RESTART_COUNT", "0"))
        procs.append(subprocess.Popen([sys.executable, *argv], env=env, start_new_session=True))
    t0 = time.monotonic()
    rc = 0
    old = None
    try:  # a SIGTERM of the launcher (e.g. `timeout`) must not orphan the rank groups
        old = signal.signal(signal.SIGTERM, _raise_interrupt)
    except ValueError:  # not the main thread
        pass
    try:
        live = list(procs)
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and rc == 0:
                    rc = code
                    # one rank died: the others would block in a collective forever
                    for q in live:
                        _kill_group(q, signal.SIGTERM)
            if timeout is not None and time.monotonic() - t0 > timeout:
                for q in live:
                    _kill_group(q, signal.SIGKILL)
                return 124
            time.sleep(0.05)
    except KeyboardInterrupt:
        for q in procs:
            _kill_group(q, signal.SIGTERM)
        raise
    finally:
        if old is not None:
            signal.signal(signal.SIGTERM, old)
        for q in procs:
            if q.poll() is None:
                try:
                    q.wait(timeout=20)
                except subprocess.TimeoutExpired:
                    _kill_group(q, signal.SIGKILL)
                    q.wait()
    return rc


def _raise_interrupt(signum, frame):
    raise KeyboardInterrupt(f"signal {signum}")


def _kill_group(p: subprocess.Popen, sig) -> None:
    try:
        os.killpg(p.pid, sig)
    except (ProcessLookupError, PermissionError):
        pass


# ------------------------------------------------------------------------ placement
def _parse_cpulist(s: str) -> list[int]:
    out = []
    for part in s.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def numa_cpus() -> dict[int, list[int]]:
    """NUMA node -> CPUs (sysfs); one pseudo-node with every CPU when unavailable."""
    nodes = {}
    base = Path("/sys/devices/system/node")
    for d in sorted(base.glob("node[0-9]*")):
        try:
            nodes[int(d.name[4:])] = _parse_cpulist((d / "cpulist").read_text())
        except (OSError, ValueError):
            continue
    if not nodes:
        nodes = {0: list(range(os.cpu_count() or 1))}
    return nodes


def gpu_numa_nodes() -> list[int]:
    """NUMA node of each AMD display/accelerator PCI function, in PCI bus order (the HIP
    enumeration order when HIP_VISIBLE_DEVICES is unset).  Read from sysfs: no GPU call."""
    out = []
    for d in sorted(Path("/sys/bus/pci/devices").glob("*")):
        try:
            if (d / "vendor").read_text().strip() != "0x1002":
                continue
            cls = (d / "class").read_text().strip()
            if not (cls.startswith("0x0380") or cls.startswith("0x0300") or cls.startswith("0x1200")):
                continue
            out.append(max(0, int((d / "numa_node").read_text().strip())))
        except (OSError, ValueError):
            continue
    return out


def visible_gpu_count() -> int:
    """GPUs a rank launcher may use, counted without any HIP call (a supervisor that never
    initialises the GPU can fork / exec ranks safely): the *_VISIBLE_DEVICES list when set,
    otherwise the AMD GPU functions in sysfs.  0 when none is visible."""
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            return len([x for x in v.split(",") if x.strip() and x.strip() != "-1"])
    return len(gpu_numa_nodes())


def plan_affinity(local_rank: int, local_world: int, allowed: list[int] | None = None,
                  nodes: dict[int, list[int]] | None = None, gpu_nodes: list[int] | None = None) -> list[int]:
    """Disjoint CPU set for one rank: the ranks that share a NUMA node split that node's
    allowed CPUs evenly.  Falls back to an even split of all allowed CPUs."""
    allowed = sorted(allowed if allowed is not None else os.sched_getaffinity(0))
    nodes = nodes if nodes is not None else numa_cpus()
    gpu_nodes = gpu_nodes if gpu_nodes is not None else gpu_numa_nodes()
    aset = set(allowed)
    if len(gpu_nodes) >= local_world and len(nodes) > 1:
        node = gpu_nodes[local_rank]
        peers = [r for r in range(local_world) if gpu_nodes[r] == node]
        cpus = [c for c in nodes.get(node, []) if c in aset]
        if cpus:
            k, n = peers.index(local_rank), len(peers)
            share = max(1, len(cpus) // n)
            mine = cpus[k * share:(k + 1) * share] if k < n - 1 else cpus[k * share:]
            return mine or cpus
    share = max(1, len(allowed) // max(1, local_world))
    lo = min(local_rank * share, max(0, len(allowed) - share))
    return allowed[lo:lo + share] if local_rank < local_world - 1 else allowed[lo:]


def pin_rank(local_rank: int, local_world: int) -> list[int]:
    """Apply :func:`plan_affinity` to this process (inherited by the engine's CABAC threads,
    which are created later).  ``TV_CPUS=N`` caps the rank at the first N CPUs of its set
    (the "1/8 of a host" experiment: an 8-GPU node's per-rank share on any box).  Pinning is
    skipped when TV_NO_PIN=1 (the cap still applies) or the platform lacks affinity."""
    if not hasattr(os, "sched_setaffinity"):
        return sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else []
    cap = int(os.environ.get("TV_CPUS", "0") or 0)
    if os.environ.get("TV_NO_PIN") == "1":
        cpus = sorted(os.sched_getaffinity(0))
    else:
        gpu_nodes = None
        phys = [int(x) for x in os.environ.get("TV_PHYS_GPUS", "").split(",") if x.strip()]
        if phys:  # a supervisor restarted this node on a subset of its GPUs (HIP_VISIBLE_DEVICES)
            allg = gpu_numa_nodes()
            gpu_nodes = [allg[g] if g < len(allg) else 0 for g in phys]
        cpus = plan_affinity(local_rank, local_world, gpu_nodes=gpu_nodes)
    if cap > 0:
        cpus = cpus[:cap]
    try:
        os.sched_setaffinity(0, cpus)
    except OSError:
        return sorted(os.sched_getaffinity(0))
    return cpus
