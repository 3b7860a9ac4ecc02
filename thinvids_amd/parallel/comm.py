"""Intra-node communication for the encode data plane (SURVEY.md §2.2 COMM, §5.8).

The reference moves segment bytes with HTTP GET/PUT between worker hosts
(reference worker/tasks.py:663-806, :1497-1525, :1655-1674).  Inside one MI355X node
the same transfers are RCCL collectives over xGMI (`torch.distributed` backend "nccl" is
RCCL on ROCm), one process per GPU:

* ``gather_bytes_to_root`` — variable-length bitstream gather to the stitch rank:
  all_gather of int64 sizes, then grouped point-to-point send/recv (one hop per peer on
  the fully connected xGMI mesh; no ring).
* ``scatter_frames_from_root`` — GOP scatter from the ingest rank with grouped sends.
* ``allreduce_stats`` — small latency-bound all-reduce of rate-control statistics.

The same functions run on the ``gloo`` backend with CPU tensors (tests, world_size > 1).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist


def _world():
    if not dist.is_available() or not dist.is_initialized():
        return 1, 0
    return dist.get_world_size(), dist.get_rank()


def _live() -> bool:
    """A process group exists: collectives run even at world size 1 (a one-rank RCCL
    communicator still executes on the GPU, so the N=1 bench exercises the same code)."""
    return dist.is_available() and dist.is_initialized()


# Per-process P2P counters of the byte gathers (bench.py reports them per rank).
COMM_STATS = {"p2p_sent_bytes": 0, "p2p_recv_bytes": 0, "p2p_ops": 0}


class _PinnedStage:
    """A reusable pinned host buffer per direction and device: a payload is copied into it
    once and moved with one asynchronous copy (no per-call ``bytearray`` + ``pin_memory``
    allocation, which is a page-locking ``hipHostMalloc`` every time).  An event guards reuse:
    the next call waits until the previous copy out of / into the buffer has completed."""

    def __init__(self):
        self.buf = None
        self.ev = None

    def get(self, n: int, device) -> "torch.Tensor":
        if self.ev is not None:
            self.ev.synchronize()
        if self.buf is None or self.buf.numel() < n:
            self.buf = torch.empty(max(n, 1 << 20, 2 * (self.buf.numel() if self.buf is not None else 0)),
                                   dtype=torch.uint8, pin_memory=True)
        return self.buf[:n]

    def mark(self, device) -> None:
        self.ev = torch.cuda.Event()
        self.ev.record(torch.cuda.current_stream(device))


_STAGES: dict = {}


def _stage(kind: str, device) -> _PinnedStage:
    key = (kind, str(device))
    if key not in _STAGES:
        _STAGES[key] = _PinnedStage()
    return _STAGES[key]


def to_device_bytes(payload: bytes, device: torch.device) -> torch.Tensor:
    """Host bytes -> a uint8 tensor on `device` (CPU: a view of the bytes, no copy)."""
    src = torch.frombuffer(memoryview(payload), dtype=torch.uint8) if len(payload) else torch.empty(0, dtype=torch.uint8)
    if device.type != "cuda":
        return src
    st = _stage("h2d", device)
    pin = st.get(len(payload), device)
    pin.copy_(src)
    out = pin.to(device, non_blocking=True)
    st.mark(device)
    return out


def from_device_bytes(t: torch.Tensor, n: int) -> bytes:
    """The first n bytes of a device (or host) uint8 tensor as bytes, through the reusable
    pinned receive buffer."""
    if t.device.type != "cuda":
        return t[:n].numpy().tobytes()
    st = _stage("d2h", t.device)
    pin = st.get(n, t.device)
    pin.copy_(t[:n], non_blocking=True)
    st.mark(t.device)
    st.ev.synchronize()
    return pin.numpy().tobytes()


def gather_bytes_to_root(payload: bytes, device: torch.device, root: int = 0):
    """Gather one byte string from every rank to `root`.  Returns list[bytes] on root, None
    elsewhere.  Sizes travel in one all_gather; payloads as one grouped isend/irecv (one
    xGMI hop per peer), staged through reusable pinned buffers."""
    world, rank = _world()
    if not _live():
        return [payload]
    n = torch.tensor([len(payload)], dtype=torch.int64, device=device)
    sizes = [torch.zeros(1, dtype=torch.int64, device=device) for _ in range(world)]
    dist.all_gather(sizes, n)
    sizes = [int(s.item()) for s in sizes]
    if rank == root:
        bufs = {r: torch.empty(sizes[r], dtype=torch.uint8, device=device)
                for r in range(world) if r != root and sizes[r] > 0}
        if bufs:
            for req in dist.batch_isend_irecv([dist.P2POp(dist.irecv, b, r) for r, b in bufs.items()]):
                req.wait()
            COMM_STATS["p2p_ops"] += len(bufs)
        out = []
        for r in range(world):
            if r == root:
                out.append(payload)
            elif r in bufs:
                out.append(from_device_bytes(bufs[r], sizes[r]))
                COMM_STATS["p2p_recv_bytes"] += sizes[r]
            else:
                out.append(b"")
        return out
    if len(payload):
        t = to_device_bytes(payload, device)
        for req in dist.batch_isend_irecv([dist.P2POp(dist.isend, t, root)]):
            req.wait()
        COMM_STATS["p2p_sent_bytes"] += len(payload)
        COMM_STATS["p2p_ops"] += 1
    return None


def scatter_frames_from_root(frames: list | None, shape: tuple, device: torch.device, root: int = 0):
    """Scatter one uint8 tensor of `shape` per rank from `root` (GOP frames of a segment).
    `frames` (root only) is a list of world tensors/arrays; device tensors are sent as they
    are (no host bounce), host arrays are uploaded first."""
    world, rank = _world()

    def dev_t(x):
        return (x if isinstance(x, torch.Tensor) else torch.as_tensor(np.asarray(x))).to(device)

    if world == 1:
        return dev_t(frames[0]).reshape(shape).clone()
    out = torch.empty(shape, dtype=torch.uint8, device=device)
    if rank == root:
        ops = []
        for r in range(world):
            t = dev_t(frames[r])
            if r == root:
                out.copy_(t)
            else:
                ops.append(dist.P2POp(dist.isend, t.contiguous(), r))
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    else:
        for req in dist.batch_isend_irecv([dist.P2POp(dist.irecv, out, root)]):
            req.wait()
    return out


def scatter_root(round_idx: int, world: int) -> int:
    """Root of scatter round `round_idx`: rotates over the ranks, so the source reads, the
    host->device staging and the world-1 sends of a job are spread evenly (each xGMI link of
    the fully connected node carries one hop per round) instead of serialising on rank 0."""
    return round_idx % max(1, world)


def stage_segment_frames(frames, shape: tuple, device: torch.device) -> torch.Tensor:
    """Pack decoded frames [(Y, U, V) host planes] into one device tensor of `shape`
    (frames x packed I420 bytes): each plane is copied straight into its slice of the device
    buffer through a pinned host staging row; no host-side concatenation."""
    buf = torch.zeros(shape, dtype=torch.uint8, device=device)
    pin = device.type == "cuda"
    row = torch.empty(shape[1], dtype=torch.uint8, pin_memory=pin) if pin else None
    for f, planes in enumerate(frames):
        o = 0
        for p in planes:
            a = torch.from_numpy(np.ascontiguousarray(p).reshape(-1))
            n = a.numel()
            if row is not None:
                row[o:o + n].copy_(a)
            else:
                buf[f, o:o + n].copy_(a)
            o += n
        if row is not None:  # one H2D copy per frame, ordered on the stream before the reuse
            buf[f].copy_(row, non_blocking=False)
    return buf


_GROUPS: dict = {}


def stream_groups(device: torch.device):
    """(control group, data group) of the streaming segment gather, created once per process
    on first use — every rank reaches its first streaming job at the same point (SPMD), so
    the collective ``new_group`` calls line up.  Control = gloo (a 16-byte header per round:
    host-side, no GPU kernel spinning while ranks wait for each other); data = the default
    backend (RCCL over xGMI for device tensors, gloo on CPU)."""
    key = (dist.get_backend(), device.type)
    if key not in _GROUPS:
        ctrl = dist.new_group(backend="gloo")
        data = dist.new_group(backend=dist.get_backend()) if device.type == "cuda" else ctrl
        if device.type == "cuda":
            # every rank joins one collective on the new data group right away, so its RCCL
            # communicator is created by all ranks together -- its first user is otherwise a
            # batch_isend_irecv among the root and the peers that happen to have a payload
            # (a first call on a subset of ranks is undefined for NCCL/RCCL)
            t = torch.zeros(1, device=device)
            dist.all_reduce(t, group=data)
            torch.cuda.synchronize(device)
        _GROUPS[key] = (ctrl, data)
    return _GROUPS[key]


class SegmentStream:
    """Per-claim bitstream gather to the stitch rank while the node encodes — the
    reference's encoder -> stitcher PUT of each finished part (worker/tasks.py:1655-1674,
    received by the stitcher's ingest loop :1898-2029), as RCCL point-to-point over xGMI.

    Ranks claim segments dynamically, so they finish different numbers of claims at
    different times; a collective schedule still needs every rank in every round.  A comm
    thread per rank therefore runs *rounds*: it waits until this rank has finished
    segments (or ``idle_s`` passes, or the rank is done), all-gathers a (payload bytes,
    done) header on the gloo control group, and then every peer with a payload sends it to
    the root with one grouped isend/irecv on the data group (one xGMI hop per peer, no
    ring).  The loop ends on every rank in the same round: the first one in which all ranks
    report done.  The root's own segments never leave the process (``put`` hands them to
    ``on_segment`` directly).  Only this thread touches the two stream groups, so the
    caller may keep issuing collectives on the default group (e.g. scatter rounds)."""

    def __init__(self, device: torch.device, on_segment, root: int = 0, idle_s: float = 0.02):
        import threading

        self.world, self.rank = _world()
        self.root, self.idle_s, self.on_segment = root, idle_s, on_segment
        self.dev = device if device.type == "cuda" and dist.get_backend() == "nccl" else torch.device("cpu")
        self.ctrl, self.data = stream_groups(self.dev)
        self.cv = threading.Condition()
        self.q: list = []
        self.done = False
        self.err: BaseException | None = None
        self.stats = {"rounds": 0, "segments": 0, "bytes": 0, "transfer_s": 0.0}
        self.th = threading.Thread(target=self._run, name="segment-stream", daemon=True)
        self.th.start()

    def put(self, key, data: bytes) -> None:
        if self.rank == self.root:
            self.on_segment(key, data)
            return
        with self.cv:
            self.q.append((key, bytes(data)))
            self.cv.notify()

    def close(self) -> dict:
        """This rank has no more segments: returns after the round in which every rank
        said so (raises the comm thread's error)."""
        with self.cv:
            self.done = True
            self.cv.notify()
        self.th.join()
        if self.err is not None:
            raise RuntimeError(f"segment stream failed: {self.err}") from self.err
        return self.stats

    def _run(self) -> None:
        import json
        import time

        try:
            if self.dev.type == "cuda":
                torch.cuda.set_device(self.dev)
            while True:
                with self.cv:
                    self.cv.wait_for(lambda: self.q or self.done, timeout=self.idle_s)
                    items, self.q = self.q, []
                    done = self.done
                blob = b""
                if items:
                    idx = json.dumps([[list(k) if isinstance(k, tuple) else k, len(b)] for k, b in items]).encode()
                    blob = len(idx).to_bytes(8, "little") + idx + b"".join(b for _, b in items)
                hdr = torch.tensor([len(blob), int(done)], dtype=torch.int64)
                hdrs = [torch.zeros(2, dtype=torch.int64) for _ in range(self.world)]
                dist.all_gather(hdrs, hdr, group=self.ctrl)
                if any(int(h[1]) == 2 for h in hdrs):  # a peer's thread failed: leave together
                    raise RuntimeError("a peer's segment stream failed")
                sizes = [int(h[0]) for h in hdrs]
                t0 = time.perf_counter()
                try:
                    self._exchange(blob, sizes)
                except BaseException as e:  # noqa: BLE001 - e.g. on_segment at the root
                    self.err = e
                    # one more header round carries the failure (2) to every rank, so no peer
                    # blocks in the next all_gather until the process-group timeout
                    dist.all_gather(hdrs, torch.tensor([0, 2], dtype=torch.int64), group=self.ctrl)
                    return
                self.stats["transfer_s"] += time.perf_counter() - t0
                self.stats["rounds"] += 1
                if all(int(h[1]) for h in hdrs):
                    return
        except BaseException as e:  # noqa: BLE001 - surfaced by close()
            if self.err is None:
                self.err = e

    def _exchange(self, blob: bytes, sizes: list) -> None:
        import json

        if self.rank == self.root:
            bufs = {r: torch.empty(sizes[r], dtype=torch.uint8, device=self.dev)
                    for r in range(self.world) if r != self.root and sizes[r] > 0}
            if not bufs:
                return
            ops = [dist.P2POp(dist.irecv, b, r, group=self.data) for r, b in bufs.items()]
            for req in dist.batch_isend_irecv(ops):
                req.wait()
            for r in sorted(bufs):
                raw = from_device_bytes(bufs[r], sizes[r])
                hl = int.from_bytes(raw[:8], "little")
                off = 8 + hl
                for k, n in json.loads(raw[8:off]):
                    self.on_segment(tuple(k) if isinstance(k, list) else k, raw[off:off + n])
                    off += n
                    self.stats["segments"] += 1
                self.stats["bytes"] += len(raw)
        elif blob:
            t = to_device_bytes(blob, self.dev)
            for req in dist.batch_isend_irecv([dist.P2POp(dist.isend, t, self.root, group=self.data)]):
                req.wait()
            self.stats["bytes"] += len(blob)


def allreduce_stats(values, device: torch.device, op: str = "sum") -> np.ndarray:
    """All-reduce a small float64 vector (e.g. per-segment complexity for 2-pass RC)."""
    t = torch.as_tensor(np.asarray(values, dtype=np.float64), device=device)
    if _live():
        dist.all_reduce(t, op=dist.ReduceOp.SUM if op == "sum" else dist.ReduceOp.MAX)
    return t.cpu().numpy()
