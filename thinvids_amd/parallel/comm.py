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


def gather_bytes_to_root(payload: bytes, device: torch.device, root: int = 0):
    """Gather one byte string from every rank to `root`.  Returns list[bytes] on root, None
    elsewhere."""
    world, rank = _world()
    if not _live():
        return [payload]
    n = torch.tensor([len(payload)], dtype=torch.int64, device=device)
    sizes = [torch.zeros(1, dtype=torch.int64, device=device) for _ in range(world)]
    dist.all_gather(sizes, n)
    sizes = [int(s.item()) for s in sizes]
    if rank == root:
        bufs = [torch.empty(max(1, sizes[r]), dtype=torch.uint8, device=device) for r in range(world)]
        ops = [dist.P2POp(dist.irecv, bufs[r], r) for r in range(world) if r != root and sizes[r] > 0]
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()
        out = []
        for r in range(world):
            if r == root:
                out.append(payload)
            else:
                out.append(bytes(bufs[r][: sizes[r]].cpu().numpy().tobytes()) if sizes[r] else b"")
        return out
    if len(payload):
        t = torch.frombuffer(bytearray(payload), dtype=torch.uint8)
        if device.type == "cuda":
            t = t.pin_memory().to(device, non_blocking=True)
        for req in dist.batch_isend_irecv([dist.P2POp(dist.isend, t, root)]):
            req.wait()
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


def allreduce_stats(values, device: torch.device, op: str = "sum") -> np.ndarray:
    """All-reduce a small float64 vector (e.g. per-segment complexity for 2-pass RC)."""
    t = torch.as_tensor(np.asarray(values, dtype=np.float64), device=device)
    if _live():
        dist.all_reduce(t, op=dist.ReduceOp.SUM if op == "sum" else dist.ReduceOp.MAX)
    return t.cpu().numpy()
