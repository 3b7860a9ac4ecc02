"""Worker process entry (reference: `huey_consumer tasks.pipeline_huey -k thread -w N` and
the encode consumer, ansible_workers.yml:340-370).

    python -m thinvids_amd.worker --role all|pipeline|encode [--pipeline-workers 4]

One process per GPU for the encode role (``LOCAL_RANK`` / ``--device`` pick the GPU); its
consumer pops up to ``TV_ENCODE_BATCH_TASKS`` encode tasks at a time and encodes them in
shared batched engine launches.  Exits with 75 when the node is disabled/quarantined.
"""
from __future__ import annotations

import argparse
import os
import signal
import sys
import threading

from ..common import get_logging
from ..queue import Consumer
from . import dataplane, tasks
from .config import get_config
from .helpers import node_is_disabled, quarantine_current_node


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--role", default=os.environ.get("TV_WORKER_ROLE", "all"), choices=("all", "pipeline", "encode"))
    ap.add_argument("--pipeline-workers", type=int, default=int(os.environ.get("TV_PIPELINE_WORKERS", "4")))
    ap.add_argument("--device", type=int, default=None)
    args = ap.parse_args(argv)
    log = get_logging("worker")
    if args.device is not None:
        os.environ["TV_DEVICE"] = str(args.device)
    if node_is_disabled():
        log.error("node %s is disabled/quarantined; refusing to start", get_config().worker_name)
        return 75
    dataplane.start_http_once()
    consumers = []
    if args.role in ("all", "pipeline"):
        consumers.append(Consumer(tasks.pipeline_q, workers=max(2, args.pipeline_workers)).start())
    if args.role in ("all", "encode"):
        from .encoder import default_cache, gpu_available

        if gpu_available():
            try:
                default_cache()
            except Exception as e:  # broken GPU stack: take this node out of rotation
                quarantine_current_node(f"GPU engine init failed: {e}")
                return 75
        consumers.append(Consumer(tasks.encode_q, workers=1,
                                  handler=lambda q: tasks.encode_batch_handler()).start())
    stop = threading.Event()
    for sig in (signal.SIGINT, signal.SIGTERM):
        signal.signal(sig, lambda *_: stop.set())
    log.info("worker %s up (role=%s)", get_config().worker_name, args.role)
    stop.wait()
    for c in consumers:
        c.stop()
    return 0


if __name__ == "__main__":
    sys.exit(main())
