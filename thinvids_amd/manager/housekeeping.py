"""Housekeeping process (reference manager/housekeeping.py): runs the
pipeline scheduler and the job watchdog outside the web server processes.

    python -m thinvids_amd.manager.housekeeping
"""
import time

from ..common import get_logging
from .core import Housekeeping


def main() -> None:  # pragma: no cover - service entry
    get_logging("housekeeping")
    hk = Housekeeping().start()
    try:
        while True:
            time.sleep(3600)
    except KeyboardInterrupt:
        hk.stop()


if __name__ == "__main__":
    main()
