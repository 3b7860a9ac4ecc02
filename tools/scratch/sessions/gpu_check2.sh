#!/bin/bash
# Whole GPU suite + smoke, then the AV1 1080p / 4K benches.  First failure ends it.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-check2}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 4 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --codec av1 --steps 6 --warmup 2 > $O/bench_av1.log 2>&1; rc=$?; tail -n 1 $O/bench_av1.log | cut -c1-1200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --codec av1 --res 4k --steps 4 --warmup 1 > $O/bench_av1_4k.log 2>&1; rc=$?; tail -n 1 $O/bench_av1_4k.log | cut -c1-1200; [ $rc -eq 0 ] || exit $rc
