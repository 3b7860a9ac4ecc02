#!/bin/bash
# Session-start check on one GPU box: all GPU tests, the smoke, the default (driver) bench,
# the 4K bench and the AV1 1080p bench.  Chained: the first failure ends it.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-start}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 8 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -n 2 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/bench.log 2>&1; rc=$?; tail -n 1 $O/bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --res 4k --steps 4 --warmup 1 > $O/bench_4k.log 2>&1; rc=$?; tail -n 1 $O/bench_4k.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --codec av1 --steps 6 --warmup 2 > $O/bench_av1.log 2>&1; rc=$?; tail -n 1 $O/bench_av1.log; [ $rc -eq 0 ] || exit $rc
