#!/bin/bash
# B-frame bring-up on one GPU box: the new B-frame GPU tests, the HEVC engine tests (IPPP
# regression), then the default bench and the hierarchical-B bench.  First failure ends it.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-bframes}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_bframes.py tests/test_gpu_engine.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 25 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 > $O/bench.log 2>&1; rc=$?; tail -n 1 $O/bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --bframes 8 > $O/bench_b8.log 2>&1; rc=$?; tail -n 1 $O/bench_b8.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --bframes 4 > $O/bench_b4.log 2>&1; rc=$?; tail -n 1 $O/bench_b4.log; [ $rc -eq 0 ] || exit $rc
