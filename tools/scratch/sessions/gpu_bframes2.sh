#!/bin/bash
# B-frame iteration: B-frame GPU tests, the B8 bench, then a rocprofv3 kernel-stats run of it.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-bframes2}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_bframes.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 8 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --bframes 8 > $O/bench_b8.log 2>&1; rc=$?; tail -n 1 $O/bench_b8.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 3 --warmup 1 --bframes 8 > $O/prof_bench.log 2>&1; rc=$?; echo "prof rc=$rc"
