#!/bin/bash
# B-frame iteration: B-frame GPU tests, the B8 bench, then single-group (no kernel overlap)
# rocprofv3 kernel stats of the IPPP and B8 benches, so kernel durations are stand-alone.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-bframes3}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_bframes.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --bframes 8 > $O/bench_b8.log 2>&1; rc=$?; tail -n 1 $O/bench_b8.log | cut -c1-900; [ $rc -eq 0 ] || exit $rc
export TV_ENGINE_GROUPS=1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_b8_g1 -o run -- python3 bench.py --steps 2 --warmup 1 --bframes 8 > $O/prof_b8_g1.log 2>&1; rc=$?; echo "prof b8 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_p_g1 -o run -- python3 bench.py --steps 2 --warmup 1 > $O/prof_p_g1.log 2>&1; rc=$?; echo "prof ippp rc=$rc"
