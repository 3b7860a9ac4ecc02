#!/bin/bash
# AV1 GPU tests, then a rocprofv3 kernel-stats run of the AV1 bench.  Usage: gpu_av1_prof.sh <tag> [bench args]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONPATH=$PWD TMPDIR=/tmp TV_NO_AUTOBUILD=1
tag=${1:-av1p}; shift
O=gpurun_out/$tag; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_av1_codec.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -n 3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --codec av1 "$@" > $O/bench.log 2>&1
rc=$?; tail -n 1 $O/bench.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
python3 tools/kstats.py $(find $O/prof -name "*kernel_stats.csv" | head -1) 16
