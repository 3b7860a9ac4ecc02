#!/bin/bash
# AV1 engine check on one GPU box: the AV1 GPU tests (bit-exact vs the golden encoder), then
# benches, one per extra argument string.  Usage: gpu_av1e.sh <tag> ["bench args" ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONPATH=$PWD TMPDIR=/tmp TV_NO_AUTOBUILD=1
tag=${1:-av1e}; shift
O=gpurun_out/$tag; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_av1_codec.py tests/test_av1_tools.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -n 12 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
i=0
for args in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python -u bench.py $args > $O/bench_$i.log 2>&1; rc=$?; tail -n 1 $O/bench_$i.log | cut -c1-900; [ $rc -eq 0 ] || exit $rc
done
