#!/bin/bash
# AV1 engine check on one GPU box: the AV1 GPU tests (bit-exact vs the golden encoder), then
# an optional bench.  Usage: gpu_av1e.sh <tag> [bench args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONPATH=$PWD TMPDIR=/tmp TV_NO_AUTOBUILD=1
tag=${1:-av1e}; shift
O=gpurun_out/$tag; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_av1_codec.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -n 30 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
if [ $# -gt 0 ]; then
  timeout -k 10 300 python -u bench.py "$@" > $O/bench.log 2>&1; rc=$?; tail -n 3 $O/bench.log; exit $rc
fi
