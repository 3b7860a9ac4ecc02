#!/bin/bash
# GPU-box step: node-executor / job-path GPU tests, then the end-to-end job bench.
set -o pipefail
TAG=${1:-job}
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests/test_node_executor.py tests/test_gpu_engine.py tests/test_parallel.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1; rc=$?; tail -15 gpurun_out/$TAG/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --job > gpurun_out/$TAG/job.log 2>&1; rc=$?; tail -3 gpurun_out/$TAG/job.log; [ $rc -eq 0 ] || exit $rc
