#!/bin/bash
# End-to-end job bench (node executor, HEVC 1080p) with the rank-0 span breakdown.  Usage: gpu_job_bench.sh <tag> [extra args]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONPATH=$PWD TMPDIR=/tmp
tag=${1:-job}; shift
O=gpurun_out/$tag; mkdir -p $O
timeout -k 10 600 python bench.py --job "$@" > $O/bench_job.log 2>&1 || { echo "job bench failed"; tail -n 30 $O/bench_job.log; exit 1; }
echo "job: $(grep '^{' $O/bench_job.log | tail -n 1 | cut -c1-3000)"
