#!/bin/bash
# Iteration script: HEVC GPU engine tests, the default bench, the AV1 2-pass bench and the
# end-to-end job bench.  Usage: gpu_round.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONPATH=$PWD TMPDIR=/tmp
tag=${1:-round}
O=gpurun_out/$tag; mkdir -p $O
[ "${2:-}" = "nopytest" ] || timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_hevc.log 2>&1 || { echo "hevc pytest failed"; tail -n 40 $O/pytest_hevc.log; exit 1; }
tail -n 3 $O/pytest_hevc.log
timeout -k 10 300 python bench.py --steps 3 --warmup 1 > $O/bench_default.log 2>&1 || { echo "bench failed"; tail -n 20 $O/bench_default.log; exit 1; }
echo "default: $(grep '^{' $O/bench_default.log | tail -n 1 | cut -c1-1500)"
timeout -k 10 300 python bench.py --kbps 2000 --steps 4 --warmup 2 > $O/bench_hevc_2pass.log 2>&1 || { echo "hevc 2pass failed"; tail -n 20 $O/bench_hevc_2pass.log; exit 1; }
echo "hevc 2pass: $(grep '^{' $O/bench_hevc_2pass.log | tail -n 1 | cut -c1-1800)"
timeout -k 10 400 python bench.py --codec av1 --kbps 6000 --steps 4 --warmup 2 > $O/bench_av1_2pass.log 2>&1 || { echo "av1 2pass failed"; tail -n 20 $O/bench_av1_2pass.log; exit 1; }
echo "av1 2pass: $(grep '^{' $O/bench_av1_2pass.log | tail -n 1 | cut -c1-1800)"
timeout -k 10 500 python bench.py --job > $O/bench_job.log 2>&1 || { echo "job bench failed"; tail -n 30 $O/bench_job.log; exit 1; }
echo "job: $(grep '^{' $O/bench_job.log | tail -n 1 | cut -c1-3000)"
