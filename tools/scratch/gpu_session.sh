#!/bin/bash
# GPU-box iteration step: GPU tests, a short bench, optional rocprofv3 kernel stats.
#   gpu_session.sh <tag> [--prof] [bench args...]
# Every GPU step has its own time limit and the steps are chained: the first failure ends it.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
tag=$1; shift
prof=0
if [ "$1" = "--prof" ]; then prof=1; shift; fi
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 $out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 "$@" > $out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 $out/bench.log
[ $rc -eq 0 ] || exit $rc
if [ $prof -eq 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python3 bench.py --steps 2 --warmup 1 "$@" > $out/prof.log 2>&1
  rc=$?; echo "prof rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  python3 tools/profsum.py $(find $out/prof -name "*kernel_trace.csv" | head -1) --skip 0.5 > $out/kernel_summary.txt 2>&1
  head -20 $out/kernel_summary.txt
fi
