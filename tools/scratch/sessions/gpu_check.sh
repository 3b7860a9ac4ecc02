#!/bin/bash
# GPU health check of the tree: gpu tests, smoke(), 1080p + 4K bench.  Usage: gpu_check.sh <tag> [bench args]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONPATH=$PWD TMPDIR=/tmp
tag=${1:-check}; shift
O=gpurun_out/$tag; mkdir -p $O
python -c "import __graft_entry__ as g; g.build()" > $O/build.log 2>&1 || { echo build failed; tail -n 20 $O/build.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { echo "pytest failed"; tail -n 40 $O/pytest_gpu.log; exit 1; }
tail -n 3 $O/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -n 20 $O/smoke.log; exit 1; }
tail -n 1 $O/smoke.log
for args in "" "--res 4k" "$@"; do
  [ -z "$args" ] && t=1080p || t=$(echo "$args" | tr -d ' -')
  timeout -k 10 300 python bench.py --steps 4 --warmup 2 $args > $O/bench_$t.log 2>&1 || { echo "bench $args failed"; tail -n 20 $O/bench_$t.log; exit 1; }
  echo "bench [$args]: $(tail -n 1 $O/bench_$t.log | cut -c1-700)"
done
