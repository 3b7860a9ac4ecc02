#!/bin/bash
# Iteration loop on the GPU box: build, GPU tests, bench, rocprofv3 stats.  Usage: gpu_iter.sh <tag> [bench args]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
tag=$1; shift
mkdir -p gpurun_out/$tag
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/$tag/build.log 2>&1 || { cat gpurun_out/$tag/build.log; exit 1; }
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/$tag/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/$tag/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 3 --warmup 1 "$@" > gpurun_out/$tag/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/$tag/bench.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$tag/prof -o run -- python3 bench.py --steps 1 --warmup 1 "$@" > gpurun_out/$tag/prof.log 2>&1
rc=$?; echo "prof rc=$rc"
find gpurun_out/$tag/prof -name "*kernel_stats.csv" -exec cut -d, -f1-4 {} \; | sed 's/(tv::gpu[^"]*//' | head -14
