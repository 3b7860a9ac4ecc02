#!/bin/bash
# First GPU session: GPU tests, smoke, 1-GPU bench, rocprofv3 kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 1; }
timeout -k 10 300 python -m pytest tests/test_gpu_engine.py -x -q > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?"; tail -20 gpurun_out/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
echo "smoke rc=$?"; tail -5 gpurun_out/smoke.log
timeout -k 10 300 python bench.py --steps 2 --warmup 1 > gpurun_out/bench_1080p.log 2>&1
echo "bench rc=$?"; tail -5 gpurun_out/bench_1080p.log
