#!/bin/bash
# AV1 tool kernels on the GPU: bit-exactness tests + throughput.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/${1:-av1}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_av1_tools.py tests/test_av1_deblock.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
  || { echo "pytest failed"; tail -n 40 $O/pytest.log; exit 1; }
tail -n 3 $O/pytest.log
timeout -k 10 300 python tools/av1_tools_bench.py --res 4k --batch 8 --iters 5 --lr > $O/bench_4k.log 2>&1 || { echo bench failed; tail -n 20 $O/bench_4k.log; exit 1; }
tail -n 1 $O/bench_4k.log
