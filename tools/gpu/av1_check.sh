#!/bin/bash
# AV1 engine check: AV1 GPU tests (GPU == golden, dav1d), 1080p + 4K benches.  Usage: av1_check.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-av1check}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_av1_codec.py tests/test_av1_conformance.py tests/test_av1_tools.py tests/test_av1_deblock.py -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR" $O/pytest.log | tail -n 30; tail -n 3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1080p 4k; do
  timeout -k 10 600 python -u bench.py --codec av1 --res $r --steps 4 --warmup 1 > $O/bench_$r.log 2>&1 || { echo "bench $r failed"; tail -n 20 $O/bench_$r.log; exit 1; }
  echo "av1 $r: $(grep '^{' $O/bench_$r.log | tail -n 1 | cut -c1-1500)"
done
