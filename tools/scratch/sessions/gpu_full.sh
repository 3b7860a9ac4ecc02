#!/bin/bash
# Round check on one GPU box: the whole GPU test suite, the smoke, then the headline bench,
# the SAO-on (production default) bench and the 4K bench.  Chained: first failure ends it.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-full}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1; rc=$?; tail -1 $O/bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --sao > $O/bench_sao.log 2>&1; rc=$?; tail -1 $O/bench_sao.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --res 4k > $O/bench_4k.log 2>&1; rc=$?; tail -1 $O/bench_4k.log; [ $rc -eq 0 ] || exit $rc
