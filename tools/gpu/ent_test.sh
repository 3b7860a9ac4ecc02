#!/bin/bash
# GPU entropy coding: its own tests, then the engine golden tests (which now run the GPU
# coder by default), then one short default bench.  First failure ends it.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-ent}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_entropy.py -x -v --timeout 120 --timeout-method thread > $O/pytest_ent.log 2>&1
rc=$?; echo "pytest_ent rc=$rc"; tail -n 3 $O/pytest_ent.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py -x -v --timeout 200 --timeout-method thread > $O/pytest_eng.log 2>&1
rc=$?; echo "pytest_eng rc=$rc"; tail -n 3 $O/pytest_eng.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -n 2 $O/bench.log
