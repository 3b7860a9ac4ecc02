#!/bin/bash
# AV1 GPU checks: engine == golden, dav1d conformance of GPU streams, AV1 tools kernels.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/${1:-av1c}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_av1_conformance.py tests/test_av1_codec.py tests/test_av1_tools.py -m gpu -x -v \
  --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -n 60 $O/pytest.log; exit 1; }
tail -n 12 $O/pytest.log
