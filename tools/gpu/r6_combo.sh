#!/bin/bash
# Round 6 combined session: engine golden tests, SDMA-vs-HIP D2H A/B, packed-SAO A/B, then the
# phase breakdown.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-r6combo}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_entropy.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu/ab_env.sh ${1:-r6combo}/d2h TV_NOP=1 TV_D2H=hip --no-4k || exit 1
bash tools/gpu/ab_env.sh ${1:-r6combo}/sao TV_NOP=1 TV_SAO_PACKED=0 --no-4k || exit 1
bash tools/gpu/r6_phases.sh ${1:-r6combo}/phase
