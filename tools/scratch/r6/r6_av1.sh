#!/bin/bash
# Round 6 AV1: codec GPU tests, stage-0 occupancy A/B at 4K, kernel trace of the 4K bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-r6av1}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_av1_codec.py tests/test_av1_conformance.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu/ab_env.sh ${1:-r6av1}/ab TV_NOP=1 TV_AV1_INTER_WPE=5 --codec av1 --res 4k || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --codec av1 --res 4k --steps 3 --warmup 1 > $O/prof.log 2>&1 || { echo "prof failed"; exit 1; }
python3 tools/profsum.py $(find $O/prof -name "*kernel_trace.csv" | head -1) --skip 0.4 > $O/summary.txt 2>&1
head -n 14 $O/summary.txt
