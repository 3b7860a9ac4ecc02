#!/bin/bash
# Round 6: engine golden tests, a single-group kernel trace and the LDS counter pass of the
# HEVC kernels (one counter group per run).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-r6mecheck}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
TV_ENGINE_GROUPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/g1 -o run -- python3 bench.py --no-4k --steps 3 --warmup 1 > $O/g1.log 2>&1 || { echo "prof failed"; exit 1; }
python3 tools/profsum.py $(find $O/g1 -name "*kernel_trace.csv" | head -1) --skip 0.4 > $O/g1_summary.txt 2>&1; head -n 6 $O/g1_summary.txt
timeout -s KILL 120 rocprofv3 --pmc LDSBankConflict LdsUtil --output-format csv -d $O/p1 -o run -- python3 bench.py --no-4k --steps 1 --warmup 1 --batch 16 --gop 8 > $O/p1.log 2>&1 || { echo "pmc failed"; exit 1; }
for k in k_inter_me k_inter_recon k_sao_decide; do python3 tools/pmcsum.py $(find $O/p1 -name "*counter_collection.csv" | head -1) $k; done
