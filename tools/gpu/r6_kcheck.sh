#!/bin/bash
# Round 6: generic kernel check -- engine golden tests, 3 default bench runs (1080p), a
# single-group kernel trace and the instruction counters of kernel $2.  Usage: r6_kcheck.sh <tag> <kernel>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD TV_NO_AUTOBUILD=1
O=gpurun_out/${1:-r6k}; K=${2:-k_inter_me}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_bframes.py tests/test_gpu_entropy.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -n 2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
val() { python3 -c "import json; L=[l for l in open('$1') if l.startswith('{')]; print(json.loads(L[-1])['value'])"; }
for r in 1 2 3; do
  timeout -k 10 300 python -u bench.py --no-4k --steps 8 --warmup 2 > $O/b$r.log 2>&1 || { echo "bench failed"; tail -n 5 $O/b$r.log; exit 1; }
  echo "bench$r $(val $O/b$r.log)"
done
TV_ENGINE_GROUPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/g1 -o run -- python3 bench.py --no-4k --steps 3 --warmup 1 > $O/g1.log 2>&1 || { echo "prof failed"; exit 1; }
python3 tools/profsum.py $(find $O/g1 -name "*kernel_trace.csv" | head -1) --skip 0.4 > $O/g1_summary.txt 2>&1; head -n 8 $O/g1_summary.txt
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --output-format csv -d $O/p1 -o run -- python3 bench.py --no-4k --steps 1 --warmup 1 --batch 16 --gop 8 > $O/p1.log 2>&1 || { echo "pmc failed"; exit 1; }
python3 tools/pmcsum.py $(find $O/p1 -name "*counter_collection.csv" | head -1) $K
