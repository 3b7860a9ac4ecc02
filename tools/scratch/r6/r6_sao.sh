#!/bin/bash
# Round 6: SAO kernel check -- engine golden tests (SAO on), bench pairs packed / per-sample
# (TV_SAO_PACKED=0), a single-group kernel trace and the instruction counters.  Usage: r6_sao.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD TV_NO_AUTOBUILD=1
O=gpurun_out/${1:-r6sao2}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_entropy.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -n 2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
val() { python3 -c "import json; L=[l for l in open('$1') if l.startswith('{')]; print(json.loads(L[-1])['value'])"; }
for r in 1 2; do
  for v in A B; do
    if [ $v = B ]; then export TV_SAO_PACKED=0; else unset TV_SAO_PACKED; fi
    timeout -k 10 300 python -u bench.py --no-4k --steps 8 --warmup 2 > $O/b_${v}$r.log 2>&1 || { echo "bench $v failed"; tail -n 5 $O/b_${v}$r.log; exit 1; }
    echo "$v$r $(val $O/b_${v}$r.log)"
  done
done
unset TV_SAO_PACKED
TV_ENGINE_GROUPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/g1 -o run -- python3 bench.py --no-4k --steps 3 --warmup 1 > $O/g1.log 2>&1 || { echo "prof failed"; exit 1; }
python3 tools/profsum.py $(find $O/g1 -name "*kernel_trace.csv" | head -1) --skip 0.4 > $O/g1_summary.txt 2>&1; head -n 8 $O/g1_summary.txt
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --output-format csv -d $O/p1 -o run -- python3 bench.py --no-4k --steps 1 --warmup 1 --batch 16 --gop 8 > $O/p1.log 2>&1 || { echo "pmc failed"; exit 1; }
python3 tools/pmcsum.py $(find $O/p1 -name "*counter_collection.csv" | head -1) k_sao_decide
