#!/bin/bash
# Round 6: k_sao_decide instruction counts per phase (TV_DIAG_SAO_STOP=1/2/3 = stop after
# staging / statistics / decision, 0 = whole kernel; timing/counting only).  Usage: r6_sao_pmc.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONPATH=$PWD TMPDIR=/tmp TV_NO_AUTOBUILD=1
O=gpurun_out/${1:-r6saopmc}; mkdir -p $O
for st in 1 2 3 0; do
  TV_DIAG_SAO_STOP=$st timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --output-format csv -d $O/p$st -o run -- python3 bench.py --no-4k --steps 1 --warmup 1 --batch 16 --gop 8 > $O/p$st.log 2>&1 || { echo "stop $st failed"; tail -n 5 $O/p$st.log; exit 1; }
  echo "== stop $st"; python3 tools/pmcsum.py $(find $O/p$st -name "*counter_collection.csv" | head -1) k_sao_decide
done 2>&1 | tee $O/summary.txt
