#!/bin/bash
# Round 6: k_inter_me phase costs now (TV_DIAG_ME_STOP 1 staging, 2 + integer search, 3 +
# half-pel; timing only) and the instruction counters per stop.  Usage: r6_me_phases.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD TV_NO_AUTOBUILD=1
O=gpurun_out/${1:-r6mep}; mkdir -p $O
for st in 1 2 3 0; do
  TV_DIAG_ME_STOP=$st TV_ENGINE_GROUPS=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/s$st -o run -- python3 bench.py --no-4k --steps 2 --warmup 1 > $O/s$st.log 2>&1 || { echo "stop $st failed"; tail -5 $O/s$st.log; exit 1; }
  echo "== stop $st"; python3 tools/profsum.py $(find $O/s$st -name "*kernel_trace.csv" | head -1) --skip 0.3 2>&1 | grep -E "inter_me"
  TV_DIAG_ME_STOP=$st timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES --output-format csv -d $O/p$st -o run -- python3 bench.py --no-4k --steps 1 --warmup 1 --batch 16 --gop 8 > $O/p$st.log 2>&1 || { echo "pmc $st failed"; exit 1; }
  python3 tools/pmcsum.py $(find $O/p$st -name "*counter_collection.csv" | head -1) k_inter_me
done 2>&1 | tee $O/summary.txt
