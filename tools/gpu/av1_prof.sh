#!/bin/bash
# AV1 engine kernel profile: per-kernel trace summary (refine rounds split) + PMC passes
# over the hot kernels.  Usage: av1_prof.sh <tag>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONPATH=$PWD
O=gpurun_out/${1:-av1prof}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t -o run -- python3 bench.py --codec av1 --res 1080p --steps 2 --warmup 1 > $O/trace.log 2>&1 || { echo "trace failed"; tail -n 20 $O/trace.log; exit 1; }
T=$(find $O/t -name "*kernel_trace.csv" | head -1)
python3 tools/profsum.py $T --skip 0.4 > $O/summary.txt 2>&1
python3 tools/profsum.py $T --seq k_av1e_mv_refine:3 >> $O/summary.txt 2>&1
rm -f $T
head -n 14 $O/summary.txt; tail -n 3 $O/summary.txt
i=0
for ctr in "LDSBankConflict LdsUtil" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES" "MeanOccupancyPerCU VALUBusy" "SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $O/p$i -o run -- python3 bench.py --codec av1 --res 1080p --steps 1 --warmup 0 --batch 8 --gop 8 > $O/p$i.log 2>&1 || { echo "pmc $i failed"; tail -n 5 $O/p$i.log; exit 1; }
  echo "== $ctr"
  for k in k_av1e_inter k_av1e_mv_refine k_av1e_mv_unify k_sgr_select k_cdef_search; do python3 tools/pmcsum.py $(find $O/p$i -name "*counter_collection.csv" | head -1) $k; done
  rm -rf $O/p$i
done
