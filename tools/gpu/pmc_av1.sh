#!/bin/bash
# Derived-counter profile of the AV1 engine's hot kernels (one counter group per run, no
# trace domains).  Usage: gpu_pmc_av1.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONPATH=$PWD TMPDIR=/tmp TV_NO_AUTOBUILD=1
O=gpurun_out/${1:-pmc_av1}; mkdir -p $O
i=0
for ctr in "MeanOccupancyPerCU VALUBusy" "VALUUtilization MemUnitStalled" "LDSBankConflict LdsUtil" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAVES"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $ctr --output-format csv -d $O/g$i -o run -- python3 bench.py --codec av1 --steps 1 --warmup 1 --batch 8 --gop 4 > $O/g$i.log 2>&1 || { echo "group $i failed"; tail -n 5 $O/g$i.log; exit 1; }
  echo "== $ctr"
  for k in k_av1e_inter k_cdef_search k_sgr_search k_deblock; do python3 tools/pmcsum.py $(find $O/g$i -name "*counter_collection.csv" | head -1) $k; done
done
