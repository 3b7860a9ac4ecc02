#!/bin/bash
# Round 6: counter passes (one group per run, no trace domains) of the hot HEVC kernels at the
# bench geometry, batch 16 / GOP 8 so each pass takes seconds.  Usage: r6_pmc.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONPATH=$PWD TMPDIR=/tmp TV_NO_AUTOBUILD=1
O=gpurun_out/${1:-r6pmc}; mkdir -p $O
i=0
for ctr in "SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM" \
           "MeanOccupancyPerCU VALUBusy" "LDSBankConflict LdsUtil" "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $O/g$i -o run -- python3 bench.py --no-4k --steps 1 --warmup 1 --batch 16 --gop 8 > $O/g$i.log 2>&1 || { echo "group $i failed"; tail -n 5 $O/g$i.log; exit 1; }
  echo "== $ctr"
  for k in k_inter_me k_inter_recon k_sao_decide k_phase_planes k_coarse_me k_deblock k_intra_recon; do python3 tools/pmcsum.py $(find $O/g$i -name "*counter_collection.csv" | head -1) $k; done
done 2>&1 | tee $O/pmc_summary.txt
