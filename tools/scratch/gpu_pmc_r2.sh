#!/bin/bash
# Counter passes (one rocprofv3 --pmc run each, no trace domains) over a short SAO-on bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-pmc_r2}; mkdir -p $O
i=0
for ctr in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA" "VALUBusy MeanOccupancyPerCU" "LDSBankConflict MemUnitStalled"; do
  i=$((i+1))
  timeout -k 10 -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d $O/g$i -o run -- python3 bench.py --steps 1 --warmup 1 --batch 8 --gop 4 --sao > $O/g$i.log 2>&1 || { echo "group $i failed"; tail -n 5 $O/g$i.log; exit 1; }
  echo "== $ctr"
  for k in k_sao_decide k_sao_apply k_inter_me k_inter_recon k_phase_planes k_intra_recon k_synth k_coarse_me k_intra_analysis; do python3 tools/pmcsum.py $(find $O/g$i -name "*counter_collection.csv" | head -1) $k; done
done
