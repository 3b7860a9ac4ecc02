#!/bin/bash
# Counter profile of the HEVC engine's hot kernels at the shipped config (SAO on, small batch
# so each pass is seconds): one counter group per run, no trace domains.  Usage: gpu_pmc_hevc.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONPATH=$PWD TMPDIR=/tmp TV_NO_AUTOBUILD=1
O=gpurun_out/${1:-pmc_hevc}; mkdir -p $O
i=0
for ctr in "MeanOccupancyPerCU VALUBusy" "VALUUtilization MemUnitStalled" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAVES" "FETCH_SIZE" "WRITE_SIZE" "LDSBankConflict LdsUtil"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $ctr --output-format csv -d $O/g$i -o run -- python3 bench.py --steps 1 --warmup 1 --batch 16 --gop 8 > $O/g$i.log 2>&1 || { echo "group $i failed"; tail -n 5 $O/g$i.log; exit 1; }
  echo "== $ctr"
  for k in k_inter_me k_inter_recon k_intra_recon k_intra_analysis k_sao_decide k_phase_planes k_coarse_me; do python3 tools/pmcsum.py $(find $O/g$i -name "*counter_collection.csv" | head -1) $k; done
done
