#!/bin/bash
# Memory-side counter passes (one rocprofv3 --pmc run each, no trace domains) over the
# 1080p headline bench: where do the ME / phase-plane / synth kernels lose time?
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-pmc_me}; mkdir -p $O
i=0
for ctr in "FETCH_SIZE MemUnitBusy" "L2CacheHit VALUBusy" "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_ANY SQ_INSTS_VALU SQ_WAVES" "MeanOccupancyPerCU LDSBankConflict"; do
  i=$((i+1))
  timeout -k 10 -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d $O/g$i -o run -- python3 bench.py --steps 1 --warmup 1 > $O/g$i.log 2>&1 || { echo "group $i failed"; tail -n 5 $O/g$i.log; exit 1; }
  echo "== $ctr"
  for k in k_inter_me k_inter_recon k_phase_planes k_intra_recon k_synth k_coarse_me k_intra_analysis k_deblock; do python3 tools/pmcsum.py $(find $O/g$i -name "*counter_collection.csv" | head -1) $k; done
done
