#!/bin/bash
# Motion-search counters (one counter group per rocprofv3 pass, no trace domains) + a
# 3-step 1080p bench whose PSNR/kbps pins the bitstream against earlier runs.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/${1:-pmc_me}; mkdir -p $O
timeout -k 10 200 python3 -u bench.py --steps 3 > $O/bench3.log 2>&1 || { echo bench failed; exit 1; }
i=0
for ctr in "LDSBankConflict LdsUtil" "MeanOccupancyPerCU VALUBusy"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $O/g$i -o run -- python3 bench.py --steps 1 --warmup 1 --batch 8 --gop 4 > $O/g$i.log 2>&1 || { echo "group $i failed"; tail -n 5 $O/g$i.log; exit 1; }
  echo "== $ctr"
  for k in k_inter_me k_inter_recon k_phase_planes; do python3 tools/pmcsum.py $O/g$i/run_counter_collection.csv $k; done
done
