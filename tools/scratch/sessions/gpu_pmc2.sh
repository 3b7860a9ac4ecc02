#!/bin/bash
# Derived-counter profile (no trace domains) of the hot kernels, one counter group per run.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/${1:-pmc3}; mkdir -p $O
python -c "import __graft_entry__ as g; g.build()" > $O/build.log 2>&1 || { echo build failed; exit 1; }
i=0
for ctr in "MeanOccupancyPerCU VALUBusy" "VALUUtilization MemUnitStalled" "LDSBankConflict LdsUtil" "SQ_IFETCH SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVES" "OccupancyPercent SALUBusy"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $ctr --output-format csv -d $O/g$i -o run -- python3 bench.py --steps 1 --warmup 1 --batch 8 --gop 4 > $O/g$i.log 2>&1 || { echo "group $i failed"; tail -n 5 $O/g$i.log; exit 1; }
  echo "== $ctr"
  for k in k_inter_me k_inter_recon k_intra_analysis k_intra_recon k_phase_planes k_synth; do python3 tools/pmcsum.py $O/g$i/run_counter_collection.csv $k; done
done
