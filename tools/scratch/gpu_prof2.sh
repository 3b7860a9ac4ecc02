#!/bin/bash
# Kernel-time profile of the default bench + derived counters of the hot kernels.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/${1:-prof2}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --steps 3 --warmup 2 > $O/trace.log 2>&1 || { echo "trace failed"; tail -n 5 $O/trace.log; exit 1; }
echo "== kernel time (warm window)"; python3 tools/profsum.py $O/trace/run_kernel_trace.csv --skip 0.5 --top 16 | tee $O/warm_summary.txt
i=0
for ctr in "MeanOccupancyPerCU VALUBusy" "VALUUtilization MemUnitStalled" "LDSBankConflict LdsUtil" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAVES" "SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $ctr --output-format csv -d $O/g$i -o run -- python3 bench.py --steps 1 --warmup 1 --batch 16 --gop 4 > $O/g$i.log 2>&1 || { echo "group $i failed"; tail -n 5 $O/g$i.log; exit 1; }
  echo "== $ctr"
  for k in k_inter_me k_inter_recon k_intra_analysis k_intra_recon k_phase_planes k_synth k_deblock; do python3 tools/pmcsum.py $O/g$i/run_counter_collection.csv $k; done
done 2>&1 | tee $O/counters.txt
