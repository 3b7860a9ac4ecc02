#!/bin/bash
# HEVC engine kernel profile at the shipped config: single-group kernel stats (clean
# per-kernel times) + the LDS / VALU counter passes of the hot kernels.  Usage: hevc_prof.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-hevcprof}; mkdir -p $O
TV_ENGINE_GROUPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/g1 -o run -- python3 bench.py --no-4k --steps 3 --warmup 1 > $O/g1.log 2>&1 || { echo "prof failed"; tail -n 20 $O/g1.log; exit 1; }
python3 tools/profsum.py $(find $O/g1 -name "*kernel_trace.csv" | head -1) --skip 0.4 > $O/g1_summary.txt 2>&1 || true
head -n 20 $O/g1_summary.txt
i=0
for ctr in "LDSBankConflict LdsUtil" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAVES" "MeanOccupancyPerCU VALUBusy"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $O/p$i -o run -- python3 bench.py --no-4k --steps 1 --warmup 1 --batch 16 --gop 8 > $O/p$i.log 2>&1 || { echo "pmc $i failed"; tail -n 5 $O/p$i.log; exit 1; }
  echo "== $ctr"
  for k in k_inter_me k_inter_recon k_sao_decide k_phase_planes k_coarse_me k_synth; do python3 tools/pmcsum.py $(find $O/p$i -name "*counter_collection.csv" | head -1) $k; done
done
