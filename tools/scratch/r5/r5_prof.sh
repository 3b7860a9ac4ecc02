#!/bin/bash
# Round-5 shipped configuration (host entropy via auto, QP cascade): kernel summary of the
# 1080p bench, then LDS-conflict / MFMA counters of the hot kernels (one group per run).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD TV_NO_AUTOBUILD=1
O=gpurun_out/${1:-r5prof}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-4k > $O/prof_bench.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/prof_bench.log; exit $rc; }
python3 tools/kstats.py $(find $O/prof -name "*kernel_stats.csv" | head -1) 22 | tee $O/kernel_summary.txt
i=0
for ctr in "LDSBankConflict LdsUtil" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAVES" "VALUBusy MeanOccupancyPerCU"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $ctr --output-format csv -d $O/g$i -o run -- python3 bench.py --steps 1 --warmup 1 --batch 16 --gop 8 --no-4k > $O/g$i.log 2>&1 || { echo "group $i failed"; tail -n 5 $O/g$i.log; exit 1; }
  echo "== $ctr"
  for k in k_inter_me k_inter_recon k_sao_decide k_phase_planes k_synth; do python3 tools/pmcsum.py $(find $O/g$i -name "*counter_collection.csv" | head -1) $k; done
done 2>&1 | tee $O/pmc_summary.txt
