#!/bin/bash
# Timing breakdown of k_inter_me by phase (TV_DIAG_ME_STOP=1 staging, 2 +integer search,
# 3 +half-pel; 0 full).  Early exits corrupt decisions: timing only, never a result.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-me_diag}; mkdir -p $O
for st in 1 2 3 0; do
  TV_DIAG_ME_STOP=$st timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/s$st -o run -- python3 bench.py --steps 2 --warmup 1 > $O/s$st.log 2>&1 || { echo "stop $st failed"; tail -5 $O/s$st.log; exit 1; }
  echo "== stop $st"; python3 tools/profsum.py $(find $O/s$st -name "*kernel_trace.csv" | head -1) --skip 0.5 | grep -E "k_inter_me|k_phase|k_inter_recon"
done
