#!/bin/bash
# Round 6: k_sao_decide phase costs (TV_DIAG_SAO_STOP=1/2/3 stop after staging / statistics /
# decision; timing only) from single-group kernel traces.  Usage: r6_sao_phases.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONPATH=$PWD TMPDIR=/tmp TV_NO_AUTOBUILD=1 TV_ENGINE_GROUPS=1
O=gpurun_out/${1:-r6sao}; mkdir -p $O
for st in 0 1 2 3; do
  TV_DIAG_SAO_STOP=$st timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/s$st -o run -- python3 bench.py --no-4k --steps 2 --warmup 1 > $O/s$st.log 2>&1 || { echo "stop $st failed"; tail -n 5 $O/s$st.log; exit 1; }
  echo "== stop $st"; python3 tools/profsum.py $(find $O/s$st -name "*kernel_trace.csv" | head -1) --skip 0.3 2>&1 | grep -E "sao|inter_me" 
done 2>&1 | tee $O/summary.txt
