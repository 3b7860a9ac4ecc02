#!/bin/bash
# SAO kernel phase costs: single-group kernel stats with TV_DIAG_SAO_STOP = 1 (staging), 2
# (+ statistics), 3 (+ decision), 0 (+ filter output).  Timing only.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD TV_ENGINE_GROUPS=1
O=gpurun_out/${1:-sao_diag}; mkdir -p $O
for d in 1 2 3 0; do
  TV_DIAG_SAO_STOP=$d timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/d$d -o run -- python3 bench.py --steps 2 --warmup 1 > $O/d$d.log 2>&1 || { echo "diag $d failed"; tail -n 5 $O/d$d.log; exit 1; }
  echo "stop=$d $(grep k_sao_decide $(find $O/d$d -name '*kernel_stats.csv') | awk -F, '{print $2, $4}')"
done
