#!/bin/bash
# Kernel-time breakdown + motion-search stage ablation (TV_ME_ABLATE; output invalid).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/${1:-meabl}; mkdir -p $O
for abl in 0 1 2 3; do
  TV_ME_ABLATE=$abl timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/a$abl -o run -- python3 bench.py --steps 2 --warmup 2 > $O/a$abl.log 2>&1 || { echo "abl $abl failed"; tail -n 5 $O/a$abl.log; exit 1; }
  echo "== ablate $abl"; python3 tools/profsum.py $O/a$abl/run_kernel_trace.csv --skip 0.55 --top 8
done
