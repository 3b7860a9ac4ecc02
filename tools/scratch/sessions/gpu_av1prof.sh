#!/bin/bash
# rocprofv3 kernel stats of the AV1 1080p bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-av1prof}; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --codec av1 --steps 2 --warmup 1 > $O/bench.log 2>&1; rc=$?; echo "prof rc=$rc"; tail -n 1 $O/bench.log | cut -c1-300
