#!/bin/bash
# Kernel-time sweep: rocprofv3 kernel stats for several bench configs.  Usage: gpu_sweep.sh <tag> "<args1>" "<args2>" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
tag=$1; shift
mkdir -p gpurun_out/$tag
[ -n "$SKIP_BUILD" ] || python -c "import __graft_entry__ as g; g.build()" > gpurun_out/$tag/build.log 2>&1 || exit 1
i=0
for a in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$tag/p$i -o run -- python3 bench.py --steps 1 --warmup 0 $a > gpurun_out/$tag/p$i.log 2>&1 || { echo "run $i failed"; exit 1; }
  echo "== $a"; tail -1 gpurun_out/$tag/p$i.log | cut -c1-120
  python3 tools/profsum.py gpurun_out/$tag/p$i/run_kernel_stats.csv | head -4
done
