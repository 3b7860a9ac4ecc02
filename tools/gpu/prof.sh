#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run.  Usage: gpu_prof.sh <tag> [bench args]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
tag=$1; shift
mkdir -p gpurun_out/prof_$tag
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- python3 bench.py "$@" > gpurun_out/prof_$tag/bench.log 2>&1
rc=$?
echo "prof rc=$rc"; tail -3 gpurun_out/prof_$tag/bench.log
find gpurun_out/prof_$tag -name "*kernel_stats.csv" -exec head -20 {} \;
