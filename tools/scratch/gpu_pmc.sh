#!/bin/bash
# Hardware counters (rocprofv3 --pmc, no trace domains) for one short bench run.
# Usage: gpu_pmc.sh <tag> "<counters>" [bench args]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
tag=$1; shift; ctrs=$1; shift
mkdir -p gpurun_out/$tag
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/$tag/build.log 2>&1 || exit 1
[ -f gpurun_out/counters.txt ] || rocprofv3 -L > gpurun_out/counters.txt 2>&1
timeout -k 10 300 rocprofv3 --pmc $ctrs --output-format csv -d gpurun_out/$tag/pmc -o run -- python3 bench.py --steps 1 --warmup 0 "$@" > gpurun_out/$tag/pmc.log 2>&1
echo "pmc rc=$?"
