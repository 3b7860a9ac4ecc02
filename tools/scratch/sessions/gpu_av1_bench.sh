#!/bin/bash
# AV1 benches (1080p, 4K) + a rocprofv3 kernel-stats run of the 1080p AV1 bench.  Usage: gpu_av1_bench.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONPATH=$PWD TMPDIR=/tmp
tag=${1:-av1b}; shift
O=gpurun_out/$tag; mkdir -p $O
for args in "--codec av1" "--codec av1 --res 4k" "$@"; do
  t=$(echo "$args" | tr -d ' -')
  timeout -k 10 400 python bench.py --steps 4 --warmup 2 $args > $O/bench_$t.log 2>&1 || { echo "bench $args failed"; tail -n 20 $O/bench_$t.log; exit 1; }
  echo "bench [$args]: $(tail -n 1 $O/bench_$t.log | cut -c1-900)"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --codec av1 --steps 3 --warmup 1 > $O/prof_bench.log 2>&1 || { echo "prof failed"; tail -n 20 $O/prof_bench.log; exit 1; }
python3 tools/kstats.py $(find $O/prof -name "*kernel_stats.csv" | head -1) 16
