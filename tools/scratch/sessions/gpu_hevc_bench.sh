#!/bin/bash
# HEVC benches: the shipped default (GOP 64, SAO on), the round-2 headline config, 4K; then a
# rocprofv3 kernel-stats run of the default.  Usage: gpu_hevc_bench.sh <tag> [extra bench arg sets...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONPATH=$PWD TMPDIR=/tmp
tag=${1:-hevcb}; shift
O=gpurun_out/$tag; mkdir -p $O
for args in "" "--gop 16 --no-sao" "--res 4k" "$@"; do
  [ -z "$args" ] && t=default || t=$(echo "$args" | tr -d ' -')
  timeout -k 10 400 python bench.py --steps 3 --warmup 1 $args > $O/bench_$t.log 2>&1 || { echo "bench $args failed"; tail -n 20 $O/bench_$t.log; exit 1; }
  echo "bench [$args]: $(tail -n 1 $O/bench_$t.log | cut -c1-1200)"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 2 --warmup 1 > $O/prof_bench.log 2>&1 || { echo "prof failed"; tail -n 20 $O/prof_bench.log; exit 1; }
python3 tools/kstats.py $(find $O/prof -name "*kernel_stats.csv" | head -1) 20
