#!/bin/bash
# rocprofv3 kernel trace + summary of a short 1080p bench (GPU entropy path).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-entprof}; shift; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-4k "$@" > $O/prof_bench.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/prof_bench.log; exit $rc; }
python3 tools/kstats.py $(find $O/prof -name "*kernel_stats.csv" | head -1) 18 | tee $O/kernel_summary.txt
