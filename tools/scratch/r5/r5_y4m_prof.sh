#!/bin/bash
# y4m file job under a kernel trace: kernel summary + GPU busy fraction over the job
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-y4mprof}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --job --source y4m > $O/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/prof.log; exit $rc; }
grep '^{' $O/prof.log | tail -1 | cut -c1-200
python3 tools/kstats.py $(find $O/prof -name "*kernel_stats.csv" | head -1) 14 | tee $O/kernel_summary.txt
ls $O/prof
