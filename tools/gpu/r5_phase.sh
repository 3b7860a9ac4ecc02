#!/bin/bash
# Phase planes: 64-column tiles (dwordx2 stores) vs the 32-column tiles (TV_PHASE_COLS=4):
# GPU golden tests, the default 1080p bench both ways, then a kernel summary.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD TV_NO_AUTOBUILD=1
O=gpurun_out/${1:-phase}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for v in 4 8 4 8; do
  TV_PHASE_COLS=$v timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 > $O/bench_c$v.log 2>&1
  rc=$?; echo "bench cols=$v rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/bench_c$v.log; exit $rc; }
  grep '^{' $O/bench_c$v.log | tail -1 | python3 -c "import json,sys; r=json.load(sys.stdin); c=r['config']; print('cols $v', r['value'], c.get('fps_4k'), c['step_ms'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-4k > $O/prof_bench.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/prof_bench.log; exit $rc; }
python3 tools/kstats.py $(find $O/prof -name "*kernel_stats.csv" | head -1) 12 | tee $O/kernel_summary.txt
