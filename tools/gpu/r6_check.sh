#!/bin/bash
# Round 6 checkpoint: whole GPU suite + smoke, default bench (1080p + 4K), the GPU-coder bench,
# then a single-group kernel-trace profile of the default bench.  First failure ends it.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-r6check}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
run() { n=$1; shift; timeout -k 10 400 python -u bench.py "$@" > $O/$n.log 2>&1 || { echo "$n failed"; tail -n 5 $O/$n.log; exit 1; }
  python3 -c "import json; L=[l for l in open('$O/$n.log') if l.startswith('{')]; [print('$n', r['value'], r['config'].get('resolution'), r['config'].get('psnr_y_db'), r['config'].get('kbps_per_30fps_stream'), r['config']['per_rank_cpu'][0]['busy_cores']) for r in map(json.loads, L)]"; }
run bench --steps 10 --warmup 3
run bench_gpuent --no-4k --steps 6 --warmup 2 --entropy gpu
TV_ENGINE_GROUPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/g1 -o run -- python3 bench.py --no-4k --steps 3 --warmup 1 > $O/g1.log 2>&1 || { echo "prof failed"; tail -n 20 $O/g1.log; exit 1; }
python3 tools/profsum.py $(find $O/g1 -name "*kernel_trace.csv" | head -1) --skip 0.4 > $O/g1_summary.txt 2>&1 || true
head -n 12 $O/g1_summary.txt
