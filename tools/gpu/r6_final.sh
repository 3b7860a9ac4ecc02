#!/bin/bash
# Round-6 end-of-round checkpoint: whole GPU suite + smoke, the default bench (1080p + 4K),
# GPU-CABAC bench, B8 (hierarchical-B quality mode), AV1 4K, the y4m and synthetic node jobs,
# a single-group kernel trace.  First failure ends it.  Usage: r6_final.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD TV_NO_AUTOBUILD=1
O=gpurun_out/${1:-r6final}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
run() { n=$1; shift; timeout -k 10 600 python -u bench.py "$@" > $O/$n.log 2>&1 || { echo "$n failed"; tail -n 5 $O/$n.log; exit 1; }
  python3 -c "import json; L=[l for l in open('$O/$n.log') if l.startswith('{')]; r=json.loads(L[-1]); c=r['config']; print('$n', r['value'], c.get('fps_4k'), c.get('psnr_y_db'), c.get('kbps_per_30fps_stream'))"; }
run bench --steps 10 --warmup 3
run bench_gpuent --no-4k --steps 6 --warmup 2 --entropy gpu
run bench_b8 --no-4k --steps 6 --warmup 2 --bframes 8
run bench_av1_4k --codec av1 --res 4k --steps 4 --warmup 2
run job_y4m --job --source y4m
run job_synth --job
TV_ENGINE_GROUPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/g1 -o run -- python3 bench.py --no-4k --steps 3 --warmup 1 > $O/g1.log 2>&1 || { echo "prof failed"; tail -n 20 $O/g1.log; exit 1; }
python3 tools/profsum.py $(find $O/g1 -name "*kernel_trace.csv" | head -1) --skip 0.4 > $O/g1_summary.txt 2>&1 || true
head -n 12 $O/g1_summary.txt
