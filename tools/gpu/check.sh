#!/bin/bash
# Session checkpoint: whole GPU suite + smoke, default bench (10 steps), 4K, B8, B8 2-pass,
# AV1 4K.  First failure ends it.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-check3}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
run() { n=$1; shift; timeout -k 10 400 python -u bench.py "$@" > $O/$n.log 2>&1 || { echo "$n failed"; tail -n 5 $O/$n.log; exit 1; }
  python -c "import json; r=json.loads([l for l in open('$O/$n.log') if l.startswith('{')][-1]); c=r['config']; print('$n', r['value'], c.get('psnr_y_db'), c.get('kbps_per_30fps_stream'), c.get('kbps_error_pct'), c['per_rank_cpu'][0]['busy_cores'])"; }
run bench --steps 10 --warmup 3
run bench_4k --res 4k --steps 4 --warmup 1
run bench_b8 --bframes 8 --steps 6 --warmup 2
run bench_b8_2pass --bframes 8 --kbps 1500 --steps 4 --warmup 2
run bench_av1_4k --codec av1 --res 4k --steps 4 --warmup 1
