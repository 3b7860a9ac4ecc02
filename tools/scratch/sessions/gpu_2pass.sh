#!/bin/bash
# HEVC 2-pass (fast first pass one step ahead on a second engine) + 1-pass default check.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-hevc_2pass}; mkdir -p $O
run() { n=$1; shift; timeout -k 10 500 python -u bench.py "$@" > $O/$n.log 2>&1 || { echo "$n failed"; tail -n 5 $O/$n.log; exit 1; }
  python -c "import json; r=json.loads([l for l in open('$O/$n.log') if l.startswith('{')][-1]); c=r['config']; print('$n', r['value'], c.get('psnr_y_db'), c.get('kbps_per_30fps_stream'), c.get('kbps_error_pct'), c['per_rank_cpu'][0]['busy_cores'], c.get('rc_steps_actual_wanted_offset'))"; }
run hevc_2pass --kbps 2000 --steps 8 --warmup 2
run hevc_b8_2pass --bframes 8 --kbps 1500 --steps 6 --warmup 2
run bench --steps 6 --warmup 2
