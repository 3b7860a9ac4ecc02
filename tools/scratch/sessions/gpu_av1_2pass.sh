#!/bin/bash
# AV1 2-pass (BASELINE config #4 rate control) at 4K and 1080p after the writer changes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-av1_2pass}; mkdir -p $O
run() { n=$1; shift; timeout -k 10 500 python -u bench.py "$@" > $O/$n.log 2>&1 || { echo "$n failed"; tail -n 5 $O/$n.log; exit 1; }
  python -c "import json; r=json.loads([l for l in open('$O/$n.log') if l.startswith('{')][-1]); c=r['config']; print('$n', r['value'], c.get('psnr_y_db'), c.get('kbps_per_30fps_stream'), c.get('kbps_error_pct'), c['per_rank_cpu'][0]['busy_cores'], c.get('step_ms'))"; }
run av1_4k_2pass --codec av1 --res 4k --kbps 20000 --steps 4 --warmup 2
run av1_1080p_2pass --codec av1 --kbps 6000 --steps 6 --warmup 2
run av1_1080p --codec av1 --steps 6 --warmup 2
