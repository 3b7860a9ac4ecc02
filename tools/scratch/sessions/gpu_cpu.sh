#!/bin/bash
# Host-CPU check after writer changes: default bench uncapped and at TV_CPUS=12 / 8, B8.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-cpu}; mkdir -p $O
run() { n=$1; shift; timeout -k 10 400 env "$@" > $O/$n.log 2>&1 || { echo "$n failed"; tail -n 5 $O/$n.log; exit 1; }
  python -c "import json; r=json.loads([l for l in open('$O/$n.log') if l.startswith('{')][-1]); c=r['config']; print('$n', r['value'], c.get('psnr_y_db'), c.get('kbps_per_30fps_stream'), c['per_rank_cpu'][0]['busy_cores'])"; }
run bench python -u bench.py --steps 10 --warmup 3
run cpus12 TV_CPUS=12 python -u bench.py --steps 10 --warmup 3
run cpus8 TV_CPUS=8 python -u bench.py --steps 10 --warmup 3
run bench_b8 python -u bench.py --bframes 8 --steps 6 --warmup 2
run bench_textured python -u bench.py --content textured --steps 6 --warmup 2
