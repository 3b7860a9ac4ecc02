#!/bin/bash
# Round-5 "before" numbers for the GPU entropy work: default bench (1080p + 4K), then smooth
# and textured 1080p with the CPU share an 8-GPU node gives one rank (TV_CPUS=8 / 4).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-r5base}; mkdir -p $O
nproc > $O/nproc.txt; python -c "import os; print(len(os.sched_getaffinity(0)))" >> $O/nproc.txt
summ() { python3 -c "import json,sys; r=json.loads([l for l in open('$O/$1.log') if l.startswith('{')][-1]); c=r['config']; print('$1', r['value'], c.get('fps_4k'), c.get('psnr_y_db'), c.get('kbps_per_30fps_stream'), c['per_rank_cpu'][0])"; }
run() { n=$1; shift; timeout -k 10 400 python -u bench.py "$@" > $O/$n.log 2>&1 || { echo "$n failed"; tail -n 5 $O/$n.log; exit 1; }; summ $n; }
run bench --steps 8 --warmup 2
TV_CPUS=8 run smooth_c8 --no-4k --steps 6 --warmup 2
TV_CPUS=8 run tex_c8 --content textured --no-4k --steps 6 --warmup 2
run tex_c0 --content textured --no-4k --steps 6 --warmup 2
