#!/bin/bash
# End-to-end job benches (add_job -> DONE through the node executor), HEVC and AV1.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-job}; mkdir -p $O
run() { n=$1; shift; timeout -k 10 500 python -u bench.py "$@" > $O/$n.log 2>&1 || { echo "$n failed"; tail -n 8 $O/$n.log; exit 1; }
  python -c "import json; r=json.loads([l for l in open('$O/$n.log') if l.startswith('{')][-1]); c=r['config']; print('$n', r['value'], {k: c.get(k) for k in ('frames', 'psnr_y_db', 'kbps_per_30fps_stream', 'engine_fps', 'rank0_spans_ms')})"; }
run job_hevc --job
run job_av1 --job --codec av1
