#!/bin/bash
# Host-wait A/B on the default bench (TV_SYNC_MODE spin / poll / block, alternating), then
# the AV1 1080p bench.  First failure ends it.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-sync_ab}; mkdir -p $O
for r in 1 2; do
  for m in spin poll block; do
    TV_SYNC_MODE=$m timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 > $O/bench_${m}_$r.log 2>&1 || { echo "bench $m failed"; tail -n 5 $O/bench_${m}_$r.log; exit 1; }
    python -c "import json,sys; r=json.loads([l for l in open('$O/bench_${m}_$r.log') if l.startswith('{')][-1]); print('$m', r['value'], r['config']['per_rank_cpu'][0]['busy_cores'])"
  done
done
timeout -k 10 300 python -u bench.py --codec av1 --steps 6 --warmup 2 > $O/bench_av1.log 2>&1; rc=$?; tail -n 1 $O/bench_av1.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
