#!/bin/bash
# Round 6 coder A/B on one box: default bench (1080p smooth, GPU coder) under coder / lane /
# slot variants given as "name:ENV=V,ENV=V" arguments.  First failure ends it.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-r6ab}; mkdir -p $O; shift
EXTRA=${BENCH_EXTRA:-}
for spec in "$@"; do
  n=${spec%%:*}; envs=${spec#*:}; envs=${envs//,/ }
  timeout -k 10 300 env $envs TV_ENT_DEBUG=1 python -u bench.py --no-4k --steps 4 --warmup 2 --entropy gpu $EXTRA > $O/$n.log 2>&1 || { echo "$n failed"; tail -n 5 $O/$n.log; exit 1; }
  python3 -c "import json; r=json.loads([l for l in open('$O/$n.log') if l.startswith('{')][-1]); c=r['config']; print('$n', r['value'], c['per_rank_cpu'][0]['busy_cores'], c['entropy']['lane_pictures'])"
  grep "tv entropy" $O/$n.log | head -1
done
