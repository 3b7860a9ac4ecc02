#!/bin/bash
# GPU CABAC with 1 / 2 / 4 substream rows per wave (TV_ENT_ROWS_PER_WAVE), smooth + textured
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-rows}; mkdir -p $O
one() {  # name, env..., -- bench args
  local n=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 --no-4k "$@" > $O/$n.log 2>&1
  local rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/$n.log; return $rc; }
  grep '^{' $O/$n.log | tail -1 > $O/$n.json
  python3 -c "import json; r=json.load(open('$O/$n.json')); c=r['config']; print('$n', r['value'], c['per_rank_cpu'][0], c['step_ms'], c['entropy'])"
}
one smooth_r1 TV_ENT_ROWS_PER_WAVE=1 -- --entropy gpu && one smooth_r2 TV_ENT_ROWS_PER_WAVE=2 -- --entropy gpu && \
one smooth_r4 TV_ENT_ROWS_PER_WAVE=4 -- --entropy gpu && \
one textured_r1 TV_ENT_ROWS_PER_WAVE=1 -- --entropy gpu --content textured && \
one textured_r2 TV_ENT_ROWS_PER_WAVE=2 -- --entropy gpu --content textured
