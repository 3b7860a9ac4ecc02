#!/bin/bash
# GPU CABAC with one / two entropy lanes per core (smooth + textured), and the per-rank CPU
# share of an 8-GPU 128-CPU node (TV_CPUS=16, entropy auto -> host writer)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-lanes}; mkdir -p $O
one() {  # name, env..., -- bench args
  local n=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 400 python -u bench.py --steps 4 --warmup 2 --no-4k "$@" > $O/$n.log 2>&1
  local rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/$n.log; return $rc; }
  grep '^{' $O/$n.log | tail -1 > $O/$n.json
  python3 -c "import json; r=json.load(open('$O/$n.json')); c=r['config']; print('$n', r['value'], c['per_rank_cpu'][0], c['step_ms'], c['entropy'])"
}
one smooth_l1 TV_ENT_LANES=1 -- --entropy gpu && one smooth_l2 TV_ENT_LANES=2 -- --entropy gpu && \
one textured_l2 TV_ENT_LANES=2 -- --entropy gpu --content textured
