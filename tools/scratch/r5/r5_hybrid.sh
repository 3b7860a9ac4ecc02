#!/bin/bash
# Hybrid entropy under a CPU cap: the GPU coder plus up to TV_ENT_HOST pictures at a time in
# the host writer, textured + smooth 1080p at TV_CPUS=8.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-hybrid}; mkdir -p $O
one() {  # name, env..., -- bench args
  local n=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 --no-4k "$@" > $O/$n.log 2>&1
  local rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/$n.log; return $rc; }
  grep '^{' $O/$n.log | tail -1 > $O/$n.json
  python3 -c "import json; r=json.load(open('$O/$n.json')); c=r['config']; print('$n', r['value'], c['per_rank_cpu'][0], c['step_ms'], c['entropy'])"
}
one tex_h0 TV_CPUS=8 TV_ENT_HOST=0 -- --entropy gpu --content textured && \
one tex_h2 TV_CPUS=8 TV_ENT_HOST=2 -- --entropy gpu --content textured && \
one tex_h4 TV_CPUS=8 TV_ENT_HOST=4 -- --entropy gpu --content textured && \
one tex_h8 TV_CPUS=8 TV_ENT_HOST=8 -- --entropy gpu --content textured && \
one smo_h0 TV_CPUS=8 TV_ENT_HOST=0 -- --entropy gpu && \
one smo_h2 TV_CPUS=8 TV_ENT_HOST=2 -- --entropy gpu && \
one smo_h4 TV_CPUS=8 TV_ENT_HOST=4 -- --entropy gpu
