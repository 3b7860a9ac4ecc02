#!/bin/bash
# Per-rank CPU share rehearsal + the host-dependence checks of item 1:
# 1-GPU bench smooth / textured uncapped, at TV_CPUS = nproc/8 (one rank's share of an 8-GPU
# node) and at TV_CPUS=8; synthetic and y4m end-to-end jobs.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-share}; mkdir -p $O
SHARE=$(( $(nproc) / 8 ))
echo "nproc $(nproc) share $SHARE"
one() {  # name, cpus (0 = uncapped), bench args...
  local n=$1 c=$2; shift 2
  TV_CPUS=$c timeout -k 10 400 python -u bench.py --steps 4 --warmup 2 --no-4k "$@" > $O/$n.json.log 2>&1
  local rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/$n.json.log; return $rc; }
  grep '^{' $O/$n.json.log | tail -1 > $O/$n.json
  python3 -c "import json; r=json.load(open('$O/$n.json')); c=r['config']; print('$n', r['value'], c.get('per_rank_cpu',[{}])[0], c.get('step_ms'), c.get('entropy'))"
}
one smooth_uncapped 0 && one smooth_share $SHARE && one textured_uncapped 0 --content textured && \
one textured_share $SHARE --content textured && one textured_cpus8 8 --content textured && \
one smooth_host_share $SHARE --entropy host && one textured_host_share $SHARE --content textured --entropy host && \
one job_synth 0 --job && one job_y4m 0 --job --source y4m && one job_y4m_share $SHARE --job --source y4m
