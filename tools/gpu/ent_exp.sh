#!/bin/bash
# entropy contention experiments (timing only): 1080p step time with the coder / binariser
# skipped (TV_ENT_SKIP, wrong bytes), and with a high-priority main stream.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-entexp}; mkdir -p $O
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 --no-4k > $O/bench_$n.log 2>&1
  local rc=$?; echo "bench $n rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/bench_$n.log; return $rc; }
  python3 -c "import json; r=json.loads([l for l in open('$O/bench_$n.log') if l.startswith('{')][-1]); c=r['config']; print('$n', r['value'], c['per_rank_cpu'][0]['busy_cores'], c['last_step_gpu_ms'], c['step_ms'], c['entropy'])"
}
run base TV_X=0 && run synthtok TV_ENT_SKIP=512
