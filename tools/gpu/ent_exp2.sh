#!/bin/bash
# WPP poll back-off: step time + coder counters (wait per row) at 1080p
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-entexp2}; mkdir -p $O
for n in dbg plain; do
  if [ $n = dbg ]; then export TV_ENT_DEBUG=1; else unset TV_ENT_DEBUG; fi
  timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 --no-4k > $O/bench_$n.log 2>&1
  rc=$?; echo "bench $n rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/bench_$n.log; exit $rc; }
  grep "tv entropy" $O/bench_$n.log | tail -1
  python3 -c "import json; r=json.loads([l for l in open('$O/bench_$n.log') if l.startswith('{')][-1]); c=r['config']; print('$n', r['value'], c['per_rank_cpu'][0]['busy_cores'], c['last_step_gpu_ms'], c['step_ms'], c['entropy'])"
done
