#!/bin/bash
# 1080p bench, GPU vs host entropy (same bytes), plus a kernel profile of the host-entropy run
# (the main-stream kernels without the entropy kernels competing for the CUs).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-cmpent}; mkdir -p $O
for e in gpu host; do
  timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 --no-4k --entropy $e > $O/bench_$e.log 2>&1
  rc=$?; echo "bench $e rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/bench_$e.log; exit $rc; }
  python3 -c "import json; r=json.loads([l for l in open('$O/bench_$e.log') if l.startswith('{')][-1]); c=r['config']; print('$e', r['value'], c['per_rank_cpu'][0], c['last_step_gpu_ms'], c['step_ms'])"
done
bash tools/gpu/ent_prof.sh ${1:-cmpent}/prof_host --entropy host
