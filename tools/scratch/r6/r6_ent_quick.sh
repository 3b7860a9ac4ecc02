#!/bin/bash
# Round 6 coder iteration: GPU entropy tests, then the GPU coder on smooth / textured (debug
# counters on), first failure ends it.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-r6entq}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_entropy.py -x -v --timeout 120 --timeout-method thread > $O/pytest_ent.log 2>&1
rc=$?; echo "pytest_ent rc=$rc"; tail -n 3 $O/pytest_ent.log; [ $rc -eq 0 ] || exit $rc
one() { n=$1; shift; timeout -k 10 300 env "$@" > $O/$n.log 2>&1 || { echo "$n failed"; tail -n 5 $O/$n.log; exit 1; }
  python3 -c "import json; r=json.loads([l for l in open('$O/$n.log') if l.startswith('{')][-1]); c=r['config']; print('$n', r['value'], c.get('psnr_y_db'), c.get('kbps_per_30fps_stream'), c['per_rank_cpu'][0]['busy_cores'], c.get('entropy'))"; grep "tv entropy" $O/$n.log | head -1; }
one gpu_smooth TV_ENT_DEBUG=1 python -u bench.py --no-4k --steps 5 --warmup 2 --entropy gpu
one gpu_tex TV_ENT_DEBUG=1 python -u bench.py --no-4k --steps 4 --warmup 2 --entropy gpu --content textured
one gpu_serial TV_ENT_SERIAL=1 TV_ENT_DEBUG=1 python -u bench.py --no-4k --steps 3 --warmup 1 --entropy gpu
