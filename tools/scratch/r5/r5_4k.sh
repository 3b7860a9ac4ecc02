#!/bin/bash
# the default run (1080p then 4K in one process) after the D2H-stream fix
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-g4k}; mkdir -p $O
timeout -k 10 400 python -u bench.py --steps 8 --warmup 2 > $O/default.log 2>&1
rc=$?; echo "default rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/default.log; exit $rc; }
python3 -c "import json; r=json.loads([l for l in open('$O/default.log') if l.startswith('{')][-1]); c=r['config']; print('default', r['value'], 'fps_4k', c.get('fps_4k'), c['per_rank_cpu'][0], c['step_ms'][:3], c.get('step_ms_4k')[:3])"
TV_ENTROPY=gpu timeout -k 10 400 python -u bench.py --steps 8 --warmup 2 > $O/default_gpu.log 2>&1
rc=$?; echo "default gpu-entropy rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/default_gpu.log; exit $rc; }
python3 -c "import json; r=json.loads([l for l in open('$O/default_gpu.log') if l.startswith('{')][-1]); c=r['config']; print('default gpu entropy', r['value'], 'fps_4k', c.get('fps_4k'), c['per_rank_cpu'][0], c['step_ms'][:3], c.get('step_ms_4k')[:3])"
