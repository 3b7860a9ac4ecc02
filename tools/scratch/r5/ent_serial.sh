#!/bin/bash
# Coder counters with the entropy stage serialised on the main stream (nothing else running
# while the coder runs) vs overlapped.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-entser}; mkdir -p $O
TV_ENT_SERIAL=1 TV_ENT_DEBUG=1 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-4k > $O/serial.log 2>&1
rc=$?; echo "serial rc=$rc"; grep "tv entropy" $O/serial.log; [ $rc -eq 0 ] || exit $rc
python3 -c "import json; r=json.loads([l for l in open('$O/serial.log') if l.startswith('{')][-1]); c=r['config']; print('serial', r['value'], c['last_step_gpu_ms'], c['step_ms'])"
