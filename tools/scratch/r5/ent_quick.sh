#!/bin/bash
# GPU entropy quick loop: entropy + engine golden tests, then the coder counters and a short
# bench (1080p only).  First failure ends it.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-entq}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_entropy.py tests/test_gpu_engine.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
TV_ENT_DEBUG=1 timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 --no-4k > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep "tv entropy" $O/bench.log; [ $rc -eq 0 ] || exit $rc
python3 -c "import json; r=json.loads([l for l in open('$O/bench.log') if l.startswith('{')][-1]); c=r['config']; print('bench', r['value'], c['psnr_y_db'], c['kbps_per_30fps_stream'], c['per_rank_cpu'][0], c['entropy'], c['last_step_gpu_ms'], c['step_ms'])"
