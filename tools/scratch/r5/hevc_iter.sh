#!/bin/bash
# HEVC kernel iteration: bit-exact engine tests, then hevc_prof.sh (single-group kernel stats +
# counter passes), then the default bench.  Usage: hevc_iter.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-hevciter}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_bframes.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu/hevc_prof.sh ${1:-hevciter}/prof || exit 1
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-4k > $O/bench.log 2>&1 || { tail -n 5 $O/bench.log; exit 1; }
python3 -c "import json; r=json.loads([l for l in open('$O/bench.log') if l.startswith('{')][-1]); print('bench', r['value'], r['config']['psnr_y_db'], r['config']['kbps_per_30fps_stream'], r['config']['per_rank_cpu'][0]['busy_cores'])"
