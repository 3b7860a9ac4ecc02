#!/bin/bash
# SAO iteration: HEVC engine tests (SAO bit-exact), SAO phase timing (stop 2 / full), bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-sao_iter}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_bframes.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for d in 2 0; do
  TV_ENGINE_GROUPS=1 TV_DIAG_SAO_STOP=$d timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/d$d -o run -- python3 bench.py --steps 2 --warmup 1 > $O/d$d.log 2>&1 || { echo "diag $d failed"; exit 1; }
done
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/bench.log 2>&1 || { tail -n 5 $O/bench.log; exit 1; }
python -c "import json; r=json.loads([l for l in open('$O/bench.log') if l.startswith('{')][-1]); print('bench', r['value'], r['config']['psnr_y_db'], r['config']['kbps_per_30fps_stream'], r['config']['per_rank_cpu'][0]['busy_cores'])"
