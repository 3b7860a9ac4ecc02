#!/bin/bash
# GPU suite + default bench + single-group kernel stats (k_synth).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-synth_iter}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 > $O/bench.log 2>&1 || { echo "bench failed"; exit 1; }
python -c "import json; r=json.loads([l for l in open('$O/bench.log') if l.startswith('{')][-1]); print('bench', r['value'], r['config']['psnr_y_db'], r['config']['per_rank_cpu'][0]['busy_cores'])"
TV_ENGINE_GROUPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/d0 -o run -- python3 bench.py --steps 3 --warmup 1 > $O/prof.log 2>&1 || { echo "prof failed"; exit 1; }
python3 tools/profsum.py $O/d0/run_kernel_stats.csv | head -12
