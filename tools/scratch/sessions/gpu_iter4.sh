#!/bin/bash
# HEVC engine tests (incl. B frames) + default bench + single-group kernel stats, then the AV1
# kernel stats.  First failure ends it.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-iter4}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_engine.py tests/test_bframes.py tests/test_parallel.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/bench.log 2>&1 || { tail -n 5 $O/bench.log; exit 1; }
python -c "import json; r=json.loads([l for l in open('$O/bench.log') if l.startswith('{')][-1]); print('bench', r['value'], r['config']['per_rank_cpu'][0]['busy_cores'], r['config']['last_step_coef_mb_d2h'])"
TV_ENGINE_GROUPS=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_p_g1 -o run -- python3 bench.py --steps 2 --warmup 1 > $O/prof_p_g1.log 2>&1; rc=$?; echo "prof ippp rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_av1 -o run -- python3 bench.py --codec av1 --steps 2 --warmup 1 > $O/prof_av1.log 2>&1; rc=$?; echo "prof av1 rc=$rc"
