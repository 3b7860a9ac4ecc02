#!/bin/bash
# GPU entropy iteration: its tests, the engine golden tests, a rocprofv3 kernel summary of a
# short 1080p bench, then the default bench.  First failure ends it.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-ent}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_entropy.py tests/test_gpu_engine.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-4k > $O/prof_bench.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/kstats.py $(find $O/prof -name "*kernel_stats.csv" | head -1) 16 | tee $O/kernel_summary.txt
timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"
python3 -c "import json; r=json.loads([l for l in open('$O/bench.log') if l.startswith('{')][-1]); c=r['config']; print('bench', r['value'], c.get('fps_4k'), c['psnr_y_db'], c['kbps_per_30fps_stream'], c['per_rank_cpu'][0], c['entropy'], c['last_step_gpu_ms'])"
