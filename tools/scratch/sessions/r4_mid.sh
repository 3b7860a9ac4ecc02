#!/bin/bash
# Mid-round check: HEVC engine tests (bit-exact), default bench (1080p + 4K), AV1 kernel
# profile (single run, kernel stats), AV1 4K 2-pass accuracy.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-r4mid}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_bframes.py tests/test_av1_codec.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 > $O/bench.log 2>&1 || { tail -n 5 $O/bench.log; exit 1; }
python3 -c "import json; r=json.loads([l for l in open('$O/bench.log') if l.startswith('{')][-1]); c=r['config']; print('bench', r['value'], c['psnr_y_db'], c['kbps_per_30fps_stream'], c['per_rank_cpu'][0]['busy_cores'], '4k', c.get('fps_4k'), c.get('psnr_y_4k'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/av1prof -o run -- python3 bench.py --codec av1 --steps 3 --warmup 1 > $O/av1prof.log 2>&1 || { echo "av1 prof failed"; tail -n 10 $O/av1prof.log; exit 1; }
python3 tools/profsum.py $(find $O/av1prof -name "*kernel_trace.csv" | head -1) --skip 0.4 > $O/av1prof_summary.txt 2>&1 || true
head -n 16 $O/av1prof_summary.txt
timeout -k 10 400 python -u bench.py --codec av1 --res 4k --kbps 20000 --steps 4 --warmup 2 > $O/av1_4k_2pass.log 2>&1 || { echo "av1 2pass failed"; tail -n 5 $O/av1_4k_2pass.log; exit 1; }
python3 -c "import json; r=json.loads([l for l in open('$O/av1_4k_2pass.log') if l.startswith('{')][-1]); c=r['config']; print('av1 4k 2pass', r['value'], c['kbps_error_pct'], c['rc_steps_actual_wanted_offset'])"
