#!/bin/bash
# In-process 4K pass (the driver's default run: 1080p then 4K in one process) against a
# standalone 4K run, same K / W; then the DVD-title job bench (MPEG-2 decode + bwdif + HEVC).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-gap}; mkdir -p $O
timeout -k 10 400 python -u bench.py --steps 8 --warmup 2 > $O/default.log 2>&1
rc=$?; echo "default rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/default.log; exit $rc; }
python3 -c "import json; r=json.loads([l for l in open('$O/default.log') if l.startswith('{')][-1]); c=r['config']; print('default', r['value'], 'fps_4k', c.get('fps_4k'), c['per_rank_cpu'][0], c['entropy'], c['step_ms'], c.get('step_ms_4k'))"
timeout -k 10 400 python -u bench.py --steps 8 --warmup 2 --res 4k > $O/4k.log 2>&1
rc=$?; echo "4k rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/4k.log; exit $rc; }
python3 -c "import json; r=json.loads([l for l in open('$O/4k.log') if l.startswith('{')][-1]); c=r['config']; print('standalone 4k', r['value'], c['per_rank_cpu'][0], c['step_ms'])"
timeout -k 10 500 python -u bench.py --job --source mpeg2 > $O/dvd_job.log 2>&1
rc=$?; echo "dvd job rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/dvd_job.log; exit $rc; }
python3 -c "import json; r=json.loads([l for l in open('$O/dvd_job.log') if l.startswith('{')][-1]); c=r['config']; print('dvd job', r['value'], c['job_wall_s'], c['psnr_y_db'], c['kbps'], {k: v['total_ms'] for k, v in c['rank0_spans_ms'].items()})"
