#!/bin/bash
# RDOQ-lite: GPU suite, same-box bench A/B (--no-rdoq vs default), then the 1080p RD points
# of the default and of --no-rdoq against round 5's cascaded default.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-r6_rdoq4}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for m in off on; do
    f=""; [ $m = off ] && f="--no-rdoq"
    timeout -k 10 300 python -u bench.py --no-4k --steps 10 --warmup 3 $f > $O/ab_${m}_$i.log 2>&1 || { echo "ab $m failed"; tail -n 5 $O/ab_${m}_$i.log; exit 1; }
    grep '^{' $O/ab_${m}_$i.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); c=r['config']; print('ab $m', r['value'], c['last_step_gpu_ms'], c['psnr_y_db'], c['kbps_per_30fps_stream'], c['coding_tools'])"
  done
done
[ "${RD:-1}" = 0 ] && exit 0
bash tools/gpu/rd_vs.sh ${1:-r6_rdoq4}/rd_on && bash tools/gpu/rd_vs.sh ${1:-r6_rdoq4}/rd_off profiles/r5_rd_cascade_1080p --no-rdoq
