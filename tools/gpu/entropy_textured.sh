#!/bin/bash
# Host entropy cost on high-bitrate content: the textured bench uncapped and at TV_CPUS=12 / 8
# (the per-rank CPU share of an 8-GPU node), plus the AV1 4K 2-pass rate accuracy.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-enttex}; mkdir -p $O
for cpus in 0 12 8; do
  TV_CPUS=$cpus timeout -k 10 300 python -u bench.py --content textured --no-4k --steps 6 --warmup 2 > $O/tex_c$cpus.log 2>&1 || { echo "tex $cpus failed"; tail -n 5 $O/tex_c$cpus.log; exit 1; }
  python3 -c "import json; r=json.loads([l for l in open('$O/tex_c$cpus.log') if l.startswith('{')][-1]); c=r['config']; print('textured cpus=$cpus', r['value'], c['psnr_y_db'], c['kbps_per_30fps_stream'], c['per_rank_cpu'][0])"
done
timeout -k 10 400 python -u bench.py --codec av1 --res 4k --kbps 20000 --steps 4 --warmup 2 > $O/av1_4k_2pass.log 2>&1 || { echo "av1 2pass failed"; tail -n 5 $O/av1_4k_2pass.log; exit 1; }
python3 -c "import json; r=json.loads([l for l in open('$O/av1_4k_2pass.log') if l.startswith('{')][-1]); c=r['config']; print('av1 4k 2pass', r['value'], c['kbps_error_pct'], c['rc_steps_actual_wanted_offset'])"
