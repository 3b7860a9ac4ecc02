#!/bin/bash
# Rate-distortion curves of the GPU engine at the bench geometry (1080p, GOP 64, SAO):
# I P P P vs hierarchical-B, QP 22/27/32/37, then the BD-rate.  Usage: gpu_rd.sh <tag> [content]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-rd}; mkdir -p $O
content=${2:-smooth}
for m in 1 8; do
  for q in 22 27 32 37; do
    timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --qp $q --bframes $m --content $content > $O/b${m}_q${q}.log 2>&1 || { echo "bench b$m q$q failed"; tail -n 5 $O/b${m}_q${q}.log; exit 1; }
    grep '^{' $O/b${m}_q${q}.log | tail -n 1 > $O/b${m}_q${q}.json
    python - "$O/b${m}_q${q}.json" <<'PY'
import json, sys
r = json.load(open(sys.argv[1])); c = r["config"]
print(f"bframes={c.get('bframes')} qp={sys.argv[1].split('_q')[1][:2]} fps={r['value']} psnr_y={c['psnr_y_db']} kbps={c['kbps_per_30fps_stream']}")
PY
  done
done
python - "$O" <<'PY'
import json, sys
sys.path.insert(0, ".")
from thinvids_amd.utils.bdrate import bd_rate
O = sys.argv[1]
cur = {}
for m in (1, 8):
    pts = [json.load(open(f"{O}/b{m}_q{q}.json"))["config"] for q in (22, 27, 32, 37)]
    cur[m] = ([p["kbps_per_30fps_stream"] for p in pts], [p["psnr_y_db"] for p in pts])
print("BD-rate B8 vs IPPP: %.2f %%" % bd_rate(cur[1][0], cur[1][1], cur[8][0], cur[8][1]))
PY
