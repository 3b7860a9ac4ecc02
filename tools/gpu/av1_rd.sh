#!/bin/bash
# AV1 vs HEVC rate-distortion at the bench geometry (1080p, GOP 64, HEVC IPPP + SAO, AV1 at
# the matched q-index), QP 22/27/32/37, then the BD-rate of AV1 against HEVC.
# Usage: av1_rd.sh <tag> [content]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-av1rd}; mkdir -p $O
content=${2:-smooth}
for q in 22 27 32 37; do
  timeout -k 10 300 python -u bench.py --no-4k --steps 2 --warmup 1 --qp $q --content $content > $O/hevc_q$q.log 2>&1 || { echo "hevc q$q failed"; tail -n 5 $O/hevc_q$q.log; exit 1; }
  timeout -k 10 300 python -u bench.py --codec av1 --steps 2 --warmup 1 --qp $q --content $content > $O/av1_q$q.log 2>&1 || { echo "av1 q$q failed"; tail -n 5 $O/av1_q$q.log; exit 1; }
done
python - "$O" <<'PY'
import json, sys
sys.path.insert(0, ".")
from thinvids_amd.utils.bdrate import bd_rate
O = sys.argv[1]
cur = {}
for c in ("hevc", "av1"):
    pts = [json.loads([l for l in open(f"{O}/{c}_q{q}.log") if l.startswith("{")][-1]) for q in (22, 27, 32, 37)]
    cur[c] = ([p["config"]["kbps_per_30fps_stream"] for p in pts], [p["config"]["psnr_y_db"] for p in pts], [p["value"] for p in pts])
    print(c, "kbps", cur[c][0], "psnr", cur[c][1], "fps", cur[c][2])
print("BD-rate AV1 vs HEVC: %.2f %%" % bd_rate(cur["hevc"][0], cur["hevc"][1], cur["av1"][0], cur["av1"][1]))
json.dump(cur, open(f"{O}/rd.json", "w"))
PY
