#!/bin/bash
# BD-rate of the default GPU engine against stored bench points of an earlier round
# (<anchor dir>/{smooth,textured}_test_q{22,27,32,37}.json, as written by rd_ab.sh),
# 1080p I P P P, QP 22/27/32/37, both contents.
# Usage: rd_vs.sh <tag> <anchor dir> ["<extra bench.py flags>"]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-rdvs}; A=${2:-profiles/r5_rd_cascade_1080p}; mkdir -p $O
for content in smooth textured; do
  for q in 22 27 32 37; do
    timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --qp $q --no-4k --content $content $3 > $O/${content}_q$q.log 2>&1 || { echo "$content q$q failed"; tail -n 5 $O/${content}_q$q.log; exit 1; }
    grep '^{' $O/${content}_q$q.log | tail -n 1 > $O/${content}_q$q.json
  done
  python - "$O" "$A" "$content" <<'PY'
import json, sys
sys.path.insert(0, ".")
from thinvids_amd.utils.bdrate import bd_rate
O, A, content = sys.argv[1:4]
qs = (22, 27, 32, 37)
a = [json.load(open(f"{A}/{content}_test_q{q}.json"))["config"] for q in qs]
t = [json.load(open(f"{O}/{content}_q{q}.json")) for q in qs]
print(content, "anchor", [(p["kbps_per_30fps_stream"], p["psnr_y_db"]) for p in a])
print(content, "now   ", [(p["config"]["kbps_per_30fps_stream"], p["config"]["psnr_y_db"]) for p in t], "fps", [p["value"] for p in t])
t = [p["config"] for p in t]
print("%s BD-rate now vs anchor: %.2f %%" % (content, bd_rate([p["kbps_per_30fps_stream"] for p in a], [p["psnr_y_db"] for p in a],
                                                           [p["kbps_per_30fps_stream"] for p in t], [p["psnr_y_db"] for p in t])))
PY
done
