#!/bin/bash
# BD-rate of the default GPU engine against the same engine with coding tools switched off
# by bench.py flags (e.g. "--no-rqt --no-pintra"), 1080p I P P P, QP 22/27/32/37, both contents.
# Usage: rd_ab.sh <tag> "<bench.py flags of the anchor>"
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-rdab}; mkdir -p $O
for content in smooth textured; do
  for v in anchor test; do
    for q in 22 27 32 37; do
      if [ $v = anchor ]; then extra="$2"; else extra=""; fi
      timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --qp $q --no-4k --content $content $extra > $O/${content}_${v}_q$q.log 2>&1 || { echo "$content $v q$q failed"; tail -n 5 $O/${content}_${v}_q$q.log; exit 1; }
      grep '^{' $O/${content}_${v}_q$q.log | tail -n 1 > $O/${content}_${v}_q$q.json
    done
  done
  python - "$O" "$content" <<'PY'
import json, sys
sys.path.insert(0, ".")
from thinvids_amd.utils.bdrate import bd_rate
O, content = sys.argv[1], sys.argv[2]
pts = {v: [json.load(open(f"{O}/{content}_{v}_q{q}.json"))["config"] for q in (22, 27, 32, 37)] for v in ("anchor", "test")}
for v in ("anchor", "test"):
    print(content, v, [(p["kbps_per_30fps_stream"], p["psnr_y_db"]) for p in pts[v]])
a, t = pts["anchor"], pts["test"]
print("%s BD-rate default vs anchor: %.2f %%" % (content, bd_rate([p["kbps_per_30fps_stream"] for p in a], [p["psnr_y_db"] for p in a],
                                                               [p["kbps_per_30fps_stream"] for p in t], [p["psnr_y_db"] for p in t])))
PY
done
