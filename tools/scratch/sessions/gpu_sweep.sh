#!/bin/bash
# Engine shape sweep at the default config: stream groups x segments per GPU.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-sweep}; mkdir -p $O
for cfg in "2 48" "3 48" "2 64" "3 63" "2 48"; do
  set -- $cfg
  TV_ENGINE_GROUPS=$1 timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --batch $2 > $O/g$1_b$2.log 2>&1 || { echo "g$1 b$2 failed"; exit 1; }
  python -c "import json; r=json.loads([l for l in open('$O/g$1_b$2.log') if l.startswith('{')][-1]); print('groups=$1 batch=$2', r['value'], r['config']['per_rank_cpu'][0]['busy_cores'])"
done
