#!/bin/bash
# bench sweep over engine stream groups and batch sizes
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/${1:-sweep2}; mkdir -p $O
run() { # groups res batch
  TV_ENGINE_GROUPS=$1 timeout -k 10 200 python bench.py --steps 3 --warmup 2 --res $2 --batch $3 > $O/g$1_$2_b$3.log 2>&1 || { echo "fail $*"; return 1; }
  python -c "import json;d=json.loads(open('$O/g$1_$2_b$3.log').read().strip().splitlines()[-1]);print('groups=$1 $2 b$3', d['value'], d['config']['last_step_entropy_cpu_ms'])"
}
run 1 1080p 32 && run 3 1080p 33 && run 4 1080p 32 && run 2 1080p 48 && run 4 1080p 64 && run 2 4k 24 && run 4 4k 16 && run 4 4k 32
