#!/bin/bash
# Same-box A/B of a runtime tuning knob: alternates `bench.py` runs with env A and env B.
#   gpu_ab_env.sh TAG "ENV_A" "ENV_B" [bench args]      e.g. "TV_ME_THREADS=256" "TV_ME_THREADS=384"
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/$1; A=$2; B=$3; shift 3; mkdir -p $O
for i in 1 2 3; do
  env $A timeout -k 10 200 python3 -u bench.py --steps 6 --warmup 2 "$@" > $O/A$i.log 2>&1 || { tail -5 $O/A$i.log; exit 1; }
  env $B timeout -k 10 200 python3 -u bench.py --steps 6 --warmup 2 "$@" > $O/B$i.log 2>&1 || { tail -5 $O/B$i.log; exit 1; }
  python3 -c "import json; a=json.loads(open('$O/A$i.log').read().strip().splitlines()[-1]); b=json.loads(open('$O/B$i.log').read().strip().splitlines()[-1]); print('$A', a['value'], '$B', b['value'], 'B/A', round(b['value']/a['value'],4))"
done
