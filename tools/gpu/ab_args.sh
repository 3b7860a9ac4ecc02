#!/bin/bash
# Same-box A/B of two bench.py argument sets, alternating A B A B.
#   gpu_ab_args.sh TAG "ARGS_A" "ARGS_B"
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/$1; A=$2; B=$3; mkdir -p $O
for i in 1 2; do
  timeout -k 10 240 python3 -u bench.py $A > $O/A$i.log 2>&1 || { tail -5 $O/A$i.log; exit 1; }
  timeout -k 10 240 python3 -u bench.py $B > $O/B$i.log 2>&1 || { tail -5 $O/B$i.log; exit 1; }
  python3 -c "import json; a=json.loads(open('$O/A$i.log').read().strip().splitlines()[-1]); b=json.loads(open('$O/B$i.log').read().strip().splitlines()[-1]); print('A[$A]', a['value'], 'B[$B]', b['value'], 'B/A', round(b['value']/a['value'],4), 'psnr', a['config']['psnr_y_db'], b['config']['psnr_y_db'])"
done
