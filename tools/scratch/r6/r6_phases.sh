#!/bin/bash
# Round 6 phase breakdown of k_inter_me (TV_DIAG_ME_STOP 1 staging, 2 + integer, 3 + half-pel)
# and k_sao_decide (TV_DIAG_SAO_STOP 1 staging, 2 + statistics, 3 + decision): single-group
# kernel traces, timing-only knobs (decisions degrade).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-r6phase}; mkdir -p $O
for spec in base:TV_NOP=1 me1:TV_DIAG_ME_STOP=1 me2:TV_DIAG_ME_STOP=2 me3:TV_DIAG_ME_STOP=3 sao1:TV_DIAG_SAO_STOP=1 sao2:TV_DIAG_SAO_STOP=2 sao3:TV_DIAG_SAO_STOP=3; do
  n=${spec%%:*}; e=${spec#*:}
  env $e TV_ENGINE_GROUPS=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n -o run -- python3 bench.py --no-4k --steps 2 --warmup 1 > $O/$n.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$n rc=$rc"; tail -5 $O/$n.log; exit $rc; }
  python3 tools/kstats.py $(find $O/$n -name "*kernel_stats.csv" | head -1) 40 | grep -E "k_inter_me|k_sao_decide" | sed "s/^/$n /" | tee $O/$n.txt
done
