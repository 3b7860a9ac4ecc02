#!/bin/bash
# k_inter_me phase breakdown for round 6: single-group kernel traces with the timing-only
# TV_DIAG_ME_STOP knob (1: staging only, 2: + integer search, 3: + half-pel, unset: full)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-mephase}; mkdir -p $O
for s in 0 1 2 3; do
  TV_ENGINE_GROUPS=1 TV_DIAG_ME_STOP=$s timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/s$s -o run -- python3 bench.py --no-4k --steps 2 --warmup 1 > $O/s$s.log 2>&1
  rc=$?; echo "stop=$s rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/s$s.log; exit $rc; }
  python3 tools/kstats.py $(find $O/s$s -name "*kernel_stats.csv" | head -1) 40 | grep -E "k_inter_me|k_inter_recon" | tee $O/s$s.txt
done
