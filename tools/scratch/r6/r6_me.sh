#!/bin/bash
# Round 6 k_inter_me A/B on one box: golden tests of the default kernel, alternating benches
# A = default vs B = $1 (env), then single-group kernel traces of both.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
T=${2:-r6_me}; O=gpurun_out/$T; mkdir -p $O; B="$1"
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu/ab_env.sh $T/ab "TV_NOP=1" "$B" --no-4k || exit 1
for v in A B; do
  E="TV_NOP=1"; [ $v = B ] && E="$B"
  env $E TV_ENGINE_GROUPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/g1_$v -o run -- python3 bench.py --no-4k --steps 3 --warmup 1 > $O/g1_$v.log 2>&1 || { echo "prof failed"; exit 1; }
  python3 tools/profsum.py $(find $O/g1_$v -name "*kernel_trace.csv" | head -1) --skip 0.4 > $O/g1_${v}_summary.txt 2>&1
  echo "== $v"; head -n 5 $O/g1_${v}_summary.txt
done
