#!/bin/bash
# Textured-content checks: GPU == golden tests (HEVC + AV1), benches on the textured variant,
# and the fetch-thread sync mode A/B.  Usage: gpu_textured.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/${1:-tex}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_engine.py tests/test_av1_codec.py -m gpu -k "textured" -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -n 40 $O/pytest.log; exit 1; }
tail -n 4 $O/pytest.log
for args in "--content textured" "--codec av1 --content textured" ; do
  t=$(echo "$args" | tr -d ' -')
  timeout -k 10 400 python bench.py --steps 3 --warmup 1 $args > $O/bench_$t.log 2>&1 || { echo "bench $args failed"; tail -n 20 $O/bench_$t.log; exit 1; }
  echo "bench [$args]: $(tail -n 1 $O/bench_$t.log | cut -c1-1500)"
done
TV_SYNC_MODE=poll timeout -k 10 300 python bench.py --steps 3 --warmup 1 > $O/bench_poll.log 2>&1 && echo "poll: $(tail -n 1 $O/bench_poll.log | cut -c1-1500)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 2 --warmup 1 > $O/prof_bench.log 2>&1 || { echo "prof failed"; tail -n 20 $O/prof_bench.log; exit 1; }
python3 tools/kstats.py $(find $O/prof -name "*kernel_stats.csv" | head -1) 16
