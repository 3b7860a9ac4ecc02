#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/${1:-r5}; mkdir -p $O
python -c "import __graft_entry__ as g; g.build()" > $O/build.log 2>&1 || { echo build failed; exit 1; }
timeout -k 10 600 python -m pytest tests -m gpu -q -x > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -n 30 $O/pytest_gpu.log; exit 1; }
tail -n 2 $O/pytest_gpu.log
prof() {
  local tag=$1; shift; local envs=$1; shift
  env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag -o run -- python3 bench.py --steps 2 --warmup 2 "$@" > $O/$tag.log 2>&1 || { echo "prof $tag failed"; return 1; }
  echo "== $tag [$envs] $*"; python3 tools/profsum.py $O/$tag/run_kernel_trace.csv --skip 0.55 --top 14
}
prof b32 "TV_X=0" && prof b32sao "TV_X=0" --sao || exit 1
for args in "" "--sao" "--res 4k"; do
  tag=b$(echo "$args" | tr -d ' -')
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 $args > $O/bench_$tag.log 2>&1 || { echo "bench $args failed"; exit 1; }
  echo "bench [$args]: $(tail -n 1 $O/bench_$tag.log | cut -c1-1000)"
done
