#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/${1:-r4}; mkdir -p $O
python -c "import __graft_entry__ as g; g.build()" > $O/build.log 2>&1 || { echo build failed; exit 1; }
timeout -k 10 600 python -m pytest tests -m gpu -q > $O/pytest_gpu.log 2>&1; echo "pytest rc=$?"; tail -n 3 $O/pytest_gpu.log
pmc() {  # tag env counters
  local tag=$1 envs=$2 ctr=$3
  env $envs timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d $O/$tag -o run -- python3 bench.py --steps 1 --warmup 1 --gop 8 > $O/$tag.log 2>&1 || { echo "pmc $tag failed"; return 1; }
  echo "== pmc $tag [$envs]"; python3 tools/pmcsum.py $O/$tag/run_counter_collection.csv k_inter_me
}
C1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
pmc pmc_ab7 "TV_ME_ABLATE=7" "$C1" && pmc pmc_base "TV_X=0" "$C1" || exit 1
prof() {
  local tag=$1; shift; local envs=$1; shift
  env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag -o run -- python3 bench.py --steps 2 --warmup 2 "$@" > $O/$tag.log 2>&1 || { echo "prof $tag failed"; return 1; }
  echo "== $tag [$envs] $*"; python3 tools/profsum.py $O/$tag/run_kernel_trace.csv --skip 0.55 --top 12
}
prof sao "TV_X=0" --sao --batch 32 || exit 1
for args in "--batch 32" "--batch 32 --sao" "--batch 32 --gop 32" "--res 4k --batch 16"; do
  tag=$(echo "$args" | tr -d ' -')
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 $args > $O/bench_$tag.log 2>&1 || { echo "bench $args failed"; exit 1; }
  echo "bench $args: $(tail -n 1 $O/bench_$tag.log | cut -c1-900)"
done
