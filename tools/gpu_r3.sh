#!/bin/bash
# Measurement batch: build, GPU tests, warm profiles (trace of the last steps only),
# ME ablations, batch-size sweep, SAO, 4K.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/${1:-r3}; mkdir -p $O
python -c "import __graft_entry__ as g; g.build()" > $O/build.log 2>&1 || { echo build failed; exit 1; }
timeout -k 10 600 python -m pytest tests -m gpu -q > $O/pytest_gpu.log 2>&1; echo "pytest rc=$?"; tail -n 3 $O/pytest_gpu.log
prof() {  # tag env args
  local tag=$1; shift; local envs=$1; shift
  env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag -o run -- python3 bench.py --steps 2 --warmup 2 "$@" > $O/$tag.log 2>&1 || { echo "prof $tag failed"; return 1; }
  echo "== $tag [$envs] $* : $(tail -n 1 $O/$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "fps")')"
  python3 tools/profsum.py $O/$tag/run_kernel_trace.csv --skip 0.55 --top 9
}
prof base "TV_X=0" && prof ab3 "TV_ME_ABLATE=3" && prof ab7 "TV_ME_ABLATE=7" && prof sao "TV_X=0" --sao && prof b32 "TV_X=0" --batch 32 || exit 1
for b in 8 16 32; do
  timeout -k 10 300 python bench.py --steps 4 --warmup 1 --batch $b > $O/bench_b$b.log 2>&1 || { echo "bench b$b failed"; exit 1; }
  echo "bench b$b: $(tail -n 1 $O/bench_b$b.log | cut -c1-600)"
done
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --res 4k --batch 8 > $O/bench_4k_b8.log 2>&1 && echo "4k b8: $(tail -n 1 $O/bench_4k_b8.log | cut -c1-600)"
