#!/bin/bash
# Round 6: instruction / wait counters of the GPU CABAC coders (lane and wave) on the 1080p
# bench with the GPU coder, one counter pass per run.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-r6entpmc}; mkdir -p $O
i=0
for coder in lanes wave; do
  i=$((i+1))
  TV_ENT_CODER=$coder timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O/p$i -o run -- python3 bench.py --no-4k --steps 1 --warmup 1 --batch 24 --gop 8 --entropy gpu > $O/p$i.log 2>&1 || { echo "pmc $coder failed"; tail -n 5 $O/p$i.log; exit 1; }
  echo "== $coder"
  python3 tools/pmcsum.py $(find $O/p$i -name "*counter_collection.csv" | head -1) k_ent_ac
done
