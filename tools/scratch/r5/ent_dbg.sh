#!/bin/bash
# GPU entropy coder diagnostics: in-kernel counters (TV_ENT_DEBUG) and one PMC pass on the
# arithmetic coder kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-entdbg}; mkdir -p $O
TV_ENT_DEBUG=1 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-4k > $O/dbg_bench.log 2>&1
rc=$?; echo "dbg rc=$rc"; grep "tv entropy" $O/dbg_bench.log; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM SQ_INSTS_BRANCH --kernel-include-regex "k_ent_ac" --output-format csv -d $O/pmc -o run -- python3 bench.py --steps 1 --warmup 0 --no-4k > $O/pmc_bench.log 2>&1
rc=$?; echo "pmc rc=$rc"
python3 tools/pmcsum.py $(find $O/pmc -name "*counter_collection.csv" | head -1) 2>&1 | head -30
