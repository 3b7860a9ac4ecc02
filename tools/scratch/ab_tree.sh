#!/bin/bash
# Same-box A/B of two built trees: abbase/ (baseline copy) vs the repo, alternating.
# Usage: ab_tree.sh <tag> <bench args...>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp TV_NO_AUTOBUILD=1
tag=$1; shift
O=$PWD/gpurun_out/$tag; mkdir -p $O
for i in 1 2; do
  (cd abbase && PYTHONPATH=$PWD timeout -k 10 300 python -u bench.py "$@" > $O/base_$i.log 2>&1) || exit 1
  echo "base $i: $(tail -1 $O/base_$i.log | cut -c1-200 | grep -o '"value": [0-9.]*')"
  PYTHONPATH=$PWD timeout -k 10 300 python -u bench.py "$@" > $O/new_$i.log 2>&1 || exit 1
  echo "new  $i: $(tail -1 $O/new_$i.log | cut -c1-200 | grep -o '"value": [0-9.]*')"
done
