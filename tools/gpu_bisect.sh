#!/bin/bash
# Run one GPU test in each pre-built variant tree under bisect/.  Usage: gpu_bisect.sh <test id>
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp TV_NO_AUTOBUILD=1
mkdir -p gpurun_out/bisect
t=${1:-"tests/test_gpu_engine.py"}
for d in . bisect/*; do
  n=$(basename $d); [ "$d" = . ] && n=HEAD
  (cd $d && PYTHONPATH=$PWD timeout -k 10 300 python -u -m pytest $t -q -x --timeout 120 --timeout-method thread -p no:cacheprovider) > gpurun_out/bisect/$n.log 2>&1
  rc=$?
  echo "$n rc=$rc $(tail -n 1 gpurun_out/bisect/$n.log)"
  [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] && exit 1
done
exit 0
