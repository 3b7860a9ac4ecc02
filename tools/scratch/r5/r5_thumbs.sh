#!/bin/bash
# scene-cut thumbnail kernel: GPU tests, then the y4m job
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-thumbs}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_scenecut.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for k in 1 2; do
  timeout -k 10 300 python -u bench.py --job --source y4m > $O/y4m_$k.log 2>&1
  rc=$?; echo "y4m rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/y4m_$k.log; exit $rc; }
  grep '^{' $O/y4m_$k.log | tail -1 | python3 -c "import json,sys; r=json.load(sys.stdin); c=r['config']; print('y4m', r['value'], c['rank0_spans_ms']['node_job.encode']['avg_ms'])"
done
