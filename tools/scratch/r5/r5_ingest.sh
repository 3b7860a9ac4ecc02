#!/bin/bash
# y4m job ingest: one DMA stream vs several (TV_INGEST_STREAMS), 1080p direct job
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-ingest}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for d in ${STREAMS:-1 2 4 1 4}; do
  TV_INGEST_STREAMS=$d timeout -k 10 300 python -u bench.py --job --source y4m > $O/y4m_d$d.log 2>&1
  rc=$?; echo "streams=$d rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/y4m_d$d.log; exit $rc; }
  grep '^{' $O/y4m_d$d.log | tail -1 > $O/y4m_d$d.json
  python3 -c "import json; r=json.load(open('$O/y4m_d$d.json')); c=r['config']; i=c['per_rank_ingest'][0]; s=c['rank0_spans_ms']; print('streams $d', r['value'], i['ingest_gb_per_s'], s['node_job.encode']['avg_ms'], s['node_job.load']['total_ms'])"
done
