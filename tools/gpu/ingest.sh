#!/bin/bash
# File-ingest check: ingest GPU tests, then the end-to-end job bench on a y4m source
# (direct and scatter) next to the synthetic-source job.  Usage: ingest.sh <tag> [frames]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-ingest}; mkdir -p $O
fr=${2:-6144}
{ df -h /tmp; free -g; nproc; python -c "import os; print('affinity', len(os.sched_getaffinity(0)))"; } > $O/box.txt 2>&1
cat $O/box.txt
timeout -k 10 600 python -u -m pytest tests/test_ingest.py tests/test_parallel.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for m in direct scatter; do
  timeout -k 10 600 python -u bench.py --job --source y4m --job-mode $m --job-frames $fr > $O/job_y4m_$m.log 2>&1 || { echo "y4m $m failed"; tail -n 30 $O/job_y4m_$m.log; exit 1; }
  echo "y4m $m: $(grep '^{' $O/job_y4m_$m.log | tail -n 1 | cut -c1-2500)"
done
timeout -k 10 600 python -u bench.py --job > $O/job_synth.log 2>&1 || { echo "synth job failed"; tail -n 30 $O/job_synth.log; exit 1; }
echo "synth: $(grep '^{' $O/job_synth.log | tail -n 1 | cut -c1-1500)"
