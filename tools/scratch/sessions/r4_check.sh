#!/bin/bash
# Round-4 feature check: ingest / HBM-budget / benchmarked-shape GPU tests, the default
# bench (1080p + the in-process 4K pass), then the y4m file-ingest job (direct, scatter).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/${1:-r4check}; mkdir -p $O
fr=${2:-12288}
timeout -k 10 900 python -u -m pytest tests/test_ingest.py tests/test_hbm_budget.py tests/test_gpu_engine.py tests/test_parallel.py -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR" $O/pytest.log | tail -n 40; tail -n 3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 > $O/bench.log 2>&1 || { echo "bench failed"; tail -n 20 $O/bench.log; exit 1; }
echo "bench: $(grep '^{' $O/bench.log | tail -n 1 | cut -c1-2500)"
for m in direct scatter; do
  timeout -k 10 600 python -u bench.py --job --source y4m --job-mode $m --job-frames $fr > $O/job_y4m_$m.log 2>&1 || { echo "y4m $m failed"; tail -n 30 $O/job_y4m_$m.log; exit 1; }
  echo "y4m $m: $(grep '^{' $O/job_y4m_$m.log | tail -n 1 | cut -c1-3000)"
done
